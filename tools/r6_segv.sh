#!/bin/bash
# Round 6: the driver's bench command (compact line + detail file), then the
# rocprofv3 kernel-trace run that faulted at exit in round 5, with the
# library's fault tracer on (MBFT_SEGV_TRACE=1: frames as module + offset).
# The traced run is last: a fault ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --detail-out $O/detail.json > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
wc -c $O/bench.json
MBFT_SEGV_TRACE=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --steps 20 --no-extra-lines --no-adversarial --c3-requests 0 --no-cpu-baseline --detail-out $O/kt_detail.json > $O/kt_bench.json 2> $O/kt.err
rc=$?
echo "[r6_segv] traced run rc $rc"
grep -A40 "mbft segv trace" $O/kt.err | head -80
exit 0

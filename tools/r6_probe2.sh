#!/bin/bash
# Round 6: the driver's bench command (sleeping resident wait, resident
# interference line), the same with the round-5 spinning wait
# (MBFT_RESIDENT_SLEEP=0), then the rocprofv3 kernel-trace run whose exit
# faulted in round 5 (CU-masked stream now destroyed at exit).  The traced
# run is last: a fault ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --detail-out $O/detail.json > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
wc -c $O/bench.json
MBFT_RESIDENT_SLEEP=0 timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-adversarial --c3-requests 0 --detail-out $O/detail_spin.json > $O/bench_spin.json 2> $O/bench_spin.err || { tail -30 $O/bench_spin.err; exit 1; }
MBFT_SEGV_TRACE=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --steps 20 --no-extra-lines --no-adversarial --c3-requests 0 --no-cpu-baseline --detail-out $O/kt_detail.json > $O/kt_bench.json 2> $O/kt.err
rc=$?
echo "[r6_probe2] traced run rc $rc"
grep -A30 "mbft segv trace" $O/kt.err | head -40
exit 0

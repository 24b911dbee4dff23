#!/bin/bash
# Round 6: the C3 message kernels' roofline from a rocprofv3 kernel trace of
# tools/c3_probe.py (after the convergent k_msg_cands / k_msg_calls), then
# the driver's bench command.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6c3}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 tools/c3_probe.py 16384 > $O/c3.json 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
K=$(find $O/kt -name "*kernel_trace.csv" | head -1)
python3 tools/trace_summary.py "$K" > $O/c3_kt_summary.json || exit 1
rm -f "$K"
python3 tools/msg_kernel_roofline.py $O/c3_kt_summary.json $O/msg_kernels_roofline.json || exit 1
cat $O/msg_kernels_roofline.json | head -c 1500; echo
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --detail-out $O/detail.json > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
head -c 700 $O/bench.json; echo
echo "[r6_c3roof] done"

#!/bin/bash
# Round 6: k_verify_quads (an item per lane quad) -- its GPU tests, then
# small-batch and device-layer latency A/Bs against lane pairs (same box),
# then the C3 message kernels' roofline trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6q}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
MBFT_QUADS=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_msgdev.py tests/test_gpu_small_check.py tests/test_gpu_check_coalesce.py > $O/pytest_q.log 2>&1 || { tail -40 $O/pytest_q.log; exit 1; }
tail -1 $O/pytest_q.log
run() {  # tag, env...
  local tag=$1; shift
  env "$@" SMALL_SIZES=300,512,640,768,1024,2048,4096 timeout -k 10 300 python3 tools/small_batch_probe.py > $O/small_$tag.json 2> $O/small_$tag.err || { tail -20 $O/small_$tag.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/small_$tag.json')); print('$tag', {k:v['p50_us'] for k,v in d['sizes'].items()})"
  env "$@" LOWLOAD_SIZES=512,1024,2048,4096 LOWLOAD_NREQ=1024 LOWLOAD_SMALL_MAX=0 timeout -k 10 300 python3 tools/lowload_probe.py > $O/lowload_$tag.json 2> $O/lowload_$tag.err || { tail -20 $O/lowload_$tag.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/lowload_$tag.json'))
print('$tag', {k:round(v['p50_us'],1) for k,v in d['go_default']['small_route'].items()})"
}
run pairs MBFT_X=1 && run quads MBFT_QUADS=1 && run quads_nosplit MBFT_QUADS=1 MBFT_SPLIT_PLANES_MAX=0 && run pairs2 MBFT_X=1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 tools/c3_probe.py 16384 > $O/c3.json 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
K=$(find $O/kt -name "*kernel_trace.csv" | head -1)
python3 tools/trace_summary.py "$K" > $O/c3_kt_summary.json || exit 1
rm -f "$K"
python3 tools/msg_kernel_roofline.py $O/c3_kt_summary.json $O/msg_kernels_roofline.json || exit 1
head -c 1200 $O/msg_kernels_roofline.json; echo
echo "[r6_quads] done"

#!/bin/bash
# Round 6: the small / mid-size verify forms as defaults -- the GPU tests
# that run them, then the small-batch and device-layer latencies against
# round 5's form (pairs, per-lane s^-1).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6p3}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_msgdev.py tests/test_gpu_multi_msg.py tests/test_gpu_check_coalesce.py tests/test_gpu_small_check.py tests/test_gpu_replies_go.py tests/test_gpu_configs.py tests/test_gpu_authen.py tests/test_gpu_failures.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 tools/small_batch_probe.py > $O/small_$tag.json 2> $O/small_$tag.err || { tail -20 $O/small_$tag.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/small_$tag.json')); print('$tag', {k:v['p50_us'] for k,v in d['sizes'].items()})"
  env "$@" LOWLOAD_SIZES=512,1024,2048,4096 LOWLOAD_NREQ=1024 LOWLOAD_SMALL_MAX=0 timeout -k 10 300 python3 tools/lowload_probe.py > $O/lowload_$tag.json 2> $O/lowload_$tag.err || { tail -20 $O/lowload_$tag.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/lowload_$tag.json'))
print('$tag', {k:round(v['p50_us'],1) for k,v in d['go_default']['small_route'].items()})"
}
SMALL_SIZES=300,512,640,768,1024,2048,4096 run default MBFT_X=1 && SMALL_SIZES=300,512,640,768,1024,2048,4096 run r5form MBFT_SPLIT_PLANES_MAX=0 MBFT_PAIRS_PLANES=0 && SMALL_SIZES=300,512,640,768,1024,2048,4096 run default2 MBFT_X=1 || exit 1
echo "[r6_planes3] done"

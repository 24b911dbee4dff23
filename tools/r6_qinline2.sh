#!/bin/bash
# Round 6: inline lane quads as the default -- the small-batch / message GPU
# tests, then the split-planes cutoff (MBFT_SPLIT_PLANES_MAX) against the
# quads at 257-768 items.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6qi2}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_msgdev.py tests/test_gpu_small_check.py tests/test_gpu_check_coalesce.py tests/test_gpu_multi_msg.py tests/test_gpu_resident.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # tag, env...
  local tag=$1; shift
  env "$@" SMALL_SIZES=260,300,400,512,640,768 timeout -k 10 300 python3 tools/small_batch_probe.py > $O/small_$tag.json 2> $O/small_$tag.err || { tail -20 $O/small_$tag.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/small_$tag.json')); print('$tag', {k:v['p50_us'] for k,v in d['sizes'].items()})"
}
run split512 MBFT_X=1 && run quads MBFT_SPLIT_PLANES_MAX=0 && run split512b MBFT_X=1 && run quadsb MBFT_SPLIT_PLANES_MAX=0 || exit 1
echo "[r6_qinline2] done"

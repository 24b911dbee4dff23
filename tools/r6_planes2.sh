#!/bin/bash
# Round 6: small / mid-size verify forms, same box: pairs with per-lane s^-1,
# pairs reading the batched per-wave s^-1 planes, and the default (planes +
# k_verify_split up to MBFT_SPLIT_PLANES_MAX items, pairs above).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6p2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_msgdev.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
MBFT_PAIRS_PLANES=1 MBFT_SPLIT_PLANES_MAX=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "small_batches or lane_and_batched" > $O/pytest_pp.log 2>&1 || { tail -40 $O/pytest_pp.log; exit 1; }
tail -1 $O/pytest_pp.log
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 tools/small_batch_probe.py > $O/small_$tag.json 2> $O/small_$tag.err || { tail -20 $O/small_$tag.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/small_$tag.json')); print('$tag', {k:v['p50_us'] for k,v in d['sizes'].items()})"
  env "$@" LOWLOAD_SIZES=256,512,1024,2048,4096 LOWLOAD_NREQ=1024 LOWLOAD_SMALL_MAX=0 timeout -k 10 300 python3 tools/lowload_probe.py > $O/lowload_$tag.json 2> $O/lowload_$tag.err || { tail -20 $O/lowload_$tag.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/lowload_$tag.json'))
print('$tag', {k:round(v['p50_us'],1) for k,v in d['go_default']['small_route'].items()})"
}
run pairs MBFT_SPLIT_PLANES_MAX=0 && run pairs_planes MBFT_SPLIT_PLANES_MAX=0 MBFT_PAIRS_PLANES=1 && run default MBFT_X=1 && run default_pp MBFT_PAIRS_PLANES=1 && run pairs2 MBFT_SPLIT_PLANES_MAX=0 || exit 1
echo "[r6_planes2] done"

#!/bin/bash
# Round 6: k_verify_quads with the s^-1 by each wave (MBFT_QUADS_INLINE=1)
# against the planes kernel first -- tests under the env, then A/Bs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6qi}
mkdir -p $O
MBFT_QUADS_INLINE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_msgdev.py tests/test_gpu_small_check.py > $O/pytest_qi.log 2>&1 || { tail -40 $O/pytest_qi.log; exit 1; }
tail -1 $O/pytest_qi.log
run() {  # tag, env...
  local tag=$1; shift
  env "$@" SMALL_SIZES=300,512,768,1024,2048,4096 timeout -k 10 300 python3 tools/small_batch_probe.py > $O/small_$tag.json 2> $O/small_$tag.err || { tail -20 $O/small_$tag.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/small_$tag.json')); print('$tag', {k:v['p50_us'] for k,v in d['sizes'].items()})"
  env "$@" LOWLOAD_SIZES=1024,2048,4096 LOWLOAD_NREQ=1024 LOWLOAD_SMALL_MAX=0 timeout -k 10 300 python3 tools/lowload_probe.py > $O/lowload_$tag.json 2> $O/lowload_$tag.err || { tail -20 $O/lowload_$tag.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/lowload_$tag.json'))
print('$tag', {k:round(v['p50_us'],1) for k,v in d['go_default']['small_route'].items() if 'messages' in k})"
}
run planes MBFT_X=1 && run inline MBFT_QUADS_INLINE=1 && run planes2 MBFT_X=1 && run inline2 MBFT_QUADS_INLINE=1 || exit 1
echo "[r6_qinline] done"

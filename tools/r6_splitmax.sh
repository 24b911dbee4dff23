#!/bin/bash
# Round 6: (R6_SUITE set: the whole GPU suite first) k_verify_split past
# 256 items (MBFT_SPLIT_MAX=1024) against the default (lane quads), same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6sm}
mkdir -p $O
if [ -n "$R6_SUITE" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
run() {  # tag, env...
  local tag=$1; shift
  env "$@" SMALL_SIZES=256,320,384,512,640,768,1024 timeout -k 10 300 python3 tools/small_batch_probe.py > $O/small_$tag.json 2> $O/small_$tag.err || { tail -20 $O/small_$tag.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/small_$tag.json')); print('$tag', {k:v['p50_us'] for k,v in d['sizes'].items()})"
}
run split768 MBFT_SPLIT_MAX=1024 && run dflt MBFT_X=1 && run split768b MBFT_SPLIT_MAX=1024 && run dfltb MBFT_X=1 || exit 1
echo "[r6_splitmax] done"

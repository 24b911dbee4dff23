#!/bin/bash
# Round 6: GPU tests of the resident paths, then the driver's bench command.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6d}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_resident.py tests/test_gpu_small_check.py tests/test_gpu_replies_go.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --detail-out $O/detail.json > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
wc -c $O/bench.json

if [ -n "$R6RAMP" ]; then
  timeout -k 10 300 python3 tools/ramp_probe.py > $O/ramp.jsonl 2> $O/ramp.err || { tail -20 $O/ramp.err; exit 1; }
  cat $O/ramp.jsonl
fi
echo "[r6_check] done"

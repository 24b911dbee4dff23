#!/bin/bash
# C3 device message layer: two-stage verify split sweep (tools/c3_probe.py,
# MBFT_MSG_VERIFY_SPLIT = the first stage's last chunk, -1 = one stage), two
# alternating passes, after the message-layer tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-sp}
timeout -k 10 600 python -u -m pytest tests/test_gpu_msgdev.py tests/test_gpu_configs.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
for pass in 1 2; do
  for sp in -1 3 2 1; do
    out=$(MBFT_MSG_VERIFY_SPLIT=$sp timeout -k 10 240 python tools/c3_probe.py 16384 2>> gpurun_out/c3split_$TAG.err) || exit 1
    echo "{\"split\": $sp, \"pass\": $pass, \"r\": $out}" >> gpurun_out/c3split_$TAG.jsonl
    echo "split $sp: $(python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(round(d['messages_per_s']/1e6,1), 'M/s', round(d['ms'],3), 'ms')" "$out")"
  done
done

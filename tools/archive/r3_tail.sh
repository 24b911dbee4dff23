#!/bin/bash
# Authenticator-level tail A/B on the GPU box: the GPU-decode path
# (tools/auth_level_probe.py pinned, 1M C2 calls, W = 29, 10 reps) over the
# chunk-plan settings below, two alternating passes; one JSON line per run in
# gpurun_out/tail_$TAG.jsonl.  Then the authenticator gate tests.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-t1}
CFGS=("MBFT_TAIL_PRIO=0"
      "MBFT_TAIL_PRIO=1"
      "MBFT_TAIL_PRIO=1 MBFT_TAIL_DIV=8"
      "MBFT_TAIL_PRIO=1 MBFT_TAIL_DIV=8 MBFT_TAIL_LOCAL=2")
for pass in 1 2; do
  for cfg in "${CFGS[@]}"; do
    out=$(env $cfg MBFT_PROBE_FORM=pinned MBFT_PROBE_WINDOW=29 timeout -k 10 200 \
      python tools/auth_level_probe.py 1048576 10 2>> gpurun_out/tail_$TAG.err) || exit 1
    echo "{\"cfg\": \"$cfg\", \"pass\": $pass, \"r\": $out}" >> gpurun_out/tail_$TAG.jsonl
    echo "$cfg p50 $(python3 -c "import json,sys; print(round(json.loads(sys.argv[1])['p50_ms'],3))" "$out")"
  done
done
MBFT_TAIL_PRIO=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_authen.py tests/test_c1.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log

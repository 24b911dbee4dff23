#!/bin/bash
# Authenticator-level sweep on the GPU box (tools/auth_level_probe.py, 1M C2
# calls, 8 reps each) over "form chunk copy_streams" configs; one JSON line
# per config in gpurun_out/auth_sweep.jsonl, stage traces in .err.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -n "$MBFT_SWEEP_FILE" ]; then mapfile -t CFGS < "$MBFT_SWEEP_FILE"; else CFGS=("items 131072 1" "items 131072 2" "pinned 131072 1" "pinned 131072 2" "pinned 262144 2"); fi
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  echo "cfg $cfg" >> gpurun_out/auth_sweep.err
  out=$(MBFT_PROBE_FORM=$1 MBFT_BATCH_CHUNK=$2 MBFT_COPY_STREAMS=$3 MBFT_STAGE_TRACE=1 \
    timeout -k 10 120 python tools/auth_level_probe.py 1048576 8 2>> gpurun_out/auth_sweep.err) || exit 1
  echo "{\"cfg\": \"$cfg\", \"r\": $out}" >> gpurun_out/auth_sweep.jsonl
done

#!/bin/bash
# Authenticator-level probe on the GPU box (tools/auth_level_probe.py) over
# host-thread / chunk settings; results in
# gpurun_out/auth_probe.jsonl, the library's per-batch stage trace in
# gpurun_out/auth_probe.err.  Config = "threads chunk".
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
CFGS=(${MBFT_PROBE_CFGS:-"16 131072" "16 262144" "16 524288" "16 131072" "16 262144"})
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  echo "cfg $cfg" >> gpurun_out/auth_probe.err
  MBFT_HOST_THREADS=$1 MBFT_BATCH_CHUNK=$2 MBFT_STAGE_TRACE=1 \
    timeout -k 10 120 python tools/auth_level_probe.py 1048576 8 >> gpurun_out/auth_probe.jsonl 2>> gpurun_out/auth_probe.err || exit 1
done

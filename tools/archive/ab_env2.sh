#!/bin/bash
# Same-box A/B of an environment setting: bench.py (headline only) alternately
# with A="$2" and B="$3" (env assignments, e.g. MBFT_VERIFY_WAVES=4), twice
# each; one JSON summary line per run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=$1; A=$2; B=$3; STEPS=${4:-200}
for rep in 1 2; do
  for cfg in "$A" "$B"; do
    env $cfg timeout -k 10 300 python bench.py --steps $STEPS --warmup 20 --no-adversarial --c3-requests 0 \
      --no-extra-lines --no-cpu-baseline --no-peak-run > gpurun_out/ab_$TAG.json 2> gpurun_out/ab_$TAG.err || exit 1
    python3 -c "
import json,sys; d=json.load(open('gpurun_out/ab_$TAG.json'))
print(json.dumps({'cfg': sys.argv[1], 'rep': $rep, 'value_M': round(d['value']/1e6,1), 'ms_per_step': round(d['ms_per_step'],4),
 'k_verify_ms': round(d['kernel_ms']['k_verify'],4), 'dev_p50_ms': round(d['p50_batch_latency_device_ms'],4)}))" "$cfg" | tee -a gpurun_out/ab_$TAG.jsonl
  done
done

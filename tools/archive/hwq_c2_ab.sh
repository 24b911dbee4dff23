#!/bin/bash
# C2 pipeline vs hardware queues per process (GPU_MAX_HW_QUEUES), alternating
# on one box (QUEUES, default "4 3 4 3 4 3").
set -o pipefail
k=0
for q in ${QUEUES:-4 3 4 3 4 3}; do
  k=$((k+1))
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-peak-run --no-adversarial --c3-requests 0 --no-extra-lines > gpurun_out/hwq2_${q}_$k.json 2> gpurun_out/hwq2_${q}_$k.err || { tail -5 gpurun_out/hwq2_${q}_$k.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/hwq2_${q}_$k.json'))
print('q=$q', round(d['value']/1e6,1), round(d['ms_per_step'],4), 'k_verify', round(d['kernel_ms']['k_verify'],4), 'dev', round(d['p50_batch_latency_device_ms'],4), 'auth', round(d['p50_batch_latency_ms'],3))"
done

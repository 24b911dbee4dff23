#!/bin/bash
# k_verify waves per SIMD A/B (MBFT_VERIFY_WAVES 3 vs 2) on one box: C2 steady
# state and the isolated launch (bench kernel_ms), alternating, twice.
set -o pipefail
for rep in 1 2; do
  for w in 3 2; do
    MBFT_VERIFY_WAVES=$w timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-peak-run --no-adversarial --c3-requests 0 --no-extra-lines > gpurun_out/waves_ab_${w}_$rep.json 2> gpurun_out/waves_ab_${w}_$rep.err || { tail -5 gpurun_out/waves_ab_${w}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/waves_ab_${w}_$rep.json'));print('waves=$w rep=$rep', round(d['value']/1e6,1), round(d['ms_per_step'],4), 'k_verify', round(d['kernel_ms']['k_verify'],4), 'dev', round(d['p50_batch_latency_device_ms'],4), 'frac', round(d['roofline']['frac'],4))"
  done
done

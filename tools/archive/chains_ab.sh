#!/bin/bash
# Level-0 chain kernels, two chains per thread (default) vs one
# (MBFT_NINV_CHAINS=1): the s^-1 parity test for both, then the C2 pipeline
# alternating on one box.
set -o pipefail
for c in 2 1; do
  MBFT_NINV_CHAINS=$c timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "inverse_forms" > gpurun_out/chains_test_$c.log 2>&1 || { tail -20 gpurun_out/chains_test_$c.log; exit 1; }
  tail -1 gpurun_out/chains_test_$c.log
done
for rep in 1 2 3; do
  for c in 2 1; do
    MBFT_NINV_CHAINS=$c timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-peak-run --no-adversarial --c3-requests 0 --no-extra-lines > gpurun_out/chains_ab_${c}_$rep.json 2> gpurun_out/chains_ab_${c}_$rep.err || { tail -5 gpurun_out/chains_ab_${c}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/chains_ab_${c}_$rep.json'));print('chains=$c rep=$rep', round(d['value']/1e6,1), round(d['ms_per_step'],4), 'inv_span', round(d['kernel_ms']['batched_inverse_span_overlapped'],4))"
  done
done

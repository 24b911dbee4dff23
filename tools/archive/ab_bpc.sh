#!/bin/bash
# A/B: k_verify grid cap (blocks per CU) -- 0 = uncapped.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  for b in 0 2 3; do
    MBFT_VERIFY_BPC=$b timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-peak-run --latency-reps 3 > gpurun_out/ab_b${b}_r${rep}.json 2> gpurun_out/ab_b${b}_r${rep}.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ab_b${b}_r${rep}.json'));print('bpc',$b,'value %.1fM'%(d['value']/1e6),'ms/step %.3f'%d['ms_per_step'],d['kernel_ms'])"
  done
done

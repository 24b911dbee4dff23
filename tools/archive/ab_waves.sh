#!/bin/bash
# A/B: k_verify at 3 vs 4 waves/SIMD, interleaved in separate processes (env var
# is read once per process).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  for w in 3 4; do
    echo "[ab] waves=$w rep=$rep"
    MBFT_VERIFY_WAVES=$w timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-peak-run --latency-reps 3 > gpurun_out/ab_w${w}_r${rep}.json 2> gpurun_out/ab_w${w}_r${rep}.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ab_w${w}_r${rep}.json'));print('waves',$w,'value %.1fM'%(d['value']/1e6),'kverify',d['kernel_ms'])"
  done
done

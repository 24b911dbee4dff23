#!/bin/bash
# Same-box A/B of the level-0 s^-1 chain length (MBFT_NINV_CHAIN0).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for c in ${MBFT_AB_CHAIN0:-16 64 32 128}; do
  MBFT_NINV_CHAIN0=$c timeout -k 10 600 python bench.py --steps 40 --warmup 10 --no-cpu-baseline --c3-requests 0 --no-adversarial > gpurun_out/bench_chain$c.json 2> gpurun_out/bench_chain$c.err || exit 1
done

#!/bin/bash
# k_verify time per mixed addition across comb windows (cache-resident vs
# 258 GiB tables): one short bench per window pair.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for w in ${MBFT_PROBE_WINDOWS:-16 22 26 29}; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --g-window $w --q-window $w --no-cpu-baseline \
    --c3-requests 0 --no-adversarial > gpurun_out/bench_w$w.json 2> gpurun_out/bench_w$w.err || exit 1
done

#!/bin/bash
# Same-box A/B of the bench's caller-stream count (batches in flight).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for k in ${MBFT_AB_STREAMS:-3 2 4}; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 --streams $k --no-cpu-baseline --c3-requests 0 --no-adversarial > gpurun_out/bench_streams$k.json 2> gpurun_out/bench_streams$k.err || exit 1
done

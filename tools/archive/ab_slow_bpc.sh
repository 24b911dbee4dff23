#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/pytest_parity_r2i.log 2>&1 || exit 1
for b in 4 1 2; do
  MBFT_SLOW_BPC=$b timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --c3-requests 0 > gpurun_out/bench_r2i_sbpc$b.json 2> gpurun_out/bench_r2i_sbpc$b.err || exit 1
done

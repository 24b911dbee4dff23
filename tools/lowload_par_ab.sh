#!/bin/bash
# Same-box A/B of the host part's worker threshold for small checks
# (MBFT_PARALLEL_MIN: 4096 = the calling thread only below 4096 calls).
mkdir -p gpurun_out
for pm in 4096 256; do
  i=$((i+1))
  MBFT_PARALLEL_MIN=$pm LOWLOAD_SIZES=64,256,512 LOWLOAD_NREQ=256 timeout -k 10 300 python -u tools/lowload_probe.py > gpurun_out/ll_pm${pm}_$i.json 2> gpurun_out/ll_pm${pm}_$i.err || { tail -5 gpurun_out/ll_pm${pm}_$i.err; exit 1; }
done

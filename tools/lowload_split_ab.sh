#!/bin/bash
# Same-box A/B of the split kernel's item limit (MBFT_SPLIT_MAX) for small
# checks of 257-512 unique calls (default 256: k_verify_pairs past it).
mkdir -p gpurun_out
for sm in 256 512 1024; do
  MBFT_STAGE_TRACE=1 MBFT_SPLIT_MAX=$sm LOWLOAD_SIZES=512 LOWLOAD_NREQ=256 timeout -k 10 300 python -u tools/lowload_probe.py > gpurun_out/ll_split$sm.json 2> gpurun_out/ll_split$sm.err || { tail -5 gpurun_out/ll_split$sm.err; exit 1; }
  grep "n=512 T=1" gpurun_out/ll_split$sm.err | tail -2
done

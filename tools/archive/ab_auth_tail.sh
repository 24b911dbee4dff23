#!/bin/bash
# Same-box A/B of the authenticator level (tools/auth_level_probe.py, GPU
# decode of 1M C2 calls in library page-locked buffers, W = 29) between the
# in-tree library and minbft_amd/libminbft_amd_base.so (tools/ab_build.sh
# REV base), three alternating reps.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2 3; do
  for L in "" "$PWD/minbft_amd/libminbft_amd_base.so"; do
    MBFT_LIB_PATH=$L MBFT_PROBE_FORM=pinned MBFT_PROBE_WINDOW=29 timeout -k 10 200 python tools/auth_level_probe.py 1048576 10 > gpurun_out/aa.json 2>gpurun_out/aa.err || exit 1
    echo "${L:-new} $(cut -c1-160 gpurun_out/aa.json)"
  done
done

#!/bin/bash
# Same-box A/B of single VerifyMessageAuthenTag calls (tools/single_call_probe.py)
# between the in-tree library and minbft_amd/libminbft_amd_base.so, three
# alternating reps; then the authenticator / C1 / parity tests.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_authen.py tests/test_c1.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_ab1.log 2>&1 || { tail -30 gpurun_out/pytest_ab1.log; exit 1; }
tail -1 gpurun_out/pytest_ab1.log
for rep in 1 2 3; do
  for L in "" "$PWD/minbft_amd/libminbft_amd_base.so"; do
    MBFT_LIB_PATH=$L timeout -k 10 120 python tools/single_call_probe.py 400 > gpurun_out/ab1.json 2> gpurun_out/ab1.err || exit 1
    echo "${L:+base}${L:-new} $(cut -c1-200 gpurun_out/ab1.json)"
  done
done

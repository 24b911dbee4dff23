#!/bin/bash
# Lane-group parallel additions in k_verify_split (round 4): tests, single-call
# probe with and without (MBFT_SPLIT_WIDE), phase timing of the wide form.
set -o pipefail
O=gpurun_out
TAG=${1:-w}
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_keys_late.py tests/test_gpu_authen.py tests/test_gpu_parity.py tests/test_c1.py > $O/pytest_wide_$TAG.log 2>&1 || { tail -30 $O/pytest_wide_$TAG.log; exit 1; }
tail -1 $O/pytest_wide_$TAG.log
for w in 1 0 1 0; do
  MBFT_SPLIT_WIDE=$w timeout -k 10 120 python -u tools/single_call_probe.py 300 > $O/single_wide${w}_$TAG.json 2> $O/single_wide${w}_$TAG.err || { tail -5 $O/single_wide${w}_$TAG.err; exit 1; }
  echo "wide=$w $(cat $O/single_wide${w}_$TAG.json)"
done
MBFT_LIB_PATH=$PWD/minbft_amd/libminbft_amd_st.so timeout -k 10 240 python -u tools/split_timing.py 200 > $O/split_timing_wide_$TAG.json 2> $O/split_timing_wide_$TAG.err && cat $O/split_timing_wide_$TAG.json

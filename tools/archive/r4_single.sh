#!/bin/bash
# Lone-call latency work (round 4): the split kernel's phase timing (timing
# build), the single-call probe with / without the status spin, a traced
# probe, and the GPU tests that cover the small-batch kernels and the
# single-call path.
#   bash tools/r4_single.sh TAG
set -o pipefail
TAG=${1:-x}
O=gpurun_out
ST=$PWD/minbft_amd/libminbft_amd_st.so
MBFT_LIB_PATH=$ST timeout -k 10 240 python -u tools/split_timing.py 200 > $O/split_timing_${TAG}.json 2> $O/split_timing_${TAG}.err &&
timeout -k 10 120 python -u tools/single_call_probe.py 300 > $O/single_${TAG}_spin.json 2> $O/single_${TAG}_spin.err &&
MBFT_SPIN_US=0 timeout -k 10 120 python -u tools/single_call_probe.py 300 > $O/single_${TAG}_nospin.json 2> $O/single_${TAG}_nospin.err &&
MBFT_HOST_INV_MAX=0 timeout -k 10 120 python -u tools/single_call_probe.py 300 > $O/single_${TAG}_waveinv.json 2> $O/single_${TAG}_waveinv.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/prof_sc_$TAG -o sc -- python3 tools/single_call_probe.py 300 > $O/single_${TAG}_traced.json 2> $O/single_${TAG}_traced.err &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_keys_late.py tests/test_gpu_authen.py tests/test_gpu_parity.py tests/test_c1.py > $O/pytest_single_${TAG}.log 2>&1
rc=$?
tail -3 $O/pytest_single_${TAG}.log
cat $O/single_${TAG}_*.json
exit $rc

set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
S=minbft_amd/libminbft_amd_stp.so
timeout -k 10 240 python -u tools/step_timing.py > gpurun_out/step_norm3.json 2>gpurun_out/step.err || exit 1
MBFT_LIB_PATH=$S timeout -k 10 240 python -u tools/step_timing.py > gpurun_out/step_stp3.json 2>>gpurun_out/step.err || exit 1
MBFT_VERIFY_BPC=1 timeout -k 10 240 python -u tools/step_timing.py > gpurun_out/step_norm1.json 2>>gpurun_out/step.err || exit 1
MBFT_VERIFY_BPC=1 MBFT_LIB_PATH=$S timeout -k 10 240 python -u tools/step_timing.py > gpurun_out/step_stp1.json 2>>gpurun_out/step.err || exit 1
for f in norm3 stp3 norm1 stp1; do echo $f; cat gpurun_out/step_$f.json; done

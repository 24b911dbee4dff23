#!/bin/bash
# FETCH_SIZE calibration for the verifier's gather shape (tools/ubench_gather.hip):
# each kernel runs twice (warm + measured) in its own process, one PMC pass each.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc_gather
export TMPDIR=/tmp
for k in stream rand64 rand128; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_gather/$k -o p -- ./tools/ubench_gather $k > gpurun_out/pmc_gather/$k.log 2>&1 || exit 1
done
echo done

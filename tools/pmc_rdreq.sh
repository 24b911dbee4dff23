#!/bin/bash
# L2 -> fabric read-request sizes (TCC_EA0_RDREQ / _64B / _128B) for the
# gather calibration kernels (tools/ubench_gather) and for k_verify at W29/29
# (tools/pmc_workload.py): whether a random 64-B comb-entry gather costs a
# 64-B or a 128-B request.
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/pmc_rdreq
mkdir -p $D
export TMPDIR=/tmp
C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
for k in ${MBFT_GATHER_KERNELS:-stream rand64 rand128}; do
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $D/$k$MBFT_GATHER_MEM -o p -- ./tools/ubench_gather $k $MBFT_GATHER_MEM > $D/$k$MBFT_GATHER_MEM.log 2>&1 || exit 1
done
[ -n "$MBFT_GATHER_ONLY" ] && { echo done; exit 0; }
timeout -s KILL 150 rocprofv3 --kernel-include-regex k_verify --pmc $C --output-format csv -d $D/verify -o p -- python3 tools/pmc_workload.py 29 29 > $D/verify.log 2>&1 || exit 1
echo done

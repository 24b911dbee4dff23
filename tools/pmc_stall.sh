#!/bin/bash
# Where k_verify's wave cycles go (G 29 / Q 29): one rocprofv3 PMC pass of the
# SQ wave-state counters -- WAIT_ANY (parked on s_waitcnt), WAIT_INST_ANY
# (issue stall), ACTIVE_INST_ANY, which sum to WAVE_CYCLES -- plus VALU and
# LDS activity; at the default grid (3 waves / SIMD) and at one wave / SIMD
# (MBFT_VERIFY_BPC=1).  Counters in their own runs, no tracing domains.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc_stall
export TMPDIR=/tmp
P="rocprofv3 --kernel-include-regex k_verify --output-format csv"
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for bpc in 0 1; do
  D=gpurun_out/pmc_stall/bpc$bpc
  mkdir -p $D
  MBFT_VERIFY_BPC=$bpc timeout -s KILL 150 $P --pmc $C -d $D -o p -- python3 tools/pmc_workload.py 29 29 > $D/run.log 2>&1 || exit 1
done
echo "[pmc_stall] done"

#!/bin/bash
# rocprofv3 PMC passes over k_verify (counters in their own runs, no tracing
# domains combined with --pmc).  FETCH_SIZE and WRITE_SIZE need separate
# passes on gfx950 (TCC slots).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
P="rocprofv3 --kernel-include-regex k_verify --output-format csv"
echo "[pmc] fetch" && \
timeout -k 10 300 $P --pmc FETCH_SIZE -d gpurun_out/pmc/fetch -o p -- python3 tools/pmc_workload.py > gpurun_out/pmc/fetch.log 2>&1 && \
echo "[pmc] write" && \
timeout -k 10 300 $P --pmc WRITE_SIZE -d gpurun_out/pmc/write -o p -- python3 tools/pmc_workload.py > gpurun_out/pmc/write.log 2>&1 && \
echo "[pmc] sq" && \
timeout -k 10 300 $P --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc/sq -o p -- python3 tools/pmc_workload.py > gpurun_out/pmc/sq.log 2>&1
rc=$?
echo "[pmc] rc=$rc"
find gpurun_out/pmc -name "*counter_collection.csv" | head
exit $rc

#!/bin/bash
# rocprofv3 PMC passes over the SHA-256 stage kernel (k_request_e_tiled):
# HBM bytes, LDS traffic and bank conflicts, VALU work.  One counter group per run.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/pmc_sha
mkdir -p $D
P="rocprofv3 --kernel-include-regex k_request_e --output-format csv"
timeout -s KILL 120 $P --pmc FETCH_SIZE -d $D/fetch -o p -- python3 tools/pmc_sha_workload.py > $D/fetch.log 2>&1 || exit 1
timeout -s KILL 120 $P --pmc WRITE_SIZE -d $D/write -o p -- python3 tools/pmc_sha_workload.py > $D/write.log 2>&1 || exit 1
timeout -s KILL 120 $P --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $D/sq -o p -- python3 tools/pmc_sha_workload.py > $D/sq.log 2>&1 || exit 1
echo "[pmc_sha] done"

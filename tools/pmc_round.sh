#!/bin/bash
# rocprofv3 PMC passes over k_verify (counters in their own runs, no tracing
# domains combined with --pmc), one set per comb-window pair.
#   WINDOWS="16,16 26,26" bash tools/pmc_round.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
P="rocprofv3 --kernel-include-regex k_verify --output-format csv"
for gq in ${WINDOWS:-16,16}; do
  g=${gq%,*}; q=${gq#*,}
  D=gpurun_out/pmc/w${g}_${q}
  mkdir -p $D
  echo "[pmc] G=$g Q=$q"
  timeout -s KILL 120 $P --pmc FETCH_SIZE -d $D/fetch -o p -- python3 tools/pmc_workload.py $g $q > $D/fetch.log 2>&1 || exit 1
  timeout -s KILL 120 $P --pmc WRITE_SIZE -d $D/write -o p -- python3 tools/pmc_workload.py $g $q > $D/write.log 2>&1 || exit 1
  timeout -s KILL 120 $P --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $D/sq -o p -- python3 tools/pmc_workload.py $g $q > $D/sq.log 2>&1 || exit 1
  timeout -s KILL 120 $P --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum -d $D/tcp -o p -- python3 tools/pmc_workload.py $g $q > $D/tcp.log 2>&1 || exit 1
done
echo "[pmc] done"

# Kernel trace of coalesced concurrent single calls (threads:slots configs).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/conc_trace -o ct -- python3 tools/conc_probe.py ${CONC_CFGS:-16:4} > gpurun_out/conc_trace.txt 2>&1 || { tail -20 gpurun_out/conc_trace.txt; exit 1; }
tail -1 gpurun_out/conc_trace.txt

# Concurrent coalesced single calls: rates, then a kernel trace of the 64:4 case.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/conc_probe.py 16:1 16:4 64:1 64:4 64:8 > gpurun_out/conc_probe.txt 2>&1 || { tail -20 gpurun_out/conc_probe.txt; exit 1; }
tail -1 gpurun_out/conc_probe.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/conc_trace -o ct -- python3 tools/conc_probe.py 64:4 > gpurun_out/conc_trace.txt 2>&1 || { tail -20 gpurun_out/conc_trace.txt; exit 1; }
tail -1 gpurun_out/conc_trace.txt

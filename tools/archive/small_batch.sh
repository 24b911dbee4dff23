# Small-batch latency (k = 1 .. 64 calls) and its kernel trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/small_batch_probe.py 200 > gpurun_out/small_batch.txt 2>&1 || { tail -20 gpurun_out/small_batch.txt; exit 1; }
cat gpurun_out/small_batch.txt | head -7
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sb_trace -o sb -- python3 tools/small_batch_probe.py 100 > gpurun_out/small_batch_tr.txt 2>&1 || { tail -20 gpurun_out/small_batch_tr.txt; exit 1; }
echo traced

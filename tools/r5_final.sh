#!/bin/bash
# Round-5 final measurement: the default bench (the driver's command), then a
# rocprofv3 kernel-trace pass over the headline loop alone (no extra lines)
# for the k_verify launch statistics.  Each GPU step under its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 400 $O/bench.json; echo
# judged by the exit status: the exit-time fault under the profiler (a
# CU-masked stream left alive for rocprofv3's destructors) is fixed in
# round 6 (resident.cpp destroy_cu_streams_at_exit)
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --steps 20 --no-extra-lines --no-adversarial --c3-requests 0 --no-cpu-baseline > $O/kt_bench.json 2> $O/kt.err || { echo "[r5_final] trace run failed"; tail -20 $O/kt.err; exit 1; }
K=$(find $O/kt -name "*kernel_trace.csv" | head -1)
[ -n "$K" ] && grep -q '"metric"' $O/kt_bench.json || { echo "[r5_final] trace run left no trace"; exit 1; }
S=$(find $O/kt -name "*kernel_stats.csv" | head -1)
python3 tools/trace_summary.py "$K" > $O/kernel_trace_summary.json || exit 1
cp "$S" $O/kernel_stats.csv
rm -f "$K"
echo "[r5_final] done"

#!/bin/bash
# One GPU-box session: tests, smoke, bench, kernel-trace profile.
# Each GPU step has its own time limit; steps are chained with &&; output
# goes to files under gpurun_out/ as it happens (the box's silence watchdog).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r3}
echo "[gpu_round] pytest -m gpu" && \
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 && \
echo "[gpu_round] smoke" && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && \
echo "[gpu_round] bench" && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
echo "[gpu_round] rocprofv3 kernel trace" && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt_$TAG -o kt -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-peak-run --no-adversarial --c3-requests 0 --no-extra-lines > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/bench_prof_$TAG.err
rc=$?
[ $rc -eq 0 ] && python3 tools/trace_summary.py gpurun_out/prof_kt_$TAG/kt_kernel_trace.csv > gpurun_out/kt_summary_$TAG.json
echo "[gpu_round] rc=$rc"
tail -3 gpurun_out/pytest_gpu_$TAG.log
cat gpurun_out/bench_$TAG.json | cut -c1-400
exit $rc

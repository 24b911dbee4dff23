#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench, kernel-trace profile of the
# bench, and a traced single-call probe.  Each GPU step has its own limit;
# steps chained with &&; output to files under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4}
SKIP_TESTS=${SKIP_TESTS:-0}
# every step runs the product defaults (zero-copy staging for the smallest
# batches, host s^-1 for lone calls, status spin); the copy path is probed
# and tested last, on its own (COPY_PROBE=1)
step() { echo "[r4_round $TAG] $*"; }
if [ "$SKIP_TESTS" != 1 ]; then
  step "pytest -m gpu" && \
  timeout -k 10 1200 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu_$TAG.log
  step "smoke" && \
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -30 gpurun_out/smoke_$TAG.log; exit 1; }
fi
step "bench" && \
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
step "rocprofv3 kernel trace of the bench" && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt_$TAG -o kt -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-peak-run --no-adversarial --c3-requests 0 --no-extra-lines > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/bench_prof_$TAG.err || { tail -20 gpurun_out/bench_prof_$TAG.err; exit 1; }
python3 tools/trace_summary.py gpurun_out/prof_kt_$TAG/kt_kernel_trace.csv > gpurun_out/kt_summary_$TAG.json
if [ "${C3_TRACE:-1}" = 1 ]; then
  step "C3 kernel trace (message-layer kernels)" && \
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3_$TAG -o c3 -- python3 tools/c3_probe.py 16384 > gpurun_out/c3_probe_$TAG.json 2> gpurun_out/c3_probe_$TAG.err || { tail -20 gpurun_out/c3_probe_$TAG.err; exit 1; }
  python3 tools/trace_summary.py gpurun_out/prof_c3_$TAG/c3_kernel_trace.csv > gpurun_out/c3_kt_summary_$TAG.json
  python3 tools/msg_kernel_roofline.py gpurun_out/c3_kt_summary_$TAG.json gpurun_out/msg_kernels_roofline_$TAG.json > /dev/null
fi
if [ "${SINGLE_TRACE:-1}" = 1 ]; then
  step "single-call trace" && \
  timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/prof_sc_$TAG -o sc -- python3 tools/single_call_probe.py 300 > gpurun_out/single_$TAG.json 2> gpurun_out/single_$TAG.err || { tail -20 gpurun_out/single_$TAG.err; exit 1; }
  python3 tools/single_trace_summary.py gpurun_out/prof_sc_$TAG gpurun_out/single_trace_summary_$TAG.json "single-call trace $TAG" > /dev/null
fi
if [ "${COPY_PROBE:-1}" = 1 ]; then
  step "copy-path single calls (probe, then tests)" && \
  MBFT_ZERO_COPY=0 timeout -k 10 120 python3 tools/single_call_probe.py 300 > gpurun_out/single_copy_$TAG.json 2> gpurun_out/single_copy_$TAG.err && \
  MBFT_ZERO_COPY=0 MBFT_SPIN_US=0 timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "single or sequences or go_error or c1 or coalesced or keys_late or live_item" --timeout 300 --timeout-method thread > gpurun_out/pytest_copy_$TAG.log 2>&1 || { tail -30 gpurun_out/single_copy_$TAG.err gpurun_out/pytest_copy_$TAG.log; exit 1; }
  tail -2 gpurun_out/pytest_copy_$TAG.log; cat gpurun_out/single_copy_$TAG.json
fi
step "done"
cut -c1-600 gpurun_out/bench_$TAG.json

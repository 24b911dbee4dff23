#!/bin/bash
# Idle-batch s^-1 forms: parity tests that take the idle path, then the
# idle-batch timeline (kernel trace) and device p50 per form.  Each GPU step
# has its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-ni}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_config.py tests/test_gpu_authen.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
for per in 8 4; do
  MBFT_NINV_PER=$per bash tools/trace_loop.sh loop_${TAG}_$per && python3 tools/idle_timeline.py gpurun_out/prof_loop_${TAG}_$per/kt_kernel_trace.csv 1 || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/bench_loop_${TAG}_$per.json')); print('PER=$per', round(d['value']/1e6,1), 'M/s  k_verify', round(d['kernel_ms']['k_verify'],4), ' dev p50', round(d['p50_batch_latency_device_ms'],4), 'unsplit', round(d['p50_batch_latency_device_unsplit_ms'],4))"
done

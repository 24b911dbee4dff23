#!/bin/bash
# Device message layer (tests + C3 probe) and the idle-batch timeline (kernel
# traces, block vs wave s^-1).  Each GPU step has its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-c2}
timeout -k 10 600 python -u -m pytest tests/test_gpu_msgdev.py tests/test_gpu_configs.py -k "flat or c3" -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
MBFT_STAGE_TRACE=1 timeout -k 10 300 python tools/c3_probe.py > gpurun_out/c3_$TAG.json 2> gpurun_out/c3_$TAG.err || { tail -20 gpurun_out/c3_$TAG.err; exit 1; }
grep 'flat dev' gpurun_out/c3_$TAG.err | tail -3
python3 -c "import json,sys; d=json.load(open('gpurun_out/c3_$TAG.json')); print('C3 device', round(d['messages_per_s']/1e6,1), 'M/s', round(d['ms'],2), 'ms; host layer', round(d['host_layer']['messages_per_s']/1e6,1), 'M/s')"
bash tools/trace_loop.sh loop_$TAG && python3 tools/idle_timeline.py gpurun_out/prof_loop_$TAG/kt_kernel_trace.csv 2 || exit 1
MBFT_NINV_FORM=wave bash tools/trace_loop.sh loopw_$TAG && python3 tools/idle_timeline.py gpurun_out/prof_loopw_$TAG/kt_kernel_trace.csv 1

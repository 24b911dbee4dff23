#!/bin/bash
# Message-layer kernels: the device message-layer tests, then the C3 copy /
# kernel timeline (tools/c3_timeline.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-mk}
timeout -k 10 600 python -u -m pytest tests/test_gpu_msgdev.py tests/test_gpu_configs.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
bash tools/c3_timeline.sh c3tl_$TAG

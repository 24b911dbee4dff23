#!/bin/bash
# Message-layer tests + the pipeline tests (queue counter zeroed by the
# chain), a quick bench, and the authenticator-level copy/kernel timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-c3}
timeout -k 10 900 python -u -m pytest tests/test_gpu_msgdev.py tests/test_gpu_parity.py tests/test_gpu_authen.py tests/test_gpu_configs.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-adversarial --c3-requests 0 --no-extra-lines --no-cpu-baseline > gpurun_out/bench_q_$TAG.json 2> gpurun_out/bench_q_$TAG.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/bench_q_$TAG.json')); print(round(d['value']/1e6,1), 'M/s ms/step', round(d['ms_per_step'],4), 'k_verify', round(d['kernel_ms']['k_verify'],4), ' dev p50', round(d['p50_batch_latency_device_ms'],4), 'auth p50', round(d['p50_batch_latency_ms'],3))"
MBFT_TL_FORMS=pinned bash tools/auth_timeline.sh && tail -45 gpurun_out/tl_pinned.txt

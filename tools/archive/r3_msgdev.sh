#!/bin/bash
# Device message layer + idle-batch s^-1 check: its GPU tests, the C3 probe
# with the stage trace, and quick bench lines for the s^-1 forms.  Each GPU
# step has its own time limit; steps chained with &&.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-md}
timeout -k 10 600 python -u -m pytest tests/test_gpu_msgdev.py tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_$TAG.log
MBFT_STAGE_TRACE=1 timeout -k 10 300 python tools/c3_probe.py > gpurun_out/c3_$TAG.json 2> gpurun_out/c3_$TAG.err || { tail -20 gpurun_out/c3_$TAG.err; exit 1; }
grep 'mbft validate\|mbft calls' gpurun_out/c3_$TAG.err | tail -8
python3 -c "import json,sys; d=json.load(open('gpurun_out/c3_$TAG.json')); print('C3 device', round(d['messages_per_s']/1e6,1), 'M/s', round(d['ms'],2), 'ms; host layer', round(d['host_layer']['messages_per_s']/1e6,1), 'M/s; pack', round(d['pack_ms'],1), 'ms; bytes', d['flat_batch_bytes'])"
for form in block wave split; do
  case $form in
    block) ENV="MBFT_NINV_FORM=block" ;;
    wave) ENV="MBFT_NINV_FORM=wave" ;;
    split) ENV="MBFT_NINV_FORM=block MBFT_SPLIT_DIV=4" ;;
  esac
  env $ENV timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-adversarial --c3-requests 0 --no-extra-lines --no-cpu-baseline > gpurun_out/bench_${TAG}_$form.json 2> gpurun_out/bench_${TAG}_$form.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$form.json')); print('$form', round(d['value']/1e6,1), 'M/s  k_verify', round(d['kernel_ms']['k_verify'],4), ' dev p50', round(d['p50_batch_latency_device_ms'],4), 'unsplit', round(d['p50_batch_latency_device_unsplit_ms'],4))"
done
echo done

set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_keys_late.py tests/test_gpu_authen.py tests/test_c1.py tests/test_gpu_parity.py > gpurun_out/pytest_hinv.log 2>&1 || { tail -30 gpurun_out/pytest_hinv.log; exit 1; }
tail -1 gpurun_out/pytest_hinv.log
for m in 64 4; do
  MBFT_HOST_INV_MAX=$m timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-peak-run --no-adversarial --c3-requests 0 > gpurun_out/hinv_$m.json 2> gpurun_out/hinv_$m.err || { tail -5 gpurun_out/hinv_$m.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/hinv_$m.json'));s=d['single_calls'];print('host_inv_max=$m single', round(s['p50_latency_us'],1), 'conc', round(s['concurrent']['calls_per_s']), 'per batch', round(s['concurrent']['mean_calls_per_batch'],1))"
done

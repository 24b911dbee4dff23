# Coalesced concurrent single calls: the coalescing tests, then the bench's
# single_calls line (Python threads; native threads at concurrency 1 and 4).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_authen.py -k "coalesced" > gpurun_out/pytest_conc.log 2>&1 || { tail -30 gpurun_out/pytest_conc.log; exit 1; }
tail -1 gpurun_out/pytest_conc.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-peak-run --no-adversarial --c3-requests 0 > gpurun_out/conc.json 2> gpurun_out/conc.err || { tail -5 gpurun_out/conc.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/conc.json'));print(json.dumps(d['single_calls']))"

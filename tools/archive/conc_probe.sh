# Concurrent coalesced single calls from OS threads: the coalescing tests, then rates.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_authen.py -k "coalesced" > gpurun_out/pytest_conc.log 2>&1 || { tail -30 gpurun_out/pytest_conc.log; exit 1; }
tail -1 gpurun_out/pytest_conc.log
timeout -k 10 150 python -u tools/conc_probe.py ${CONC_CFGS:-16:1 16:4 64:1 64:4} > gpurun_out/conc_probe.txt 2>&1 || { tail -20 gpurun_out/conc_probe.txt; exit 1; }
tail -1 gpurun_out/conc_probe.txt

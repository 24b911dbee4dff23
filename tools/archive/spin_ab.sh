# Front-waiter spin of coalesced single calls (MBFT_COALESCE_SPIN_US 0 / 200 / 1000).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_authen.py -k "coalesced" > gpurun_out/pytest_conc.log 2>&1 || { tail -30 gpurun_out/pytest_conc.log; exit 1; }
tail -1 gpurun_out/pytest_conc.log
for ch in 0 200 1000; do
  MBFT_COALESCE_SPIN_US=$ch timeout -k 10 200 python -u tools/conc_probe.py 16:1 64:1 64:4 > gpurun_out/chain_$ch.txt 2>&1 || { tail -20 gpurun_out/chain_$ch.txt; exit 1; }
  echo "chain $ch: $(tail -1 gpurun_out/chain_$ch.txt)"
done

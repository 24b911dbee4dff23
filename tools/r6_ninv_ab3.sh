#!/bin/bash
# Round 6: the pipelined s^-1 (now the default path) -- chain length per
# lane, and the block form, alternated; then the GPU parity tests that cover
# the verifier's paths.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6m}
mkdir -p $O
for rep in 1 2; do
for cfg in "wave 16" "wave 32" "wave 8" "block 8"; do
  set -- $cfg
  MBFT_NINV_PIPE_FORM=$1 MBFT_NINV_PIPE_PER=$2 timeout -k 10 300 python3 tools/steady_ab.py --streams 3 --tag "$1_$2" >> $O/ninv.jsonl 2>> $O/ninv.err || { tail -20 $O/ninv.err; exit 1; }
done
done
cat $O/ninv.jsonl
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bench_config.py tests/test_gpu_configs.py tests/test_gpu_msgdev.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 tools/lowload_probe.py > $O/lowload.json 2> $O/lowload.err || { tail -20 $O/lowload.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/lowload.json'))
print({k:(round(v['p50_us'],1), round(v.get('cpu_us_per_window',0),1)) for k,v in d['go_default']['small_route'].items()})"

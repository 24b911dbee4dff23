#!/bin/bash
# Round 6: mid-size batches through the batched s^-1 + k_verify_split form
# (MBFT_SPLIT_PLANES_MAX) -- the GPU tests that run 257..12288-item device
# batches, then latency A/Bs against k_verify_pairs (=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6p}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_msgdev.py tests/test_gpu_multi_msg.py tests/test_gpu_check_coalesce.py tests/test_gpu_small_check.py tests/test_gpu_replies_go.py tests/test_gpu_parity.py tests/test_gpu_authen.py tests/test_gpu_configs.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for pm in 0 12288; do
  MBFT_SPLIT_PLANES_MAX=$pm timeout -k 10 300 python3 tools/small_batch_probe.py > $O/small_$pm.json 2> $O/small_$pm.err || { tail -20 $O/small_$pm.err; exit 1; }
  cat $O/small_$pm.json
  MBFT_SPLIT_PLANES_MAX=$pm LOWLOAD_SIZES=256,512,1024,2048,4096 LOWLOAD_NREQ=1024 LOWLOAD_SMALL_MAX=0 timeout -k 10 300 python3 tools/lowload_probe.py > $O/lowload_$pm.json 2> $O/lowload_$pm.err || { tail -20 $O/lowload_$pm.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/lowload_$pm.json'))
print($pm, {k:(round(v['p50_us'],1), round(v.get('cpu_us_per_window',0),1)) for k,v in d['go_default']['small_route'].items()})"
done
MBFT_SPLIT_PLANES_MAX=12288 LOWLOAD_SIZES=1024,4096 LOWLOAD_NREQ=1024 LOWLOAD_SMALL_MAX=0 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/t -o t --output-format csv -- python3 tools/lowload_probe.py > $O/lowload_tr.json 2> $O/lowload_tr.err || { tail -20 $O/lowload_tr.err; exit 1; }
python3 tools/pass_timeline.py $O/t > $O/timeline.json
rm -f $(find $O/t -name "*kernel_trace.csv") $(find $O/t -name "*memory_copy_trace.csv")
echo "[r6_planes] done"

#!/bin/bash
# Round 6: the dedup table inserts inside k_msg_cands -- message GPU tests,
# the 1,024-message timeline, latencies, and C3.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6fi}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_msgdev.py tests/test_gpu_multi_msg.py tests/test_gpu_check_coalesce.py tests/test_gpu_small_check.py tests/test_gpu_replies_go.py tests/test_gpu_configs.py tests/test_reference_scenarios.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
LOWLOAD_SIZES=1024 LOWLOAD_NREQ=1024 LOWLOAD_SMALL_MAX=0 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/t -o t --output-format csv -- python3 tools/lowload_probe.py > $O/lowload_tr.json 2> $O/lowload_tr.err || { tail -20 $O/lowload_tr.err; exit 1; }
python3 tools/pass_timeline.py $O/t > $O/timeline_1024.json
rm -f $(find $O/t -name "*kernel_trace.csv") $(find $O/t -name "*memory_copy_trace.csv")
python3 -c "
import json; d=json.load(open('$O/timeline_1024.json')); print(d['median_span_us'], [(o['op'][:14], round(o['dur_us'],1), round(o['gap_before_us'],1)) for o in d['ops']])"
LOWLOAD_SIZES=512,1024,2048,4096 LOWLOAD_NREQ=1024 LOWLOAD_SMALL_MAX=0 timeout -k 10 300 python3 tools/lowload_probe.py > $O/lowload_mid.json 2> $O/lowload_mid.err || { tail -20 $O/lowload_mid.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/lowload_mid.json'))
print({k:round(v['p50_us'],1) for k,v in d['go_default']['small_route'].items()})"
timeout -k 10 300 python3 tools/c3_probe.py > $O/c3.json 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/c3.json')); g=d['go_wiring']
print('c3', round(d['messages_per_s']/1e6,1), 'go', round(g['messages_per_s']/1e6,1), {k:round(v['messages_per_s']/1e6,1) for k,v in g['coalesced'].items()})"
echo "[r6_fuseins] done"

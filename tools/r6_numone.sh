#!/bin/bash
# Round 6: one-workgroup call numbering for one-chunk passes
# (msg_number_one) -- the message GPU tests, the 1,024-message timeline, and
# an A/B against the hipcub scan + two kernels (MBFT_MSG_NUMBER_ONE=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6n1}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_msgdev.py tests/test_gpu_multi_msg.py tests/test_gpu_check_coalesce.py tests/test_gpu_small_check.py tests/test_gpu_replies_go.py tests/test_gpu_configs.py tests/test_reference_scenarios.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
LOWLOAD_SIZES=1024 LOWLOAD_NREQ=1024 LOWLOAD_SMALL_MAX=0 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/t -o t --output-format csv -- python3 tools/lowload_probe.py > $O/lowload_tr.json 2> $O/lowload_tr.err || { tail -20 $O/lowload_tr.err; exit 1; }
python3 tools/pass_timeline.py $O/t > $O/timeline_1024.json
rm -f $(find $O/t -name "*kernel_trace.csv") $(find $O/t -name "*memory_copy_trace.csv")
python3 -c "
import json; d=json.load(open('$O/timeline_1024.json')); print(d['median_span_us'], [(o['op'][:14], round(o['dur_us'],1), round(o['gap_before_us'],1)) for o in d['ops']])"
run() {  # tag, env...
  local tag=$1; shift
  env "$@" LOWLOAD_SIZES=512,1024,2048,4096 LOWLOAD_NREQ=1024 LOWLOAD_SMALL_MAX=0 timeout -k 10 300 python3 tools/lowload_probe.py > $O/lowload_$tag.json 2> $O/lowload_$tag.err || { tail -20 $O/lowload_$tag.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/lowload_$tag.json'))
print('$tag', {k:round(v['p50_us'],1) for k,v in d['go_default']['small_route'].items()})"
}
run one MBFT_X=1 && run hipcub MBFT_MSG_NUMBER_ONE=0 && run one2 MBFT_X=1 && run hipcub2 MBFT_MSG_NUMBER_ONE=0 || exit 1
echo "[r6_numone] done"

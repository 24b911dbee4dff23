#!/bin/bash
# Round 6: the one-wait check form past 1,365 messages (the verifier's s^-1
# now batched per wave), A/B against the two-wait form, same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6ow}
mkdir -p $O
MBFT_MSG_ONE_WAIT_MAX=4096 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_msgdev.py tests/test_gpu_check_coalesce.py tests/test_gpu_multi_msg.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # tag, env...
  local tag=$1; shift
  env "$@" LOWLOAD_SIZES=1024,2048,4096 LOWLOAD_NREQ=1024 LOWLOAD_SMALL_MAX=0 timeout -k 10 300 python3 tools/lowload_probe.py > $O/lowload_$tag.json 2> $O/lowload_$tag.err || { tail -20 $O/lowload_$tag.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/lowload_$tag.json'))
print('$tag', {k:(round(v['p50_us'],1),round(v['cpu_us_per_window'],1)) for k,v in d['go_default']['small_route'].items() if 'messages' in k})"
}
run two MBFT_X=1 && run one MBFT_MSG_ONE_WAIT_MAX=4096 && run two2 MBFT_X=1 && run one2 MBFT_MSG_ONE_WAIT_MAX=4096 || exit 1
MBFT_MSG_ONE_WAIT_MAX=4096 LOWLOAD_SIZES=4096 LOWLOAD_NREQ=1024 LOWLOAD_SMALL_MAX=0 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/t -o t --output-format csv -- python3 tools/lowload_probe.py > $O/lowload_tr.json 2> $O/lowload_tr.err || { tail -20 $O/lowload_tr.err; exit 1; }
python3 tools/pass_timeline.py $O/t > $O/timeline_4096_one.json
rm -f $(find $O/t -name "*kernel_trace.csv") $(find $O/t -name "*memory_copy_trace.csv")
echo "[r6_onewait] done"

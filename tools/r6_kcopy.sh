#!/bin/bash
# Round 6: small message passes upload their records and arena from
# k_msg_init's threads (MBFT_MSG_KCOPY_MAX) -- the message-layer GPU tests,
# the mid-size timelines, and A/Bs against the copy-engine uploads (=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6kc}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_msgdev.py tests/test_gpu_multi_msg.py tests/test_gpu_check_coalesce.py tests/test_gpu_small_check.py tests/test_gpu_replies_go.py tests/test_gpu_configs.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for w in 1024 4096; do
  LOWLOAD_SIZES=$w LOWLOAD_NREQ=1024 LOWLOAD_SMALL_MAX=0 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/t$w -o t --output-format csv -- python3 tools/lowload_probe.py > $O/lowload_tr$w.json 2> $O/lowload_tr$w.err || { tail -20 $O/lowload_tr$w.err; exit 1; }
  python3 tools/pass_timeline.py $O/t$w > $O/timeline_$w.json
  rm -f $(find $O/t$w -name "*kernel_trace.csv") $(find $O/t$w -name "*memory_copy_trace.csv")
  python3 -c "
import json; d=json.load(open('$O/timeline_$w.json')); print($w, d['median_span_us'], [(o['op'][:14], round(o['dur_us'],1), round(o['gap_before_us'],1)) for o in d['ops']])"
done
run() {  # tag, env...
  local tag=$1; shift
  env "$@" LOWLOAD_SIZES=512,1024,2048,4096 LOWLOAD_NREQ=1024 LOWLOAD_SMALL_MAX=0 timeout -k 10 300 python3 tools/lowload_probe.py > $O/lowload_$tag.json 2> $O/lowload_$tag.err || { tail -20 $O/lowload_$tag.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/lowload_$tag.json'))
print('$tag', {k:(round(v['p50_us'],1), round(v.get('cpu_us_per_window',0),1)) for k,v in d['go_default']['small_route'].items()})"
  env "$@" timeout -k 10 300 python3 tools/c3_probe.py > $O/c3_$tag.json 2> $O/c3_$tag.err || { tail -20 $O/c3_$tag.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/c3_$tag.json')); g=d['go_wiring']
print('$tag c3', round(d['messages_per_s']/1e6,1), 'go', round(g['messages_per_s']/1e6,1), {k:round(v['messages_per_s']/1e6,1) for k,v in g['coalesced'].items()})"
}
run kcopy MBFT_X=1 && run dma MBFT_MSG_KCOPY_MAX=0 && run kcopy2 MBFT_X=1 || exit 1
echo "[r6_kcopy] done"

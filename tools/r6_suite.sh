#!/bin/bash
# Round 6: the whole GPU suite and smoke(), then the 1,024-message pass timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6s}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
LOWLOAD_SIZES=1024 LOWLOAD_NREQ=1024 LOWLOAD_SMALL_MAX=0 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/t -o t --output-format csv -- python3 tools/lowload_probe.py > $O/lowload_tr.json 2> $O/lowload_tr.err || { tail -20 $O/lowload_tr.err; exit 1; }
python3 tools/pass_timeline.py $O/t > $O/timeline_1024.json
rm -f $(find $O/t -name "*kernel_trace.csv") $(find $O/t -name "*memory_copy_trace.csv")
python3 -c "
import json; d=json.load(open('$O/timeline_1024.json')); print(d['median_span_us'], [(o['op'][:14], round(o['dur_us'],1), round(o['gap_before_us'],1)) for o in d['ops']])"
echo "[r6_suite] done"

#!/bin/bash
# Round 6: a kernel + copy trace of mid-size message passes (windows of
# 1,024 and 4,096 messages through the device message layer).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6r}
mkdir -p $O
for w in 1024 4096; do
  LOWLOAD_SIZES=$w LOWLOAD_NREQ=1024 LOWLOAD_SMALL_MAX=0 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/t$w -o t --output-format csv -- python3 tools/lowload_probe.py > $O/lowload_$w.json 2> $O/lowload_$w.err || { tail -20 $O/lowload_$w.err; exit 1; }
  python3 tools/pass_timeline.py $O/t$w > $O/timeline_$w.json
  rm -f $(find $O/t$w -name "*kernel_trace.csv") $(find $O/t$w -name "*memory_copy_trace.csv")
done
echo "[r6_midsize] done"

#!/bin/bash
# Round 6: k_msg_init's upload spread (MBFT_MSG_KCOPY_BLOCK bytes per
# workgroup) -- traced 1,024- and 4,096-message passes per setting.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6kb}
mkdir -p $O
for b in ${KCB_LIST:-8192 2048 1024 4096}; do
  for w in 1024 4096; do
    MBFT_MSG_KCOPY_UBLOCKS=${KCU:-2048} MBFT_MSG_KCOPY_BLOCK=$b LOWLOAD_SIZES=$w LOWLOAD_NREQ=1024 LOWLOAD_SMALL_MAX=0 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/t${b}_$w -o t --output-format csv -- python3 tools/lowload_probe.py > $O/lowload_${b}_$w.json 2> $O/lowload_${b}_$w.err || { tail -20 $O/lowload_${b}_$w.err; exit 1; }
    K=$(find $O/t${b}_$w -name "*kernel_trace.csv" | head -1)
    python3 - "$K" $b $w <<'PY'
import csv, sys, statistics
rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Kernel_Name"].startswith("k_msg_init")]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows][-32:]
print("ublocks", __import__("os").environ.get("KCU","2048"), "block", sys.argv[2], "msgs", sys.argv[3], "k_msg_init us median", round(statistics.median(d), 1), "n", len(d))
PY
    rm -f "$K"
  done
done
echo "[r6_kcblock] done"

"""Summarize a rocprofv3 --kernel-trace CSV per kernel, separating dispatches
that ran alone from those that overlapped another dispatch of the same
kernel (bench.py's timed loop overlaps consecutive batches on two streams;
its latency loop runs one batch at a time).  The isolated average is the
launch duration bench.py's roofline uses.

    python3 tools/trace_summary.py gpurun_out/prof_kt/kt_kernel_trace.csv > profiles/<name>.json
"""
import csv
import json
import sys
from collections import defaultdict


def main(path):
    rows = list(csv.DictReader(open(path)))
    by = defaultdict(list)
    for r in rows:
        by[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    out = {}
    for name, iv in by.items():
        iv.sort()
        iso, ovl = [], []
        for i, (s, e) in enumerate(iv):
            prev_end = iv[i - 1][1] if i else -1
            next_start = iv[i + 1][0] if i + 1 < len(iv) else 1 << 62
            (iso if prev_end <= s and next_start >= e else ovl).append((e - s) / 1e6)
        key = name if len(name) < 80 else name[:77] + "..."
        out[key] = {
            "calls": len(iv),
            "avg_ms_all": sum((e - s) for s, e in iv) / len(iv) / 1e6,
            "isolated_calls": len(iso),
            "avg_ms_isolated": sum(iso) / len(iso) if iso else None,
            "overlapped_calls": len(ovl),
            "avg_ms_overlapped": sum(ovl) / len(ovl) if ovl else None,
        }
    json.dump(dict(sorted(out.items(), key=lambda kv: -kv[1]["avg_ms_all"] * kv[1]["calls"])),
              sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])

#!/usr/bin/env python3
"""One device message pass, kernel by kernel and copy by copy, from a
rocprofv3 trace (kernel_trace.csv, memory_copy_trace.csv): passes are cut at
each k_msg_init dispatch; for the median-length pass of the trace's last
`--last` passes, every operation's start offset and duration (us), and the
gaps.  Used for the mid-size windows.

    python3 tools/pass_timeline.py <dir with *_kernel_trace.csv> [--last 32]
"""
import csv
import glob
import json
import os
import sys


def main():
    d = sys.argv[1]
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 32
    ops = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "?")))
    ops.sort()
    starts = [i for i, o in enumerate(ops) if "k_msg_init" in o[2]]
    passes = []
    for a, b in zip(starts, starts[1:] + [len(ops)]):
        passes.append(ops[a:b])
    passes = passes[-last:]
    if not passes:
        print(json.dumps({"error": "no k_msg_init in the trace"}))
        return
    spans = sorted((p[-1][1] - p[0][0], k) for k, p in enumerate(passes))
    span, k = spans[len(spans) // 2]
    p = passes[k]
    t0 = p[0][0]
    rows = []
    busy_end = t0
    for s, e, n in p:
        rows.append({"op": n, "start_us": round((s - t0) / 1e3, 1), "dur_us": round((e - s) / 1e3, 1),
                     "gap_before_us": round(max(0, s - busy_end) / 1e3, 1)})
        busy_end = max(busy_end, e)
    print(json.dumps({"passes": len(passes), "median_span_us": round(span / 1e3, 1), "ops": rows}, indent=1))


if __name__ == "__main__":
    main()

"""Summarize a rocprofv3 --kernel-trace CSV per (kernel, grid size),
separating dispatches that ran alone from those that overlapped another
dispatch (any kernel) in time.  bench.py's timed loop overlaps consecutive
batches on several streams; its latency loop runs one batch at a time, so
the isolated average of the 1M-item k_verify grid is the launch duration
bench.py's roofline (`roofline.launch_ms`) is checked against.

Keys are "<kernel> [grid=<threads>]": one kernel launched over different
batch sizes (the 1M C2 grid, the 4K-65K grids of the authenticator chunks
and the exact-path queue) is never averaged together.

    python3 tools/trace_summary.py gpurun_out/prof_kt/kt_kernel_trace.csv > profiles/<name>.json
"""
import csv
import json
import sys
from collections import defaultdict


def short(name: str) -> str:
    return name if len(name) < 80 else name[:77] + "..."


def main(path):
    rows = list(csv.DictReader(open(path)))
    allv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
    by = defaultdict(list)
    for r in rows:
        grid = int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1) * int(r.get("Grid_Size_Z", 1) or 1)
        by[(r["Kernel_Name"], grid)].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    # overlap with ANY other dispatch: sweep the sorted intervals once
    overl = set()
    end_max, end_idx = -1, -1
    for i, (s, e) in enumerate(allv):
        if s < end_max:
            overl.add(allv[i])
            overl.add(allv[end_idx])
        if e > end_max:
            end_max, end_idx = e, i
    out = {}
    for (name, grid), iv in by.items():
        iv.sort()
        iso = [(e - s) / 1e6 for s, e in iv if (s, e) not in overl]
        ovl = [(e - s) / 1e6 for s, e in iv if (s, e) in overl]
        out[f"{short(name)} [grid={grid}]"] = {
            "kernel": short(name),
            "grid_threads": grid,
            "calls": len(iv),
            "avg_ms_all": sum((e - s) for s, e in iv) / len(iv) / 1e6,
            "isolated_calls": len(iso),
            "avg_ms_isolated": sum(iso) / len(iso) if iso else None,
            "min_ms_isolated": min(iso) if iso else None,
            "overlapped_calls": len(ovl),
            "avg_ms_overlapped": sum(ovl) / len(ovl) if ovl else None,
        }
    json.dump(dict(sorted(out.items(), key=lambda kv: -kv[1]["avg_ms_all"] * kv[1]["calls"])),
              sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])

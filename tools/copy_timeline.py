"""Timeline of the last batch of an authenticator-level probe from a
rocprofv3 run with --kernel-trace --memory-copy-trace (CSV): every copy
(direction, bytes, duration, GB/s) and kernel in start order, relative to
the first copy of the last `window_ms` of the trace.

    python tools/copy_timeline.py <prefix> [window_ms]
"""
import csv
import sys


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main():
    pre = sys.argv[1]
    win = float(sys.argv[2]) if len(sys.argv) > 2 else 6.0
    ev = []
    mc = rows(pre + "_memory_copy_trace.csv")
    if mc:
        print("# memory copy columns:", list(mc[0].keys()))
    for r in mc:
        b = int(r.get("Bytes") or r.get("Size") or r.get("Copy_Bytes") or 0)
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r["Direction"], b))
    for r in rows(pre + "_kernel_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40], 0))
    ev.sort()
    end = max(e[1] for e in ev)
    lo = end - int(win * 1e6)
    ev = [e for e in ev if e[0] >= lo]
    t0 = ev[0][0]
    tot = {}
    for s, e, name, b in ev:
        gbs = b / (e - s) if b and e > s else 0.0
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} us  {name:42s} "
              f"{b:>10d} B {gbs:6.1f} GB/s")
        if name.startswith("copy"):
            a = tot.setdefault(name, [0, 0, 0])
            a[0] += 1
            a[1] += b
            a[2] += e - s
    for k, (c, b, d) in tot.items():
        print(f"# {k}: {c} copies, {b / 1e6:.1f} MB, busy {d / 1e3:.1f} us, {b / max(d, 1):.1f} GB/s while busy")


if __name__ == "__main__":
    main()

"""Timeline of the bench's one-batch-at-a-time (idle GPU) loop from a
rocprofv3 kernel trace: each 1M-item batch's one-launch s^-1 (k_ninv_block /
k_ninv_local), its k_verify and k_verify_slow, with the gaps between them
and the span from the s^-1 start to the last kernel's end.

    python tools/idle_timeline.py gpurun_out/prof_loop/kt_kernel_trace.csv [max_batches]
"""
import csv
import statistics
import sys


def main() -> None:
    rows = list(csv.DictReader(open(sys.argv[1])))
    cap = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    spans, invs, vers, gaps = [], [], [], []
    shown = 0
    for i, r in enumerate(rows):
        if "k_ninv_block" not in r["Kernel_Name"] and "k_ninv_local" not in r["Kernel_Name"]:
            continue
        seq = [r]
        for q in rows[i + 1:i + 6]:
            seq.append(q)
            if q["Kernel_Name"].startswith("k_verify_slow"):
                break
        names = [q["Kernel_Name"] for q in seq]
        if not any(n.startswith("void k_verify<") for n in names):
            continue
        v = next(q for q in seq if q["Kernel_Name"].startswith("void k_verify<"))
        if int(v["Grid_Size_X"]) < 1 << 20:
            continue
        t0 = int(r["Start_Timestamp"])
        end = max(int(q["End_Timestamp"]) for q in seq)
        spans.append((end - t0) / 1e3)
        invs.append((int(r["End_Timestamp"]) - t0) / 1e3)
        vers.append((int(v["End_Timestamp"]) - int(v["Start_Timestamp"])) / 1e3)
        gaps.append((int(v["Start_Timestamp"]) - int(r["End_Timestamp"])) / 1e3)
        if shown < cap:
            shown += 1
            for q in seq:
                s = (int(q["Start_Timestamp"]) - t0) / 1e3
                e = (int(q["End_Timestamp"]) - t0) / 1e3
                print("%9.1f %9.1f %7.1f %-34s grid=%s" % (s, e, e - s, q["Kernel_Name"][:34], q["Grid_Size_X"]))
            print()
    if spans:
        print("batches %d: s^-1 %.1f us, gap %.1f us, k_verify %.1f us, span %.1f us (medians)"
              % (len(spans), statistics.median(invs), statistics.median(gaps), statistics.median(vers),
                 statistics.median(spans)))


if __name__ == "__main__":
    main()

"""Timeline of the bench's timed loop from a rocprofv3 kernel trace: the
1M-item k_verify launches and the kernels around them (start / end in us
relative to one verify), and the step period.

    python tools/loop_timeline.py gpurun_out/prof_loop/kt_kernel_trace.csv [first] [count]
"""
import csv
import sys


def main() -> None:
    rows = list(csv.DictReader(open(sys.argv[1])))
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    count = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    v = [i for i, r in enumerate(rows)
         if r["Kernel_Name"].startswith("void k_verify") and int(r["Grid_Size_X"]) >= 1 << 20]
    if len(v) < first + count:
        first, count = 0, len(v)
    t0 = int(rows[v[first]]["Start_Timestamp"])
    for r in rows[v[first] - 6:v[first + count - 1] + 2]:
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        e = (int(r["End_Timestamp"]) - t0) / 1e3
        print("%9.1f %9.1f %7.1f q%-2s s%-2s %-30s grid=%s" % (s, e, e - s, r["Queue_Id"], r["Stream_Id"],
                                                            r["Kernel_Name"][:30], r["Grid_Size_X"]))
    starts = [int(rows[i]["Start_Timestamp"]) for i in v[first:first + count]]
    if len(starts) > 1:
        print("mean verify start-to-start: %.1f us" % ((starts[-1] - starts[0]) / 1e3 / (len(starts) - 1)))


if __name__ == "__main__":
    main()

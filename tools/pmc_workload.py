"""Small fixed workload for rocprofv3 PMC passes: 3 verify launches of the
bench batch (1,048,576 single-signer REQUEST items, inputs in HBM).

    python3 tools/pmc_workload.py [G_WINDOW Q_WINDOW]
"""
import sys

sys.path.insert(0, ".")
import bench  # noqa: E402


def main():
    g, q = (sys.argv[1], sys.argv[2]) if len(sys.argv) > 2 else ("16", "16")
    sys.argv = ["bench.py", "--steps", "3", "--warmup", "0", "--latency-reps", "0",
                "--no-cpu-baseline", "--no-peak-run", "--g-window", g, "--q-window", q]
    bench.main()


if __name__ == "__main__":
    main()

"""Small fixed workload for rocprofv3 PMC passes: 3 verify launches of the
bench batch (1,048,576 single-signer REQUEST items, inputs in HBM)."""
import sys

sys.path.insert(0, ".")
import bench  # noqa: E402


def main():
    sys.argv = ["bench.py", "--steps", "3", "--warmup", "0", "--latency-reps", "0",
                "--no-cpu-baseline", "--no-peak-run"]
    bench.main()


if __name__ == "__main__":
    main()

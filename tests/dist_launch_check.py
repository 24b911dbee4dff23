"""bench.py's `--gpus N` dispatch on CPU (gloo): tests/test_dist.py runs this
script without a launcher.  With N > 1 it restarts itself as N ranks of a
child torch.distributed.run exactly as bench.py does (minbft_amd.dist:
launch_mode / relaunch), each rank joins a gloo group, and rank 0 prints ONE
JSON line (world size, MAX over ranks of a per-rank value), which the parent
relays on its stdout."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from minbft_amd import dist as mdist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    if mdist.launch_mode(args.gpus) == "relaunch":
        sys.exit(mdist.relaunch(os.path.abspath(__file__), sys.argv[1:], args.gpus))
    import torch
    import torch.distributed as dist
    world, rank, _ = mdist.env_ranks()
    if world > 1:
        dist.init_process_group("gloo")
    tmax = mdist.max_over_ranks(dist, float(rank + 1) * args.steps, torch.device("cpu"))
    if rank == 0:
        print(json.dumps({"n_gpus": world, "tmax": tmax, "launched_by": "torchrun" if "WORLD_SIZE" in
                          os.environ else "direct"}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

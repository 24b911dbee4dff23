"""One rank of the world_size-2 CPU rehearsal of the multi-process path
(tests/test_dist.py launches it with torch.distributed.run over gloo, the
way the driver launches bench.py over RCCL).

Each rank verifies its contiguous shard of the golden prehashed vectors with
a stand-in verifier (the oracle's C restatement: there is no GPU here; on a
GPU rank this is Authenticator.verify_prehashed), rank 0 gathers every
status in index order through minbft_amd.dist and writes a JSON report."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from golden_util import prehashed_arrays  # noqa: E402
from minbft_amd import dist as mdist  # noqa: E402


def main(out_path):
    world, rank, _ = mdist.env_ranks()
    dist.init_process_group("gloo")
    dev = torch.device("cpu")
    assert dist.get_world_size() == world == 2

    from oracle import c_oracle
    xy, e, r, s, exp, labels = prehashed_arrays()
    # slot = index of the vector's key in a per-run key list
    keys, slots = {}, np.zeros(len(labels), dtype=np.uint32)
    for i in range(len(labels)):
        slots[i] = keys.setdefault(xy[i].tobytes(), len(keys))
    qxy = np.zeros((len(keys), 64), dtype=np.uint8)
    for k, v in keys.items():
        qxy[v] = np.frombuffer(k, dtype=np.uint8)

    seen = []

    def verify(e_, r_, s_, sl_):
        seen.append(int(e_.shape[0]))
        return c_oracle.verify_prehashed_batch(qxy, e_, r_, s_, sl_, nthreads=2)

    st = mdist.verify_sharded(dist, verify, e, r, s, slots, dev)
    # a ragged total that does not divide by the world size, and an empty one
    st7 = mdist.verify_sharded(dist, verify, e[:7], r[:7], s[:7], slots[:7], dev)
    st0 = mdist.verify_sharded(dist, verify, e[:0], r[:0], s[:0], slots[:0], dev)
    tmax = mdist.max_over_ranks(dist, float(rank + 1) * 1.5, dev)
    # bench.py's per-rank synthetic batches must differ between ranks
    import bench
    msgs = bench.make_requests(rank, 64)
    digest = torch.tensor(msgs[:, 15:47].reshape(-1)[:32].astype(np.int64))
    parts = [torch.empty_like(digest) for _ in range(world)]
    dist.all_gather(parts, digest)
    distinct = not torch.equal(parts[0], parts[1])
    dist.barrier()
    if rank == 0:
        rep = {"world": world, "shard_sizes_rank0": seen,
               "match": bool((((st == 0).astype(np.int64)) == exp).all()),
               "n": int(st.shape[0]),
               "ragged_ok": bool(st7.shape[0] == 7 and (((st7 == 0).astype(np.int64)) == exp[:7]).all()),
               "empty_ok": bool(st0.shape[0] == 0), "tmax": tmax, "distinct_ranks": bool(distinct)}
        with open(out_path, "w") as f:
            json.dump(rep, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])

"""World-size-2 rehearsal of the multi-process (one process per GPU) path on
CPU: torch.distributed.run launches tests/dist_worker.py twice over gloo on
127.0.0.1, exactly as the driver launches bench.py over RCCL.  Checks that
the contiguous shards cover the batch, that rank 0 receives every status in
index order (including a ragged and an empty batch), the MAX-over-ranks
timing rule, and that bench.py's per-rank synthetic batches differ."""
import json
import os
import socket
import subprocess
import sys

import numpy as np

from minbft_amd.dist import shard_range

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shard_range_partitions():
    for n in (0, 1, 7, 551, 1 << 20):
        for world in (1, 2, 3, 8):
            got = [shard_range(n, world, r) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(got, got[1:]))
            sizes = [b - a for a, b in got]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_gloo(tmp_path):
    out = tmp_path / "rep.json"
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "dist_worker.py"), str(out)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    rep = json.loads(out.read_text())
    assert rep["world"] == 2
    assert rep["match"] and rep["ragged_ok"] and rep["empty_ok"]
    assert rep["n"] == 551
    assert rep["shard_sizes_rank0"][0] == 551 // 2
    assert rep["tmax"] == 3.0
    assert rep["distinct_ranks"]
    assert np.isfinite(rep["tmax"])

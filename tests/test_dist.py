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


def _run_check(args, launcher_nproc=0):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    script = os.path.join(ROOT, "tests", "dist_launch_check.py")
    cmd = [sys.executable, script, *args]
    if launcher_nproc:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={launcher_nproc}", "--master-addr=127.0.0.1",
               f"--master-port={_free_port()}", script, *args]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)


def test_gpus_flag_relaunches_two_ranks():
    """`--gpus 2` with no launcher: the script restarts itself as 2 ranks of a
    child torch.distributed.run (bench.py's dispatch) and the parent relays
    rank 0's single JSON line."""
    p = _run_check(["--gpus", "2", "--steps", "3"])
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    rep = json.loads(lines[0])
    assert rep == {"n_gpus": 2, "tmax": 6.0, "launched_by": "torchrun"}


def test_gpus_flag_one_is_direct():
    p = _run_check(["--gpus", "1"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert json.loads(p.stdout.strip()) == {"n_gpus": 1, "tmax": 3.0, "launched_by": "direct"}


def test_gpus_flag_must_match_launcher():
    p = _run_check(["--gpus", "3"], launcher_nproc=2)
    assert p.returncode != 0
    assert "WORLD_SIZE=2" in p.stderr


def test_launch_mode():
    from minbft_amd.dist import launch_mode
    assert launch_mode(1, {}) == "direct"
    assert launch_mode(8, {}) == "relaunch"
    assert launch_mode(8, {"WORLD_SIZE": "8"}) == "direct"
    import pytest
    with pytest.raises(SystemExit):
        launch_mode(8, {"WORLD_SIZE": "1"})

"""Multi-process sharding: one process per GPU.

Verification has no cross-item dependency, so a global batch is split into
contiguous index ranges, one per rank; each rank verifies its own range on
its own GPU with its own tables, and only the status bytes travel (to rank 0,
in index order).  There is no data-path collective: the only collectives are
the timing barrier / max-over-ranks of bench.py and this final status
gather.  The same functions run over RCCL (``nccl`` backend, GPU tensors) on
a node and over ``gloo`` on CPU in tests/test_dist.py.

The in-process alternative (one Go process driving all GPUs of a node) is
``mbft_ctx_add_device`` in the C-ABI; its sharding is the same contiguous
split.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
from typing import Callable, Mapping, Optional, Sequence, Tuple

import numpy as np


def env_ranks() -> Tuple[int, int, int]:
    """(world, rank, local_rank) from torch.distributed.run's environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def launch_mode(gpus: int, env: Mapping[str, str] = os.environ) -> str:
    """How a `--gpus N` run starts (bench.py's contract: N is authoritative).

    * Under torch.distributed.run (WORLD_SIZE set): "direct", and WORLD_SIZE
      must equal N -- a mismatch is an error, not a silently different run.
    * No launcher, N > 1: "relaunch" -- the caller starts N ranks as a child
      torch.distributed.run (relaunch below) before touching any GPU.
    * No launcher, N == 1: "direct" (one process, no process group)."""
    if gpus < 1:
        raise SystemExit(f"--gpus {gpus}: need at least one GPU")
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            raise SystemExit(f"--gpus {gpus} but the launcher started WORLD_SIZE={world} ranks")
        return "direct"
    return "relaunch" if gpus > 1 else "direct"


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def relaunch_cmd(script: str, argv: Sequence[str], nproc: int, port: int) -> list:
    """The torch.distributed.run command the driver itself would use."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr=127.0.0.1", f"--master-port={port}", script, *argv]


def relaunch(script: str, argv: Sequence[str], nproc: int, env: Optional[Mapping[str, str]] = None) -> int:
    """Run `script argv` as nproc ranks of a child torch.distributed.run (one
    process per GPU) and relay its stdout (rank 0's JSON line) line by line;
    stderr passes through.  Returns the child's exit code.  The caller must
    not have initialized a GPU: this process only waits (a child, never an
    exec)."""
    cmd = relaunch_cmd(script, argv, nproc, free_port())
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=dict(env or os.environ))
    assert p.stdout is not None
    for line in p.stdout:
        sys.stdout.write(line)
        sys.stdout.flush()
    return p.wait()


def shard_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous shard [lo, hi) of rank `rank` (sizes differ by at most 1)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    return n * rank // world, n * (rank + 1) // world


def max_over_ranks(dist, value: float, device) -> float:
    """MAX of a per-rank float (bench.py's timing rule)."""
    import torch
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_status(dist, status: np.ndarray, n_total: int, device) -> Optional[np.ndarray]:
    """Concatenate every rank's shard of status bytes in index order; the full
    array is returned on rank 0, None elsewhere.  Shards are padded to a
    common length for all_gather (works on gloo and RCCL)."""
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    lo, hi = shard_range(n_total, world, rank)
    if status.shape[0] != hi - lo:
        raise ValueError(f"rank {rank}: shard has {status.shape[0]} statuses, expected {hi - lo}")
    width = max(1, -(-n_total // world))
    buf = torch.zeros(width, dtype=torch.uint8, device=device)
    if hi > lo:
        buf[: hi - lo] = torch.from_numpy(np.ascontiguousarray(status, dtype=np.uint8)).to(device)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    if rank != 0:
        return None
    out = np.empty(n_total, dtype=np.uint8)
    for r, p in enumerate(parts):
        a, b = shard_range(n_total, world, r)
        out[a:b] = p[: b - a].cpu().numpy()
    return out


def verify_sharded(dist, verify: Callable, e: np.ndarray, r: np.ndarray, s: np.ndarray,
                   slots: np.ndarray, device) -> Optional[np.ndarray]:
    """Each rank verifies its contiguous shard of the global (e, r, s, slot)
    batch with `verify` (Authenticator.verify_prehashed on a GPU rank) and
    rank 0 receives all statuses in index order."""
    n = e.shape[0]
    world, rank = dist.get_world_size(), dist.get_rank()
    lo, hi = shard_range(n, world, rank)
    st = verify(e[lo:hi], r[lo:hi], s[lo:hi], slots[lo:hi]) if hi > lo else \
        np.zeros(0, dtype=np.uint8)
    return gather_status(dist, np.asarray(st, dtype=np.uint8), n, device)

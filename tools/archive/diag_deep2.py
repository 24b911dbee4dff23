"""Diagnostic (round 5): tests/test_gpu_bench_config.py::test_full_batch_w29_mix
with per-item detail of mismatches (kind, lane, whether its wave mixes key
windows)."""
import hashlib, sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np
import torch
torch.cuda.init()
from minbft_amd.authenticator import Authenticator
from oracle import p256 as o
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
W = 29
with Authenticator(0) as a:
    a.set_generator_window(29)
    ds = [int.from_bytes(hashlib.sha256(b"bench config key %d" % i).digest(), "big") % (o.N - 1) + 1 for i in range(2)]
    qs = [o.pubkey(d) for d in ds]
    xy = np.array([list(q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big")) for q in qs], dtype=np.uint8)
    a.set_key_window(W)
    sl_a, va = a.register_points(xy[:1])
    a.set_key_window(8)
    sl_b, vb = a.register_points(xy[1:])
    rng = np.random.Generator(np.random.PCG64(0x29))
    e = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    priv = np.frombuffer(ds[0].to_bytes(32, "big"), dtype=np.uint8)[None, :]
    r, s = a.sign_prehashed(priv, e)
    slot = np.full(n, sl_a[0], dtype=np.uint32)
    kind = np.full(n, -1)
    sel = np.arange(n)[np.arange(n) % 97 == 0]
    kind[sel] = rng.integers(0, 7, size=sel.size)
    Nb = np.frombuffer(o.N.to_bytes(32, "big"), dtype=np.uint8)
    pos = rng.integers(0, 32, size=n)
    t = kind == 0; e[t, pos[t]] ^= 0x04
    t = kind == 1; r[t, pos[t]] ^= 0x20
    t = kind == 2; s[t, pos[t]] ^= 0x01
    r[kind == 3] = 0
    s[kind == 4] = Nb
    slot[kind == 5] = sl_b[0]
    for i in np.nonzero(kind == 6)[0]:
        s[i] = np.frombuffer((o.N - int.from_bytes(s[i].tobytes(), "big")).to_bytes(32, "big"), dtype=np.uint8)
    st = a.verify_prehashed(e, r, s, slot)
    want_accept = (kind == -1) | (kind == 6)
    bad = np.nonzero((st == 0) != want_accept)[0]
    mixed = np.zeros(n // 64, bool)
    mixed[np.unique(np.nonzero(kind == 5)[0] // 64)] = True
    print("n", n, "mismatches", len(bad), "kinds", np.unique(kind[bad], return_counts=True),
          "in mixed-window waves", int(mixed[bad // 64].sum()), "status", np.unique(st[bad], return_counts=True))
    print("first", bad[:20], "waves", len(np.unique(bad // 64)), "mixed waves total", int(mixed.sum()))
    # same batch, the valid items only with slot a everywhere
    slot2 = slot.copy(); slot2[kind == 5] = sl_a[0]
    st2 = a.verify_prehashed(e, r, s, slot2)
    print("without the W=8 key: accepted valid", int((st2[kind == -1] == 0).sum()), "of", int((kind == -1).sum()))

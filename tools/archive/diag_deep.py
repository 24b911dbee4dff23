import hashlib, sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np
import torch
torch.cuda.init()
from minbft_amd.authenticator import Authenticator
from oracle import p256 as o
for W in (16, 29):
    with Authenticator(0) as a:
        a.set_generator_window(W)
        a.set_key_window(W)
        d = int.from_bytes(hashlib.sha256(b"diag").digest(), "big") % (o.N - 1) + 1
        q = o.pubkey(d)
        xy = np.array([list(q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big"))], dtype=np.uint8)
        sl, va = a.register_points(xy)
        n = 1 << 16
        rng = np.random.Generator(np.random.PCG64(5))
        e = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
        priv = np.frombuffer(d.to_bytes(32, "big"), dtype=np.uint8)[None, :]
        r, s = a.sign_prehashed(priv, e)
        slot = np.full(n, sl[0], dtype=np.uint32)
        st = a.verify_prehashed(e, r, s, slot)
        bad = np.nonzero(st != 0)[0]
        print("W", W, "rejects", len(bad), "of", n, "lanes", np.bincount(bad % 64, minlength=64)[:16] if len(bad) else "", "waves", len(np.unique(bad // 64)))
        # dead lanes in a wave: every 7th item r = 0
        r2 = r.copy(); r2[::7] = 0
        st2 = a.verify_prehashed(e, r2, s, slot)
        want = np.ones(n, bool); want[::7] = False
        print("  with dead lanes: mismatches", int(((st2 == 0) != want).sum()))

"""Quick GPU sanity + timing (development aid, not the bench contract)."""
import hashlib
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from minbft_amd.authenticator import Authenticator  # noqa: E402
from oracle import p256 as o  # noqa: E402


def main(n=1 << 20):
    a = Authenticator(0)
    d = int.from_bytes(hashlib.sha256(b"k").digest(), "big") % o.N
    q = o.pubkey(d)
    xy = np.frombuffer(q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big"), dtype=np.uint8)
    slots, valid = a.register_points(xy[None, :])
    print("valid", valid, "slot", slots, flush=True)
    rng = np.random.default_rng(1)
    e = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    priv = np.frombuffer(d.to_bytes(32, "big"), dtype=np.uint8)[None, :]
    t = time.time()
    r, s = a.sign_prehashed(priv, e)
    print("sign %d: %.3f s" % (n, time.time() - t), flush=True)
    # oracle check of a few signatures
    for i in range(4):
        rr = int.from_bytes(r[i].tobytes(), "big")
        ss = int.from_bytes(s[i].tobytes(), "big")
        print("oracle verify", i, o.go_ecdsa_verify(q, e[i].tobytes(), rr, ss), flush=True)
    sl = np.zeros(n, dtype=np.uint32) + slots[0]
    for rep in range(3):
        t = time.time()
        st = a.verify_prehashed(e, r, s, sl)
        dt = time.time() - t
        print("verify %d: %.3f s  %.3f M/s  accept=%d" % (n, dt, n / dt / 1e6, int((st == 0).sum())), flush=True)
    e2 = e.copy()
    e2[:, 5] ^= 1
    st = a.verify_prehashed(e2, r, s, sl)
    print("tampered accept", int((st == 0).sum()), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20)

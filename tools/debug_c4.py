"""Debug aid: reproduce test_c4_adversarial_gpu_share's valid-item rejects and
classify them (signature valid per the C oracle? rejected again when
verified alone? which digits / key?)."""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import torch  # noqa: E402

torch.cuda.init()
from minbft_amd.authenticator import Authenticator  # noqa: E402
from oracle import c_oracle  # noqa: E402
from oracle import p256 as o  # noqa: E402
from test_gpu_configs import _keys  # noqa: E402


def main(n=8 << 20):
    a = Authenticator(0)
    rng = np.random.Generator(np.random.PCG64(0xC4))
    priv, xy = _keys(8)
    slots, valid = a.register_points(xy)
    kidx = rng.integers(0, 8, size=n).astype(np.uint32)
    e = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    r, s = a.sign_prehashed(priv, e, kidx)
    slot = slots[kidx].copy()
    got = a.verify_prehashed(e, r, s, slot)
    bad = np.nonzero(got != 0)[0]
    print("rejected", bad.size, flush=True)
    qx = np.zeros((int(slots.max()) + 1, 64), dtype=np.uint8)
    qx[slots] = xy
    ref = c_oracle.verify_prehashed_batch(qx, e[bad], r[bad], s[bad], slot[bad], nthreads=8)
    print("oracle says valid:", int((ref == 0).sum()), "of", bad.size, flush=True)
    alone = a.verify_prehashed(e[bad], r[bad], s[bad], slot[bad])
    print("GPU alone accepts:", int((alone == 0).sum()), flush=True)
    for i in bad[:8]:
        ri = int.from_bytes(r[i].tobytes(), "big")
        si = int.from_bytes(s[i].tobytes(), "big")
        ei = int.from_bytes(e[i].tobytes(), "big")
        w = pow(si, -1, o.N)
        u1, u2 = ei * w % o.N, ri * w % o.N
        d1 = [(u1 >> (16 * k)) & 0xFFFF for k in range(16)]
        d2 = [(u2 >> (16 * k)) & 0xFFFF for k in range(16)]
        print(int(i), "key", int(kidx[i]), "zero digits G", [k for k, d in enumerate(d1) if d == 0],
              "Q", [k for k, d in enumerate(d2) if d == 0], "ri<2^255", ri < (1 << 255), flush=True)
    from collections import Counter
    cnt = Counter()
    for i in bad:
        ri = int.from_bytes(r[i].tobytes(), "big")
        si = int.from_bytes(s[i].tobytes(), "big")
        ei = int.from_bytes(e[i].tobytes(), "big")
        w = pow(si, -1, o.N)
        u1, u2 = ei * w % o.N, ri * w % o.N
        for k in range(16):
            cnt[("Q", k, (u2 >> (16 * k)) & 0xFFFF)] += 1
            cnt[("G", k, (u1 >> (16 * k)) & 0xFFFF)] += 1
    print("most common (phase, window, digit):", cnt.most_common(6), flush=True)
    b = Authenticator(0)
    s3, v3 = b.register_points(xy[3:4])
    alone3 = b.verify_prehashed(e[bad], r[bad], s[bad], np.full(bad.size, s3[0], np.uint32))
    print("fresh ctx, key 3 alone, accepts:", int((alone3 == 0).sum()), "of", bad.size, flush=True)
    b.close()
    c = Authenticator(0)
    sl8, _ = c.register_points(xy)
    again = c.verify_prehashed(e[bad], r[bad], s[bad], sl8[kidx[bad]])
    print("fresh ctx, 8 keys again, accepts:", int((again == 0).sum()), flush=True)
    c.close()
    # rerun full batch: same items?
    got2 = a.verify_prehashed(e, r, s, slot)
    bad2 = np.nonzero(got2 != 0)[0]
    print("second run rejected", bad2.size, "same set", bool(np.array_equal(bad, bad2)), flush=True)
    a.close()


if __name__ == "__main__":
    main()

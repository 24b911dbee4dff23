"""GPU parity at the EXACT kernel configuration bench.py measures: generator
and key comb windows G = 29 / Q = 29 (258 GiB of tables on one MI355X).

One 129 GiB key table fits beside the 129 GiB generator table, so each key
gets the context to itself in turn (mbft_clear_keys between keys):

* every prehashed golden vector (550 vectors over 50 keys: valid, tampered,
  wrong key, high-s, range edges, e = 0 / N, e >= N, R.x >= N, final
  infinity, u1 G = u2 Q, Q = +-G, and the comb8 / comb16 collision vectors,
  which at W = 29 are ordinary vectors), under its own key at W = 29;
* the comb29 accumulator-collision vectors (tests/golden/comb_windows.json,
  built for the signed 29-bit key windows by make_golden.py);
* a full 1,048,576-item batch, as bench.py runs it, with a reject mix every
  97th item (tampered e, r, s; r = 0; s = N; a wrong key registered at
  W = 8 beside the W = 29 key; high-s, which Go accepts): every status
  checked against its construction and 4,096 items against the C oracle.
"""
import numpy as np
import pytest

from golden_util import prehashed_arrays

pytestmark = pytest.mark.gpu

W = 29


@pytest.fixture(scope="module")
def auth29(lib):
    from minbft_amd.authenticator import Authenticator
    a = Authenticator(0)
    a.set_generator_window(W)
    a.set_key_window(W)
    assert a.windows() == (W, W)
    yield a
    a.close()


def _run_per_key(a, xy, e, r, s):
    """Verify (xy, e, r, s) grouped by key, each key alone at W = 29."""
    st = np.full(len(e), 0xFF, dtype=np.uint8)
    keys = {}
    for i in range(len(e)):
        keys.setdefault(xy[i].tobytes(), []).append(i)
    for k, (kb, idx) in enumerate(keys.items()):
        print(f"key {k + 1}/{len(keys)}: {len(idx)} vectors", flush=True)
        a.clear_keys()
        a.set_key_window(W)
        slots, valid = a.register_points(np.frombuffer(kb, dtype=np.uint8)[None, :])
        assert valid.all()
        idx = np.array(idx)
        st[idx] = a.verify_prehashed(e[idx], r[idx], s[idx],
                                     np.full(len(idx), slots[0], dtype=np.uint32))
    return st


def _check(st, exp, labels):
    got = (st == 0).astype(np.int64)
    bad = [(labels[i], int(st[i]), int(exp[i])) for i in range(len(exp)) if got[i] != exp[i]]
    assert not bad, bad[:20]


def test_golden_prehashed_w29(auth29):
    xy, e, r, s, exp, labels = prehashed_arrays()
    _check(_run_per_key(auth29, xy, e, r, s), exp, labels)


def test_comb29_collisions_w29(auth29):
    xy, e, r, s, exp, labels = prehashed_arrays("comb_windows.json")
    sel = np.array([i for i, l in enumerate(labels) if l.startswith("comb29_")])
    assert len(sel) >= 5
    _check(_run_per_key(auth29, xy[sel], e[sel], r[sel], s[sel]), exp[sel],
           [labels[i] for i in sel])


def test_full_batch_w29_mix(auth29):
    import hashlib

    from oracle import c_oracle
    from oracle import p256 as o
    n = 1 << 20
    a = auth29
    a.clear_keys()
    ds = [int.from_bytes(hashlib.sha256(b"bench config key %d" % i).digest(), "big") % (o.N - 1) + 1
          for i in range(2)]
    qs = [o.pubkey(d) for d in ds]
    xy = np.array([list(q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big")) for q in qs],
                  dtype=np.uint8)
    a.set_key_window(W)
    sl_a, va = a.register_points(xy[:1])
    a.set_key_window(8)
    sl_b, vb = a.register_points(xy[1:])
    assert va.all() and vb.all()
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
    t = kind == 0
    e[t, pos[t]] ^= 0x04                                     # tampered e
    t = kind == 1
    r[t, pos[t]] ^= 0x20                                     # tampered r
    t = kind == 2
    s[t, pos[t]] ^= 0x01                                     # tampered s
    r[kind == 3] = 0                                         # r = 0
    s[kind == 4] = Nb                                        # s = N
    slot[kind == 5] = sl_b[0]                                # wrong key (W = 8 table)
    for i in np.nonzero(kind == 6)[0]:                       # high-s: Go accepts
        s[i] = np.frombuffer((o.N - int.from_bytes(s[i].tobytes(), "big")).to_bytes(32, "big"),
                             dtype=np.uint8)
    st = a.verify_prehashed(e, r, s, slot)
    want_accept = (kind == -1) | (kind == 6)
    assert (st[want_accept] == 0).all()
    assert (st[~want_accept] == 1).all()
    # 4,096 items (every kind represented) against the C oracle
    idx = np.unique(np.concatenate([np.nonzero(kind >= 0)[0][:2048],
                                    rng.choice(n, size=2048, replace=False)]))
    qx = np.zeros((int(max(sl_a[0], sl_b[0])) + 1, 64), dtype=np.uint8)
    qx[sl_a[0]] = xy[0]
    qx[sl_b[0]] = xy[1]
    want = c_oracle.verify_prehashed_batch(qx, e[idx], r[idx], s[idx], slot[idx], nthreads=16)
    assert (st[idx] == want).all()


def _craft(o, q, u1, u2):
    """A valid signature whose verification computes exactly (u1, u2):
    R = u1 G + u2 Q, r = x(R) mod N, s = r / u2, e = u1 s."""
    R = o.combined_mult(u1, u2, q)
    r = R[0] % o.N
    s = r * pow(u2, -1, o.N) % o.N
    return u1 * s % o.N, r, s


def test_zero_windows_w29(auth29):
    """Zero comb digits and an accumulator at infinity are exact in the FAST
    path (k_verify's rare branches; an attacker who picks s controls u1 or u2
    and can force them): crafted valid signatures whose u1 has its first, its
    second, both first, a middle or all but the top G window zero (the last
    two start the accumulator at infinity), u1 = 0, and u2 with a zero low /
    middle / top window -- each also tampered.  Statuses against the
    construction and the C oracle."""
    import hashlib
    import random

    from oracle import c_oracle
    from oracle import p256 as o
    N = o.N
    d = int.from_bytes(hashlib.sha256(b"zero windows w29").digest(), "big") % (N - 1) + 1
    q = o.pubkey(d)
    rng = random.Random(0x2929)

    def clear(u, k):
        return u & ~(((1 << W) - 1) << (W * k)) or 1

    kinds = {
        "g0": lambda: (rng.randrange(1, N >> W) << W, rng.randrange(1, N)),
        "g1": lambda: (rng.randrange(1, 1 << (W - 1)) + (rng.randrange(1, N >> (2 * W)) << (2 * W)),
                       rng.randrange(1, N)),
        "g01_inf": lambda: (rng.randrange(1, N >> (2 * W)) << (2 * W), rng.randrange(1, N)),
        "g_top_only_inf": lambda: (rng.randrange(1, N >> (8 * W)) << (8 * W), rng.randrange(1, N)),
        "g_mid": lambda: (clear(rng.randrange(1, N), rng.randrange(2, 8)), rng.randrange(1, N)),
        "u1_zero": lambda: (0, rng.randrange(1, N)),
        "q_low": lambda: (rng.randrange(1, N), rng.randrange(1, N >> W) << W),
        "q_mid": lambda: (rng.randrange(1, N), clear(rng.randrange(1, N), rng.randrange(1, 8))),
        "q_top": lambda: (rng.randrange(1, N), rng.randrange(1, 1 << (8 * W))),
    }
    rows, labels, exp = [], [], []
    for name, gen in kinds.items():
        for _ in range(12):
            u1, u2 = gen()
            e, r, s = _craft(o, q, u1, u2)
            if r == 0:
                continue
            rows.append((e, r, s))
            labels.append(name)
            exp.append(1)
            rows.append((e ^ 1, r, s))
            labels.append(name + "_tampered")
            exp.append(0)
    be = lambda v: list(v.to_bytes(32, "big"))  # noqa: E731
    e = np.array([be(x[0]) for x in rows], dtype=np.uint8)
    r = np.array([be(x[1]) for x in rows], dtype=np.uint8)
    s = np.array([be(x[2]) for x in rows], dtype=np.uint8)
    xy = np.array([list(q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big"))] * len(rows),
                  dtype=np.uint8)
    st = _run_per_key(auth29, xy, e, r, s)
    _check(st, np.array(exp), labels)
    want = c_oracle.verify_prehashed_batch(xy[:1], e, r, s, np.zeros(len(rows), dtype=np.uint32),
                                           nthreads=8)
    assert (st == want).all()

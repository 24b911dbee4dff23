"""GPU parity tests: the HIP path vs the oracle's golden fixtures, through
the C-ABI.  Run on the MI355X box: pytest -m gpu.

Comb windows: the verify kernel takes the generator and key
windows at run time, so every window size the library accepts is one code
path; these tests cover the key windows 8/16 on the full golden set, each
large generator window (20..29) on the full set, and each large key window
with its own accumulator-collision vectors (tests/golden/comb_windows.json),
all in the signed-digit layout (kernels.hip comb_digit).
"""
import numpy as np
import pytest

from golden_util import prehashed_arrays

pytestmark = pytest.mark.gpu


def _check(st, exp, labels):
    got = (st == 0).astype(np.int64)
    bad = [(labels[i], int(st[i]), int(exp[i])) for i in range(len(exp)) if got[i] != exp[i]]
    assert not bad, bad[:20]


@pytest.mark.parametrize("wbits", [16, 8])
def test_prehashed_golden(lib, wbits):
    from minbft_amd.authenticator import Authenticator
    xy, e, r, s, exp, labels = prehashed_arrays()
    with Authenticator(0) as a:
        a.set_key_window(wbits)
        slots, valid = a.register_points(xy)
        assert valid.all()
        st = a.verify_prehashed(e, r, s, slots)
    _check(st, exp, labels)


@pytest.mark.parametrize("form", ["split", "pairs", "pairs_lane_inv", "quads", "quads_planes"])
def test_prehashed_golden_small_batches(lib, form):
    """The full golden set in batches of <= 200 items: the small-batch
    kernels (k_verify_split: one item per 4-wave workgroup, the windows
    split over the waves and joined, s^-1 per wave; k_verify_pairs reading
    the batched per-wave s^-1 planes, or inverting per lane; k_verify_quads,
    each lane half a scalar's windows, inverting per wave or reading the
    planes), key windows 8 and 16, against the golden
    expectation (every crafted edge case: u1 G == u2 Q, final infinity,
    R.x >= N, comb collisions, high s)."""
    from minbft_amd.authenticator import Authenticator
    xy, e, r, s, exp, labels = prehashed_arrays()
    for wbits in (16, 8):
        with Authenticator(0) as a:
            a.set_small_batch_form(256 if form == "split" else 0)
            a.set_small_batch_inverse({"pairs_lane_inv": 0, "quads": 2, "quads_planes": 3}.get(form, 1))
            a.set_key_window(wbits)
            slots, valid = a.register_points(xy)
            assert valid.all()
            st = np.concatenate([a.verify_prehashed(e[k:k + 200], r[k:k + 200], s[k:k + 200], slots[k:k + 200])
                                 for k in range(0, len(labels), 200)])
        _check(st, exp, labels)


@pytest.mark.parametrize("gbits", [20, 22, 24, 26, 29])
def test_generator_windows(lib, gbits):
    """Full golden set with a large generator comb (partial last window for
    every one of these sizes); key tables at window 8 to keep HBM small."""
    from minbft_amd.authenticator import Authenticator
    xy, e, r, s, exp, labels = prehashed_arrays()
    with Authenticator(0) as a:
        a.set_generator_window(gbits)
        a.set_key_window(8)
        assert a.windows() == (gbits, 8)
        slots, valid = a.register_points(xy)
        assert valid.all()
        st = a.verify_prehashed(e, r, s, slots)
    _check(st, exp, labels)


@pytest.mark.parametrize("qbits", [20, 22, 24, 26, 29])
def test_key_windows(lib, qbits):
    """Large key windows: the collision vectors built for this window, plus
    valid / tampered / wrong-key / high-s vectors of one key, in contexts of
    at most 147 GiB of key tables each (one 129 GiB table at W = 29)."""
    from minbft_amd.authenticator import Authenticator
    cxy, ce, cr, cs, cexp, clab = prehashed_arrays("comb_windows.json")
    sel = [i for i, l in enumerate(clab) if l.startswith("comb%d_" % qbits)]
    assert len(sel) >= 5
    xy, e, r, s, exp, labels = prehashed_arrays()
    key0 = xy[0]
    same = [i for i in range(len(labels)) if (xy[i] == key0).all()]
    assert len(same) >= 8
    per_ctx = 1 if qbits >= 29 else 8
    groups = [[("c", i) for i in sel[k:k + per_ctx]] for k in range(0, len(sel), per_ctx)]
    groups.append([("p", i) for i in same])
    for grp in groups:
        src = {"c": (cxy, ce, cr, cs, cexp, clab), "p": (xy, e, r, s, exp, labels)}
        pick = lambda j: np.stack([src[t][j][i] for t, i in grp])  # noqa: E731
        gexp = np.array([src[t][4][i] for t, i in grp])
        glab = [src[t][5][i] for t, i in grp]
        with Authenticator(0) as a:
            a.set_key_window(qbits)
            slots, valid = a.register_points(pick(0))
            assert valid.all()
            st = a.verify_prehashed(pick(1), pick(2), pick(3), slots)
        _check(st, gexp, glab)


def test_mixed_key_windows(lib):
    """Keys registered under different windows in one context: each slot
    keeps its own table and window."""
    from minbft_amd.authenticator import Authenticator
    xy, e, r, s, exp, labels = prehashed_arrays()
    n = len(labels)
    with Authenticator(0) as a:
        a.set_key_window(8)
        slots8, v8 = a.register_points(xy[: n // 2])
        a.set_key_window(12)
        slots12, v12 = a.register_points(xy[n // 2:])
        assert v8.all() and v12.all()
        slots = np.concatenate([slots8, slots12])
        st = a.verify_prehashed(e, r, s, slots)
    _check(st, exp, labels)


@pytest.mark.parametrize("wbits", [16, 8])
def test_lane_and_batched_inverse_agree(lib, wbits):
    """Small batches (<= MBFT_LANE_INV_MAX, 4096) invert s per lane inside
    k_verify (divsteps); larger ones use the batched chain.  The golden set
    alone (551 vectors) takes the lane path, the same vectors tiled past
    4,096 items the batched one: identical statuses, every golden
    expectation."""
    from minbft_amd.authenticator import Authenticator
    xy, e, r, s, exp, labels = prehashed_arrays()
    reps = 4096 // len(labels) + 2
    with Authenticator(0) as a:
        a.set_key_window(wbits)
        slots, valid = a.register_points(xy)
        assert valid.all()
        lane = a.verify_prehashed(e, r, s, slots)
        tile = lambda x: np.concatenate([x] * reps)  # noqa: E731
        batched = a.verify_prehashed(tile(e), tile(r), tile(s), tile(slots))
    assert len(batched) > 4096
    _check(lane, exp, labels)
    assert (batched == tile(lane)).all()


@pytest.mark.parametrize("wbits", [16, 8])
def test_small_batch_forms_agree(lib, wbits):
    """The golden set tiled to 3,306 items (the small-batch range, past the
    split kernel's): lane pairs inverting per lane (form 0), lane pairs on
    the batched per-wave s^-1 planes (1), lane quads inverting per wave (2)
    or on the planes (3) -- every golden expectation, in every copy, for
    each form."""
    from minbft_amd.authenticator import Authenticator
    xy, e, r, s, exp, labels = prehashed_arrays()
    reps = 6
    tile = lambda x: np.concatenate([x] * reps)  # noqa: E731
    with Authenticator(0) as a:
        a.set_key_window(wbits)
        slots, valid = a.register_points(xy)
        assert valid.all()
        a.set_small_batch_form(0)
        for form in (0, 1, 2, 3):
            a.set_small_batch_inverse(form)
            st = a.verify_prehashed(tile(e), tile(r), tile(s), tile(slots))
            _check(st, tile(exp), labels * reps)


@pytest.mark.parametrize("n", [1, 17, 5000, 65537])
def test_batch_sizes_tree_shapes(gpu_auth, n):
    """Batch sizes that give every shape of the s^-1 tree: one item, a
    single partial chain, one level into k_ninv_top, and 16 * 4096 + 1 (two
    chain levels, 257 totals at the top).  Valid signatures accept, every
    7th digest flipped rejects."""
    import hashlib

    from oracle import p256 as o
    d = int.from_bytes(hashlib.sha256(b"tree shapes").digest(), "big") % (o.N - 1) + 1
    q = o.pubkey(d)
    xy = np.frombuffer(q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big"), dtype=np.uint8)
    slots, valid = gpu_auth.register_points(xy[None, :])
    rng = np.random.Generator(np.random.PCG64(n))
    e = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    priv = np.frombuffer(d.to_bytes(32, "big"), dtype=np.uint8)[None, :]
    r, s = gpu_auth.sign_prehashed(priv, e)
    e[::7, 3] ^= 0x08
    st = gpu_auth.verify_prehashed(e, r, s, np.full(n, slots[0], dtype=np.uint32))
    want = np.zeros(n, dtype=np.uint8)
    want[::7] = 1
    assert (st == want).all(), np.nonzero(st != want)[0][:10]


def test_exact_path_queue(gpu_auth):
    """Items whose u2 has a zero comb window (crafted with the signer's key:
    u2 = v 2^W, s = r / u2, e = r (k / u2 - d)) leave the fast loop for the
    queued exact path (k_verify_slow): 96 of them, valid and with a flipped
    digest, spread over a 4,096-item batch of ordinary signatures at key
    window 16 -- a wave holding several, one, or none -- against the C oracle."""
    import hashlib
    import random

    from oracle import c_oracle
    from oracle import p256 as o
    rng = random.Random(0x51)
    d = int.from_bytes(hashlib.sha256(b"exact path queue").digest(), "big") % (o.N - 1) + 1
    q = o.pubkey(d)
    xy = np.frombuffer(q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big"), dtype=np.uint8)
    n = 4096
    npr = np.random.Generator(np.random.PCG64(0x51))
    e = npr.integers(0, 256, size=(n, 32), dtype=np.uint8)
    priv = np.frombuffer(d.to_bytes(32, "big"), dtype=np.uint8)[None, :]
    slots, _ = gpu_auth.register_points(xy[None, :])   # default key window 16
    r, s = gpu_auth.sign_prehashed(priv, e)
    pos = sorted(rng.sample(range(n), 96))
    for j, i in enumerate(pos):
        k = rng.randrange(1, o.N)
        u2 = rng.randrange(1, o.N >> 16) << 16 if j % 2 else rng.randrange(1, o.N >> 48) << 48
        rr = o.scalar_mult(k, o.G)[0] % o.N
        iu = pow(u2, -1, o.N)
        ss = rr * iu % o.N
        ee = rr * ((k * iu - d) % o.N) % o.N
        if j % 3 == 0:
            ee ^= 1 << 200                                        # tampered: must reject
        e[i] = np.frombuffer(ee.to_bytes(32, "big"), dtype=np.uint8)
        r[i] = np.frombuffer(rr.to_bytes(32, "big"), dtype=np.uint8)
        s[i] = np.frombuffer(ss.to_bytes(32, "big"), dtype=np.uint8)
    sl = np.full(n, slots[0], dtype=np.uint32)
    st = gpu_auth.verify_prehashed(e, r, s, sl)
    qx = np.zeros((int(slots[0]) + 1, 64), dtype=np.uint8)
    qx[slots[0]] = xy
    want = c_oracle.verify_prehashed_batch(qx, e, r, s, sl, nthreads=16)
    assert (st == want).all(), np.nonzero(st != want)[0][:10]
    got = st[pos]
    assert (got[0::3] == 1).all() and (got[1::3] == 0).all() and (got[2::3] == 0).all()


def test_exact_path_queue_many(gpu_auth):
    """A long exact-path queue: 8,192 crafted items (u2 = v 2^16: a zero
    first key window at window 16), every third with a flipped digest, at
    every 4th position of a 32,768-item batch, run twice back to back (the
    queue buffers are reused); every status against the construction."""
    import random

    import torch

    N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
    rng = random.Random(0x57EA1)
    d = rng.randrange(1, N)
    from oracle import p256 as o
    q = o.pubkey(d)
    xy = np.frombuffer(q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big"), dtype=np.uint8)
    slots, _ = gpu_auth.register_points(xy[None, :])   # default key window 16
    n, m = 32768, 8192
    dev = torch.device("cuda", 0)

    def rows(vals):
        return np.frombuffer(b"".join(v.to_bytes(32, "big") for v in vals), dtype=np.uint8).reshape(-1, 32).copy()

    ks = [rng.randrange(1, N) for _ in range(m)]
    u2 = [rng.randrange(1, N >> 16) << 16 for _ in range(m)]
    priv = torch.from_numpy(np.frombuffer(d.to_bytes(32, "big"), dtype=np.uint8).copy()).to(dev)
    d_k = torch.from_numpy(rows(ks)).to(dev)
    d_z = torch.zeros((m, 32), dtype=torch.uint8, device=dev)
    d_r = torch.empty((m, 32), dtype=torch.uint8, device=dev)
    d_s = torch.empty((m, 32), dtype=torch.uint8, device=dev)
    gpu_auth.sign_nonce_device(priv.data_ptr(), 0, d_z.data_ptr(), d_k.data_ptr(), m, d_r.data_ptr(),
                               d_s.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    rs = [int.from_bytes(b.tobytes(), "big") for b in d_r.cpu().numpy()]
    iu = [pow(v, -1, N) for v in u2]
    cs = [rs[i] * iu[i] % N for i in range(m)]
    ce = [rs[i] * ((ks[i] * iu[i] - d) % N) % N for i in range(m)]
    for j in range(0, m, 3):
        ce[j] ^= 1 << 100                                   # tampered: must reject
    npr = np.random.Generator(np.random.PCG64(0x57EA1))
    e = npr.integers(0, 256, size=(n, 32), dtype=np.uint8)
    r, s = gpu_auth.sign_prehashed(np.frombuffer(d.to_bytes(32, "big"), dtype=np.uint8)[None, :], e)
    pos = np.arange(0, n, 4)
    e[pos], r[pos], s[pos] = rows(ce), rows(rs), rows(cs)
    want = np.zeros(n, dtype=np.uint8)
    want[pos[0::3]] = 1
    sl = np.full(n, slots[0], dtype=np.uint32)
    for _ in range(2):
        st = gpu_auth.verify_prehashed(e, r, s, sl)
        assert (st == want).all(), np.nonzero(st != want)[0][:10]


def test_exact_path_queue_degenerate(gpu_auth):
    """The exact-path queue itself: items whose key-phase mixed addition is
    DEGENERATE (accumulator == +-entry, crafted with the key's discrete log,
    bench.craft_degenerate) at every 8th position of a 16,384-item batch (the
    batched-chain path, > 4,096 items), every third tampered; k_verify queues
    them for k_verify_slow.  Every status against the construction, twice
    (queue buffers reused)."""
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from oracle import p256 as o
    d = 0x5EED0F
    q = o.pubkey(d)
    xy = np.frombuffer(q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big"), dtype=np.uint8)
    slots, _ = gpu_auth.register_points(xy[None, :])   # default key window 16
    W = gpu_auth.windows()[1]
    rows = bench.craft_degenerate(d, W, 48, 0xDE6)
    for e_, r_, s_ in rows[:8]:
        assert o.go_ecdsa_verify(q, e_.to_bytes(32, "big"), r_, s_)
    n = 16384
    npr = np.random.Generator(np.random.PCG64(0xDE6))
    e = npr.integers(0, 256, size=(n, 32), dtype=np.uint8)
    r, s = gpu_auth.sign_prehashed(np.frombuffer(d.to_bytes(32, "big"), dtype=np.uint8)[None, :], e)
    pos = np.arange(0, n, 8)
    want = np.zeros(n, dtype=np.uint8)
    be = lambda v: np.frombuffer(v.to_bytes(32, "big"), dtype=np.uint8)  # noqa: E731
    for k, p in enumerate(pos):
        e_, r_, s_ = rows[k % len(rows)]
        if k % 3 == 0:
            e_ ^= 1 << 77
            want[p] = 1
        e[p], r[p], s[p] = be(e_), be(r_), be(s_)
    sl = np.full(n, slots[0], dtype=np.uint32)
    for _ in range(2):
        st = gpu_auth.verify_prehashed(e, r, s, sl)
        assert (st == want).all(), np.nonzero(st != want)[0][:10]


@pytest.mark.parametrize("n", [4097, 2048 * 5 + 77, 100_003])
def test_inverse_forms_agree(lib, monkeypatch, n):
    """The two batched s^-1 forms verify_device picks from (host.cpp: the
    one-launch k_ninv_local on an idle GPU, the level chain k_ninv_up / _top
    / _down beside batches in flight) give the golden statuses on the same
    tiled batch: ragged sizes around the local form's 2,048-item blocks and
    above the per-lane inversion's 4,096-item limit, every golden vector
    (range edges, high s, infinity, collisions) present."""
    from minbft_amd.authenticator import Authenticator
    xy, e, r, s, exp, labels = prehashed_arrays()
    reps = -(-n // len(labels))
    idx = np.tile(np.arange(len(labels)), reps)[:n]
    got = {}
    with Authenticator(0) as a:
        a.set_key_window(16)
        slots, valid = a.register_points(xy)
        assert valid.all()
        for form in ("local", "levels"):
            monkeypatch.setenv("MBFT_NINV", form)
            got[form] = a.verify_prehashed(e[idx], r[idx], s[idx], slots[idx])
            _check(got[form], exp[idx], [labels[i] for i in idx])
    assert (got["local"] == got["levels"]).all()

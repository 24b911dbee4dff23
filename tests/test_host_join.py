"""The host end of a resident-kernel verify (join_host.cpp, through the
mbft_debug_host_join hook; no GPU): four partial comb sums in the device's
limb format -- Chudnovsky (X, Y, ZZ, ZZZ) at random Z, 9 x 29-bit limbs in
Montgomery form (R = 2^261), canonical, plus a multiple of p, or with lazy
limbs -- joined and x-checked against r.  The result must be the oracle's
crypto/ecdsa.Verify outcome (oracle/p256.py go_ecdsa_verify, restating Go's
verifyGeneric as called at sample/authentication/crypto.go:86) for valid
and tampered signatures, partial sums at infinity, equal partial sums (the
join doubles), opposite ones (they cancel), a sum at infinity (reject) and
x(R) >= N (the r + N < p branch)."""
import ctypes
import random

import pytest

from oracle import p256 as o

R_DEV = pow(2, 261, o.P)


@pytest.fixture(scope="module")
def join():
    from minbft_amd import load_library
    lib = load_library()
    f = lib.mbft_debug_host_join
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p]
    return f


def _limbs(v, rng, form):
    """9 x 29-bit limbs of v (< 2^261): canonical, v + k p, or lazy (a limb
    borrows 2^29 from the next one, up to 2^32)."""
    if form == 1:
        for k in (3, 2, 1):
            if v + k * o.P < 2 ** 261:
                v += k * o.P
                break
    w = [(v >> (29 * k)) & (2 ** 29 - 1) for k in range(9)]
    if form == 2:
        for k in range(8):
            if w[k + 1] >= 7 and rng.random() < 0.5:
                t = rng.randrange(1, 8)
                w[k] += t << 29
                w[k + 1] -= t
    assert sum(x << (29 * k) for k, x in enumerate(w)) % o.P == v % o.P
    return w


def _part(pt, rng, form, affine=False):
    """One partial sum's 40 words (or infinity); affine: Z = 1 (the kernel's
    single-window partials)."""
    if pt is None:
        return [0] * 36 + [1, 0, 0, 0]
    x, y = pt
    z = 1 if affine else rng.randrange(1, o.P)
    vals = [x * z * z % o.P, y * pow(z, 3, o.P) % o.P, z * z % o.P, pow(z, 3, o.P)]
    words = []
    for v in vals:
        words += _limbs(v * R_DEV % o.P, rng, form)
    return words + [0, 0, 0, 0]


def _run(join, parts, r):
    arr = (ctypes.c_uint32 * (40 * len(parts)))(*[w for p in parts for w in p])
    return join(arr, len(parts), r.to_bytes(32, "big"))


def _sig_case(rng, tamper=False):
    d = rng.randrange(1, o.N)
    q = o.pubkey(d)
    h = rng.randbytes(32)
    r, s = o.ecdsa_sign(d, h)
    if tamper:
        h = bytes([h[0] ^ 1]) + h[1:]
    e = o.hash_to_int(h)
    w = pow(s, -1, o.N)
    return q, e * w % o.N, r * w % o.N, r, o.go_ecdsa_verify(q, h, r, s)


def _split(rng, u1, u2, q, mode="random"):
    if mode == "equal":  # G partials equal (doubling), Q partials random
        a = u1 * pow(2, -1, o.N) % o.N
        b = a
    elif mode == "zero":
        a, b = 0, u1
    else:
        a = rng.randrange(o.N)
        b = (u1 - a) % o.N
    c = rng.randrange(o.N)
    dd = (u2 - c) % o.N
    pts = [o.scalar_mult(k, o.G) if k else None for k in (a, b)]
    pts += [o.scalar_mult(k, q) if k else None for k in (c, dd)]
    return pts


@pytest.mark.parametrize("form", [0, 1, 2])
def test_valid_and_tampered(join, form):
    rng = random.Random(0x701 + form)
    for k in range(24):
        q, u1, u2, r, want = _sig_case(rng, tamper=(k % 3 == 2))
        mode = ("random", "equal", "zero")[k % 3]
        parts = [_part(p, rng, form) for p in _split(rng, u1, u2, q, mode)]
        assert _run(join, parts, r) == (0 if want else 1), (k, mode)


def test_cancel_and_infinity(join):
    rng = random.Random(0x702)
    q, u1, u2, r, want = _sig_case(rng)
    assert want
    a = rng.randrange(1, o.N)
    # G partials opposite (cancel), Q partials carry the whole sum
    pts = [o.scalar_mult(a, o.G), o.scalar_mult(o.N - a, o.G),
           o.scalar_mult(u2, q), o.scalar_mult(u1, o.G)]
    assert _run(join, [_part(p, rng, 0) for p in pts], r) == 0
    # every partial at infinity, and a sum at infinity: reject
    assert _run(join, [_part(None, rng, 0)] * 4, r) == 1
    p1 = o.scalar_mult(a, o.G)
    pts = [p1, o.point_neg(p1), None, None]
    assert _run(join, [_part(p, rng, 1) for p in pts], r) == 1


def test_x_at_least_n(join):
    """x(R) in [N, p): Go accepts r = x - N (x mod N == r)."""
    rng = random.Random(0x703)
    for _ in range(200):
        x = rng.randrange(o.N, o.P)
        y2 = (pow(x, 3, o.P) - 3 * x + o.B) % o.P
        y = pow(y2, (o.P + 1) // 4, o.P)
        if y * y % o.P == y2:
            break
    else:
        pytest.skip("no point found")
    pt = (x, y)
    a = rng.randrange(1, o.N)
    pa = o.scalar_mult(a, o.G)
    pts = [pa, o.point_add(pt, o.point_neg(pa)), None, None]
    parts = [_part(p, rng, 2) for p in pts]
    assert _run(join, parts, x - o.N) == 0
    assert _run(join, parts, (x - o.N + 1) % o.N) == 1


def test_eight_partials(join):
    """The 8-wave form: each scalar's windows in 4 ranges, 8 partial sums."""
    rng = random.Random(0x704)
    for k in range(12):
        q, u1, u2, r, want = _sig_case(rng, tamper=(k % 4 == 3))
        a = [rng.randrange(o.N) for _ in range(3)]
        c = [rng.randrange(o.N) for _ in range(3)]
        ks_g = a + [(u1 - sum(a)) % o.N]
        ks_q = c + [(u2 - sum(c)) % o.N]
        if k % 4 == 1:
            ks_g[1] = 0  # a range at infinity
            ks_g[3] = (u1 - ks_g[0] - ks_g[2]) % o.N
        pts = [o.scalar_mult(x, o.G) if x else None for x in ks_g] + \
              [o.scalar_mult(x, q) if x else None for x in ks_q]
        parts = [_part(p, rng, k % 3, affine=(i % 3 == 2)) for i, p in enumerate(pts)]
        assert _run(join, parts, r) == (0 if want else 1), k


def test_sixteen_partials_with_affine(join):
    """The two-workgroup form's layout: 16 slots, 8 per scalar (4 range sums
    and up to 4 affine single-window entries, the rest at infinity)."""
    rng = random.Random(0x705)
    for k in range(10):
        q, u1, u2, r, want = _sig_case(rng, tamper=(k % 5 == 4))
        parts = []
        for u, base in ((u1, o.G), (u2, q)):
            ks = [rng.randrange(o.N) for _ in range(5)]
            ks.append((u - sum(ks)) % o.N)
            pts = [o.scalar_mult(x, base) for x in ks]
            slots = [_part(pts[i], rng, i % 3) for i in range(4)]
            slots += [_part(pts[4], rng, 0, affine=True), None, _part(pts[5], rng, 2, affine=True), None]
            parts += [s_ if s_ is not None else _part(None, rng, 0) for s_ in slots]
        assert _run(join, parts, r) == (0 if want else 1), k


def test_host_scalars():
    """u1 = e s^-1, u2 = r s^-1 mod N on the host (winv_host.cpp host_scalars,
    what the resident kernel's comb digits start from) against Python big
    integers: e at and above N (no reduction before the product), extreme r
    and s, and invalid s (zeros)."""
    from minbft_amd import load_library
    f = load_library().mbft_debug_host_scalars
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_char_p] * 3 + [ctypes.c_void_p]
    rng = random.Random(0x706)
    cases = [(rng.randrange(2 ** 256), rng.randrange(1, o.N), rng.randrange(1, o.N)) for _ in range(200)]
    cases += [(0, 1, 1), (o.N, o.N - 1, o.N - 1), (2 ** 256 - 1, 1, o.N - 1), (o.N - 1, o.N - 1, 1),
              (2 ** 256 - 1, 5, 0), (7, 5, o.N), (7, 5, 2 ** 256 - 1)]
    for e, r, s in cases:
        out = (ctypes.c_uint32 * 16)()
        assert f(e.to_bytes(32, "big"), r.to_bytes(32, "big"), s.to_bytes(32, "big"), out) == 0
        u1 = sum(out[j] << (32 * j) for j in range(8))
        u2 = sum(out[8 + j] << (32 * j) for j in range(8))
        if 0 < s < o.N:
            w = pow(s, -1, o.N)
            assert (u1, u2) == (e * w % o.N, r * w % o.N), (e, r, s)
        else:
            assert (u1, u2) == (0, 0)

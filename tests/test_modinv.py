"""The divsteps inversion mod N at the root of the batched s^-1 tree
(minbft_amd/csrc/modinv.h, run by k_ninv_top on one lane) checked on the
HOST against Python big integers: the same header compiled into the test-only
tests/libmodinv_check.so (tests/csrc/modinv_check.cpp)."""
import ctypes
import os
import random

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551


@pytest.fixture(scope="module")
def modinv():
    from __graft_entry__ import build_modinv_check
    lib = ctypes.CDLL(build_modinv_check())
    lib.modinv_check_run.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int]
    lib.modinv_check_run.restype = ctypes.c_int

    def run(xs):
        n = len(xs)
        x = np.zeros((n, 8), dtype=np.uint32)
        for i, v in enumerate(xs):
            for j in range(8):
                x[i, j] = (v >> (32 * j)) & 0xFFFFFFFF
        out = np.zeros((n, 8), dtype=np.uint32)
        ok = np.zeros(n, dtype=np.uint8)
        lib.modinv_check_run(x.ctypes.data, out.ctypes.data, ok.ctypes.data, n)
        return [(bool(ok[i]), sum(int(out[i, j]) << (32 * j) for j in range(8))) for i in range(n)]
    return run


def test_random_and_edges(modinv):
    rng = random.Random(0x1A7)
    xs = [1, 2, 3, N - 1, N - 2, N >> 1, (N >> 1) + 1, 1 << 255, (1 << 128) - 1, 0xFFFFFFFF]
    xs += [rng.randrange(1, N) for _ in range(30000)]
    xs += [rng.randrange(1, 1 << rng.randrange(1, 256)) for _ in range(5000)]
    xs += [N - rng.randrange(1, 1 << 64) for _ in range(2000)]
    for x, (ok, got) in zip(xs, modinv(xs)):
        assert ok and got == pow(x, -1, N), hex(x)


def test_not_invertible(modinv):
    """0 and N have no inverse: reported, never a wrong value."""
    for ok, _ in modinv([0, N]):
        assert not ok


def test_host_winv_planes():
    """The lone calls' host s^-1 (minbft_amd/csrc/winv_host.cpp host_winv):
    s^-1 2^261 mod N in 9 planes of 29-bit limbs, zeros for s = 0 or s >= N
    (k_verify_split rejects those before reading w)."""
    from __graft_entry__ import build_modinv_check
    lib = ctypes.CDLL(build_modinv_check())
    lib.winv_check_run.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    rng = random.Random(0x5117)
    ss = [1, 2, N - 1, N, N + 1, 0, (1 << 256) - 1, 1 << 255, 1 << 200, 0xFFFFFFFF]
    ss += [rng.randrange(1, N) for _ in range(3000)]
    ss += [rng.randrange(1, 1 << rng.randrange(1, 256)) for _ in range(1000)]
    n = len(ss)
    sb = np.frombuffer(b"".join(v.to_bytes(32, "big") for v in ss), dtype=np.uint8).copy()
    # one call (the divsteps alone), small batches and the whole set
    # (Montgomery's trick with invalid values among valid ones)
    for lo, m in ((0, 1), (3, 1), (0, 2), (2, 3), (0, 7), (5, 64), (0, n)):
        sub = np.ascontiguousarray(sb[32 * lo:32 * (lo + m)])
        planes = np.full((9, m), 0xDEADBEEF, dtype=np.uint32)
        lib.winv_check_run(sub.ctypes.data, m, planes.ctypes.data)
        for i, v in enumerate(ss[lo:lo + m]):
            got = sum(int(planes[k, i]) << (29 * k) for k in range(9))
            want = pow(v, -1, N) * (1 << 261) % N if 0 < v < N else 0
            assert got == want, (lo, m, i, hex(v))


def test_host_winv_u():
    """host_winv_u (the small batches' host-staged scalars, read by
    k_verify_split): the same s^-1 planes, then u1 = e s^-1 and u2 = r s^-1
    mod N as 16 LE words per call, zeros for an invalid s -- one call
    (host_scalars) and batches by Montgomery's trick; e and r up to 2^256 - 1
    (no reduction first, as Go's u1 = e w mod N)."""
    from __graft_entry__ import build_modinv_check
    lib = ctypes.CDLL(build_modinv_check())
    lib.winv_u_check_run.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_size_t, ctypes.c_void_p]
    rng = random.Random(0x5118)
    ss = [1, N - 1, N, 0, (1 << 256) - 1] + [rng.randrange(1, N) for _ in range(300)]
    es = [rng.randrange(1 << 256) for _ in ss]
    rs = [rng.randrange(1, N) for _ in ss]
    es[1], rs[1] = (1 << 256) - 1, N - 1
    n = len(ss)
    pack = lambda xs: np.frombuffer(b"".join(v.to_bytes(32, "big") for v in xs), dtype=np.uint8).copy()
    eb, rb, sb = pack(es), pack(rs), pack(ss)
    for lo, m in ((0, 1), (5, 1), (1, 1), (0, 2), (2, 3), (0, 7), (5, 64), (0, n)):
        sub = [np.ascontiguousarray(x[32 * lo:32 * (lo + m)]) for x in (eb, rb, sb)]
        buf = np.full(25 * m, 0xDEADBEEF, dtype=np.uint32)
        lib.winv_u_check_run(sub[0].ctypes.data, sub[1].ctypes.data, sub[2].ctypes.data, m, buf.ctypes.data)
        planes = buf[:9 * m].reshape(9, m)
        u = buf[9 * m:].reshape(m, 16)
        for i in range(m):
            e, r, s = es[lo + i], rs[lo + i], ss[lo + i]
            got_w = sum(int(planes[k, i]) << (29 * k) for k in range(9))
            u1 = sum(int(u[i, j]) << (32 * j) for j in range(8))
            u2 = sum(int(u[i, 8 + j]) << (32 * j) for j in range(8))
            if 0 < s < N:
                w = pow(s, -1, N)
                assert (got_w, u1, u2) == (w * (1 << 261) % N, e * w % N, r * w % N), (lo, m, i)
            else:
                assert (got_w, u1, u2) == (0, 0, 0), (lo, m, i)

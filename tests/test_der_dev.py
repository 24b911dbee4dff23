"""The device DER decoder (minbft_amd/csrc/der_dev.h, run per lane by
k_prepare when flat calls are decoded on the GPU) against the host product
parser (der.cpp, mbft_der_parse_sig) and the golden Go outcomes, rule by
rule: the same header compiled for the HOST into the test-only
tests/libder_dev_check.so (tests/csrc/der_dev_check.cpp).  The GPU run of
the same code is compared with the host decode in
tests/test_gpu_authen.py::test_device_decode_*."""
import ctypes
import json
import os
import random

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def der_dev():
    from __graft_entry__ import build_der_dev_check
    lib = ctypes.CDLL(build_der_dev_check())
    lib.der_dev_run.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_int] + [ctypes.c_void_p] * 4
    lib.der_dev_run.restype = ctypes.c_int

    def run(sigs):
        n = len(sigs)
        off = np.zeros(n + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(b) for b in sigs])
        data = np.frombuffer(b"".join(sigs) + b"\0", dtype=np.uint8).copy()
        ok = np.zeros(n, dtype=np.uint8)
        r = np.zeros((n, 32), dtype=np.uint8)
        s = np.zeros((n, 32), dtype=np.uint8)
        used = np.zeros(n, dtype=np.uint32)
        lib.der_dev_run(data.ctypes.data, off.ctypes.data, n, ok.ctypes.data, r.ctypes.data,
                        s.ctypes.data, used.ctypes.data)
        return [(bool(ok[i]), bytes(r[i]), bytes(s[i]), int(used[i])) for i in range(n)]
    return run


def _host(sig):
    from minbft_amd import _lib
    return _lib.der_parse_sig(sig)


def _same(dev, host):
    ok, r, s, used = dev
    if host is None:
        return not ok and r == bytes(32) and s == bytes(32)
    return ok and (r, s, used) == host


def test_golden_strings(der_dev):
    with open(os.path.join(ROOT, "tests", "golden", "der.json")) as f:
        vs = json.load(f)
    sigs = [bytes.fromhex(v["sig"]) for v in vs]
    for v, sig, got in zip(vs, sigs, der_dev(sigs)):
        assert got[0] == (v["ok"] == 1), v
        assert _same(got, _host(sig)), (v, got)


def test_mutations_match_host_parser(der_dev):
    """~60K mutated encodings (byte edits, deletions, insertions, length-byte
    and tag edits, long-form lengths, random strings) decode identically."""
    from oracle import p256 as o
    rng = random.Random(0xDE5)
    bases = [o.der_encode_sig(rng.randrange(1, o.N), rng.randrange(1, o.N)) for _ in range(16)]
    bases += [o.der_encode_sig(rng.randrange(1, 1 << rng.randrange(1, 256)),
                               rng.randrange(1, 1 << rng.randrange(1, 256))) for _ in range(16)]
    sigs = []
    for _ in range(60000):
        b = bytearray(rng.choice(bases) if rng.random() < 0.8 else rng.randbytes(rng.randrange(0, 90)))
        for _ in range(rng.randrange(0, 4)):
            k = rng.randrange(6)
            if k == 0 and b:
                b[rng.randrange(len(b))] = rng.randrange(256)
            elif k == 1 and b:
                del b[rng.randrange(len(b))]
            elif k == 2:
                b.insert(rng.randrange(len(b) + 1), rng.randrange(256))
            elif k == 3 and len(b) > 1:
                b[1] = rng.choice([0x80, 0x81, 0x82, 0x84, 0x7f, len(b) - 2, len(b), 0xff])
            elif k == 4 and len(b) > 3:
                b[rng.choice([0, 2])] = rng.choice([0x30, 0x02, 0x1f, 0x3f, 0x22, 0x10, 0xa0])
            else:
                b += rng.randbytes(rng.randrange(1, 4))
        sigs.append(bytes(b))
    got = der_dev(sigs)
    bad = [sig.hex() for sig, g in zip(sigs, got) if not _same(g, _host(sig))]
    assert not bad, bad[:5]
    assert sum(g[0] for g in got) > 10000  # plenty of accepted encodings too

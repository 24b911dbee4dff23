"""CPU-side checks of the product library: it loads, exports every symbol
the C-ABI header declares, and its host-only logic (Go encoding/asn1 DER
decode, SHA-256) matches the oracle.  No compute call needs a GPU here."""
import hashlib
import os
import random
import re

import pytest

from golden_util import load

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    with open(os.path.join(ROOT, "include", "minbft_gpu.h")) as f:
        txt = f.read()
    decl = r"^\s*(?:int|void|uint64_t|size_t|const char\s*\*)\s+(mbft_[a-z_0-9]+)\s*\("
    return sorted(set(re.findall(decl, txt, flags=re.M)))


def test_header_symbols_exported(lib):
    from minbft_amd import _lib
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(_lib.EXPORTED) == syms


def test_version(lib):
    assert lib.mbft_version() >= 1


def test_no_gpu_fails_loudly(lib):
    import ctypes
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except Exception:
        pass
    ctx = ctypes.c_void_p()
    rc = lib.mbft_ctx_create(0, ctypes.byref(ctx))
    assert rc < 0 and not ctx.value


def test_der_parse_matches_go_rules(lib):
    from minbft_amd import _lib
    for v in load("der.json"):
        sig = bytes.fromhex(v["sig"])
        got = _lib.der_parse_sig(sig)
        assert (got is not None) == (v["ok"] == 1), (v, got)
        if got is not None:
            clip = lambda x: x if 0 < x < (1 << 256) else 0  # noqa: E731
            assert int.from_bytes(got[0], "big") == clip(int(v["r"], 16))
            assert int.from_bytes(got[1], "big") == clip(int(v["s"], 16))
            assert len(sig) - got[2] == v["rest"]


def test_der_parse_random_fuzz(lib):
    from minbft_amd import _lib
    from oracle import p256 as o
    rng = random.Random(11)
    base = o.der_encode_sig(rng.randrange(1, o.N), rng.randrange(1, o.N))
    for _ in range(3000):
        b = bytearray(base if rng.random() < 0.7 else rng.randbytes(rng.randrange(0, 80)))
        for _ in range(rng.randrange(0, 4)):
            k = rng.randrange(3)
            if k == 0 and b:
                b[rng.randrange(len(b))] = rng.randrange(256)
            elif k == 1 and b:
                del b[rng.randrange(len(b))]
            else:
                b.insert(rng.randrange(len(b) + 1), rng.randrange(256))
        b = bytes(b)
        try:
            r, s, rest = o.der_parse_sig(b)
            ok = True
        except o.Asn1Error:
            ok = False
        got = _lib.der_parse_sig(b)
        assert (got is not None) == ok, b.hex()
        if ok:
            clip = lambda x: x if 0 < x < (1 << 256) else 0  # noqa: E731
            assert int.from_bytes(got[0], "big") == clip(r)
            assert int.from_bytes(got[1], "big") == clip(s)
            assert len(b) - got[2] == len(rest)


def test_sha256(lib):
    from minbft_amd import _lib
    rng = random.Random(3)
    for n in [0, 1, 3, 55, 56, 57, 63, 64, 65, 127, 128, 129, 256, 1000]:
        m = rng.randbytes(n)
        assert _lib.sha256(m) == hashlib.sha256(m).digest()


def test_sha256_host_forms(lib):
    """Both host compressions (sha256_host.cpp: the portable one and the x86
    SHA extensions, when this CPU has them) against hashlib at every length
    0..300 (one and two padding blocks, every tail length) and a few long
    inputs."""
    from minbft_amd import _lib
    rng = random.Random(0x5A)
    forms = [f for f in (0, 1) if _lib.sha256_form(f, b"") is not None]
    assert 0 in forms
    for n in list(range(301)) + [1000, 4096, 65537]:
        m = rng.randbytes(n)
        want = hashlib.sha256(m).digest()
        for f in forms:
            assert _lib.sha256_form(f, m) == want, (f, n)


def test_authen_bytes_all_types(lib):
    """mbft_authen_bytes (messages/authen.go:27-82) vs the oracle, host only."""
    from minbft_amd import _lib
    from oracle import p256 as o
    rng = random.Random(4)
    for t in (o.MSG_REQUEST, o.MSG_REPLY, o.MSG_PREPARE, o.MSG_COMMIT, o.MSG_REQ_VIEW_CHANGE):
        for _ in range(20):
            m = o.Msg(type=t, replica_id=rng.randrange(1 << 32), prep_replica_id=rng.randrange(1 << 32),
                      view=rng.randrange(1 << 64), client_id=rng.randrange(1 << 32),
                      seq=rng.randrange(1 << 64), op=rng.randbytes(rng.randrange(0, 300)),
                      prep_ui_counter=rng.randrange(1 << 64))
            assert _lib.authen_bytes(m) == o.msg_authen_bytes(m)
    # the sizes SURVEY.md §8(a) A1 lists
    sizes = {o.MSG_REQUEST: 47, o.MSG_REPLY: 49, o.MSG_PREPARE: 59, o.MSG_COMMIT: 70,
             o.MSG_REQ_VIEW_CHANGE: 23}
    for t, n in sizes.items():
        assert len(_lib.authen_bytes(o.Msg(type=t, op=b"x"))) == n


def test_pack_messages_layout(lib):
    """mbft_pack_messages (host only): each record carries the message's
    fields and the offsets / lengths of its bytes in the arena, in message
    order, and a size query (no records) reports the arena size."""
    import ctypes
    import numpy as np
    from minbft_amd import _lib
    from minbft_amd.authenticator import Authenticator
    from oracle import p256 as o
    rng = random.Random(9)
    msgs = []
    for k in range(50):
        msgs.append(o.Msg(type=rng.randrange(1, 6), stream=k, replica_id=rng.randrange(40),
                          prep_replica_id=rng.randrange(40), view=rng.randrange(1 << 64),
                          client_id=rng.randrange(1 << 32), seq=rng.randrange(1 << 64),
                          op=rng.randbytes(rng.randrange(0, 90)), sig=rng.randbytes(rng.randrange(0, 80)),
                          ui_counter=rng.randrange(1 << 64), ui_cert=rng.randbytes(rng.randrange(0, 90)),
                          prep_ui_counter=rng.randrange(1 << 64),
                          prep_ui_cert=rng.randbytes(rng.randrange(0, 90))))
    arr, keep = _lib.make_messages(msgs)
    packed = np.frombuffer(arr, dtype=_lib.message_dtype(), count=len(msgs))
    recs, arena = Authenticator.pack_messages(packed, pinned=False)
    total = sum(len(m.op) + len(m.sig) + len(m.ui_cert) + len(m.prep_ui_cert) for m in msgs)
    assert arena.nbytes == total
    raw = bytes(arena)
    for m, r in zip(msgs, recs):
        for f in ("type", "stream", "replica_id", "prep_replica_id", "view", "client_id", "seq",
                  "ui_counter", "prep_ui_counter"):
            assert int(r[f]) == getattr(m, f), f
        for f in ("op", "sig", "ui_cert", "prep_ui_cert"):
            off, n = int(r[f + "_off"]), int(r[f + "_len"])
            assert raw[off:off + n] == getattr(m, f), f
    used = ctypes.c_size_t(0)
    lib_ = _lib.load()
    assert lib_.mbft_pack_messages(ctypes.cast(packed.ctypes.data, ctypes.c_void_p), len(msgs), None, None,
                                   0, ctypes.byref(used)) == 0
    assert used.value == total
    small = np.zeros(total - 1, dtype=np.uint8)
    rr = np.zeros(len(msgs), dtype=_lib.msg_rec_dtype())
    assert lib_.mbft_pack_messages(ctypes.cast(packed.ctypes.data, ctypes.c_void_p), len(msgs),
                                   ctypes.c_void_p(rr.ctypes.data), ctypes.c_void_p(small.ctypes.data),
                                   total - 1, ctypes.byref(used)) == -1
    del keep

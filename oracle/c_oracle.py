"""ctypes loader for oracle/liboracle.so and oracle/libossl_baseline.so
(TEST INFRASTRUCTURE ONLY: the C restatement in oracle/c/p256_oracle.c and
the OpenSSL CPU baseline in oracle/c/openssl_baseline.c; used by tests/,
smoke() and the cpu_baseline leg of bench.py -- never by the product)."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
OSSL_LIB = os.path.join(HERE, "libossl_baseline.so")
_lib = None
_ossl = None


def build():
    srcs = [(LIB, os.path.join(HERE, "c", "p256_oracle.c")),
            (OSSL_LIB, os.path.join(HERE, "c", "openssl_baseline.c"))]
    if all(os.path.exists(o) and os.path.getmtime(o) >= os.path.getmtime(s) for o, s in srcs):
        return LIB
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)
    return LIB


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = ctypes.CDLL(LIB)
        vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        lib.oracle_ecdsa_verify.argtypes = [vp, vp, vp, vp]
        lib.oracle_ecdsa_verify.restype = i
        lib.oracle_der_parse.argtypes = [vp, sz, vp, vp, ctypes.POINTER(sz)]
        lib.oracle_der_parse.restype = i
        lib.oracle_sha256.argtypes = [vp, sz, vp]
        lib.oracle_sha256.restype = None
        lib.oracle_verify_ecdsa_role.argtypes = [vp, vp, sz, vp, sz]
        lib.oracle_verify_ecdsa_role.restype = i
        lib.oracle_verify_usig_sig.argtypes = [vp, vp, sz, ctypes.c_uint64, ctypes.c_uint64, vp, sz]
        lib.oracle_verify_usig_sig.restype = i
        lib.oracle_verify_prehashed_batch.argtypes = [vp, vp, vp, vp, vp, sz, vp, i]
        lib.oracle_verify_prehashed_batch.restype = i
        lib.oracle_verify_ecdsa_role_batch.argtypes = [vp, vp, vp, vp, vp, vp, sz, vp, i]
        lib.oracle_verify_ecdsa_role_batch.restype = i
        _lib = lib
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def verify(qxy: bytes, e: bytes, r: bytes, s: bytes) -> int:
    return load().oracle_ecdsa_verify(qxy, e, r, s)


def der_parse(sig: bytes):
    r = ctypes.create_string_buffer(32)
    s = ctypes.create_string_buffer(32)
    rest = ctypes.c_size_t(0)
    ok = load().oracle_der_parse(sig, len(sig), r, s, ctypes.byref(rest))
    return (r.raw, s.raw, rest.value) if ok else None


def sha256(m: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    load().oracle_sha256(m, len(m), out)
    return out.raw


def verify_prehashed_batch(qxy, e, r, s, slot, nthreads=8) -> np.ndarray:
    qxy = np.ascontiguousarray(qxy, dtype=np.uint8)
    e = np.ascontiguousarray(e, dtype=np.uint8)
    r = np.ascontiguousarray(r, dtype=np.uint8)
    s = np.ascontiguousarray(s, dtype=np.uint8)
    slot = np.ascontiguousarray(slot, dtype=np.uint32)
    n = slot.shape[0]
    out = np.zeros(n, dtype=np.uint8)
    rc = load().oracle_verify_prehashed_batch(_p(qxy), _p(e), _p(r), _p(s), _p(slot), n, _p(out),
                                              nthreads)
    assert rc == 0
    return out


def verify_ecdsa_role_batch(qxy, slot, msgs, tags, nthreads=8) -> np.ndarray:
    """msgs/tags: lists of bytes.  Returns status per item (0/1/2)."""
    qxy = np.ascontiguousarray(qxy, dtype=np.uint8)
    slot = np.ascontiguousarray(slot, dtype=np.uint32)
    moff = np.zeros(len(msgs) + 1, dtype=np.uint64)
    toff = np.zeros(len(tags) + 1, dtype=np.uint64)
    moff[1:] = np.cumsum([len(m) for m in msgs])
    toff[1:] = np.cumsum([len(t) for t in tags])
    mb = np.frombuffer(b"".join(msgs) + b"\0", dtype=np.uint8)
    tb = np.frombuffer(b"".join(tags) + b"\0", dtype=np.uint8)
    out = np.zeros(len(msgs), dtype=np.uint8)
    rc = load().oracle_verify_ecdsa_role_batch(_p(qxy), _p(slot), _p(mb), _p(moff), _p(tb), _p(toff),
                                               len(msgs), _p(out), nthreads)
    assert rc == 0
    return out


def _ossl_load():
    global _ossl
    if _ossl is None:
        if not os.path.exists(OSSL_LIB):
            build()
        lib = ctypes.CDLL(OSSL_LIB)
        vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        lib.ossl_verify_ecdsa_role_batch.argtypes = [vp, sz, vp, vp, vp, vp, vp, sz, vp, i]
        lib.ossl_verify_ecdsa_role_batch.restype = i
        _ossl = lib
    return _ossl


def ossl_verify_ecdsa_role_batch(qxy, slot, msgs, tags, nthreads=8) -> np.ndarray:
    """OpenSSL 3 d2i_ECDSA_SIG + ECDSA_do_verify over the ECDSA-role call
    (digest = msg || SHA256("")), one thread per `nthreads`.  Status per
    item: 0 accept, 1 reject, 2 malformed DER."""
    qxy = np.ascontiguousarray(qxy, dtype=np.uint8).reshape(-1, 64)
    slot = np.ascontiguousarray(slot, dtype=np.uint32)
    moff = np.zeros(len(msgs) + 1, dtype=np.uint64)
    toff = np.zeros(len(tags) + 1, dtype=np.uint64)
    moff[1:] = np.cumsum([len(m) for m in msgs])
    toff[1:] = np.cumsum([len(t) for t in tags])
    mb = np.frombuffer(b"".join(msgs) + b"\0", dtype=np.uint8)
    tb = np.frombuffer(b"".join(tags) + b"\0", dtype=np.uint8)
    out = np.zeros(len(msgs), dtype=np.uint8)
    rc = _ossl_load().ossl_verify_ecdsa_role_batch(_p(qxy), qxy.shape[0], _p(slot), _p(mb), _p(moff),
                                                   _p(tb), _p(toff), len(msgs), _p(out), nthreads)
    assert rc == 0
    return out

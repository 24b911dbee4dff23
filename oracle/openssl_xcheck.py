"""Independent cross-check of the oracle's ECDSA core via OpenSSL libcrypto
(TEST INFRASTRUCTURE ONLY -- used by tests/ to pin ``oracle.p256``).

OpenSSL's ``ECDSA_do_verify`` implements the same textbook verification as
Go's ``crypto/ecdsa.Verify`` (range checks on r, s; leftmost-256-bit digest
truncation; ``x(u1*G + u2*Q) mod N == r``), so agreeing with it on random and
adversarial ``(Q, e, r, s)`` vectors pins the oracle's arithmetic to an
independent implementation.  Loaded via ctypes; absent libcrypto => the
caller skips.
"""
from __future__ import annotations

import ctypes
import ctypes.util
from typing import Optional

NID_X9_62_prime256v1 = 415

_lib: Optional[ctypes.CDLL] = None


def load() -> Optional[ctypes.CDLL]:
    global _lib
    if _lib is not None:
        return _lib
    for name in ("libcrypto.so.3", ctypes.util.find_library("crypto")):
        if not name:
            continue
        try:
            lib = ctypes.CDLL(name)
        except OSError:
            continue
        vp = ctypes.c_void_p
        lib.EC_KEY_new_by_curve_name.restype = vp
        lib.EC_KEY_new_by_curve_name.argtypes = [ctypes.c_int]
        lib.EC_KEY_free.argtypes = [vp]
        lib.EC_KEY_set_public_key_affine_coordinates.argtypes = [vp, vp, vp]
        lib.EC_KEY_set_public_key_affine_coordinates.restype = ctypes.c_int
        lib.BN_bin2bn.restype = vp
        lib.BN_bin2bn.argtypes = [ctypes.c_char_p, ctypes.c_int, vp]
        lib.BN_free.argtypes = [vp]
        lib.ECDSA_SIG_new.restype = vp
        lib.ECDSA_SIG_free.argtypes = [vp]
        lib.ECDSA_SIG_set0.argtypes = [vp, vp, vp]
        lib.ECDSA_SIG_set0.restype = ctypes.c_int
        lib.ECDSA_do_verify.argtypes = [ctypes.c_char_p, ctypes.c_int, vp, vp]
        lib.ECDSA_do_verify.restype = ctypes.c_int
        _lib = lib
        return lib
    return None


def _bn(lib, x: int):
    b = x.to_bytes(max(1, (x.bit_length() + 7) // 8), "big")
    return lib.BN_bin2bn(b, len(b), None)


def verify(qx: int, qy: int, digest32: bytes, r: int, s: int) -> Optional[bool]:
    """Returns True/False, or None if OpenSSL refused the key (off-curve)."""
    lib = load()
    assert lib is not None
    key = lib.EC_KEY_new_by_curve_name(NID_X9_62_prime256v1)
    bx, by = _bn(lib, qx), _bn(lib, qy)
    try:
        if lib.EC_KEY_set_public_key_affine_coordinates(key, bx, by) != 1:
            return None
        sig = lib.ECDSA_SIG_new()
        if lib.ECDSA_SIG_set0(sig, _bn(lib, r), _bn(lib, s)) != 1:
            raise RuntimeError("ECDSA_SIG_set0 failed")
        rc = lib.ECDSA_do_verify(digest32, len(digest32), sig, key)
        lib.ECDSA_SIG_free(sig)
        if rc < 0:
            # OpenSSL reports r/s out of range as an error; Go returns false.
            return False
        return rc == 1
    finally:
        lib.BN_free(bx)
        lib.BN_free(by)
        lib.EC_KEY_free(key)

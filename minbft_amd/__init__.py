"""minbft_amd -- MI355X-native batch message authenticator for MinBFT.

The product is ``libminbft_amd.so`` (HIP kernels for gfx950 + C++ host
runtime behind the C-ABI in ``include/minbft_gpu.h``).  This package holds
its sources (``csrc/``), the in-tree build (``build.py``), the ctypes binding
(``_lib.py``) and a Python mirror of ``api.Authenticator``
(``authenticator.py``).
"""
from ._lib import (ACCEPT, BAD_CERT, BAD_KEY, BAD_UI, DER_TRAILING, EPOCH_MISMATCH,  # noqa: F401
                   MALFORMED_DER, REJECT_SIG, ROLE_CLIENT, ROLE_REPLICA, ROLE_USIG,
                   UNKNOWN_KEY, UNKNOWN_ROLE, ZERO_COUNTER, LIB_PATH)

__all__ = ["Authenticator", "AuthenticationError", "SignaturePanic", "load_library"]


def load_library():
    from . import _lib
    return _lib.load()


def __getattr__(name):
    if name in ("Authenticator", "AuthenticationError", "SignaturePanic", "GpuError",
                "der_encode_sig"):
        from . import authenticator
        return getattr(authenticator, name)
    raise AttributeError(name)

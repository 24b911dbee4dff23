"""ctypes binding of the C-ABI in include/minbft_gpu.h.

The library is the in-tree ``minbft_amd/libminbft_amd.so`` (built by
``minbft_amd.build``).  There is no fallback: if the library cannot be
loaded, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

HERE = os.path.dirname(os.path.abspath(__file__))
# MBFT_LIB_PATH: load another build of the same C-ABI (A/B timing of kernel
# variants, tools/ab_build.sh); default is the in-tree library.
LIB_PATH = os.environ.get("MBFT_LIB_PATH") or os.path.join(HERE, "libminbft_amd.so")

# enum mbft_status
ACCEPT = 0
REJECT_SIG = 1
MALFORMED_DER = 2
DER_TRAILING = 3
UNKNOWN_KEY = 4
BAD_KEY = 5
BAD_UI = 6
BAD_CERT = 7
ZERO_COUNTER = 8
EPOCH_MISMATCH = 9
UNKNOWN_ROLE = 10

# enum mbft_err
OK = 0
ERR_ARG = -1
ERR_HIP = -2
ERR_NOMEM = -3
ERR_KEY = -4
ERR_STATE = -5
ERR_NODEV = -6

# enum mbft_role (api/api.go:98-115)
ROLE_REPLICA = 1
ROLE_USIG = 2
ROLE_CLIENT = 3

#: every symbol include/minbft_gpu.h declares (checked by tests/test_abi.py)
EXPORTED = [
    "mbft_version", "mbft_device_count", "mbft_ctx_create", "mbft_ctx_destroy",
    "mbft_last_error", "mbft_add_role", "mbft_set_public_key_pkix",
    "mbft_set_public_key_xy", "mbft_register_points", "mbft_key_slot",
    "mbft_enable_usig", "mbft_set_private_key", "mbft_verify_message_authen_tag",
    "mbft_verify_batch", "mbft_generate_message_authen_tag", "mbft_verify_prehashed",
    "mbft_verify_prehashed_device", "mbft_sign_prehashed", "mbft_sign_prehashed_device",
    "mbft_der_parse_sig", "mbft_sha256", "mbft_profile_enable", "mbft_profile_read",
    "mbft_set_key_window", "mbft_authen_bytes", "mbft_validate_messages",
    "mbft_validate_messages_flat", "mbft_pack_messages",
    "mbft_set_generator_window", "mbft_get_windows", "mbft_request_digests_device",
    "mbft_sha256_device", "mbft_usig_digests_device", "mbft_ctx_add_device",
    "mbft_ctx_devices", "mbft_set_shard_min", "mbft_validate_replies", "mbft_clear_keys",
    "mbft_profile_stages", "mbft_sign_nonce_device", "mbft_verify_batch_flat",
    "mbft_check_batch", "mbft_check_batch_flat", "mbft_resolve_checked", "mbft_authen_digests",
    "mbft_set_coalescing", "mbft_set_coalescing_slots", "mbft_host_alloc", "mbft_host_free", "mbft_set_device_prepare",
    "mbft_set_concurrency", "mbft_get_concurrency", "mbft_plan_windows",
    "mbft_check_messages_flat", "mbft_resolve_message", "mbft_msg_batch_free",
    "mbft_resolve_messages", "mbft_profile_msg_layer", "mbft_verify_batch_flat32",
    "mbft_check_batch_flat32", "mbft_set_small_batch_form", "mbft_set_small_batch_inverse", "mbft_set_check_coalescing",
    "mbft_check_coalescing_stats", "mbft_set_small_check", "mbft_debug_sha256",
    "mbft_validate_replies_flat", "mbft_set_resident", "mbft_resident_stats", "mbft_resident_wait_stats", "mbft_debug_threads_started",
    "mbft_debug_host_join", "mbft_debug_host_scalars",
]

# enum mbft_msg_type / mbft_stage / mbft_validate_flags
MSG_REQUEST, MSG_REPLY, MSG_PREPARE, MSG_COMMIT, MSG_REQ_VIEW_CHANGE = 1, 2, 3, 4, 5
ST_REQUEST_SIG, ST_NOT_PRIMARY, ST_PREPARE_UI, ST_COMMIT_FROM_PRIMARY = 1, 2, 3, 4
ST_COMMIT_UI, ST_NOT_IMPLEMENTED, ST_STREAM_STOPPED, ST_REPLY_SIG, ST_AFTER_PANIC = 5, 6, 7, 8, 9
ST_UNKNOWN_TYPE, ST_REPLY_CLIENT_ID = 10, 11
VF_NO_STREAM_STOP, VF_NO_PANIC_STOP = 1, 2


class MbftMessage(ctypes.Structure):
    _fields_ = [
        ("type", ctypes.c_uint32),
        ("stream", ctypes.c_uint32),
        ("replica_id", ctypes.c_uint32),
        ("prep_replica_id", ctypes.c_uint32),
        ("view", ctypes.c_uint64),
        ("client_id", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
        ("seq", ctypes.c_uint64),
        ("op", ctypes.c_void_p),
        ("op_len", ctypes.c_size_t),
        ("sig", ctypes.c_void_p),
        ("sig_len", ctypes.c_size_t),
        ("ui_counter", ctypes.c_uint64),
        ("ui_cert", ctypes.c_void_p),
        ("ui_cert_len", ctypes.c_size_t),
        ("prep_ui_counter", ctypes.c_uint64),
        ("prep_ui_cert", ctypes.c_void_p),
        ("prep_ui_cert_len", ctypes.c_size_t),
    ]


def message_dtype():
    """numpy view of mbft_message (the MbftMessage layout), for packed batches."""
    import numpy as np
    names = [f[0] for f in MbftMessage._fields_]
    fmt = {ctypes.c_uint32: "<u4", ctypes.c_uint64: "<u8", ctypes.c_void_p: "<u8",
           ctypes.c_size_t: "<u8"}
    return np.dtype({"names": names,
                     "formats": [fmt[f[1]] for f in MbftMessage._fields_],
                     "offsets": [getattr(MbftMessage, nm).offset for nm in names],
                     "itemsize": ctypes.sizeof(MbftMessage)})


# mbft_msg_rec (include/minbft_gpu.h): the flat batch record
MSG_REC_DTYPE_FIELDS = [
    ("type", "<u4"), ("stream", "<u4"), ("replica_id", "<u4"), ("prep_replica_id", "<u4"),
    ("client_id", "<u4"), ("op_len", "<u4"), ("sig_len", "<u4"), ("ui_cert_len", "<u4"),
    ("prep_ui_cert_len", "<u4"), ("reserved", "<u4"), ("view", "<u8"), ("seq", "<u8"),
    ("ui_counter", "<u8"), ("prep_ui_counter", "<u8"), ("op_off", "<u8"), ("sig_off", "<u8"),
    ("ui_cert_off", "<u8"), ("prep_ui_cert_off", "<u8"),
]


def msg_rec_dtype():
    """numpy view of mbft_msg_rec (104 bytes, no padding)."""
    import numpy as np
    dt = np.dtype(MSG_REC_DTYPE_FIELDS)
    assert dt.itemsize == 104
    return dt


def make_messages(msgs):
    """list of objects with the oracle Msg fields -> (ctypes array, keepalive)."""
    arr = (MbftMessage * max(len(msgs), 1))()
    keep = []

    def b(x):
        buf = ctypes.create_string_buffer(bytes(x), len(x) or 1)
        keep.append(buf)
        return ctypes.cast(buf, ctypes.c_void_p), len(x)

    for k, m in enumerate(msgs):
        op, opl = b(m.op)
        sg, sgl = b(m.sig)
        uc, ucl = b(m.ui_cert)
        pc, pcl = b(m.prep_ui_cert)
        arr[k] = MbftMessage(m.type, m.stream, m.replica_id, m.prep_replica_id, m.view, m.client_id,
                             0, m.seq, op, opl, sg, sgl, m.ui_counter, uc, ucl, m.prep_ui_counter,
                             pc, pcl)
    return arr, keep


def authen_bytes(m) -> bytes:
    """Host-only messages.AuthenBytes through the C-ABI."""
    lib = load()
    arr, keep = make_messages([m])
    n = ctypes.c_size_t(0)
    out = ctypes.create_string_buffer(256)
    rc = lib.mbft_authen_bytes(arr, out, 256, ctypes.byref(n))
    if rc != OK:
        raise ValueError(f"mbft_authen_bytes: {rc}")
    return out.raw[:n.value]


class MbftItem(ctypes.Structure):
    _fields_ = [
        ("role", ctypes.c_uint32),
        ("id", ctypes.c_uint32),
        ("msg", ctypes.c_void_p),
        ("msg_len", ctypes.c_size_t),
        ("tag", ctypes.c_void_p),
        ("tag_len", ctypes.c_size_t),
    ]


# numpy view of mbft_item (same layout as MbftItem), for packed batches
ITEM_DTYPE = None
try:
    import numpy as _np
    ITEM_DTYPE = _np.dtype({"names": ["role", "id", "msg", "msg_len", "tag", "tag_len"],
                            "formats": ["<u4", "<u4", "<u8", "<u8", "<u8", "<u8"],
                            "offsets": [0, 4, 8, 16, 24, 32], "itemsize": 40})
    assert ctypes.sizeof(MbftItem) == 40
except ImportError:  # pragma: no cover
    pass

_lib: Optional[ctypes.CDLL] = None


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load (once) and type the C-ABI.  Raises OSError if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise OSError(f"{path} not built: run `python -m minbft_amd.build`")
    lib = ctypes.CDLL(path)
    vp, sz, u32, u8p, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int
    sig = {
        "mbft_version": (i, []),
        "mbft_device_count": (i, []),
        "mbft_ctx_create": (i, [i, ctypes.POINTER(vp)]),
        "mbft_ctx_destroy": (None, [vp]),
        "mbft_last_error": (ctypes.c_char_p, [vp]),
        "mbft_ctx_add_device": (i, [vp, i]),
        "mbft_ctx_devices": (i, [vp, vp, i]),
        "mbft_set_shard_min": (i, [vp, sz]),
        "mbft_add_role": (i, [vp, u32]),
        "mbft_set_public_key_pkix": (i, [vp, u32, u32, u8p, sz]),
        "mbft_set_public_key_xy": (i, [vp, u32, u32, u8p]),
        "mbft_register_points": (i, [vp, u8p, sz, vp, vp]),
        "mbft_key_slot": (i, [vp, u32, u32]),
        "mbft_clear_keys": (i, [vp]),
        "mbft_enable_usig": (i, [vp, i]),
        "mbft_set_key_window": (i, [vp, i]),
        "mbft_set_generator_window": (i, [vp, i]),
        "mbft_get_windows": (i, [vp, ctypes.POINTER(i), ctypes.POINTER(i)]),
        "mbft_request_digests_device": (i, [vp, vp, vp, u32, sz, vp, vp]),
        "mbft_sha256_device": (i, [vp, vp, vp, sz, vp, vp]),
        "mbft_usig_digests_device": (i, [vp, vp, vp, vp, vp, sz, vp, vp]),
        "mbft_authen_bytes": (i, [ctypes.POINTER(MbftMessage), vp, sz, ctypes.POINTER(sz)]),
        "mbft_validate_messages": (i, [vp, ctypes.POINTER(MbftMessage), sz, u32, u32, vp]),
        "mbft_validate_messages_flat": (i, [vp, vp, sz, vp, sz, u32, u32, vp]),
        "mbft_pack_messages": (i, [vp, sz, vp, vp, sz, ctypes.POINTER(sz)]),
        "mbft_check_messages_flat": (i, [vp, vp, sz, vp, sz, u32, ctypes.POINTER(vp)]),
        "mbft_resolve_message": (i, [vp, vp, sz]),
        "mbft_resolve_messages": (i, [vp, vp, sz, sz, vp]),
        "mbft_verify_batch_flat32": (i, [vp, vp, vp, vp, vp, vp, vp, sz, vp]),
        "mbft_set_small_batch_form": (i, [vp, ctypes.c_long]),
        "mbft_set_small_batch_inverse": (i, [vp, ctypes.c_int]),
        "mbft_check_batch_flat32": (i, [vp, vp, vp, vp, vp, vp, vp, sz, vp]),
        "mbft_profile_msg_layer": (i, [vp, ctypes.POINTER(ctypes.c_double)]),
        "mbft_msg_batch_free": (None, [vp]),
        "mbft_validate_replies": (i, [vp, ctypes.POINTER(MbftMessage), sz, u32, u32, vp]),
        "mbft_authen_digests": (i, [vp, ctypes.POINTER(MbftMessage), sz, u32, vp, vp, vp]),
        "mbft_set_private_key": (i, [vp, u32, u8p]),
        "mbft_verify_message_authen_tag": (i, [vp, u32, u32, u8p, sz, u8p, sz]),
        "mbft_verify_batch": (i, [vp, ctypes.POINTER(MbftItem), sz, vp]),
        "mbft_set_coalescing": (i, [vp, i, u32, u32]),
        "mbft_set_coalescing_slots": (i, [vp, i]),
        "mbft_set_resident": (i, [vp, i]),
        "mbft_debug_host_join": (i, [vp, i, vp]),
        "mbft_debug_host_scalars": (i, [vp, vp, vp, vp]),
        "mbft_debug_threads_started": (ctypes.c_uint64, []),
        "mbft_resident_stats": (i, [vp, ctypes.POINTER(ctypes.c_double)]),
        "mbft_resident_wait_stats": (i, [vp, ctypes.POINTER(ctypes.c_double)]),
        "mbft_set_check_coalescing": (i, [vp, i, u32, sz]),
        "mbft_check_coalescing_stats": (i, [vp, ctypes.POINTER(ctypes.c_double)]),
        "mbft_set_small_check": (i, [vp, sz]),
        "mbft_validate_replies_flat": (i, [vp, vp, sz, vp, sz, u32, u32, vp]),
        "mbft_debug_sha256": (i, [i, u8p, sz, vp]),
        "mbft_set_concurrency": (i, [vp, i]),
        "mbft_get_concurrency": (i, [vp]),
        "mbft_plan_windows": (i, [i, sz, sz, sz] + [ctypes.POINTER(i)] * 4),
        "mbft_host_alloc": (i, [sz, ctypes.POINTER(vp)]),
        "mbft_host_free": (i, [vp]),
        "mbft_set_device_prepare": (i, [vp, i]),
        "mbft_verify_batch_flat": (i, [vp, vp, vp, vp, vp, vp, vp, sz, vp]),
        "mbft_check_batch": (i, [vp, ctypes.POINTER(MbftItem), sz, vp]),
        "mbft_check_batch_flat": (i, [vp, vp, vp, vp, vp, vp, vp, sz, vp]),
        "mbft_resolve_checked": (i, [vp, u32, u32, u8p, sz, u8p, sz, ctypes.c_uint8]),
        "mbft_generate_message_authen_tag": (i, [vp, u32, u8p, sz, u8p, sz, ctypes.POINTER(sz)]),
        "mbft_verify_prehashed": (i, [vp, u8p, u8p, u8p, vp, sz, vp]),
        "mbft_verify_prehashed_device": (i, [vp, vp, vp, vp, vp, sz, vp, vp]),
        "mbft_sign_prehashed": (i, [vp, u8p, sz, vp, u8p, sz, vp, vp]),
        "mbft_sign_prehashed_device": (i, [vp, vp, vp, vp, sz, vp, vp, vp]),
        "mbft_sign_nonce_device": (i, [vp, vp, vp, vp, vp, sz, vp, vp, vp]),
        "mbft_der_parse_sig": (i, [u8p, sz, vp, vp, ctypes.POINTER(sz)]),
        "mbft_sha256": (None, [u8p, sz, vp]),
        "mbft_profile_enable": (i, [vp, i]),
        "mbft_profile_read": (i, [vp, ctypes.POINTER(ctypes.c_double)]),
        "mbft_profile_stages": (i, [vp, ctypes.POINTER(ctypes.c_double)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def der_parse_sig(sig: bytes):
    """Host-only Go encoding/asn1 decode: (r32, s32, consumed) or None."""
    lib = load()
    r = ctypes.create_string_buffer(32)
    s = ctypes.create_string_buffer(32)
    n = ctypes.c_size_t(0)
    ok = lib.mbft_der_parse_sig(sig, len(sig), r, s, ctypes.byref(n))
    if not ok:
        return None
    return r.raw, s.raw, n.value


def sha256(data: bytes) -> bytes:
    lib = load()
    out = ctypes.create_string_buffer(32)
    lib.mbft_sha256(data, len(data), out)
    return out.raw


def sha256_form(form: int, data: bytes) -> Optional[bytes]:
    """Host SHA-256 through one compression (mbft_debug_sha256): 0 portable,
    1 the x86 SHA extensions (None when the CPU lacks them)."""
    lib = load()
    out = ctypes.create_string_buffer(32)
    rc = lib.mbft_debug_sha256(form, data, len(data), out)
    if rc == ERR_STATE:
        return None
    if rc != OK:
        raise ValueError(f"mbft_debug_sha256: {rc}")
    return out.raw

"""Python mirror of MinBFT's ``api.Authenticator`` over the GPU C-ABI.

Mirrors the reference plugin interface (api/api.go:133-144,
sample/authentication/authenticator.go:121-141) for tests and benchmarks,
the way the cgo wrapper in INTEGRATION.md does for Go:

* ``VerifyMessageAuthenTag(role, id, msg, tag)`` returns ``None`` (Go nil),
  raises :class:`AuthenticationError` (a Go error) or
  :class:`SignaturePanic` (where Go's EcdsaSigCipher.Verify panics on a
  malformed DER signature, crypto.go:82-84).
* ``GenerateMessageAuthenTag(role, msg)`` returns the DER tag (ECDSA roles).
* ``verify_batch`` is the new batched entry point; ``verify_prehashed`` is
  the decoded ``crypto/ecdsa.Verify`` core.

Every call goes through ``libminbft_amd.so``; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import sys as _sys
from typing import Iterable, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import (ACCEPT, MALFORMED_DER, ROLE_CLIENT, ROLE_REPLICA, ROLE_USIG,  # noqa: F401
                   MbftItem)

STATUS_TEXT = {
    0: "ok", 1: "invalid signature", 2: "ECDSA signature is not ASN.1-DER encoded",
    3: "extra bytes in USIG signature", 4: "public key not found", 5: "invalid public key",
    6: "failed to unmarshal UI", 7: "failed to parse UI cert", 8: "UI counter is zero",
    9: "epoch value mismatch", 10: "Unknown role",
}


class AuthenticationError(Exception):
    """Go: VerifyMessageAuthenTag returned a non-nil error."""

    def __init__(self, status: int):
        super().__init__(f"Invalid authentication tag: {STATUS_TEXT.get(status, status)}")
        self.status = status


class SignaturePanic(Exception):
    """Go: EcdsaSigCipher.Verify panics (crypto.go:82-84)."""


class GpuError(RuntimeError):
    pass


def _buf(a) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data) if a is not None else ctypes.c_void_p(0)


def host_array(n: int, dtype=np.uint8) -> np.ndarray:
    """A numpy array in library-owned page-locked host memory
    (mbft_host_alloc), freed when the array is collected.  Flat batches
    built in such arrays are decoded on the GPU (include/minbft_gpu.h)."""
    import weakref
    lib = _lib.load()
    dt = np.dtype(dtype)
    nbytes = max(1, int(n) * dt.itemsize)
    p = ctypes.c_void_p()
    rc = lib.mbft_host_alloc(nbytes, ctypes.byref(p))
    if rc != 0 or not p.value:
        raise MemoryError(f"mbft_host_alloc({nbytes}) failed: {rc}")
    raw = (ctypes.c_uint8 * nbytes).from_address(p.value)
    arr = np.frombuffer(raw, dtype=np.uint8)[: int(n) * dt.itemsize].view(dt)
    weakref.finalize(raw, lib.mbft_host_free, ctypes.c_void_p(p.value))
    return arr


#: SHA256("") -- the digest Sum(m) appends in the ECDSA roles (crypto.go:121)
SHA256_EMPTY = bytes.fromhex("e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855")


def ecdsa_e_prefix(msg: bytes) -> bytes:
    """(msg || SHA256(""))[0:32]: all of an ECDSA-role message the verdict
    depends on (copied, not hashed) -- what the compact flat form may carry
    instead of the message (include/minbft_gpu.h mbft_verify_batch_flat32)."""
    return (bytes(msg) + SHA256_EMPTY)[:32]


def flat_calls(items, pinned: bool = False, compact: bool = False):
    """(roles, ids, msgs, msg_off, tags, tag_off) of the flat entry points for
    calls (role, id, msg, tag); in library page-locked memory if `pinned`;
    compact: u8 roles and u32 offsets (mbft_verify_batch_flat32)."""
    n = len(items)
    mlen = np.array([len(it[2]) for it in items], dtype=np.uint64)
    tlen = np.array([len(it[3]) for it in items], dtype=np.uint64)
    alloc = host_array if pinned else (lambda k, dt=np.uint8: np.zeros(k, dtype=dt))
    odt = np.uint32 if compact else np.uint64
    roles, ids = alloc(n, np.uint8 if compact else np.uint32), alloc(n, np.uint32)
    mo, to = alloc(n + 1, odt), alloc(n + 1, odt)
    roles[:] = [it[0] for it in items]
    ids[:] = [it[1] for it in items]
    mo[0] = to[0] = 0
    mo[1:] = np.cumsum(mlen)
    to[1:] = np.cumsum(tlen)
    mb, tb = alloc(int(mo[n]) + 1), alloc(int(to[n]) + 1)
    mb[: int(mo[n])] = np.frombuffer(b"".join(bytes(it[2]) for it in items), dtype=np.uint8)
    tb[: int(to[n])] = np.frombuffer(b"".join(bytes(it[3]) for it in items), dtype=np.uint8)
    return roles, ids, mb, mo, tb, to


class Authenticator:
    """One authenticator (mbft_ctx).  `devices` adds engines on further GPUs
    (mbft_ctx_add_device): host-buffer batches are then sharded across all of
    them; device-pointer calls stay on `device`."""

    def __init__(self, device: int = 0, devices: Sequence[int] = ()):
        self.lib = _lib.load()
        ctx = ctypes.c_void_p()
        rc = self.lib.mbft_ctx_create(device, ctypes.byref(ctx))
        if rc != _lib.OK:
            raise GpuError(f"mbft_ctx_create(device={device}) failed: {rc}")
        self.ctx = ctx
        self.device = device
        for d in devices:
            self.add_device(d)

    def add_device(self, device: int):
        self._check(self.lib.mbft_ctx_add_device(self.ctx, device), f"add_device({device})")

    def devices(self) -> list:
        buf = (ctypes.c_int * 64)()
        n = self._check(self.lib.mbft_ctx_devices(self.ctx, buf, 64), "ctx_devices")
        return list(buf[:n])

    def set_shard_min(self, items: int):
        self._check(self.lib.mbft_set_shard_min(self.ctx, items), "set_shard_min")

    # ------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "ctx", None):
            self.lib.mbft_ctx_destroy(self.ctx)
            self.ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        # Never touch the HIP runtime during interpreter shutdown (its own
        # teardown may already have run): call close() explicitly instead.
        if _sys is None or _sys.is_finalizing():
            return
        try:
            self.close()
        except Exception:
            pass

    def last_error(self) -> str:
        """The context's last error message (mbft_last_error)."""
        msg = self.lib.mbft_last_error(self.ctx)
        return msg.decode() if msg else ""

    def _check(self, rc: int, what: str) -> int:
        if rc < 0:
            msg = self.lib.mbft_last_error(self.ctx)
            raise GpuError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
        return rc

    # ------------------------------------------------------------ key store
    def add_role(self, role: int):
        self._check(self.lib.mbft_add_role(self.ctx, role), "add_role")

    def set_key_window(self, wbits: int):
        """Comb window (4..29 bits, default 16) for keys registered after the
        call; include/minbft_gpu.h lists the HBM cost per window."""
        self._check(self.lib.mbft_set_key_window(self.ctx, wbits), "set_key_window")

    def set_generator_window(self, wbits: int):
        """Rebuild the generator comb table with a window of 4..29 bits."""
        self._check(self.lib.mbft_set_generator_window(self.ctx, wbits), "set_generator_window")

    def windows(self) -> Tuple[int, int]:
        g, q = ctypes.c_int(), ctypes.c_int()
        self._check(self.lib.mbft_get_windows(self.ctx, ctypes.byref(g), ctypes.byref(q)),
                    "get_windows")
        return g.value, q.value

    def enable_usig(self, enabled: bool = True):
        self._check(self.lib.mbft_enable_usig(self.ctx, int(enabled)), "enable_usig")

    def set_public_key(self, role: int, id_: int, key: bytes):
        """``key``: 91-byte PKIX DER or 64-byte X||Y.  Raises ValueError for
        an invalid / off-curve key (x509.ParsePKIXPublicKey error)."""
        if len(key) == 64:
            rc = self.lib.mbft_set_public_key_xy(self.ctx, role, id_, key)
        else:
            rc = self.lib.mbft_set_public_key_pkix(self.ctx, role, id_, key, len(key))
        if rc == _lib.ERR_KEY:
            raise ValueError("invalid public key")
        self._check(rc, "set_public_key")

    def set_private_key(self, role: int, d: bytes):
        assert len(d) == 32
        self._check(self.lib.mbft_set_private_key(self.ctx, role, d), "set_private_key")

    def clear_keys(self):
        """Drop every key, slot and comb table (mbft_clear_keys)."""
        self._check(self.lib.mbft_clear_keys(self.ctx), "clear_keys")

    def key_slot(self, role: int, id_: int) -> int:
        return self._check(self.lib.mbft_key_slot(self.ctx, role, id_), "key_slot")

    def register_points(self, xy: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        xy = np.ascontiguousarray(xy, dtype=np.uint8).reshape(-1, 64)
        n = xy.shape[0]
        slots = np.zeros(n, dtype=np.uint32)
        valid = np.zeros(n, dtype=np.uint8)
        self._check(self.lib.mbft_register_points(self.ctx, _buf(xy), n, _buf(slots), _buf(valid)),
                    "register_points")
        return slots, valid

    # ------------------------------------------------------- authenticator
    def set_coalescing(self, enabled: bool, max_wait_us: int = 0, max_batch: int = 0) -> None:
        """Coalesce concurrent single calls into batches (mbft_set_coalescing)."""
        self._check(self.lib.mbft_set_coalescing(self.ctx, 1 if enabled else 0, max_wait_us, max_batch),
                    "set_coalescing")

    def set_coalescing_slots(self, slots: int) -> None:
        """Coalesced batches in flight at once (mbft_set_coalescing_slots;
        default 1, at most the concurrency's lanes)."""
        self._check(self.lib.mbft_set_coalescing_slots(self.ctx, slots), "set_coalescing_slots")

    def set_resident(self, slots: int) -> None:
        """The resident single-call verifier (mbft_set_resident): a kernel
        kept on the GPU serving verify_status / VerifyMessageAuthenTag calls
        through `slots` host-mapped mailbox slots; 0 turns it off."""
        self._check(self.lib.mbft_set_resident(self.ctx, slots), "set_resident")

    def resident_stats(self) -> dict:
        """mbft_resident_stats: slots, calls served, launches, calls that
        found every slot taken, relaunches found by a stream query, whether
        the kernel's stream has its own hardware queue."""
        out = (ctypes.c_double * 6)()
        self._check(self.lib.mbft_resident_stats(self.ctx, out), "resident_stats")
        keys = ("slots", "calls", "launches", "fallbacks", "stream_relaunches", "own_queue")
        return {k: (int(v) if k != "own_queue" else bool(v)) for k, v in zip(keys, out)}

    def resident_wait_stats(self) -> dict:
        """mbft_resident_wait_stats: the callers' sleeps, sleeps that woke
        after the items were done, the estimates (ns) of a lone item's post ->
        done and of the wake-up delay, whether the wait sleeps."""
        out = (ctypes.c_double * 5)()
        self._check(self.lib.mbft_resident_wait_stats(self.ctx, out), "resident_wait_stats")
        return {"sleeps": int(out[0]), "woke_late": int(out[1]), "done_ns": out[2], "wake_delay_ns": out[3],
                "sleeping": bool(out[4])}

    def set_check_coalescing(self, enabled: bool, max_wait_us: int = 0, max_messages: int = 0) -> None:
        """Coalesce concurrent check_messages_flat calls into one device pass
        (mbft_set_check_coalescing)."""
        self._check(self.lib.mbft_set_check_coalescing(self.ctx, 1 if enabled else 0, max_wait_us,
                                                       max_messages), "set_check_coalescing")

    def set_small_check(self, max_messages: int) -> None:
        """Checks of at most max_messages messages take the small route
        (mbft_set_small_check; default 512, 0 = always the device message
        layer)."""
        self._check(self.lib.mbft_set_small_check(self.ctx, max_messages), "set_small_check")

    def check_coalescing_stats(self) -> dict:
        """Passes, caller batches and messages since the last call
        (mbft_check_coalescing_stats; resets them)."""
        out = (ctypes.c_double * 3)()
        self._check(self.lib.mbft_check_coalescing_stats(self.ctx, out), "check_coalescing_stats")
        return {"passes": int(out[0]), "batches": int(out[1]), "messages": int(out[2])}

    def set_concurrency(self, lanes: int) -> None:
        """Run up to `lanes` batch calls at once on this GPU (mbft_set_concurrency)."""
        self._check(self.lib.mbft_set_concurrency(self.ctx, lanes), "set_concurrency")

    def concurrency(self) -> int:
        return self._check(self.lib.mbft_get_concurrency(self.ctx), "get_concurrency")

    def verify_status(self, role: int, id_: int, msg: bytes, tag: bytes) -> int:
        return self._check(
            self.lib.mbft_verify_message_authen_tag(self.ctx, role, id_, msg, len(msg), tag, len(tag)),
            "verify")

    def VerifyMessageAuthenTag(self, role: int, id_: int, msg: bytes, tag: bytes) -> None:
        st = self.verify_status(role, id_, msg, tag)
        if st == ACCEPT:
            return None
        if st == MALFORMED_DER and role != ROLE_USIG:
            raise SignaturePanic("ECDSA signature is not ASN.1-DER encoded")
        raise AuthenticationError(st)

    def GenerateMessageAuthenTag(self, role: int, msg: bytes) -> bytes:
        out = ctypes.create_string_buffer(80)
        n = ctypes.c_size_t(0)
        self._check(self.lib.mbft_generate_message_authen_tag(self.ctx, role, msg, len(msg), out, 80,
                                                              ctypes.byref(n)), "generate")
        return out.raw[:n.value]

    def verify_batch(self, items: Sequence[Tuple[int, int, bytes, bytes]]) -> np.ndarray:
        n = len(items)
        arr = (MbftItem * max(n, 1))()
        keep = []
        for k, (role, id_, msg, tag) in enumerate(items):
            mb = ctypes.create_string_buffer(bytes(msg), len(msg) or 1)
            tb = ctypes.create_string_buffer(bytes(tag), len(tag) or 1)
            keep.append((mb, tb))
            arr[k] = MbftItem(role, id_, ctypes.cast(mb, ctypes.c_void_p), len(msg),
                              ctypes.cast(tb, ctypes.c_void_p), len(tag))
        out = np.zeros(n, dtype=np.uint8)
        self._check(self.lib.mbft_verify_batch(self.ctx, arr, n, _buf(out)), "verify_batch")
        return out

    def verify_batch_packed(self, roles, ids, msgs: np.ndarray, msg_lens, tags: np.ndarray,
                            tag_lens, out: Optional[np.ndarray] = None) -> np.ndarray:
        """mbft_verify_batch over row-packed buffers (no per-item Python
        objects): item i = (roles[i], ids[i], msgs[i, :msg_lens[i]],
        tags[i, :tag_lens[i]]).  Returns the status bytes."""
        items = self.pack_items(roles, ids, msgs, msg_lens, tags, tag_lens)
        return self.verify_batch_items(items, out)

    @staticmethod
    def pack_items(roles, ids, msgs: np.ndarray, msg_lens, tags: np.ndarray, tag_lens):
        """An mbft_item array (numpy structured, C layout) pointing into msgs /
        tags (which must stay alive while the items are used)."""
        n = msgs.shape[0]
        assert msgs.flags.c_contiguous and tags.flags.c_contiguous and tags.shape[0] == n
        it = np.zeros(n, dtype=_lib.ITEM_DTYPE)
        it["role"] = roles
        it["id"] = ids
        it["msg"] = msgs.ctypes.data + np.arange(n, dtype=np.uint64) * np.uint64(msgs.shape[1])
        it["msg_len"] = msg_lens
        it["tag"] = tags.ctypes.data + np.arange(n, dtype=np.uint64) * np.uint64(tags.shape[1])
        it["tag_len"] = tag_lens
        return it

    def verify_batch_items(self, items: np.ndarray, out: Optional[np.ndarray] = None) -> np.ndarray:
        n = items.shape[0]
        if out is None:
            out = np.zeros(n, dtype=np.uint8)
        self._check(self.lib.mbft_verify_batch(self.ctx, ctypes.cast(items.ctypes.data,
                                                                     ctypes.POINTER(MbftItem)),
                                               n, _buf(out)), "verify_batch")
        return out

    def set_small_batch_form(self, split_max: int) -> None:
        """mbft_set_small_batch_form: batches <= split_max take k_verify_split,
        larger small ones k_verify_pairs (0: pairs only; -1: default)."""
        self._check(self.lib.mbft_set_small_batch_form(self.ctx, split_max), "set_small_batch_form")

    def set_small_batch_inverse(self, mode: int) -> None:
        """mbft_set_small_batch_inverse: the batches past the split kernel's
        take lane quads inverting per wave (2), the batched per-wave s^-1
        planes and lane quads (3) or lane pairs (1), lane pairs inverting per
        lane (0), or the default (-1)."""
        self._check(self.lib.mbft_set_small_batch_inverse(self.ctx, mode), "set_small_batch_inverse")

    def set_device_prepare(self, enabled: bool) -> None:
        """mbft_set_device_prepare: decode flat calls in library page-locked
        memory on the GPU (default) or always on the host."""
        self._check(self.lib.mbft_set_device_prepare(self.ctx, 1 if enabled else 0),
                    "set_device_prepare")

    def verify_batch_flat(self, items, pinned: bool = False) -> np.ndarray:
        """mbft_verify_batch_flat (the form the Go binding uses).  `pinned`:
        the flat buffers (and the status output) in library page-locked
        memory, so the calls are decoded on the GPU."""
        return self.verify_flat_arrays(*flat_calls(items, pinned), pinned=pinned)

    def verify_flat_arrays(self, roles, ids, mb, mo, tb, to, out=None, pinned: bool = False):
        """mbft_verify_batch_flat over prepared flat arrays."""
        n = len(roles)
        if out is None:
            out = host_array(n) if pinned else np.zeros(n, dtype=np.uint8)
        self._check(self.lib.mbft_verify_batch_flat(self.ctx, _buf(roles), _buf(ids), _buf(mb), _buf(mo),
                                                    _buf(tb), _buf(to), n, _buf(out)),
                    "verify_batch_flat")
        return out

    def verify_batch_flat32(self, items, pinned: bool = False, ecdsa_e: bool = False) -> np.ndarray:
        """mbft_verify_batch_flat32 (compact form); ecdsa_e: ECDSA-role
        messages passed as their 32-byte e prefix (ecdsa_e_prefix)."""
        if ecdsa_e:
            items = [(r, i, ecdsa_e_prefix(m) if r != ROLE_USIG else m, t) for (r, i, m, t) in items]
        roles, ids, mb, mo, tb, to = flat_calls(items, pinned, compact=True)
        return self.verify_flat32_arrays(roles, ids, mb, mo, tb, to, pinned=pinned)

    def verify_flat32_arrays(self, roles, ids, mb, mo, tb, to, out=None, pinned: bool = False):
        """mbft_verify_batch_flat32 over prepared compact arrays."""
        n = len(roles)
        if out is None:
            out = host_array(n) if pinned else np.zeros(n, dtype=np.uint8)
        self._check(self.lib.mbft_verify_batch_flat32(self.ctx, _buf(roles), _buf(ids), _buf(mb), _buf(mo),
                                                      _buf(tb), _buf(to), n, _buf(out)),
                    "verify_batch_flat32")
        return out

    def check_batch_flat32(self, items, pinned: bool = False) -> np.ndarray:
        """mbft_check_batch_flat32: pure statuses, compact form."""
        roles, ids, mb, mo, tb, to = flat_calls(items, pinned, compact=True)
        n = len(items)
        out = host_array(n) if pinned else np.zeros(n, dtype=np.uint8)
        self._check(self.lib.mbft_check_batch_flat32(self.ctx, _buf(roles), _buf(ids), _buf(mb), _buf(mo),
                                                     _buf(tb), _buf(to), n, _buf(out)),
                    "check_batch_flat32")
        return out

    def check_batch_flat(self, items, pinned: bool = False) -> np.ndarray:
        """mbft_check_batch_flat: pure statuses, no epoch state touched."""
        roles, ids, mb, mo, tb, to = flat_calls(items, pinned)
        out = host_array(len(items)) if pinned else np.zeros(len(items), dtype=np.uint8)
        self._check(self.lib.mbft_check_batch_flat(self.ctx, _buf(roles), _buf(ids), _buf(mb), _buf(mo),
                                                   _buf(tb), _buf(to), len(items), _buf(out)),
                    "check_batch_flat")
        return np.array(out)

    def resolve_checked(self, role: int, id_: int, msg: bytes, tag: bytes, pure: int) -> int:
        return self._check(self.lib.mbft_resolve_checked(self.ctx, role, id_, msg, len(msg), tag,
                                                         len(tag), pure), "resolve_checked")

    # ---------------------------------------------------- message layer
    def validate_messages(self, msgs, n_replicas: int, flags: int = 0) -> np.ndarray:
        """Batched core validators (include/minbft_gpu.h mbft_validate_messages):
        per message 0 = valid, else (stage << 8) | status."""
        arr, keep = _lib.make_messages(msgs)
        out = np.zeros(len(msgs), dtype=np.int32)
        self._check(self.lib.mbft_validate_messages(self.ctx, arr, len(msgs), n_replicas, flags,
                                                    _buf(out)), "validate_messages")
        del keep
        return out

    def authen_digests(self, msgs, kind: int, epochs=None, counters=None) -> np.ndarray:
        """mbft_authen_digests: e of AuthenBytes(msg) per message, on the GPU
        (kind 0 REQUEST, 1 REPLY: ECDSA quirk; 2 PREPARE, 3 COMMIT: USIG chain)."""
        arr, keep = _lib.make_messages(msgs)
        n = len(msgs)
        ep = None if epochs is None else np.ascontiguousarray(epochs, dtype=np.uint64)
        ct = None if counters is None else np.ascontiguousarray(counters, dtype=np.uint64)
        out = np.zeros((n, 32), dtype=np.uint8)
        self._check(self.lib.mbft_authen_digests(self.ctx, arr, n, kind, _buf(ep), _buf(ct), _buf(out)),
                    "authen_digests")
        del keep
        return out

    def validate_messages_packed(self, arr: np.ndarray, n_replicas: int, flags: int = 0,
                                 out: Optional[np.ndarray] = None) -> np.ndarray:
        """mbft_validate_messages over a packed mbft_message array
        (_lib.message_dtype(); its pointers must stay valid)."""
        n = arr.shape[0]
        if out is None:
            out = np.zeros(n, dtype=np.int32)
        self._check(self.lib.mbft_validate_messages(
            self.ctx, ctypes.cast(arr.ctypes.data, ctypes.POINTER(_lib.MbftMessage)), n, n_replicas,
            flags, _buf(out)), "validate_messages")
        return out

    @staticmethod
    def pack_messages(arr: np.ndarray, pinned: bool = True):
        """mbft_pack_messages over a packed mbft_message array ->
        (records, byte arena): the flat batch of mbft_validate_messages_flat,
        in library page-locked memory if `pinned` (then validated on the GPU)."""
        lib = _lib.load()
        n = arr.shape[0]
        msgs = ctypes.cast(arr.ctypes.data, ctypes.c_void_p)
        used = ctypes.c_size_t(0)
        lib.mbft_pack_messages(msgs, n, None, None, 0, ctypes.byref(used))  # size only
        alloc = host_array if pinned else (lambda k, dt=np.uint8: np.zeros(k, dtype=dt))
        recs = alloc(n, _lib.msg_rec_dtype())
        arena = alloc(max(int(used.value), 1))
        rc = lib.mbft_pack_messages(msgs, n, _buf(recs), _buf(arena), int(used.value), ctypes.byref(used))
        if rc != _lib.OK:
            raise ValueError(f"mbft_pack_messages: {rc}")
        return recs, arena[: int(used.value)] if used.value else arena[:0]

    def validate_messages_flat(self, recs: np.ndarray, arena: np.ndarray, n_replicas: int, flags: int = 0,
                               out: Optional[np.ndarray] = None) -> np.ndarray:
        """mbft_validate_messages_flat: the same results as validate_messages;
        on the GPU end to end when recs and arena are library page-locked
        memory (pack_messages(pinned=True), host_array)."""
        n = recs.shape[0]
        if out is None:
            out = np.zeros(n, dtype=np.int32)
        self._check(self.lib.mbft_validate_messages_flat(self.ctx, _buf(recs), n, _buf(arena), arena.nbytes,
                                                         n_replicas, flags, _buf(out)),
                    "validate_messages_flat")
        return out

    def check_messages_flat(self, recs: np.ndarray, arena: np.ndarray, n_replicas: int) -> "MessageBatch":
        """mbft_check_messages_flat: every pure check of the batch on the GPU,
        no state touched; resolve the messages later (MessageBatch.resolve)."""
        h = ctypes.c_void_p()
        self._check(self.lib.mbft_check_messages_flat(self.ctx, _buf(recs), recs.shape[0], _buf(arena),
                                                      arena.nbytes, n_replicas, ctypes.byref(h)),
                    "check_messages_flat")
        return MessageBatch(self, h, recs.shape[0])

    def validate_messages_via_flat(self, msgs, n_replicas: int, flags: int = 0, pinned: bool = True) -> np.ndarray:
        """validate_messages through the flat entry point (packed from the
        oracle-style message objects)."""
        arr, keep = _lib.make_messages(msgs)
        packed = np.frombuffer(arr, dtype=_lib.message_dtype(), count=len(msgs))
        recs, arena = self.pack_messages(packed, pinned)
        del keep
        return self.validate_messages_flat(recs, arena, n_replicas, flags)

    def authen_digests_packed(self, arr: np.ndarray, kind: int, epochs=None, counters=None) -> np.ndarray:
        n = arr.shape[0]
        ep = None if epochs is None else np.ascontiguousarray(epochs, dtype=np.uint64)
        ct = None if counters is None else np.ascontiguousarray(counters, dtype=np.uint64)
        out = np.zeros((n, 32), dtype=np.uint8)
        self._check(self.lib.mbft_authen_digests(
            self.ctx, ctypes.cast(arr.ctypes.data, ctypes.POINTER(_lib.MbftMessage)), n, kind,
            _buf(ep), _buf(ct), _buf(out)), "authen_digests")
        return out

    def validate_replies(self, msgs, client_id: int, flags: int = 0) -> np.ndarray:
        """Client-side REPLY checks (mbft_validate_replies): per REPLY 0 =
        valid, else (stage << 8) | status; no stream stop."""
        arr, keep = _lib.make_messages(msgs)
        out = np.zeros(len(msgs), dtype=np.int32)
        self._check(self.lib.mbft_validate_replies(self.ctx, arr, len(msgs), client_id, flags,
                                                   _buf(out)), "validate_replies")
        del keep
        return out

    def validate_replies_flat(self, recs: np.ndarray, arena: np.ndarray, client_id: int,
                              flags: int = 0) -> np.ndarray:
        """mbft_validate_replies_flat over records + arena (pack_messages)."""
        n = recs.shape[0]
        out = np.zeros(n, dtype=np.int32)
        self._check(self.lib.mbft_validate_replies_flat(self.ctx, _buf(recs), n, _buf(arena), arena.nbytes,
                                                        client_id, flags, _buf(out)), "validate_replies_flat")
        return out

    # ------------------------------------------------------------- core
    def verify_prehashed(self, e: np.ndarray, r: np.ndarray, s: np.ndarray,
                         slots: np.ndarray) -> np.ndarray:
        e = np.ascontiguousarray(e, dtype=np.uint8).reshape(-1, 32)
        r = np.ascontiguousarray(r, dtype=np.uint8).reshape(-1, 32)
        s = np.ascontiguousarray(s, dtype=np.uint8).reshape(-1, 32)
        slots = np.ascontiguousarray(slots, dtype=np.uint32).reshape(-1)
        n = e.shape[0]
        assert r.shape[0] == n and s.shape[0] == n and slots.shape[0] == n
        out = np.zeros(n, dtype=np.uint8)
        self._check(self.lib.mbft_verify_prehashed(self.ctx, _buf(e), _buf(r), _buf(s), _buf(slots),
                                                   n, _buf(out)), "verify_prehashed")
        return out

    def verify_prehashed_device(self, d_e: int, d_r: int, d_s: int, d_slots: int, n: int,
                                d_status: int, stream: int = 0) -> None:
        self._check(self.lib.mbft_verify_prehashed_device(
            self.ctx, ctypes.c_void_p(d_e), ctypes.c_void_p(d_r), ctypes.c_void_p(d_s),
            ctypes.c_void_p(d_slots), n, ctypes.c_void_p(d_status), ctypes.c_void_p(stream)),
            "verify_prehashed_device")

    def sign_prehashed(self, priv: np.ndarray, e: np.ndarray,
                       key_idx: Optional[np.ndarray] = None) -> Tuple[np.ndarray, np.ndarray]:
        priv = np.ascontiguousarray(priv, dtype=np.uint8).reshape(-1, 32)
        e = np.ascontiguousarray(e, dtype=np.uint8).reshape(-1, 32)
        n = e.shape[0]
        ki = None if key_idx is None else np.ascontiguousarray(key_idx, dtype=np.uint32)
        r = np.zeros((n, 32), dtype=np.uint8)
        s = np.zeros((n, 32), dtype=np.uint8)
        self._check(self.lib.mbft_sign_prehashed(self.ctx, _buf(priv), priv.shape[0], _buf(ki),
                                                 _buf(e), n, _buf(r), _buf(s)), "sign_prehashed")
        return r, s

    # ---------------------------------------------------------- profiling
    def profile(self, enable: bool = True):
        """Record HIP events around the inversion and verify kernels of every
        batch (on the stream they are launched on)."""
        self._check(self.lib.mbft_profile_enable(self.ctx, int(enable)), "profile_enable")

    def profile_read(self) -> dict:
        out = (ctypes.c_double * 4)()
        self._check(self.lib.mbft_profile_read(self.ctx, out), "profile_read")
        return {"verify_ms": out[0], "inverse_ms": out[1], "batches": int(out[2]), "items": int(out[3])}

    def msg_layer_profile(self) -> dict:
        """mbft_profile_msg_layer (HIP events; profiling enabled): calls,
        H2D ms, device ms, bytes uploaded -- summed since the last read."""
        out = (ctypes.c_double * 4)()
        self._check(self.lib.mbft_profile_msg_layer(self.ctx, out), "profile_msg_layer")
        return {"calls": out[0], "h2d_ms": out[1], "device_ms": out[2], "bytes": out[3]}

    def stage_profile(self) -> dict:
        """Host-side stage times of verify_batch since the last call, per
        batch (mbft_profile_stages); resets them."""
        out = (ctypes.c_double * 6)()
        self._check(self.lib.mbft_profile_stages(self.ctx, out), "profile_stages")
        b = max(out[0], 1.0)
        return {"batches": int(out[0]), "items": int(out[1]),
                "host_prepare_ms": out[2] / b, "gpu_wait_after_last_chunk_ms": out[3] / b,
                "resolve_ms": out[4] / b, "total_ms": out[5] / b}

    def sign_prehashed_device(self, d_priv: int, d_key_idx: int, d_e: int, n: int, d_r: int,
                              d_s: int, stream: int = 0) -> None:
        self._check(self.lib.mbft_sign_prehashed_device(
            self.ctx, ctypes.c_void_p(d_priv), ctypes.c_void_p(d_key_idx), ctypes.c_void_p(d_e), n,
            ctypes.c_void_p(d_r), ctypes.c_void_p(d_s), ctypes.c_void_p(stream)),
            "sign_prehashed_device")

    def sign_nonce_device(self, d_priv: int, d_key_idx: int, d_e: int, d_k: int, n: int, d_r: int,
                          d_s: int, stream: int = 0) -> None:
        """Signatures with given nonces (crafted-input generation)."""
        self._check(self.lib.mbft_sign_nonce_device(
            self.ctx, ctypes.c_void_p(d_priv), ctypes.c_void_p(d_key_idx), ctypes.c_void_p(d_e),
            ctypes.c_void_p(d_k), n, ctypes.c_void_p(d_r), ctypes.c_void_p(d_s),
            ctypes.c_void_p(stream)), "sign_nonce_device")

    # ------------------------------------------------------ SHA-256 stage
    def request_digests_device(self, d_seq: int, d_ops: int, op_len: int, n: int, d_e: int,
                               stream: int = 0) -> None:
        """e_i = (AuthenBytes(REQUEST_i) || SHA256(""))[0:32] on the GPU."""
        self._check(self.lib.mbft_request_digests_device(
            self.ctx, ctypes.c_void_p(d_seq), ctypes.c_void_p(d_ops), op_len, n,
            ctypes.c_void_p(d_e), ctypes.c_void_p(stream)), "request_digests_device")

    def sha256_device(self, d_data: int, d_off: int, n: int, d_out: int, stream: int = 0) -> None:
        self._check(self.lib.mbft_sha256_device(
            self.ctx, ctypes.c_void_p(d_data), ctypes.c_void_p(d_off), n, ctypes.c_void_p(d_out),
            ctypes.c_void_p(stream)), "sha256_device")

    def usig_digests_device(self, d_data: int, d_off: int, d_epoch: int, d_counter: int, n: int,
                            d_e: int, stream: int = 0) -> None:
        self._check(self.lib.mbft_usig_digests_device(
            self.ctx, ctypes.c_void_p(d_data), ctypes.c_void_p(d_off), ctypes.c_void_p(d_epoch),
            ctypes.c_void_p(d_counter), n, ctypes.c_void_p(d_e), ctypes.c_void_p(stream)),
            "usig_digests_device")


class MessageBatch:
    """A device-checked message batch (mbft_check_messages_flat): resolve(i)
    is message i's result with the USIG epoch step applied now
    (mbft_resolve_message); close() frees it."""

    def __init__(self, auth: "Authenticator", handle: ctypes.c_void_p, n: int):
        self.auth, self.h, self.n = auth, handle, n

    def resolve(self, i: int) -> int:
        return self.auth._check(self.auth.lib.mbft_resolve_message(self.auth.ctx, self.h, i),
                                "resolve_message")

    def resolve_range(self, i0: int, count: int, out: Optional[np.ndarray] = None) -> np.ndarray:
        """mbft_resolve_messages: messages i0 .. i0+count-1 in order."""
        if out is None:
            out = np.zeros(count, dtype=np.int32)
        self.auth._check(self.auth.lib.mbft_resolve_messages(self.auth.ctx, self.h, i0, count, _buf(out)),
                         "resolve_messages")
        return out

    def close(self) -> None:
        if self.h:
            self.auth.lib.mbft_msg_batch_free(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def der_encode_sig(r: bytes, s: bytes) -> bytes:
    """asn1.Marshal(ecdsaSignature{r, s}) for 32-byte big-endian r, s."""
    def i(v: bytes) -> bytes:
        v = v.lstrip(b"\x00") or b"\x00"
        if v[0] & 0x80:
            v = b"\x00" + v
        return b"\x02" + bytes([len(v)]) + v
    body = i(r) + i(s)
    return b"\x30" + bytes([len(body)]) + body


def items_from(iterable: Iterable) -> list:
    return list(iterable)


def der_encode_rows(r: np.ndarray, s: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Vectorized asn1.Marshal(ecdsaSignature{r, s}) for n rows of 32-byte
    big-endian r, s: returns (tags (n, 72) uint8, lens (n,) uint64).  Rows
    are grouped by (leading zeros, pad byte) of r and s, so each group is a
    handful of slice copies."""
    r = np.ascontiguousarray(r, dtype=np.uint8).reshape(-1, 32)
    s = np.ascontiguousarray(s, dtype=np.uint8).reshape(-1, 32)
    n = r.shape[0]

    def shape(v):
        nzm = v != 0
        nz = np.where(nzm.any(axis=1), np.argmax(nzm, axis=1), 31)  # first nonzero byte (0 -> one 00)
        pad = (v[np.arange(n), nz] >= 0x80).astype(np.int64)
        return nz, pad

    rz, rp = shape(r)
    sz, sp = shape(s)
    rl = 32 - rz + rp
    sl = 32 - sz + sp
    tags = np.zeros((n, 72), dtype=np.uint8)
    lens = (6 + rl + sl).astype(np.uint64)
    key = ((rz * 2 + rp) * 64 + sz * 2 + sp)
    for k in np.unique(key):
        rows = np.nonzero(key == k)[0]
        a, b = int(rz[rows[0]]), int(rp[rows[0]])
        c, d = int(sz[rows[0]]), int(sp[rows[0]])
        la, lc = 32 - a + b, 32 - c + d
        t = tags[rows]
        t[:, 0] = 0x30
        t[:, 1] = 4 + la + lc
        t[:, 2] = 0x02
        t[:, 3] = la
        t[:, 4 + b:4 + la] = r[rows, a:]
        o = 4 + la
        t[:, o] = 0x02
        t[:, o + 1] = lc
        t[:, o + 2 + d:o + 2 + lc] = s[rows, c:]
        tags[rows] = t
    return tags, lens


def plan_windows(device: int, n_replica: int, n_usig: int, n_client: int) -> dict:
    """mbft_plan_windows: comb windows from the device's free HBM and the key
    counts (what the Go binding uses by default)."""
    lib = _lib.load()
    out = [ctypes.c_int(0) for _ in range(4)]
    rc = lib.mbft_plan_windows(device, n_replica, n_usig, n_client, *[ctypes.byref(x) for x in out])
    if rc != _lib.OK:
        raise RuntimeError(f"mbft_plan_windows: {rc}")
    return dict(zip(("generator", "replica", "usig", "client"), (x.value for x in out)))

"""CPU restatement of MinBFT's message-authentication path (TEST INFRASTRUCTURE).

This module is the *oracle*: a plain-Python restatement of the reference's
verification semantics, used only by ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg as the checker.  Nothing in the
product (``minbft_amd/``) imports it.

What it restates (reference = hyperledger-labs/minbft snapshot at
/root/reference, Go stdlib pinned by go.mod:30 ``go 1.11`` and CI Go 1.11/1.14,
.github/workflows/continuous-integration.yml:15):

* ``sample/authentication/crypto.go:113-126`` -- PublicAuthenScheme: the
  digest is ``HashScheme.New().Sum(m)`` which APPENDS SHA256("") to ``m``
  (``md = m || e3b0c442...``), then ECDSA over ``md`` (left-most 256 bits).
* ``sample/authentication/crypto.go:79-89`` -- EcdsaSigCipher.Verify:
  ``asn1.Unmarshal`` error => panic; trailing bytes ignored.
* ``usig/sgx/usig-enclave.go:198-229`` -- USIG VerifySignature:
  ``h = SHA256(digest || epoch_le64 || counter_le64)``; DER error => error;
  trailing bytes => error.
* ``usig/sgx/sgx-usig.go:81-168`` -- VerifyUI / MakeID / ParseCert.
* ``sample/authentication/crypto.go:134-144,186-239`` -- USIG key
  fingerprint and epoch capture.
* ``usig/usig.go:54-86`` -- UI = counter_be64 || cert.
* ``messages/authen.go:27-82`` -- AuthenBytes layouts.
* ``sample/authentication/authenticator.go:121-134`` and
  ``keymanager.go:96-101`` -- role/key dispatch.
* Go stdlib ``crypto/ecdsa.Verify`` (Go 1.11/1.14): range checks,
  ``hashToInt``, ``w = s^-1``, ``u1 = e*w``, ``u2 = r*w``,
  ``(x, y) = u1*G + u2*Q`` (CombinedMult, complete), ``(0,0)`` => false,
  accept iff ``x mod N == r``.  No low-s rule.
* Go stdlib ``encoding/asn1`` DER rules for ``struct{R, S *big.Int}``
  (parseTagAndLength, checkInteger, parseBigInt; extra SEQUENCE elements
  ignored).

Independent cross-checks of this restatement (``tests/test_oracle.py``):
RFC 6979 A.2.5 P-256/SHA-256 known-answer signatures, the reference's own
fixture key pair (``sample/authentication/keymanager_test.go:68-69``:
private scalar * G must equal the stored public key) and OpenSSL 3
``ECDSA_do_verify`` via ctypes on random and adversarial vectors.
"""
from __future__ import annotations

import hashlib
import hmac
import struct
from dataclasses import dataclass, field
from typing import Dict, Optional, Tuple

# --------------------------------------------------------------------------
# Curve constants (FIPS 186-4 D.1.2.3, the curve behind elliptic.P256()).
P = 0xFFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFF
N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
A = P - 3
B = 0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B
GX = 0x6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296
GY = 0x4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5

SHA256_EMPTY = hashlib.sha256(b"").digest()  # e3b0c442...7852b855

# Status codes -- must match include/minbft_gpu.h (enum mbft_status).
ACCEPT = 0
REJECT_SIG = 1        # range / infinity / x-mismatch (ecdsa.Verify == false)
MALFORMED_DER = 2     # asn1.Unmarshal error (ECDSA roles: Go panics)
DER_TRAILING = 3      # USIG only: "extra bytes in USIG signature"
UNKNOWN_KEY = 4       # known role, unknown id (pk == nil)
BAD_KEY = 5           # key slot holds an invalid (off-curve) key
BAD_UI = 6            # USIG tag shorter than 8 bytes
BAD_CERT = 7          # USIG cert shorter than 8 bytes
ZERO_COUNTER = 8      # core/usig-ui.go:65-67 (core-level check)
EPOCH_MISMATCH = 9    # usig/sgx/sgx-usig.go:92-94
UNKNOWN_ROLE = 10     # keymanager.go:100 / authenticator.go:126-129

STATUS_NAMES = {
    ACCEPT: "ACCEPT", REJECT_SIG: "REJECT_SIG", MALFORMED_DER: "MALFORMED_DER",
    DER_TRAILING: "DER_TRAILING", UNKNOWN_KEY: "UNKNOWN_KEY", BAD_KEY: "BAD_KEY",
    BAD_UI: "BAD_UI", BAD_CERT: "BAD_CERT", ZERO_COUNTER: "ZERO_COUNTER",
    EPOCH_MISMATCH: "EPOCH_MISMATCH", UNKNOWN_ROLE: "UNKNOWN_ROLE",
}

# api/api.go:98-115
ROLE_REPLICA = 1
ROLE_USIG = 2
ROLE_CLIENT = 3


# --------------------------------------------------------------------------
# Point arithmetic (affine, None = point at infinity).  Deliberately simple
# and obviously-correct; speed is irrelevant for the oracle.
def on_curve(x: int, y: int) -> bool:
    """x509.ParsePKIXPublicKey -> elliptic.Unmarshal on-curve check
    (sample/authentication/keymanager.go:357, usig/sgx/sgx-usig.go:133)."""
    if not (0 <= x < P and 0 <= y < P):
        return False
    return (y * y - (x * x * x + A * x + B)) % P == 0


def point_add(p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    x1, y1 = p1
    x2, y2 = p2
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = (3 * x1 * x1 + A) * pow(2 * y1, -1, P) % P
    else:
        lam = (y2 - y1) * pow(x2 - x1, -1, P) % P
    x3 = (lam * lam - x1 - x2) % P
    y3 = (lam * (x1 - x3) - y1) % P
    return (x3, y3)


def point_neg(p1):
    if p1 is None:
        return None
    return (p1[0], (-p1[1]) % P)


def scalar_mult(k: int, pt):
    """Left-to-right double-and-add; complete for any k >= 0."""
    acc = None
    for bit in bin(k)[2:] if k > 0 else "":
        acc = point_add(acc, acc)
        if bit == "1":
            acc = point_add(acc, pt)
    return acc


G = (GX, GY)


def combined_mult(u1: int, u2: int, q):
    """u1*G + u2*Q, the math of Go's CombinedMult (p256_asm.go: handles
    u1 == 0, equal points via doubling, and opposite points -> infinity)."""
    return point_add(scalar_mult(u1, G), scalar_mult(u2, q))


# --------------------------------------------------------------------------
# Go crypto/ecdsa
def hash_to_int(h: bytes) -> int:
    """crypto/ecdsa hashToInt for a 256-bit order: take the left-most 32
    bytes; shorter hashes are used as-is (no shift since excess <= 0)."""
    h = h[:32]
    return int.from_bytes(h, "big")


def go_ecdsa_verify(q, h: bytes, r: int, s: int) -> bool:
    """crypto/ecdsa.Verify (Go 1.11/1.14).  ``q`` must be an on-curve point
    (the reference only ever reaches Verify with x509-validated keys)."""
    if r <= 0 or s <= 0:
        return False
    if r >= N or s >= N:
        return False
    e = hash_to_int(h)
    w = pow(s, -1, N)
    u1 = e * w % N
    u2 = r * w % N
    pt = combined_mult(u1, u2, q)
    if pt is None:  # Go: x.Sign()==0 && y.Sign()==0 -> false
        return False
    return pt[0] % N == r


# --------------------------------------------------------------------------
# Go encoding/asn1 restatement for struct { R, S *big.Int }
class Asn1Error(Exception):
    pass


def _parse_base128(b: bytes, off: int):
    ret = 0
    shifted = 0
    while off < len(b):
        if shifted == 5:
            raise Asn1Error("base 128 integer too large")
        ret = (ret << 7) | (b[off] & 0x7F)
        c = b[off]
        off += 1
        shifted += 1
        if c & 0x80 == 0:
            if ret > 0x7FFFFFFF:
                raise Asn1Error("base 128 integer too large")
            return ret, off
    raise Asn1Error("truncated base 128 integer")


def _parse_tag_and_length(b: bytes, off: int):
    """encoding/asn1 parseTagAndLength."""
    if off >= len(b):
        raise Asn1Error("internal error in parseTagAndLength")
    c = b[off]
    off += 1
    cls = c >> 6
    compound = (c & 0x20) != 0
    tag = c & 0x1F
    if tag == 0x1F:
        tag, off = _parse_base128(b, off)
        if tag < 0x1F:
            raise Asn1Error("non-minimal tag")
    if off >= len(b):
        raise Asn1Error("truncated tag or length")
    c = b[off]
    off += 1
    if c & 0x80 == 0:
        length = c & 0x7F
    else:
        nbytes = c & 0x7F
        if nbytes == 0:
            raise Asn1Error("indefinite length found (not DER)")
        length = 0
        for _ in range(nbytes):
            if off >= len(b):
                raise Asn1Error("truncated tag or length")
            c = b[off]
            off += 1
            if length >= 1 << 23:
                raise Asn1Error("length too large")
            length = (length << 8) | c
            if length == 0:
                raise Asn1Error("superfluous leading zeros in length")
        if length < 0x80:
            raise Asn1Error("non-minimal length")
    return cls, tag, compound, length, off


def _parse_big_int(v: bytes) -> int:
    """encoding/asn1 checkInteger + parseBigInt (two's complement)."""
    if len(v) == 0:
        raise Asn1Error("empty integer")
    if len(v) > 1 and ((v[0] == 0 and v[1] & 0x80 == 0) or
                       (v[0] == 0xFF and v[1] & 0x80 == 0x80)):
        raise Asn1Error("integer not minimally-encoded")
    x = int.from_bytes(v, "big")
    if v[0] & 0x80:
        x -= 1 << (8 * len(v))
    return x


def _parse_int_field(inner: bytes, off: int):
    if off == len(inner):
        raise Asn1Error("sequence truncated")
    cls, tag, compound, length, off = _parse_tag_and_length(inner, off)
    if cls != 0 or tag != 2 or compound:
        raise Asn1Error("tags don't match")
    if off + length > len(inner):
        raise Asn1Error("data truncated")
    return _parse_big_int(inner[off:off + length]), off + length


def der_parse_sig(sig: bytes) -> Tuple[int, int, bytes]:
    """asn1.Unmarshal(sig, &struct{R, S *big.Int}) -> (R, S, rest).
    Raises Asn1Error exactly where Go returns an error."""
    if len(sig) == 0:
        raise Asn1Error("sequence truncated")
    cls, tag, compound, length, off = _parse_tag_and_length(sig, 0)
    if cls != 0 or tag != 16 or not compound:
        raise Asn1Error("tags don't match")
    if off + length > len(sig):
        raise Asn1Error("data truncated")
    inner = sig[off:off + length]
    r, ioff = _parse_int_field(inner, 0)
    s, ioff = _parse_int_field(inner, ioff)
    # extra bytes inside the SEQUENCE are ignored (encoding/asn1 parseField)
    return r, s, sig[off + length:]


def _der_int(x: int) -> bytes:
    assert x >= 0
    v = x.to_bytes(max(1, (x.bit_length() + 7) // 8), "big")
    if v[0] & 0x80:
        v = b"\x00" + v
    return b"\x02" + _der_len(len(v)) + v


def _der_len(n: int) -> bytes:
    if n < 0x80:
        return bytes([n])
    v = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(v)]) + v


def der_encode_sig(r: int, s: int) -> bytes:
    """asn1.Marshal(ecdsaSignature{r, s}) for non-negative r, s."""
    body = _der_int(r) + _der_int(s)
    return b"\x30" + _der_len(len(body)) + body


# --------------------------------------------------------------------------
# Deterministic signer (RFC 6979, SHA-256) -- generation side only, used to
# make fixtures; the reference signs with crypto/rand (crypto.go:65) but the
# verification semantics do not depend on the nonce.
def _bits2int(b: bytes) -> int:
    return int.from_bytes(b[:32], "big")


def rfc6979_k(d: int, h1: bytes) -> int:
    x = d.to_bytes(32, "big")
    hv = (_bits2int(h1) % N).to_bytes(32, "big")
    v = b"\x01" * 32
    k = b"\x00" * 32
    k = hmac.new(k, v + b"\x00" + x + hv, hashlib.sha256).digest()
    v = hmac.new(k, v, hashlib.sha256).digest()
    k = hmac.new(k, v + b"\x01" + x + hv, hashlib.sha256).digest()
    v = hmac.new(k, v, hashlib.sha256).digest()
    while True:
        v = hmac.new(k, v, hashlib.sha256).digest()
        kk = _bits2int(v)
        if 1 <= kk < N:
            return kk
        k = hmac.new(k, v + b"\x00", hashlib.sha256).digest()
        v = hmac.new(k, v, hashlib.sha256).digest()


def ecdsa_sign(d: int, h: bytes, k: Optional[int] = None) -> Tuple[int, int]:
    e = hash_to_int(h)
    if k is None:
        k = rfc6979_k(d, h[:32])
    R = scalar_mult(k, G)
    r = R[0] % N
    s = pow(k, -1, N) * (e + r * d) % N
    assert r != 0 and s != 0
    return r, s


def pubkey(d: int):
    return scalar_mult(d, G)


# --------------------------------------------------------------------------
# messages/authen.go:27-82
def _h(data: bytes) -> bytes:
    return hashlib.sha256(data).digest()


def authen_request(seq: int, op: bytes) -> bytes:
    return b"REQUEST" + struct.pack(">Q", seq) + _h(op)


def authen_reply(client_id: int, seq: int, result: bytes) -> bytes:
    return b"REPLY" + struct.pack(">IQ", client_id, seq) + _h(result)


def _prepare_fields(view: int, client_id: int, seq: int, op: bytes) -> bytes:
    return struct.pack(">QI", view, client_id) + struct.pack(">Q", seq) + _h(op)


def authen_prepare(view: int, client_id: int, seq: int, op: bytes) -> bytes:
    return b"PREPARE" + _prepare_fields(view, client_id, seq, op)


def authen_commit(primary_id: int, view: int, client_id: int, seq: int,
                  op: bytes, prepare_counter: int) -> bytes:
    return (b"COMMIT" + struct.pack(">I", primary_id) +
            _prepare_fields(view, client_id, seq, op) +
            struct.pack(">Q", prepare_counter))


def authen_req_view_change(new_view: int) -> bytes:
    return b"REQ-VIEW-CHANGE" + struct.pack(">Q", new_view)


# --------------------------------------------------------------------------
# Digest rules
def quirk_digest(msg: bytes) -> bytes:
    """crypto.go:114,121: HashScheme.New().Sum(m) == m || SHA256("")."""
    return msg + SHA256_EMPTY


def usig_digest(msg: bytes, epoch: int, counter: int) -> bytes:
    """usig-enclave.go:204-214 with messageDigest sgx-usig.go:99-101."""
    return _h(_h(msg) + struct.pack("<QQ", epoch, counter))


# --------------------------------------------------------------------------
# PKIX / fingerprint (crypto.go:134-144, Appendix A of SURVEY.md)
PKIX_P256_PREFIX = bytes.fromhex(
    "3059301306072a8648ce3d020106082a8648ce3d030107034200")


def pkix_encode(q) -> bytes:
    return PKIX_P256_PREFIX + b"\x04" + q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big")


def pkix_decode(der: bytes):
    if len(der) != 91 or not der.startswith(PKIX_P256_PREFIX + b"\x04"):
        raise ValueError("unsupported PKIX public key")
    x = int.from_bytes(der[27:59], "big")
    y = int.from_bytes(der[59:91], "big")
    if not on_curve(x, y):
        raise ValueError("x509: invalid elliptic curve public key")
    return (x, y)


def usig_fingerprint(q) -> bytes:
    return _h(pkix_encode(q))[:8]


def ui_marshal(counter: int, cert: bytes) -> bytes:
    return struct.pack(">Q", counter) + cert


def make_cert(epoch: int, sig_der: bytes) -> bytes:
    return struct.pack(">Q", epoch) + sig_der


def usig_create_ui(d: int, msg: bytes, epoch: int, counter: int) -> bytes:
    """Software stand-in for the enclave's ecall_usig_create_ui
    (usig/sgx/enclave/usig.c:36-76): returns the marshalled UI tag."""
    r, s = ecdsa_sign(d, usig_digest(msg, epoch, counter))
    return ui_marshal(counter, make_cert(epoch, der_encode_sig(r, s)))


# --------------------------------------------------------------------------
# Authenticator model (authenticator.go:121-134 + the two schemes)
@dataclass
class KeyStore:
    # role -> id -> point (None means registered-but-invalid key slot)
    keys: Dict[int, Dict[int, Optional[Tuple[int, int]]]] = field(default_factory=dict)
    usig_enabled: bool = True


class Authenticator:
    """Status-code restatement of Authenticator.VerifyMessageAuthenTag.
    ``verify`` returns one of the status constants instead of Go's
    nil/error/panic; ``MALFORMED_DER`` in the ECDSA roles is the Go panic."""

    def __init__(self, ks: KeyStore):
        self.ks = ks
        self.epoch: Dict[bytes, int] = {}  # crypto.go:152 fingerprint -> epoch

    def verify(self, role: int, id_: int, msg: bytes, tag: bytes) -> int:
        keymap = self.ks.keys.get(role)
        if keymap is None:
            return UNKNOWN_ROLE           # keymanager.go:100
        if role == ROLE_USIG and not self.ks.usig_enabled:
            return UNKNOWN_ROLE           # authenticator.go:126-129
        if role not in (ROLE_REPLICA, ROLE_CLIENT, ROLE_USIG):
            return UNKNOWN_ROLE
        known = id_ in keymap
        q = keymap.get(id_)
        if role == ROLE_USIG:
            return self._verify_usig(known, q, msg, tag)
        return self._verify_ecdsa(known, q, msg, tag)

    @staticmethod
    def _verify_ecdsa(known, q, msg, tag) -> int:
        try:
            r, s, _rest = der_parse_sig(tag)   # crypto.go:81, rest ignored
        except Asn1Error:
            return MALFORMED_DER               # crypto.go:82-84 panic
        if not known:
            return UNKNOWN_KEY                 # crypto.go:85-88 (pk nil)
        if q is None:
            return BAD_KEY
        ok = go_ecdsa_verify(q, quirk_digest(msg), r, s)
        return ACCEPT if ok else REJECT_SIG

    def _verify_usig(self, known, q, msg, tag) -> int:
        if len(tag) < 8:
            return BAD_UI                      # usig.go:75-80
        counter = struct.unpack(">Q", tag[:8])[0]
        cert = tag[8:]
        if not known:
            return UNKNOWN_KEY                 # crypto.go:193-196
        if q is None:
            return BAD_KEY
        fp = usig_fingerprint(q)
        epoch = self.epoch.get(fp)
        if epoch is None:
            if counter == 1:                   # crypto.go:219-225
                if len(cert) < 8:
                    return BAD_CERT
                epoch = struct.unpack(">Q", cert[:8])[0]
            else:
                epoch = 0
        if len(cert) < 8:
            return BAD_CERT                    # sgx-usig.go:87-90
        ui_epoch = struct.unpack(">Q", cert[:8])[0]
        if ui_epoch != epoch:
            return EPOCH_MISMATCH              # sgx-usig.go:92-94
        sig = cert[8:]
        try:
            r, s, rest = der_parse_sig(sig)    # usig-enclave.go:217
        except Asn1Error:
            return MALFORMED_DER
        if len(rest) != 0:
            return DER_TRAILING                # usig-enclave.go:220-221
        if not go_ecdsa_verify(q, usig_digest(msg, epoch, counter), r, s):
            return REJECT_SIG
        self.epoch[fp] = epoch                 # crypto.go:236
        return ACCEPT


def core_verify_ui(auth: Authenticator, replica_id: int, msg: bytes, tag: bytes) -> int:
    """core/usig-ui.go:62-77: zero counter rejected before the authenticator."""
    if len(tag) >= 8 and struct.unpack(">Q", tag[:8])[0] == 0:
        return ZERO_COUNTER
    return auth.verify(ROLE_USIG, replica_id, msg, tag)


# --------------------------------------------------------------------------
# Message layer: AuthenBytes for a flattened message and the core validators
# (core/message-handling.go:409-424 and the validators it dispatches to).
MSG_REQUEST, MSG_REPLY, MSG_PREPARE, MSG_COMMIT, MSG_REQ_VIEW_CHANGE = 1, 2, 3, 4, 5
ST_REQUEST_SIG, ST_NOT_PRIMARY, ST_PREPARE_UI, ST_COMMIT_FROM_PRIMARY = 1, 2, 3, 4
ST_COMMIT_UI, ST_NOT_IMPLEMENTED, ST_STREAM_STOPPED, ST_REPLY_SIG, ST_AFTER_PANIC = 5, 6, 7, 8, 9
ST_UNKNOWN_TYPE, ST_REPLY_CLIENT_ID = 10, 11
VF_NO_STREAM_STOP, VF_NO_PANIC_STOP = 1, 2


@dataclass
class Msg:
    """Flattened authenticated fields (mirrors include/minbft_gpu.h
    mbft_message)."""
    type: int
    stream: int = 0
    replica_id: int = 0
    prep_replica_id: int = 0
    view: int = 0
    client_id: int = 0
    seq: int = 0
    op: bytes = b""
    sig: bytes = b""
    ui_counter: int = 0
    ui_cert: bytes = b""
    prep_ui_counter: int = 0
    prep_ui_cert: bytes = b""


def msg_authen_bytes(m: Msg, as_type: Optional[int] = None) -> bytes:
    """messages/authen.go:27-82 for the message (or its embedded parts)."""
    t = m.type if as_type is None else as_type
    if t == MSG_REQUEST:
        return authen_request(m.seq, m.op)
    if t == MSG_REPLY:
        return authen_reply(m.client_id, m.seq, m.op)
    if t == MSG_PREPARE:
        return authen_prepare(m.view, m.client_id, m.seq, m.op)
    if t == MSG_COMMIT:
        return authen_commit(m.prep_replica_id, m.view, m.client_id, m.seq, m.op, m.prep_ui_counter)
    if t == MSG_REQ_VIEW_CHANGE:
        return authen_req_view_change(m.view)
    raise ValueError("unknown message type")


def validate_messages(auth: Authenticator, msgs, n_replicas: int, flags: int = 0):
    """Sequential restatement of the validators with the stream loop and
    panic semantics; returns (stage << 8) | status per message (0 = valid)."""
    out = []
    stopped = set()
    panicked = False

    def sig_call(role, id_, ab, tag, stage):
        st = auth.verify(role, id_, ab, tag)
        return 0 if st == ACCEPT else ((stage << 8) | st, st == MALFORMED_DER and role != ROLE_USIG)

    def ui_call(rid, ab, ctr, cert, stage):
        if ctr == 0:  # core/usig-ui.go:65-67
            return ((stage << 8) | ZERO_COUNTER, False)
        st = auth.verify(ROLE_USIG, rid, ab, ui_marshal(ctr, cert))
        return 0 if st == ACCEPT else ((stage << 8) | st, False)

    def prepare(m, primary, ctr, cert):
        if primary != m.view % n_replicas:  # core/prepare.go:51-53
            return (ST_NOT_PRIMARY << 8, False)
        r = sig_call(ROLE_CLIENT, m.client_id, msg_authen_bytes(m, MSG_REQUEST), m.sig, ST_REQUEST_SIG)
        if r:
            return r
        return ui_call(primary, msg_authen_bytes(m, MSG_PREPARE), ctr, cert, ST_PREPARE_UI)

    for m in msgs:
        if panicked:
            out.append(ST_AFTER_PANIC << 8)
            continue
        if not (flags & VF_NO_STREAM_STOP) and m.stream in stopped:
            out.append(ST_STREAM_STOPPED << 8)
            continue
        if m.type == MSG_REQUEST:
            r = sig_call(ROLE_CLIENT, m.client_id, msg_authen_bytes(m), m.sig, ST_REQUEST_SIG)
        elif m.type == MSG_REPLY:
            # core/message-handling.go:420-421: a replica's message validator
            # panics on any other type ("Unknown message type")
            r = (ST_UNKNOWN_TYPE << 8, True)
        elif m.type == MSG_PREPARE:
            r = prepare(m, m.replica_id, m.ui_counter, m.ui_cert)
        elif m.type == MSG_COMMIT:
            if m.replica_id == m.prep_replica_id:  # core/commit.go:78-80
                r = (ST_COMMIT_FROM_PRIMARY << 8, False)
            else:
                r = prepare(m, m.prep_replica_id, m.prep_ui_counter, m.prep_ui_cert)
                if not r:
                    r = ui_call(m.replica_id, msg_authen_bytes(m), m.ui_counter, m.ui_cert, ST_COMMIT_UI)
        else:
            r = (ST_NOT_IMPLEMENTED << 8, False)
        if r:
            code, panic = r
            out.append(code)
            stopped.add(m.stream)
            if panic and not (flags & VF_NO_PANIC_STOP):
                panicked = True
        else:
            out.append(0)
    return out


def validate_replies(auth: Authenticator, msgs, client_id: int, flags: int = 0):
    """Client side (client/message-handling.go:93-110,140-170): each REPLY is
    checked on its own -- ClientID mismatch => error, else
    VerifyMessageAuthenTag(ReplicaAuthen, replicaID, AuthenBytes, sig); a
    rejected REPLY is only logged and the stream goes on (no stream stop),
    but a malformed DER signature still panics (crypto.go:82-84)."""
    out = []
    panicked = False
    for m in msgs:
        if m.type != MSG_REPLY:
            raise ValueError("validate_replies takes REPLY messages only")
        if panicked:
            out.append(ST_AFTER_PANIC << 8)
            continue
        if m.client_id != client_id:                  # message-handling.go:163-165
            out.append(ST_REPLY_CLIENT_ID << 8)
            continue
        st = auth.verify(ROLE_REPLICA, m.replica_id, msg_authen_bytes(m), m.sig)
        if st == ACCEPT:
            out.append(0)
            continue
        out.append((ST_REPLY_SIG << 8) | st)
        if st == MALFORMED_DER and not (flags & VF_NO_PANIC_STOP):
            panicked = True
    return out

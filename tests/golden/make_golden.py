#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Run from the repo root:  python tests/golden/make_golden.py

Every expected value comes from the oracle (oracle/p256.py), which is pinned
by RFC 6979 A.2.5 known answers, the reference's fixture key pair
(sample/authentication/keymanager_test.go:68-69) and OpenSSL 3
ECDSA_do_verify (tests/test_oracle.py re-checks all of these).  The Go
reference itself cannot run here (no Go toolchain).

Fixtures:
  kat.json        RFC 6979 P-256/SHA-256 vectors + reference fixture key.
  prehashed.json  (Q, e, r, s) -> accept/reject, random + adversarial,
                  including R.x >= N, u1 == 0, e >= N, final infinity, and
                  accumulator collisions (doubling / infinity mid-way) of
                  the GPU's 8-bit fixed-window comb.
  comb_windows.json  accumulator collisions for the 20..29-bit key windows.
  der.json        DER signature strings -> Go encoding/asn1 outcome.
  authen.json     Authenticator-level call sequences (ECDSA roles with the
                  Sum(m) quirk, USIG roles with epoch capture), with the
                  expected status of each call, in order.
"""
from __future__ import annotations

import base64
import hashlib
import json
import os
import random
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import p256 as o  # noqa: E402

RNG = random.Random(0x4D696E42)  # "MinB"


def h32(x: int) -> str:
    return x.to_bytes(32, "big").hex()


def rand_scalar() -> int:
    return RNG.randrange(1, o.N)


def key_from_seed(i: int) -> int:
    return int.from_bytes(hashlib.sha256(b"minbft-amd key %d" % i).digest(), "big") % (o.N - 1) + 1


# ----------------------------------------------------------------------------
def make_kat():
    pk_b64 = ("MFkwEwYHKoZIzj0CAQYIKoZIzj0DAQcDQgAEh6uiVdr+3EgyT3YEilvrvzQINr8eo"
              "lxR22/0JudQrpGbLQQQIK+7RdnoLaIyZIlakZkb1tAws0iQN263EkwzGw==")
    sk_b64 = ("MHcCAQEEIFxopskcl2LyZ/LLsDMBfQk/82WZQI/YhvXNSYZNmUSFoAoGCCqGSM49A"
              "wEHoUQDQgAEh6uiVdr+3EgyT3YEilvrvzQINr8eolxR22/0JudQrpGbLQQQIK+7R"
              "dnoLaIyZIlakZkb1tAws0iQN263EkwzGw==")
    return {
        "rfc6979_p256_sha256": {
            "d": "C9AFA9D845BA75166B5C215767B1D6934E50C3DB36E89B127B8A622B120F6721",
            "ux": "60FED4BA255A9D31C961EB74C6356D68C049B8923B61FA6CE669622E60F29FB6",
            "uy": "7903FE1008B8BC99A41AE9E95628BC64F2F1B20C2D7E9F5177A3C294D4462299",
            "vectors": [
                {"msg": "sample",
                 "k": "A6E3C57DD01ABE90086538398355DD4C3B17AA873382B0F24D6129493D8AAD60",
                 "r": "EFD48B2AACB6A8FD1140DD9CD45E81D69D2C877B56AAF991C34D0EA84EAF3716",
                 "s": "F7CB1C942D657C41D436C7A1B6E29F65F3E900DBB9AFF4064DC4AB2F843ACDA8"},
                {"msg": "test",
                 "k": "D16B6AE827F17175E040871A1C7EC3500192C4C92677336EC2537ACAEE0008E0",
                 "r": "F1ABB023518351CD71D881567B1EA663ED3EFCF6C5132B354F28D3B0B7D38367",
                 "s": "019F4113742A2B14BD25926B49C649155F267E60D3814B4C0CC84250E46F0083"},
            ],
        },
        # sample/authentication/keymanager_test.go:68-69 (data, base64 DER)
        "reference_fixture_key": {"sec1_private_b64": sk_b64, "pkix_public_b64": pk_b64},
        "sha256_empty": o.SHA256_EMPTY.hex(),
    }


# ----------------------------------------------------------------------------
def lift_x(x: int):
    """A curve point with the given x, or None."""
    rhs = (x * x * x + o.A * x + o.B) % o.P
    y = pow(rhs, (o.P + 1) // 4, o.P)
    if y * y % o.P != rhs:
        return None
    return (x, y)


def vec(q, e_int, r, s, label):
    e_b = e_int.to_bytes(32, "big")
    ok = o.go_ecdsa_verify(q, e_b, r, s)
    return {"qx": h32(q[0]), "qy": h32(q[1]), "e": e_b.hex(), "r": h32(r), "s": h32(s),
            "expect": 1 if ok else 0, "label": label}


def signed_instance(d, e_int):
    r, s = o.ecdsa_sign(d, e_int.to_bytes(32, "big"))
    return r, s


def signed_digits(u, W):
    """The GPU comb's signed-digit recoding of a scalar u < 2^256 (W-bit
    windows, low to high; minbft_amd/csrc/kernels.hip comb_digit): x = window
    bits + carry, x > 2^(W-1) -> digit x - 2^W and carry 1; the last window
    takes its bits + carry unrecoded.  sum(d_i 2^(W i)) == u."""
    S = -(-256 // W)
    out, carry = [], 0
    for i in range(S):
        x = ((u >> (W * i)) & ((1 << W) - 1)) + carry
        if i < S - 1 and x > (1 << (W - 1)):
            out.append(x - (1 << W))
            carry = 1
        else:
            out.append(x)
            carry = 0
    assert sum(d << (W * i) for i, d in enumerate(out)) == u
    return out


def comb_collision(i, infinity, W=8, rng=None):
    """Accepting instance where, in the comb's Q phase, the accumulator hits
    +addend (doubling) or -addend (infinity) at window i (W-bit signed-digit
    windows, processed low to high, after all G windows)."""
    rs = (lambda: rng.randrange(1, o.N)) if rng is not None else rand_scalar
    while True:
        k = rs()
        R = o.scalar_mult(k, o.G)
        r = R[0] % o.N
        s = rs()
        u2 = r * pow(s, -1, o.N) % o.N
        dig = signed_digits(u2, W)
        di = dig[i]
        if di == 0:
            continue
        # accumulator before window i: u1*G + partial*Q; addend di*2^(W i)*Q
        partial = sum(d << (W * j) for j, d in enumerate(dig[:i]))
        if not infinity:
            # acc == +addend  <=>  u1 == (di 2^(W i) - partial) * d
            denom = (u2 + (di << (W * i)) - partial) % o.N
        else:
            # acc == -addend  <=>  u1 == -(partial + di 2^(W i)) * d
            denom = (u2 - partial - (di << (W * i))) % o.N
        if denom == 0:
            continue
        d = k * pow(denom, -1, o.N) % o.N
        if d == 0:
            continue
        q = o.scalar_mult(d, o.G)
        u1 = (k - u2 * d) % o.N
        e = u1 * s % o.N
        return q, e, r, s


def make_prehashed():
    out = []
    keys = [key_from_seed(i) for i in range(8)]
    pubs = [o.pubkey(d) for d in keys]
    # random valid / tampered / wrong-key / high-s
    for i in range(96):
        d, q = keys[i % 8], pubs[i % 8]
        e = int.from_bytes(hashlib.sha256(b"msg %d" % i).digest(), "big")
        r, s = signed_instance(d, e)
        out.append(vec(q, e, r, s, "valid"))
        out.append(vec(q, e ^ (1 << RNG.randrange(256)), r, s, "tampered_e"))
        out.append(vec(pubs[(i + 1) % 8], e, r, s, "wrong_key"))
        out.append(vec(q, e, r, o.N - s, "high_s_accept"))
        out.append(vec(q, e, r, s ^ (1 << RNG.randrange(250)), "tampered_s"))
    # range edges
    d, q = keys[0], pubs[0]
    e = int.from_bytes(hashlib.sha256(b"edge").digest(), "big")
    r, s = signed_instance(d, e)
    for rr, ss, lab in [(0, s, "r_zero"), (r, 0, "s_zero"), (o.N, s, "r_eq_N"),
                        (r, o.N, "s_eq_N"), (o.N + 1, s, "r_gt_N"), (r, o.N + 1, "s_gt_N"),
                        ((1 << 256) - 1, s, "r_max"), (r, (1 << 256) - 1, "s_max"),
                        (r + o.N if r + o.N < (1 << 256) else r, s, "r_plus_N"),
                        (1, 1, "r1_s1"), (o.N - 1, o.N - 1, "rN1_sN1")]:
        out.append(vec(q, e, rr, ss, lab))
    # e == 0 and e == N (u1 == 0), accept cases
    for e_raw, lab in [(0, "e_zero_u1_zero"), (o.N, "e_eq_N_u1_zero")]:
        k = rand_scalar()
        R = o.scalar_mult(k, o.G)
        r = R[0] % o.N
        s = rand_scalar()
        u2 = r * pow(s, -1, o.N) % o.N
        dd = k * pow(u2, -1, o.N) % o.N
        out.append(vec(o.pubkey(dd), e_raw, r, s, lab))
    # e >= N accept: sign e_small, present e_small + N
    for j in range(4):
        e_small = RNG.randrange(0, (1 << 256) - o.N)
        r, s = signed_instance(keys[j], e_small)
        out.append(vec(pubs[j], e_small + o.N, r, s, "e_ge_N_accept"))
    # R.x >= N accept: Q = u2^-1 (R - u1 G)
    cnt = 0
    x = o.N
    while cnt < 4:
        x += RNG.randrange(1, 1 << 100)
        if x >= o.P:
            x = o.N + RNG.randrange(1, 1 << 64)
        R = lift_x(x)
        if R is None:
            continue
        r = x - o.N
        s = rand_scalar()
        e = RNG.randrange(1 << 256)
        w = pow(s, -1, o.N)
        u1, u2 = e * w % o.N, r * w % o.N
        q = o.scalar_mult(pow(u2, -1, o.N), o.point_add(R, o.point_neg(o.scalar_mult(u1, o.G))))
        out.append(vec(q, e, r, s, "Rx_ge_N_accept"))
        # and the r = x (not reduced) variant, which Go rejects if x >= N
        out.append(vec(q, e, x if x < (1 << 256) else r, s, "Rx_ge_N_unreduced_r"))
        cnt += 1
    # final result at infinity: e == -r*d
    for j in range(4):
        d = keys[j]
        r = rand_scalar()
        s = rand_scalar()
        e = (-r * d) % o.N
        out.append(vec(pubs[j], e, r, s, "final_infinity"))
    # classic Straus collision u1*G == u2*Q (e == r*d)
    for j in range(4):
        d = keys[j]
        r, s = rand_scalar(), rand_scalar()
        out.append(vec(pubs[j], r * d % o.N, r, s, "u1G_eq_u2Q"))
    # Q = G, Q = -G
    for d, lab in [(1, "Q_eq_G"), (o.N - 1, "Q_eq_negG")]:
        e = RNG.randrange(1 << 256)
        r, s = signed_instance(d, e)
        out.append(vec(o.pubkey(d), e, r, s, lab))
        out.append(vec(o.pubkey(d), e ^ 1, r, s, lab + "_tampered"))
    # comb accumulator collisions, for both key-table windows (8 and 16 bits)
    for W in (8, 16):
        last = 256 // W - 1
        for i in sorted(set(list(range(0, last + 1, 3)) + [last])):
            for inf in ((False, True) if i < last else (False,)):
                q, e, r, s = comb_collision(i, inf, W)
                lab = ("comb%d_inf_w%d" if inf else "comb%d_dbl_w%d") % (W, i)
                out.append(vec(q, e, r, s, lab))
    return out


def make_comb_windows():
    """Comb-collision vectors for the large key windows (20..29 bits): for
    each window W, windows 0, a middle one and the last (partial) one, as a
    doubling and (except the last) an infinity collision.  Own RNG stream so
    that prehashed.json is unchanged."""
    rng = random.Random(0x57494E44)  # "WIND"
    out = []
    for W in (20, 22, 24, 26, 29):
        last = -(-256 // W) - 1
        for i in (0, last // 2, last):
            for inf in ((False, True) if i < last else (False,)):
                q, e, r, s = comb_collision(i, inf, W, rng)
                lab = ("comb%d_inf_w%d" if inf else "comb%d_dbl_w%d") % (W, i)
                out.append(vec(q, e, r, s, lab))
    return out


# ----------------------------------------------------------------------------
def make_der():
    good_r = int("EFD48B2AACB6A8FD1140DD9CD45E81D69D2C877B56AAF991C34D0EA84EAF3716", 16)
    good_s = int("19F4113742A2B14BD25926B49C649155F267E60D3814B4C0CC84250E46F0083", 16)
    g = o.der_encode_sig(good_r, good_s)
    cases = [
        g, g + b"\x00", g + b"\x01\x02\x03",  # trailing bytes
        b"", b"\x30", b"\x30\x00", b"\x30\x80" + g[2:], b"\x31" + g[1:], b"\x10" + g[1:],
        g[:-1], g[:10], b"\x30\x81" + bytes([len(g) - 2]) + g[2:],  # non-minimal long length
        b"\x30\x81\x80" + b"\x02\x01\x01" * 42 + b"\x02\x02\x01",  # long form ok but truncated
        b"\x30\x06\x02\x01\x01\x02\x01\x01",
        b"\x30\x06\x02\x01\x01\x02\x01\x01\xff",
        b"\x30\x07\x02\x01\x01\x02\x01\x01\x05",  # extra byte inside SEQUENCE: ignored
        b"\x30\x09\x02\x01\x01\x02\x01\x01\x05\x00\x00",
        b"\x30\x03\x02\x01\x01",  # missing S
        b"\x30\x05\x02\x00\x02\x01\x01",  # empty integer
        b"\x30\x07\x02\x02\x00\x01\x02\x01\x01",  # non-minimal integer (00 01)
        b"\x30\x07\x02\x02\x00\x80\x02\x01\x01",  # minimal (00 80)
        b"\x30\x07\x02\x02\xff\x80\x02\x01\x01",  # non-minimal negative (ff 80)
        b"\x30\x07\x02\x02\xff\x7f\x02\x01\x01",  # negative minimal
        b"\x30\x06\x02\x01\x80\x02\x01\x01",      # -128
        b"\x30\x06\x22\x01\x01\x02\x01\x01",      # constructed INTEGER
        b"\x30\x06\x42\x01\x01\x02\x01\x01",      # wrong class
        b"\x30\x06\x03\x01\x01\x02\x01\x01",      # wrong tag
        b"\x30\x06\x02\x01\x01\x02\x02\x01",      # S overruns SEQUENCE
        b"\x30\x06\x02\x05\x01\x02\x01\x01",      # R overruns
        b"\x3f\x10\x06\x02\x01\x01\x02\x01\x01",  # high tag number form
        b"\x3f\x81\x80\x00",                      # base128 tag
        b"\x30\x84\x00\x00\x00\x06\x02\x01\x01\x02\x01\x01",  # leading zero in length
        b"\x30\x82\x00\x80",
        b"\x30\x88\x7f\xff\xff\xff\xff\xff\xff\xff",  # length too large
        b"\x30\x06\x02\x81\x01\x01\x02\x01\x01",  # non-minimal INTEGER length
        b"\x30\x08\x02\x83\x00\x00\x01\x01\x02\x01\x01",
        b"\x30\x25\x02\x21\x00" + b"\xff" * 32 + b"\x02\x01\x01",  # 2^256-1
        b"\x30\x26\x02\x22\x01" + b"\x00" * 33 + b"\x02\x01\x01",  # > 2^256
        b"\x30\x06\x02\x01\x00\x02\x01\x00",
        b"\x30\x04\x02\x01\x01\x02",               # truncated S tag/len
        b"\x30\x05\x02\x01\x01\x02\x80",          # indefinite S length
    ]
    for _ in range(200):  # random mutations of a valid encoding
        b = bytearray(g)
        for _ in range(RNG.randrange(1, 4)):
            op = RNG.randrange(3)
            if op == 0 and b:
                b[RNG.randrange(len(b))] ^= 1 << RNG.randrange(8)
            elif op == 1 and b:
                del b[RNG.randrange(len(b))]
            else:
                b.insert(RNG.randrange(len(b) + 1), RNG.randrange(256))
        cases.append(bytes(b))
    out = []
    for c in cases:
        try:
            r, s, rest = o.der_parse_sig(c)
            out.append({"sig": c.hex(), "ok": 1, "r": hex(r), "s": hex(s), "rest": len(rest)})
        except o.Asn1Error as ex:
            out.append({"sig": c.hex(), "ok": 0, "err": str(ex)})
    return out


# ----------------------------------------------------------------------------
def make_authen():
    """Sequences of Authenticator calls.  Keys: replicas 0..3 (ECDSA and USIG
    keys), clients 10..11; replica 3's USIG key slot is deliberately absent."""
    rep = {i: key_from_seed(100 + i) for i in range(4)}
    usig = {i: key_from_seed(200 + i) for i in range(3)}
    cli = {10: key_from_seed(300), 11: key_from_seed(301)}
    ks = {
        o.ROLE_REPLICA: {i: o.pkix_encode(o.pubkey(d)).hex() for i, d in rep.items()},
        o.ROLE_USIG: {i: o.pkix_encode(o.pubkey(d)).hex() for i, d in usig.items()},
        o.ROLE_CLIENT: {i: o.pkix_encode(o.pubkey(d)).hex() for i, d in cli.items()},
    }
    calls = []

    def add(role, id_, msg, tag, note):
        calls.append({"role": role, "id": id_, "msg": msg.hex(), "tag": tag.hex(), "note": note})

    def sig_quirk(d, msg):
        r, s = o.ecdsa_sign(d, o.quirk_digest(msg))
        return o.der_encode_sig(r, s)

    op = bytes(range(256))
    for seq in range(1, 9):
        msg = o.authen_request(seq, op)
        tag = sig_quirk(cli[10], msg)
        add(o.ROLE_CLIENT, 10, msg, tag, "request_valid")
        t = bytearray(msg)
        t[5] ^= 1
        add(o.ROLE_CLIENT, 10, bytes(t), tag, "request_tamper_lt32")
        t = bytearray(msg)
        t[32 + seq] ^= 0x40
        add(o.ROLE_CLIENT, 10, bytes(t), tag, "request_tamper_ge32_accepted")
        add(o.ROLE_CLIENT, 11, msg, tag, "request_wrong_client")
        add(o.ROLE_CLIENT, 12, msg, tag, "request_unknown_client")
        add(o.ROLE_CLIENT, 12, msg, tag[:-2], "request_unknown_client_malformed")
        add(o.ROLE_CLIENT, 10, msg, tag[:-1], "request_truncated_der")
        add(o.ROLE_CLIENT, 10, msg, tag + b"\x00\x01", "request_trailing_ignored")
        r, s, _ = o.der_parse_sig(tag)
        add(o.ROLE_CLIENT, 10, msg, o.der_encode_sig(r, o.N - s), "request_high_s")
        add(7, 10, msg, tag, "unknown_role")
    # short messages (< 32 bytes): e = msg || SHA256("")[..]
    for m in [b"hello", b"", b"REQ-VIEW-CHANGE" + struct.pack(">Q", 5)]:
        add(o.ROLE_REPLICA, 1, m, sig_quirk(rep[1], m), "short_msg")
    # reply
    msg = o.authen_reply(10, 3, b"result")
    add(o.ROLE_REPLICA, 2, msg, sig_quirk(rep[2], msg), "reply")
    add(o.ROLE_REPLICA, 0, msg, sig_quirk(rep[2], msg), "reply_wrong_replica")

    # USIG stream: primary 0 PREPAREs, replicas 1,2 COMMITs
    epochs = {i: RNG.randrange(1 << 64) for i in usig}
    ctr = {i: 0 for i in usig}

    def ui(i, msg, epoch=None, counter=None):
        ctr[i] += 1
        c = ctr[i] if counter is None else counter
        return o.usig_create_ui(usig[i], msg, epochs[i] if epoch is None else epoch, c)

    # a UI with counter 2 before any capture: epoch defaults to 0 -> mismatch
    early = o.authen_prepare(0, 10, 99, op)
    add(o.ROLE_USIG, 0, early, o.usig_create_ui(usig[0], early, epochs[0], 2), "usig_no_epoch_yet")
    for seq in range(1, 7):
        prep = o.authen_prepare(0, 10, seq, op)
        tag = ui(0, prep)
        add(o.ROLE_USIG, 0, prep, tag, "prepare_valid")
        add(o.ROLE_USIG, 0, prep, tag, "prepare_replay_same_ui")
        pc = ctr[0]
        for rid in (1, 2):
            com = o.authen_commit(0, 0, 10, seq, op, pc)
            t = ui(rid, com)
            add(o.ROLE_USIG, rid, com, t, "commit_valid")
            bad = bytearray(com)
            bad[-1] ^= 1
            add(o.ROLE_USIG, rid, bytes(bad), t, "commit_tampered")
    # wrong epoch (a second USIG instance with same key), short tag/cert, etc.
    prep = o.authen_prepare(0, 10, 50, op)
    add(o.ROLE_USIG, 0, prep, o.usig_create_ui(usig[0], prep, epochs[0] ^ 1, 7), "epoch_mismatch")
    add(o.ROLE_USIG, 0, prep, b"\x00\x00\x00", "bad_ui_short")
    add(o.ROLE_USIG, 0, prep, struct.pack(">Q", 7) + b"\x01\x02", "bad_cert_short")
    t = o.usig_create_ui(usig[0], prep, epochs[0], 7)
    add(o.ROLE_USIG, 0, prep, t + b"\x00", "der_trailing")
    add(o.ROLE_USIG, 0, prep, t[:-3], "der_truncated")
    add(o.ROLE_USIG, 3, prep, t, "usig_unknown_replica")
    add(o.ROLE_USIG, 1, prep, t, "usig_wrong_replica")
    # replica 2 never captured? (it did above) -- fresh replica scenario
    # captured with counter 1 but failing signature must NOT store the epoch
    return {"keystore": {str(k): {str(i): v for i, v in m.items()} for k, m in ks.items()},
            "sequences": [calls]}


def expected_authen(fx):
    ks = o.KeyStore()
    for role, m in fx["keystore"].items():
        ks.keys[int(role)] = {int(i): o.pkix_decode(bytes.fromhex(v)) for i, v in m.items()}
    for seq in fx["sequences"]:
        a = o.Authenticator(ks)
        for c in seq:
            c["expect"] = a.verify(c["role"], c["id"], bytes.fromhex(c["msg"]), bytes.fromhex(c["tag"]))


def make_usig_epoch_edge():
    """Fresh-authenticator sequences exercising epoch capture rules
    (crypto.go:219-236)."""
    d = key_from_seed(400)
    q = o.pubkey(d)
    m = o.authen_prepare(1, 10, 1, b"op")
    seqs = []
    e1 = 0x1122334455667788
    # 1: counter-1 UI with a bad signature: epoch captured for the check but
    #    not stored; a later valid counter-2 UI (epoch e1) then mismatches (epoch 0)
    bad = o.usig_create_ui(d, m + b"x", e1, 1)
    s1 = [(m, bad), (m, o.usig_create_ui(d, m, e1, 2)), (m, o.usig_create_ui(d, m, e1, 1)),
          (m, o.usig_create_ui(d, m, e1, 2))]
    # 2: cert epoch 0 with counter != 1 is accepted when nothing captured
    s2 = [(m, o.usig_create_ui(d, m, 0, 5)), (m, o.usig_create_ui(d, m, 0, 6)),
          (m, o.usig_create_ui(d, m, e1, 1))]
    for s in (s1, s2):
        seqs.append([{"role": o.ROLE_USIG, "id": 0, "msg": mm.hex(), "tag": tt.hex(),
                      "note": "epoch_edge"} for mm, tt in s])
    return {"keystore": {str(o.ROLE_USIG): {"0": o.pkix_encode(q).hex()}}, "sequences": seqs}


def make_messages():
    """MinBFT message streams (n = 4, f = 1) for the batched validators:
    a backup's view of REQUESTs, PREPAREs (primary 0) and COMMITs (replicas
    1..3) and adversarial cases for every validator branch; plus the client
    side: REPLY sequences for client/message-handling.go:140-170.  Each
    sequence runs on a fresh authenticator."""
    n = 4
    rep = {i: key_from_seed(500 + i) for i in range(n)}
    usig = {i: key_from_seed(600 + i) for i in range(n)}
    cli = {10: key_from_seed(700), 11: key_from_seed(701)}
    ks = {
        o.ROLE_REPLICA: {i: o.pkix_encode(o.pubkey(d)).hex() for i, d in rep.items()},
        o.ROLE_USIG: {i: o.pkix_encode(o.pubkey(d)).hex() for i, d in usig.items()},
        o.ROLE_CLIENT: {i: o.pkix_encode(o.pubkey(d)).hex() for i, d in cli.items()},
    }
    epochs = {i: RNG.randrange(1 << 64) for i in usig}

    def csig(cid, m):
        r, s_ = o.ecdsa_sign(cli[cid], o.quirk_digest(o.msg_authen_bytes(m, o.MSG_REQUEST)))
        return o.der_encode_sig(r, s_)

    def ui(rid, ab, ctr, epoch=None):
        tag = o.usig_create_ui(usig[rid], ab, epochs[rid] if epoch is None else epoch, ctr)
        return tag[8:]  # cert

    def enc(m):
        d = dict(m.__dict__)
        for k in ("op", "sig", "ui_cert", "prep_ui_cert"):
            d[k] = d[k].hex()
        return d

    def stream_normal(nreq, tamper=None):
        msgs = []
        ctr = {i: 0 for i in range(n)}
        for k in range(nreq):
            cid = 10 + (k % 2)
            op = RNG.randbytes(64 + k)
            rq = o.Msg(type=o.MSG_REQUEST, stream=100 + cid, client_id=cid, seq=k + 1, op=op)
            rq.sig = csig(cid, rq)
            msgs.append(rq)
            ctr[0] += 1
            pr = o.Msg(type=o.MSG_PREPARE, stream=0, replica_id=0, view=0, client_id=cid, seq=k + 1,
                       op=op, sig=rq.sig, ui_counter=ctr[0])
            pr.ui_cert = ui(0, o.msg_authen_bytes(pr), ctr[0])
            msgs.append(pr)
            for rid in (1, 2, 3):
                ctr[rid] += 1
                cm = o.Msg(type=o.MSG_COMMIT, stream=rid, replica_id=rid, prep_replica_id=0, view=0,
                           client_id=cid, seq=k + 1, op=op, sig=rq.sig, prep_ui_counter=pr.ui_counter,
                           prep_ui_cert=pr.ui_cert, ui_counter=ctr[rid])
                cm.ui_cert = ui(rid, o.msg_authen_bytes(cm), ctr[rid])
                msgs.append(cm)
        return msgs

    def reply(rid, cid, k, signer=None):
        rp = o.Msg(type=o.MSG_REPLY, stream=200 + rid, replica_id=rid, client_id=cid,
                   seq=k + 1, op=b"result-%d" % k)
        r_, s_ = o.ecdsa_sign(rep[rid if signer is None else signer],
                              o.quirk_digest(o.msg_authen_bytes(rp)))
        rp.sig = o.der_encode_sig(r_, s_)
        return rp

    seqs = []
    base = stream_normal(6)
    seqs.append({"n": n, "flags": 0, "msgs": base})
    # adversarial variants of the same traffic
    adv = stream_normal(6)
    import copy
    extra = []
    p0 = next(m for m in adv if m.type == o.MSG_PREPARE)
    bad = copy.copy(p0); bad.replica_id = 1; bad.stream = 1            # PREPARE from a backup
    extra.append(bad)
    c0 = next(m for m in adv if m.type == o.MSG_COMMIT)
    bad = copy.copy(c0); bad.replica_id = 0; bad.stream = 50           # COMMIT from the primary
    extra.append(bad)
    bad = copy.copy(c0); bad.op = c0.op + b"x"; bad.stream = 51        # embedded request tampered
    extra.append(bad)
    bad = copy.copy(c0); bad.ui_counter = 0; bad.stream = 52           # zero counter
    extra.append(bad)
    bad = copy.copy(c0); bad.prep_ui_counter = 0; bad.stream = 53      # zero prepare counter
    extra.append(bad)
    bad = copy.copy(c0); bad.prep_ui_cert = c0.ui_cert; bad.stream = 54  # wrong prepare UI
    extra.append(bad)
    bad = copy.copy(p0); bad.view = 4; bad.stream = 55                 # view 4: primary 0 (4 mod 4)
    extra.append(bad)
    bad = copy.copy(p0); bad.view = 1; bad.stream = 56                 # primary of view 1 is 1
    extra.append(bad)
    extra.append(o.Msg(type=o.MSG_REQ_VIEW_CHANGE, stream=57, view=1))
    # the same stream continues after a reject: stopped
    bad2 = copy.copy(c0); bad2.stream = 51
    extra.append(bad2)
    seqs.append({"n": n, "flags": 0, "msgs": adv + extra})
    seqs.append({"n": n, "flags": 1, "msgs": adv + extra})             # no stream stop
    # malformed DER in an ECDSA role: Go panics -> everything after stops
    pan = stream_normal(2)
    bad = copy.copy(pan[0]); bad.sig = pan[0].sig[:-3]; bad.stream = 60
    seqs.append({"n": n, "flags": 0, "msgs": pan[:3] + [bad] + pan[3:]})
    seqs.append({"n": n, "flags": 2, "msgs": pan[:3] + [bad] + pan[3:]})
    # a REPLY on a replica's peer stream: the message validator panics
    # ("Unknown message type", core/message-handling.go:420-421)
    seqs.append({"n": n, "flags": 0, "msgs": pan[:2] + [reply(1, 10, 0)] + pan[2:]})
    seqs.append({"n": n, "flags": 2, "msgs": pan[:2] + [reply(1, 10, 0)] + pan[2:]})

    # client side (client 10): REPLY checks, no stream stop
    rps = [reply(rid, 10, k) for k in range(3) for rid in range(n)]
    rbad = []
    b = copy.copy(rps[0]); b.client_id = 11; rbad.append(b)            # ClientID mismatch
    rbad.append(reply(3, 10, 5, signer=1))                              # signed by another replica
    b = copy.copy(rps[1]); b.op = b"forged"; rbad.append(b)            # result tampered
    b = copy.copy(rps[2]); b.replica_id = 9; rbad.append(b)            # unknown replica id
    b = copy.copy(rps[3]); b.seq += 1 << 40; rbad.append(b)            # seq tampered (offset < 32)
    rseq = rps[:4] + rbad + rps[4:]
    pan_r = copy.copy(rps[5]); pan_r.sig = rps[5].sig[:10]               # malformed DER: panic
    replies = [{"client_id": 10, "flags": 0, "msgs": rseq},
               {"client_id": 10, "flags": 0, "msgs": rps[:5] + [pan_r] + rps[5:]},
               {"client_id": 10, "flags": 2, "msgs": rps[:5] + [pan_r] + rps[5:]},
               {"client_id": 11, "flags": 0, "msgs": rps[:4]}]
    out = {"keystore": {str(k): {str(i): v for i, v in m.items()} for k, m in ks.items()},
           "sequences": [], "replies": []}
    kst = o.KeyStore()
    for role, m in out["keystore"].items():
        kst.keys[int(role)] = {int(i): o.pkix_decode(bytes.fromhex(v)) for i, v in m.items()}
    for sq in seqs:
        a = o.Authenticator(kst)
        exp = o.validate_messages(a, sq["msgs"], sq["n"], sq["flags"])
        out["sequences"].append({"n": sq["n"], "flags": sq["flags"],
                                 "msgs": [enc(m) for m in sq["msgs"]], "expect": exp})
    for sq in replies:
        a = o.Authenticator(kst)
        exp = o.validate_replies(a, sq["msgs"], sq["client_id"], sq["flags"])
        out["replies"].append({"client_id": sq["client_id"], "flags": sq["flags"],
                               "msgs": [enc(m) for m in sq["msgs"]], "expect": exp})
    return out


def main():
    def dump(name, obj):
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(obj, f, indent=0, sort_keys=True)
            f.write("\n")

    dump("kat.json", make_kat())
    dump("prehashed.json", make_prehashed())
    dump("comb_windows.json", make_comb_windows())
    dump("der.json", make_der())
    a = make_authen()
    expected_authen(a)
    dump("authen.json", a)
    b = make_usig_epoch_edge()
    expected_authen(b)
    dump("usig_epoch.json", b)
    dump("messages.json", make_messages())


if __name__ == "__main__":
    main()

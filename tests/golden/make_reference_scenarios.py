#!/usr/bin/env python3
"""Generate tests/golden/reference_scenarios.json: the reference's OWN test
scenarios for the authentication path, restated as call sequences with the
reference's fixture key pair and the reference tests' literal inputs.

Run from the repo root:  python tests/golden/make_reference_scenarios.py

The reference holds no ECDSA known-answer vectors;
what it does hold is this key pair and these scenarios.  Each scenario below
cites the reference test it restates and keeps that test's inputs and
expected outcome (NoError -> ACCEPT, Error -> the reject kind the oracle's
restatement gives):

  ecdsa_sig_cipher      sample/authentication/crypto_test.go:49-58
  ecdsa_authen_scheme   sample/authentication/crypto_test.go:60-68
  usig_second_instance  sample/authentication/crypto_test.go:70-98
  sgx_usig_wrong_msg    usig/sgx/sgx-usig_test.go:30-83
  ui_marshal            usig/usig_test.go:31-45
  ui_verifier           core/usig-ui_test.go:39-82 (through the PREPARE validator)
  authenticator_roles   sample/authentication/authenticator_test.go:29-69
  keystore_lookup       sample/authentication/keymanager_test.go:86-113

Keys: the fixture pair of keymanager_test.go:68-69 (also the public key of
every replica, client and USIG entry in keymanager_test.go:51-83).  The
reference signs with crypto/rand (crypto.go:69) and its USIG signs inside
SGX with a random epoch (usig.c:168-197); here the signer is RFC 6979 and
the epochs are fixed constants -- verification does not depend on either.
Only the data (inputs, tags, expected statuses) is committed; the generating
logic is this script plus oracle/p256.py.
"""
from __future__ import annotations

import base64
import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import p256 as o  # noqa: E402

# sample/authentication/keymanager_test.go:68-69
PK_B64 = ("MFkwEwYHKoZIzj0CAQYIKoZIzj0DAQcDQgAEh6uiVdr+3EgyT3YEilvrvzQINr8eolxR22/0JudQrpGbLQQQIK+7"
          "RdnoLaIyZIlakZkb1tAws0iQN263EkwzGw==")
SK_B64 = ("MHcCAQEEIFxopskcl2LyZ/LLsDMBfQk/82WZQI/YhvXNSYZNmUSFoAoGCCqGSM49AwEHoUQDQgAEh6uiVdr+3Egy"
          "T3YEilvrvzQINr8eolxR22/0JudQrpGbLQQQIK+7RdnoLaIyZIlakZkb1tAws0iQN263EkwzGw==")

EPOCH1 = 0x0123456789ABCDEF   # "usig1" enclave epoch (random in the reference)
EPOCH2 = 0x0FEDCBA987654321   # "usig2": same sealed key, fresh epoch


def fixture_key():
    pkix = base64.b64decode(PK_B64)
    sec1 = base64.b64decode(SK_B64)
    # SEC1 ECPrivateKey: 30 77 02 01 01 04 20 <d (32 B)> ...
    assert sec1[:7] == bytes.fromhex("30770201010420")
    d = int.from_bytes(sec1[7:39], "big")
    q = o.pkix_decode(pkix)
    assert o.pubkey(d) == q
    return d, q, pkix


def ecdsa_tag(d: int, msg: bytes) -> bytes:
    """PublicAuthenScheme.GenerateAuthenticationTag (crypto.go:113-116)."""
    r, s = o.ecdsa_sign(d, o.quirk_digest(msg))
    return o.der_encode_sig(r, s)


def call(role, id_, msg, tag, note, ref):
    return {"role": role, "id": id_, "msg": msg.hex(), "tag": tag.hex(), "note": note, "ref": ref}


def main():
    d, q, pkix = fixture_key()
    hello = b"hello"                      # crypto_test.go:34
    usig_msg, wrong = b"Test message", b"Another message"   # sgx-usig_test.go:31-32
    # every role of the example key stores maps ids 0..2 (replica), 10
    # (client) and the USIG keys to the fixture public key
    keystore = {str(o.ROLE_REPLICA): {"0": pkix.hex(), "1": pkix.hex(), "2": pkix.hex()},
                str(o.ROLE_CLIENT): {"10": pkix.hex()},
                str(o.ROLE_USIG): {"0": pkix.hex(), "1": pkix.hex(), "2": pkix.hex()}}
    sc = {}

    # crypto_test.go:49-58: md = SHA256.New().Sum(msg); Sign; Verify(md, sig)
    md = o.quirk_digest(hello)
    r, s = o.ecdsa_sign(d, md)
    sc["ecdsa_sig_cipher"] = {
        "ref": "sample/authentication/crypto_test.go:49-58",
        "prehashed": [{"e": md[:32].hex(), "r": r.to_bytes(32, "big").hex(),
                       "s": s.to_bytes(32, "big").hex(), "note": "Sign(md) then Verify(md)"}]}

    # crypto_test.go:60-68: scheme round trip (GenerateAuthenticationTag ->
    # VerifyAuthenticationTag), here through the Authenticator boundary
    tag = ecdsa_tag(d, hello)
    sc["ecdsa_authen_scheme"] = {
        "ref": "sample/authentication/crypto_test.go:60-68",
        "calls": [call(o.ROLE_REPLICA, 0, hello, tag, "scheme round trip", "crypto_test.go:64-67"),
                  call(o.ROLE_CLIENT, 10, hello, tag, "same tag, client role", "crypto_test.go:64-67")]}

    # crypto_test.go:70-98: usig1 (epoch 1) tag verifies; usig2 = same sealed
    # key, new epoch: its first UI is rejected by scheme 1 (epoch captured)
    t1 = o.usig_create_ui(d, hello, EPOCH1, 1)
    t2 = o.usig_create_ui(d, hello, EPOCH2, 1)
    sc["usig_second_instance"] = {
        "ref": "sample/authentication/crypto_test.go:70-98",
        "calls": [call(o.ROLE_USIG, 0, hello, t1, "usig1 tag1", "crypto_test.go:79-80"),
                  call(o.ROLE_USIG, 0, hello, t2, "usig2 tag2 on scheme1", "crypto_test.go:96-97")]}

    # sgx-usig_test.go:30-83: UIs counter 1, 2 of one instance; ui2 verifies
    # for msg, not for wrongMsg
    u1 = o.usig_create_ui(d, usig_msg, EPOCH1, 1)
    u2 = o.usig_create_ui(d, usig_msg, EPOCH1, 2)
    sc["sgx_usig_wrong_msg"] = {
        "ref": "usig/sgx/sgx-usig_test.go:30-83",
        "calls": [call(o.ROLE_USIG, 1, usig_msg, u1, "ui counter 1", "sgx-usig_test.go:61-65"),
                  call(o.ROLE_USIG, 1, usig_msg, u2, "VerifyUI(msg, ui2)", "sgx-usig_test.go:75-76"),
                  call(o.ROLE_USIG, 1, wrong, u2, "VerifyUI(wrongMsg, ui2)", "sgx-usig_test.go:78-82")]}

    # usig/usig_test.go:31-45: UI{Counter, Cert: 1 random byte} marshals to
    # counter_be64 || cert and back.  Through the authenticator that UI
    # parses (usig.go:75-80) and then fails ParseCert (cert < 8 B); a 7-byte
    # tag fails the UI unmarshal itself.
    ctr = 0x8BADF00D12345678
    ui_bytes = o.ui_marshal(ctr, b"\x5a")
    assert ui_bytes == struct.pack(">Q", ctr) + b"\x5a"
    sc["ui_marshal"] = {
        "ref": "usig/usig_test.go:31-45",
        "ui": {"counter": ctr, "cert": "5a", "bytes": ui_bytes.hex()},
        "calls": [call(o.ROLE_USIG, 2, hello, ui_bytes, "UI with 1-byte cert", "usig.go:75-86"),
                  call(o.ROLE_USIG, 2, hello, ui_bytes[:7], "7-byte UI", "usig.go:75-80")]}

    # core/usig-ui_test.go:39-82 through makePrepareValidator (primary 0,
    # view 0, n = 3): correct UI; failed USIG certificate; zero counter
    op = b"reference scenario op"
    req_tag = ecdsa_tag(d, o.authen_request(1, op))
    ab_prep = o.authen_prepare(0, 10, 1, op)
    good = o.usig_create_ui(d, ab_prep, EPOCH1, 1)
    bad = bytearray(good)
    bad[-1] ^= 0x01
    msgs = []
    for stream, (ctr_, cert) in enumerate([(1, good[8:]), (1, bytes(bad[8:])), (0, good[8:])]):
        msgs.append({"type": o.MSG_PREPARE, "stream": stream, "replica_id": 0, "prep_replica_id": 0,
                     "view": 0, "client_id": 10, "seq": 1, "op": op.hex(), "sig": req_tag.hex(),
                     "ui_counter": ctr_, "ui_cert": cert.hex(), "prep_ui_counter": 0,
                     "prep_ui_cert": ""})
    sc["ui_verifier"] = {"ref": "core/usig-ui_test.go:39-82", "n": 3, "flags": 0,
                         "notes": ["Correct UI", "Failed USIG certificate verification",
                                   "Invalid (zero) counter value"],
                         "msgs": msgs}

    # authenticator_test.go:29-69: a0 generates, a1 verifies, per role
    sc["authenticator_roles"] = {
        "ref": "sample/authentication/authenticator_test.go:29-69",
        "calls": [call(o.ROLE_REPLICA, 0, hello, ecdsa_tag(d, hello), "ReplicaAuthen a0 -> a1",
                       "authenticator_test.go:40-44"),
                  call(o.ROLE_USIG, 0, hello, o.usig_create_ui(d, hello, EPOCH2, 1),
                       "USIGAuthen a0 -> a1", "authenticator_test.go:46-50"),
                  call(o.ROLE_CLIENT, 10, hello, ecdsa_tag(d, hello), "ClientAuthen a0 -> a1",
                       "authenticator_test.go:64-68")]}

    # keymanager_test.go:86-113 testLoadSimpleKeyStore cases: (role, id) found?
    sc["keystore_lookup"] = {
        "ref": "sample/authentication/keymanager_test.go:86-113",
        "cases": [[o.ROLE_REPLICA, 0, True], [o.ROLE_REPLICA, 1, True], [o.ROLE_REPLICA, 2, True],
                  [o.ROLE_CLIENT, 10, True], [0xFFFFFFFF, 0, False], [o.ROLE_REPLICA, 4, False]]}

    # expected outcomes from the oracle's restatement (each scenario starts
    # from a fresh authenticator: fresh epoch map)
    ks = o.KeyStore(keys={int(r): {int(i): q for i in m} for r, m in keystore.items()})
    for name, s_ in sc.items():
        if "calls" in s_:
            auth = o.Authenticator(ks)
            for c in s_["calls"]:
                c["expect"] = auth.verify(c["role"], c["id"], bytes.fromhex(c["msg"]),
                                          bytes.fromhex(c["tag"]))
        if "prehashed" in s_:
            for v in s_["prehashed"]:
                ok = o.go_ecdsa_verify(q, bytes.fromhex(v["e"]), int(v["r"], 16), int(v["s"], 16))
                v["expect"] = o.ACCEPT if ok else o.REJECT_SIG
        if "msgs" in s_:
            auth = o.Authenticator(ks)
            ms = []
            for m in s_["msgs"]:
                m2 = dict(m)
                for k in ("op", "sig", "ui_cert", "prep_ui_cert"):
                    m2[k] = bytes.fromhex(m2[k])
                ms.append(o.Msg(**m2))
            s_["expect"] = o.validate_messages(auth, ms, s_["n"], s_["flags"])
    out = {"key": {"d": d.to_bytes(32, "big").hex(), "pkix": pkix.hex(),
                   "source": "sample/authentication/keymanager_test.go:68-69"},
           "keystore": keystore, "scenarios": sc}
    with open(os.path.join(HERE, "reference_scenarios.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    main()

"""Pins the oracle (CPU only): RFC 6979 known answers, the reference's own
fixture key pair, OpenSSL cross-checks, the committed golden fixtures, and
agreement of the C restatement with the Python restatement."""
import base64
import hashlib
import random

import numpy as np
import pytest

from golden_util import load
from oracle import p256 as o


def test_rfc6979_known_answers():
    kat = load("kat.json")["rfc6979_p256_sha256"]
    d = int(kat["d"], 16)
    q = o.pubkey(d)
    assert q == (int(kat["ux"], 16), int(kat["uy"], 16))
    for v in kat["vectors"]:
        h = hashlib.sha256(v["msg"].encode()).digest()
        assert o.rfc6979_k(d, h) == int(v["k"], 16)
        r, s = o.ecdsa_sign(d, h)
        assert (r, s) == (int(v["r"], 16), int(v["s"], 16))
        assert o.go_ecdsa_verify(q, h, r, s)
        assert not o.go_ecdsa_verify(q, h, r, (s + 1) % o.N)


def test_reference_fixture_key_pair():
    """sample/authentication/keymanager_test.go:68-69: d*G == stored key."""
    k = load("kat.json")["reference_fixture_key"]
    sk = base64.b64decode(k["sec1_private_b64"])
    pk = base64.b64decode(k["pkix_public_b64"])
    assert sk[:7] == bytes.fromhex("30770201010420")
    d = int.from_bytes(sk[7:39], "big")
    assert o.pubkey(d) == o.pkix_decode(pk)
    assert o.pkix_encode(o.pkix_decode(pk)) == pk


def test_quirk_digest_constant():
    assert o.SHA256_EMPTY.hex() == load("kat.json")["sha256_empty"]
    e = o.quirk_digest(o.authen_request(1, bytes(range(256))))[:32]
    # SURVEY.md §0 finding 1 (verified independently there)
    assert e.hex() == "52455155455354000000000000000140aff2e9d2d8922e47afd4648e69674971"


PREHASHED = ["prehashed.json", "comb_windows.json"]


@pytest.mark.parametrize("name", PREHASHED)
def test_prehashed_golden_consistent(name):
    for v in load(name):
        q = (int(v["qx"], 16), int(v["qy"], 16))
        got = o.go_ecdsa_verify(q, bytes.fromhex(v["e"]), int(v["r"], 16), int(v["s"], 16))
        assert int(got) == v["expect"], v["label"]


@pytest.mark.parametrize("name", PREHASHED)
def test_prehashed_golden_vs_openssl(name):
    from oracle import openssl_xcheck as x
    if x.load() is None:
        pytest.skip("libcrypto not available")
    for v in load(name):
        got = x.verify(int(v["qx"], 16), int(v["qy"], 16), bytes.fromhex(v["e"]),
                       int(v["r"], 16), int(v["s"], 16))
        assert got is not None
        assert int(got) == v["expect"], v["label"]


def test_random_vs_openssl():
    from oracle import openssl_xcheck as x
    if x.load() is None:
        pytest.skip("libcrypto not available")
    rng = random.Random(5)
    for i in range(40):
        d = rng.randrange(1, o.N)
        q = o.pubkey(d)
        h = rng.randbytes(32)
        r, s = o.ecdsa_sign(d, h)
        for rr, ss in [(r, s), (r, o.N - s), (r ^ 1, s), (rng.randrange(1, o.N), s)]:
            assert x.verify(q[0], q[1], h, rr, ss) == o.go_ecdsa_verify(q, h, rr, ss)


def test_der_golden_consistent():
    for v in load("der.json"):
        sig = bytes.fromhex(v["sig"])
        try:
            r, s, rest = o.der_parse_sig(sig)
            assert v["ok"] == 1 and int(v["r"], 16) == r and int(v["s"], 16) == s and v["rest"] == len(rest)
        except o.Asn1Error:
            assert v["ok"] == 0


def test_authen_golden_replay():
    for name in ("authen.json", "usig_epoch.json"):
        fx = load(name)
        ks = o.KeyStore()
        for role, m in fx["keystore"].items():
            ks.keys[int(role)] = {int(i): o.pkix_decode(bytes.fromhex(p)) for i, p in m.items()}
        for seq in fx["sequences"]:
            a = o.Authenticator(ks)
            for c in seq:
                got = a.verify(c["role"], c["id"], bytes.fromhex(c["msg"]), bytes.fromhex(c["tag"]))
                assert got == c["expect"], c["note"]


def test_usig_epoch_rules():
    """crypto.go:219-236: failed first UI does not capture; epoch 0 accepted
    with counter != 1 when nothing is captured."""
    seqs = load("usig_epoch.json")["sequences"]
    assert [c["expect"] for c in seqs[0]] == [o.REJECT_SIG, o.EPOCH_MISMATCH, o.ACCEPT, o.ACCEPT]
    assert [c["expect"] for c in seqs[1]] == [o.ACCEPT, o.ACCEPT, o.EPOCH_MISMATCH]


# ------------------------------------------------------------- C oracle
@pytest.fixture(scope="module")
def coracle():
    from oracle import c_oracle
    c_oracle.build()
    return c_oracle


@pytest.mark.parametrize("name", PREHASHED)
def test_c_oracle_prehashed_golden(coracle, name):
    for v in load(name):
        got = coracle.verify(bytes.fromhex(v["qx"] + v["qy"]), bytes.fromhex(v["e"]),
                             bytes.fromhex(v["r"]), bytes.fromhex(v["s"]))
        assert int(got == 1) == v["expect"], v["label"]


def test_c_oracle_der_golden(coracle):
    for v in load("der.json"):
        got = coracle.der_parse(bytes.fromhex(v["sig"]))
        assert (got is not None) == (v["ok"] == 1), v
        if got is not None:
            r = int(v["r"], 16)
            s = int(v["s"], 16)
            clip = lambda x: x if 0 < x < (1 << 256) else 0  # noqa: E731
            assert int.from_bytes(got[0], "big") == clip(r)
            assert int.from_bytes(got[1], "big") == clip(s)
            assert got[2] == v["rest"]


def test_c_oracle_sha256(coracle):
    rng = random.Random(1)
    for n in [0, 1, 55, 56, 63, 64, 65, 119, 120, 200, 256, 1000]:
        m = rng.randbytes(n)
        assert coracle.sha256(m) == hashlib.sha256(m).digest()


def test_c_oracle_batch_threads(coracle):
    v = load("prehashed.json")
    qxy = np.array([list(bytes.fromhex(x["qx"] + x["qy"])) for x in v], dtype=np.uint8)
    arr = lambda k: np.array([list(bytes.fromhex(x[k])) for x in v], dtype=np.uint8)  # noqa: E731
    out = coracle.verify_prehashed_batch(qxy, arr("e"), arr("r"), arr("s"),
                                         np.arange(len(v), dtype=np.uint32), nthreads=4)
    assert [int(x == 0) for x in out] == [x["expect"] for x in v]


def test_message_streams_golden_replay():
    """The committed validator expectations (tests/golden/messages.json)
    replay from the oracle's sequential restatement: replica-side
    validate_messages and client-side validate_replies."""
    import copy
    fx = load("messages.json")
    ks = o.KeyStore()
    for role, m in fx["keystore"].items():
        ks.keys[int(role)] = {int(i): o.pkix_decode(bytes.fromhex(v)) for i, v in m.items()}

    def msgs(ds):
        out = []
        for d in ds:
            d = dict(d)
            for k in ("op", "sig", "ui_cert", "prep_ui_cert"):
                d[k] = bytes.fromhex(d[k])
            out.append(o.Msg(**d))
        return out
    for sq in fx["sequences"][-2:]:
        assert o.validate_messages(o.Authenticator(copy.deepcopy(ks)), msgs(sq["msgs"]), sq["n"],
                                   sq["flags"]) == sq["expect"]
    for sq in fx["replies"]:
        assert o.validate_replies(o.Authenticator(copy.deepcopy(ks)), msgs(sq["msgs"]),
                                  sq["client_id"], sq["flags"]) == sq["expect"]


def test_openssl_baseline_agrees_with_c_oracle(coracle):
    """The OpenSSL CPU baseline (oracle/c/openssl_baseline.c, bench.py's
    second cpu_baseline line) makes the same ECDSA-role decisions as the C
    oracle on the golden Authenticator calls of the ECDSA roles (valid,
    quirk-mode tampers, wrong key, malformed DER is status 2 in both)."""
    fx = load("authen.json")
    keys = {}
    msgs, tags, slots = [], [], []
    for seq in fx["sequences"]:
        for c in seq:
            if c["role"] not in (1, 3):
                continue
            pk = fx["keystore"].get(str(c["role"]), {}).get(str(c["id"]))
            if pk is None:
                continue
            xy = bytes.fromhex(pk)[27:]
            slots.append(keys.setdefault(xy, len(keys)))
            msgs.append(bytes.fromhex(c["msg"]))
            tags.append(bytes.fromhex(c["tag"]))
    assert len(msgs) > 20
    qxy = np.frombuffer(b"".join(sorted(keys, key=keys.get)), dtype=np.uint8).reshape(-1, 64)
    slot = np.array(slots, dtype=np.uint32)
    a = coracle.verify_ecdsa_role_batch(qxy, slot, msgs, tags, nthreads=2)
    b = coracle.ossl_verify_ecdsa_role_batch(qxy, slot, msgs, tags, nthreads=2)
    assert (a == b).all(), list(zip(a, b))
    assert (a == 0).any() and (a == 1).any()

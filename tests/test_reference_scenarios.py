"""The reference's own test scenarios for the authentication path, with the
reference's fixture key pair (sample/authentication/keymanager_test.go:68-69),
replayed (a) through the oracle on the CPU and (b) through the HIP library's
C-ABI on the GPU.  Fixture: tests/golden/reference_scenarios.json, made by
tests/golden/make_reference_scenarios.py (each scenario cites the reference
test it restates: crypto_test.go:49-98, sgx-usig_test.go:30-83,
usig_test.go:31-45, core/usig-ui_test.go:39-82, authenticator_test.go:29-69,
keymanager_test.go:86-113).

These are the only pinning material the reference holds for this path: the
expected outcome of every scenario is the reference test's own assertion
(NoError -> ACCEPT, Error -> reject), with the reject KIND from the oracle."""
import struct

import numpy as np
import pytest

from golden_util import load

FX = load("reference_scenarios.json")
SC = FX["scenarios"]
# the reference assertions, independent of the oracle: 0 = NoError, else Error
REF_NOERROR = {
    "ecdsa_sig_cipher": [True],                   # crypto_test.go:56-57 assert.True(ok)
    "ecdsa_authen_scheme": [True, True],          # crypto_test.go:66-67 NoError
    "usig_second_instance": [True, False],        # crypto_test.go:80, 97
    "sgx_usig_wrong_msg": [True, True, False],    # sgx-usig_test.go:75-82
    "ui_marshal": [False, False],                 # 1-byte cert / short UI: errors
    "ui_verifier": [True, False, False],          # usig-ui_test.go:63, 72, 77
    "authenticator_roles": [True, True, True],    # authenticator_test.go:44, 50, 68
}


def _msgs(sc):
    from oracle import p256 as o
    out = []
    for m in sc["msgs"]:
        m = dict(m)
        for k in ("op", "sig", "ui_cert", "prep_ui_cert"):
            m[k] = bytes.fromhex(m[k])
        out.append(o.Msg(**m))
    return out


def _expects(name):
    sc = SC[name]
    if "calls" in sc:
        return [c["expect"] for c in sc["calls"]]
    if "prehashed" in sc:
        return [v["expect"] for v in sc["prehashed"]]
    return sc["expect"]


# ----------------------------------------------------------------- CPU
def test_fixture_key_is_the_reference_pair():
    """d decodes from the SEC1 private key and d*G is the PKIX public key."""
    from oracle import p256 as o
    d = int(FX["key"]["d"], 16)
    assert o.pubkey(d) == o.pkix_decode(bytes.fromhex(FX["key"]["pkix"]))


@pytest.mark.parametrize("name", sorted(REF_NOERROR))
def test_expectations_match_reference_assertions(name):
    """The fixture's expected statuses agree with the reference test's own
    NoError/Error assertions."""
    got = [e == 0 for e in _expects(name)]
    assert got == REF_NOERROR[name]


def test_oracle_replays_scenarios():
    """The oracle restatement, replayed from the fixture inputs, reproduces
    every expected status (fresh authenticator per scenario)."""
    from oracle import p256 as o
    q = o.pkix_decode(bytes.fromhex(FX["key"]["pkix"]))
    ks = o.KeyStore(keys={int(r): {int(i): q for i in m} for r, m in FX["keystore"].items()})
    for name, sc in SC.items():
        if "calls" in sc:
            a = o.Authenticator(ks)
            got = [a.verify(c["role"], c["id"], bytes.fromhex(c["msg"]), bytes.fromhex(c["tag"]))
                   for c in sc["calls"]]
            assert got == _expects(name), name
        elif "msgs" in sc:
            got = o.validate_messages(o.Authenticator(ks), _msgs(sc), sc["n"], sc["flags"])
            assert got == _expects(name), name


def test_ui_marshal_layout_host():
    """usig/usig_test.go:31-45: UI = counter_be64 || cert (usig.go:54-70)."""
    ui = SC["ui_marshal"]["ui"]
    b = bytes.fromhex(ui["bytes"])
    assert b == struct.pack(">Q", ui["counter"]) + bytes.fromhex(ui["cert"])
    assert struct.unpack(">Q", b[:8])[0] == ui["counter"] and b[8:].hex() == ui["cert"]


def test_reference_tags_parse_host(lib):
    """Host-side C-ABI (no GPU): every ECDSA-role tag of the scenarios decodes
    with the Go-exact DER parser to the signer's (r, s)."""
    from minbft_amd import _lib
    from oracle import p256 as o
    for name in ("ecdsa_authen_scheme", "authenticator_roles"):
        for c in SC[name]["calls"]:
            if c["role"] == o.ROLE_USIG:
                continue
            tag = bytes.fromhex(c["tag"])
            r, s, n = _lib.der_parse_sig(tag)
            rr, ss, rest = o.der_parse_sig(tag)
            assert (int.from_bytes(r, "big"), int.from_bytes(s, "big"), n) == (rr, ss, len(tag))
            assert rest == b""


# ----------------------------------------------------------------- GPU
def _auth():
    from minbft_amd.authenticator import Authenticator
    a = Authenticator(0)
    for role, m in FX["keystore"].items():
        a.add_role(int(role))
        for id_, pk in m.items():
            a.set_public_key(int(role), int(id_), bytes.fromhex(pk))
    a.enable_usig(True)
    return a


@pytest.mark.gpu
@pytest.mark.parametrize("name", [n for n in sorted(SC) if "calls" in SC[n]])
@pytest.mark.parametrize("mode", ["one_at_a_time", "batch"])
def test_gpu_scenario_calls(lib, name, mode):
    """VerifyMessageAuthenTag through mbft_verify_message_authen_tag (one
    call at a time) and mbft_verify_batch (the whole scenario as one batch)."""
    calls = SC[name]["calls"]
    with _auth() as a:
        if mode == "batch":
            got = [int(x) for x in a.verify_batch(
                [(c["role"], c["id"], bytes.fromhex(c["msg"]), bytes.fromhex(c["tag"])) for c in calls])]
        else:
            got = [a.verify_status(c["role"], c["id"], bytes.fromhex(c["msg"]), bytes.fromhex(c["tag"]))
                   for c in calls]
    assert got == _expects(name), [(c["note"], g) for c, g in zip(calls, got)]


@pytest.mark.gpu
def test_gpu_ecdsa_sig_cipher_prehashed(lib):
    """crypto_test.go:49-58 at the crypto/ecdsa.Verify boundary
    (mbft_verify_prehashed), plus the same signature under every single-bit
    flip of e (each must reject)."""
    from minbft_amd.authenticator import Authenticator
    v = SC["ecdsa_sig_cipher"]["prehashed"][0]
    pk = bytes.fromhex(FX["key"]["pkix"])
    e0 = np.frombuffer(bytes.fromhex(v["e"]), dtype=np.uint8)
    e = np.tile(e0, (257, 1))
    for k in range(256):
        e[1 + k, k // 8] ^= 0x80 >> (k % 8)
    r = np.tile(np.frombuffer(bytes.fromhex(v["r"]), dtype=np.uint8), (257, 1))
    s = np.tile(np.frombuffer(bytes.fromhex(v["s"]), dtype=np.uint8), (257, 1))
    with Authenticator(0) as a:
        slots, valid = a.register_points(np.frombuffer(pk[27:], dtype=np.uint8)[None, :])
        assert valid.all()
        st = a.verify_prehashed(e, r, s, np.full(257, slots[0], dtype=np.uint32))
    assert st[0] == v["expect"] == 0
    assert (st[1:] == 1).all()


@pytest.mark.gpu
def test_gpu_ui_verifier_through_prepare_validator(lib):
    """core/usig-ui_test.go:39-82 through mbft_validate_messages: correct UI,
    failed USIG certificate, zero counter (rejected before the
    authenticator)."""
    sc = SC["ui_verifier"]
    with _auth() as a:
        got = [int(x) for x in a.validate_messages(_msgs(sc), sc["n"], sc["flags"])]
    assert got == sc["expect"]


@pytest.mark.gpu
def test_gpu_generate_then_verify_fixture_key(lib):
    """crypto_test.go:60-68 / authenticator_test.go:29-69 with the GPU signer:
    GenerateMessageAuthenTag(role, "hello") with the fixture private key, then
    VerifyMessageAuthenTag on another authenticator (a1) for every ECDSA role
    entry of the key store; and the oracle accepts the same tag."""
    from minbft_amd.authenticator import ROLE_CLIENT, ROLE_REPLICA, Authenticator
    from oracle import p256 as o
    d = bytes.fromhex(FX["key"]["d"])
    q = o.pkix_decode(bytes.fromhex(FX["key"]["pkix"]))
    with Authenticator(0) as a0, _auth() as a1:
        for role, ids in ((ROLE_REPLICA, (0, 1, 2)), (ROLE_CLIENT, (10,))):
            a0.set_private_key(role, d)
            tag = a0.GenerateMessageAuthenTag(role, b"hello")
            r, s, _ = o.der_parse_sig(tag)
            assert o.go_ecdsa_verify(q, o.quirk_digest(b"hello"), r, s)
            for id_ in ids:
                assert a1.VerifyMessageAuthenTag(role, id_, b"hello", tag) is None
            # wrong message: error (not accept, not panic)
            assert a1.verify_status(role, ids[0], b"hellp", tag) == 1


@pytest.mark.gpu
def test_gpu_keystore_lookup(lib):
    """keymanager_test.go:86-113 cases: (role, id) present in the example key
    store or not (mbft_key_slot; an unknown role / id is an error)."""
    with _auth() as a:
        for role, id_, found in SC["keystore_lookup"]["cases"]:
            rc = a.lib.mbft_key_slot(a.ctx, role, id_)
            assert (rc >= 0) == found, (role, id_, rc)

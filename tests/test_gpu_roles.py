"""Roles outside the reference's three at the boundary.

api.AuthenticationRole is a Go int (api/api.go:95-115); the reference
rejects any role it has no key set / scheme for ("key set not found",
keymanager.go:96-101; "Unknown role", authenticator.go:121-134).  The Go
binding hands the library roleByte(role) (go/gpuauth/gpuauth.go): the three
roles as themselves, anything else as 0 -- so 257 can no longer alias
ReplicaAuthen.  Here every such role, after that mapping (compact u8 forms)
and raw (u32 forms, single calls), must come back MBFT_UNKNOWN_ROLE, equal to
the oracle's verdict on the unmapped role, with valid calls around it
accepted, through mbft_verify_batch_flat32 / mbft_check_batch_flat32 (host
and GPU decode), mbft_verify_batch_flat and mbft_verify_message_authen_tag.
"""
import hashlib

import pytest

pytestmark = pytest.mark.gpu

ODD_ROLES = [0, 4, 5, 255, 256, 257, 258, 259, 1 << 16, (1 << 31) - 1, (1 << 32) + 1, (1 << 32) + 3]


def go_role_byte(role: int) -> int:
    """go/gpuauth/gpuauth.go roleByte."""
    return role if role in (1, 2, 3) else 0


def test_unknown_roles_reject_like_the_reference(lib):
    from minbft_amd.authenticator import Authenticator, ROLE_CLIENT, ROLE_REPLICA, ROLE_USIG
    from oracle import p256 as o
    d = int.from_bytes(hashlib.sha256(b"roles").digest(), "big") % o.N
    q = o.pubkey(d)
    ks = o.KeyStore()
    ks.keys = {ROLE_CLIENT: {7: q}, ROLE_REPLICA: {1: q}, ROLE_USIG: {0: q}}
    oracle = o.Authenticator(ks)
    msg = o.authen_request(3, bytes(range(200)))
    r, s = o.ecdsa_sign(d, o.quirk_digest(msg))
    tag = o.der_encode_sig(r, s)
    with Authenticator(0) as a:
        a.set_key_window(8)
        for role, m in ks.keys.items():
            a.add_role(role)
            for id_, pt in m.items():
                a.set_public_key(role, id_, o.pkix_encode(pt))
        a.enable_usig(True)
        for role in ODD_ROLES:
            assert oracle.verify(role, 1, msg, tag) == o.UNKNOWN_ROLE
            assert oracle.verify(role, 7, msg, tag) == o.UNKNOWN_ROLE
        want_ok = [oracle.verify(ROLE_CLIENT, 7, msg, tag), oracle.verify(ROLE_REPLICA, 1, msg, tag)]
        assert want_ok == [0, 0]
        # compact form (u8 roles) after the binding's mapping, a valid call on either side
        items = []
        for role in ODD_ROLES:
            for id_ in (1, 7):
                items += [(ROLE_CLIENT, 7, msg, tag), (go_role_byte(role), id_, msg, tag),
                          (ROLE_REPLICA, 1, msg, tag)]
        want = [0, o.UNKNOWN_ROLE, 0] * (len(items) // 3)
        for pinned in (False, True):  # host decode, GPU decode (k_prepare)
            got = a.verify_batch_flat32(items, pinned=pinned, ecdsa_e=True)
            assert [int(x) for x in got] == want, pinned
            got = a.check_batch_flat32(items, pinned=pinned)
            assert [int(x) for x in got] == want, pinned
        # wide form (u32 roles) and single calls with the raw role (mod 2^32,
        # what a C caller can pass): never an alias of a known role
        raw = [(rl & 0xFFFFFFFF) for rl in ODD_ROLES if (rl & 0xFFFFFFFF) not in (1, 2, 3)]
        wide = [(rl, 7, msg, tag) for rl in raw] + [(ROLE_CLIENT, 7, msg, tag)]
        for pinned in (False, True):
            got = a.verify_batch_flat(wide, pinned=pinned)
            assert [int(x) for x in got] == [o.UNKNOWN_ROLE] * len(raw) + [0], pinned
        for rl in raw:
            assert a.verify_status(rl, 7, msg, tag) == o.UNKNOWN_ROLE, rl
        # what a role narrowed to a byte would have done: 257 -> ReplicaAuthen accepts
        assert a.verify_status(257 & 0xFF, 1, msg, tag) == 0

"""The Go client's batched reply loop (go/client/message-handling-batch.go +
go/gpuauth/replies.go) as its C-ABI call sequence, against the oracle's
validate_replies (client/message-handling.go:93-110,138-170):

per window of REPLYs already received from a replica -- records + arena
(the Go marshal), mbft_validate_replies_flat with MBFT_VF_NO_PANIC_STOP --
then each REPLY in arrival order: its result, where a malformed DER
signature is the reference's panic (the loop ends there: every earlier
REPLY handled, nothing after it).  Windows of 1, 3 and the whole stream,
through the small route (AuthenBytes hashed on the host, one zero-copy
launch) and through the GPU digest stage (small route off)."""
import hashlib
import random

import numpy as np
import pytest

from test_gpu_authen import _msgs, load

pytestmark = pytest.mark.gpu

ST_REPLY_SIG, ST_AFTER_PANIC = 8, 9
MALFORMED_DER = 2
NO_PANIC_STOP = 2


def _go_loop(a, msgs, client_id, window):
    """The Go loop's sequence; returns the per-REPLY results up to the panic
    (inclusive) and the panic position (or None)."""
    out = []
    i = 0
    while i < len(msgs):
        part = msgs[i:i + window]
        from minbft_amd import _lib
        arr, keep = _lib.make_messages(part)
        packed = np.frombuffer(arr, dtype=_lib.message_dtype(), count=len(part))
        recs, arena = a.pack_messages(packed, True)
        res = a.validate_replies_flat(recs, arena, client_id, NO_PANIC_STOP)
        del keep
        for r in res:
            out.append(int(r))
            if (int(r) >> 8) == ST_REPLY_SIG and (int(r) & 0xFF) == MALFORMED_DER:
                return out, len(out) - 1  # Result(i) panics: the client process ends here
        i += len(part)
    return out, None


def _synthetic(rng, n_replicas=4, count=60):
    """Replies of replicas 0..3 to client 7 (and a few to client 8), some
    tampered, unknown-replica, trailing-DER (accepted for ECDSA roles) and
    one malformed DER signature near the end."""
    from oracle import p256 as o
    keys = {r: int.from_bytes(hashlib.sha256(b"reply key %d" % r).digest(), "big") % o.N
            for r in range(n_replicas)}
    msgs = []
    for k in range(count):
        rid = rng.randrange(n_replicas + 1)  # n_replicas: no key for it
        m = o.Msg(type=o.MSG_REPLY, replica_id=rid, client_id=7 if k % 9 else 8, seq=k // 3 + 1,
                  op=rng.randbytes(rng.choice([0, 5, 64, 300])))
        d = keys.get(rid, keys[0])
        r, s = o.ecdsa_sign(d, o.quirk_digest(o.msg_authen_bytes(m)))
        m.sig = o.der_encode_sig(r, s)
        kind = k % 11
        if kind == 3:
            m.op = m.op + b"!"  # tampered result
        elif kind == 5:
            m.sig = m.sig + b"\x00\x01"  # trailing bytes: ignored in the ECDSA roles
        msgs.append(m)
    bad = msgs[count - 7]
    bad.client_id = 7
    bad.sig = b"\x30\x81" + bad.sig[2:]  # malformed DER (long-form length < 128)
    ks = {o.ROLE_REPLICA: {r: o.pubkey(d) for r, d in keys.items()}}
    return msgs, ks


@pytest.mark.parametrize("small", [256, 0])
def test_go_reply_loop_vs_oracle(lib, small):
    from minbft_amd.authenticator import Authenticator
    from oracle import p256 as o
    fx = load("messages.json")
    cases = []
    for sq in fx["replies"]:
        keys = {int(role): {int(i): bytes.fromhex(pk) for i, pk in m.items()} for role, m in fx["keystore"].items()}
        cases.append((_msgs(sq["msgs"]), sq["client_id"], keys, None))
    msgs, ks = _synthetic(random.Random(0x9E7))
    cases.append((msgs, 7, {role: {i: o.pkix_encode(q) for i, q in m.items()} for role, m in ks.items()}, ks))
    for msgs, client_id, keys, okeys in cases:
        oks = o.KeyStore()
        if okeys is None:
            oks.keys = {role: {i: o.pkix_decode(pk) for i, pk in m.items()} for role, m in keys.items()}
        else:
            oks.keys = okeys
        want = o.validate_replies(o.Authenticator(oks), msgs, client_id, 0)
        stop = next((i for i, w in enumerate(want) if w == (ST_AFTER_PANIC << 8)), None)
        for window in (1, 3, len(msgs)):
            with Authenticator(0) as a:
                a.set_key_window(8)
                a.set_small_check(small)
                for role, m in keys.items():
                    a.add_role(role)
                    for i, pk in m.items():
                        a.set_public_key(role, i, pk)
                got, panic_at = _go_loop(a, msgs, client_id, window)
            if stop is None:
                assert panic_at is None and got == want, (window, small)
            else:
                assert panic_at == stop - 1, (window, small, panic_at, stop)
                assert got == want[:stop], (window, small)
    assert any((w >> 8) == ST_REPLY_SIG and (w & 0xFF) == 1 for w in want)  # a tampered REPLY rejected

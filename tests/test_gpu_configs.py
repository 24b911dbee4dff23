"""BASELINE.json configs as parity cases (the bench line is C2; these are
the other configs):

* C3 -- USIG UI verification for PREPARE/COMMIT streams, n = 2f+1 replicas
  for f in 1..16, mixed COMMIT signers, through the batched core validators
  (mbft_validate_messages), against the oracle's sequential restatement of
  the validators and the USIG epoch logic.
* C4 -- the adversarial mix at one GPU's share of the 64M batch
  (8,388,608 items: 2% tampered, 2% wrong key, 2% r/s out of range, 1%
  off-curve key slot, 1% high-s), every status checked against its
  construction plus a C-oracle sample; and the Authenticator-level part of
  the mix (malformed DER, quirk-mode tamper at offset >= 32, trailing DER
  bytes) through mbft_verify_batch against the C oracle.
"""
import hashlib
import random
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _seeded_key(tag: str) -> int:
    from oracle import p256 as o
    return int.from_bytes(hashlib.sha256(tag.encode()).digest(), "big") % (o.N - 1) + 1


def _fast_oracle(monkeypatch):
    """The oracle's validators with its ECDSA core swapped for the C
    restatement (same rules, pinned by tests/test_oracle.py) for speed."""
    from oracle import c_oracle
    from oracle import p256 as o
    slow = o.go_ecdsa_verify

    def fast(q, h, r, s):
        if not (0 < r < (1 << 256) and 0 < s < (1 << 256)):
            return slow(q, h, r, s)
        e = h[:32] if len(h) >= 32 else b"\0" * (32 - len(h)) + h
        qxy = q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big")
        return c_oracle.verify(qxy, e, r.to_bytes(32, "big"), s.to_bytes(32, "big")) == 1
    monkeypatch.setattr(o, "go_ecdsa_verify", fast)


def _c3_streams(f: int, nreq: int, rng: random.Random, faults: bool):
    """A backup's view of nreq requests in view 0 (primary 0): REQUEST,
    PREPARE and the COMMITs of replicas 1..n-1 in a shuffled (mixed-signer)
    order, sequential USIG counters per replica from 1, a random epoch per
    replica.  With faults: a tampered COMMIT certificate, a COMMIT under the
    wrong epoch, a zero-counter COMMIT and a PREPARE UI from the wrong USIG."""
    from oracle import p256 as o
    n = 2 * f + 1
    usig = {i: _seeded_key(f"c3 usig {f} {i}") for i in range(n)}
    cli = _seeded_key(f"c3 client {f}")
    epoch = {i: rng.randrange(1, 1 << 64) for i in range(n)}
    ctr = {i: 0 for i in range(n)}
    msgs = []
    for k in range(nreq):
        op = rng.randbytes(256)
        rq = o.Msg(type=o.MSG_REQUEST, stream=1000, client_id=7, seq=k + 1, op=op)
        r, s = o.ecdsa_sign(cli, o.quirk_digest(o.msg_authen_bytes(rq)))
        rq.sig = o.der_encode_sig(r, s)
        msgs.append(rq)
        ctr[0] += 1
        pr = o.Msg(type=o.MSG_PREPARE, stream=0, replica_id=0, view=0, client_id=7, seq=k + 1,
                   op=op, sig=rq.sig, ui_counter=ctr[0])
        pr.ui_cert = o.usig_create_ui(usig[0], o.msg_authen_bytes(pr), epoch[0], ctr[0])[8:]
        msgs.append(pr)
        backups = list(range(1, n))
        rng.shuffle(backups)
        for rid in backups:
            ctr[rid] += 1
            cm = o.Msg(type=o.MSG_COMMIT, stream=rid, replica_id=rid, prep_replica_id=0, view=0,
                       client_id=7, seq=k + 1, op=op, sig=rq.sig, prep_ui_counter=pr.ui_counter,
                       prep_ui_cert=pr.ui_cert, ui_counter=ctr[rid])
            cm.ui_cert = o.usig_create_ui(usig[rid], o.msg_authen_bytes(cm), epoch[rid],
                                          ctr[rid])[8:]
            msgs.append(cm)
    if faults:
        import copy
        cms = [m for m in msgs if m.type == o.MSG_COMMIT]
        b = copy.copy(cms[0])
        cert = bytearray(b.ui_cert)
        cert[-1] ^= 1
        b.ui_cert = bytes(cert)
        b.stream = 5000
        msgs.insert(len(msgs) // 2, b)                                # bad signature
        b = copy.copy(cms[1])
        b.ui_cert = struct.pack(">Q", epoch[b.replica_id] ^ 1) + b.ui_cert[8:]
        b.stream = 5001
        msgs.insert(len(msgs) // 3, b)                                # epoch mismatch
        b = copy.copy(cms[-1])
        b.ui_counter = 0
        msgs.append(b)                                                # zero counter (stops stream)
        b = copy.copy(cms[2])
        b.prep_ui_cert = cms[2].ui_cert
        b.stream = 5002
        msgs.append(b)                                                # wrong PREPARE UI
    keys = {o.ROLE_USIG: {i: o.pubkey(d) for i, d in usig.items()},
            o.ROLE_CLIENT: {7: o.pubkey(cli)}}
    return n, msgs, keys


@pytest.mark.parametrize("f", [1, 2, 4, 8, 16])
def test_c3_usig_streams(lib, monkeypatch, f):
    from minbft_amd.authenticator import Authenticator
    from oracle import p256 as o
    _fast_oracle(monkeypatch)
    rng = random.Random(0xC3 * 100 + f)
    for faults in (False, True):
        n, msgs, keys = _c3_streams(f, 3, rng, faults)
        ks = o.KeyStore()
        ks.keys = {role: dict(m) for role, m in keys.items()}
        want = o.validate_messages(o.Authenticator(ks), msgs, n, 0)
        with Authenticator(0) as a:
            a.set_key_window(16)
            for role, m in keys.items():
                a.add_role(role)
                for id_, q in m.items():
                    a.set_public_key(role, id_, o.pkix_encode(q))
            a.enable_usig(True)
            got = a.validate_messages(msgs, n, 0)
        bad = [(i, int(g), w) for i, (g, w) in enumerate(zip(got, want)) if g != w]
        assert not bad, (f, faults, bad[:10])
        if not faults:
            assert all(w == 0 for w in want)
        else:
            assert sum(w != 0 for w in want) >= 4


def test_c3_usig_streams_large(lib, monkeypatch):
    """C3 at f = 16 with 121 requests (4,118 messages): past the batch size
    at which the message layer builds its checks and deduplicates its calls
    on the worker pool (4,096), with the faults injected; against the
    oracle's sequential validators."""
    from minbft_amd.authenticator import Authenticator
    from oracle import p256 as o
    _fast_oracle(monkeypatch)
    rng = random.Random(0xC3B16)
    n, msgs, keys = _c3_streams(16, 121, rng, True)
    assert len(msgs) > 4096
    ks = o.KeyStore()
    ks.keys = {role: dict(m) for role, m in keys.items()}
    want = o.validate_messages(o.Authenticator(ks), msgs, n, 0)
    with Authenticator(0) as a:
        a.set_key_window(16)
        for role, m in keys.items():
            a.add_role(role)
            for id_, q in m.items():
                a.set_public_key(role, id_, o.pkix_encode(q))
        a.enable_usig(True)
        got = a.validate_messages(msgs, n, 0)
    bad = [(i, int(g), w) for i, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not bad, bad[:10]
    assert sum(w != 0 for w in want) >= 4


def _keys(k):
    from oracle import p256 as o
    ds = [_seeded_key(f"c4 key {i}") for i in range(k)]
    qs = [o.pubkey(d) for d in ds]
    priv = np.array([list(d.to_bytes(32, "big")) for d in ds], dtype=np.uint8)
    xy = np.array([list(q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big")) for q in qs],
                  dtype=np.uint8)
    return priv, xy


def test_c4_adversarial_gpu_share(gpu_auth):
    """8,388,608 items (64M / 8 GPUs) with the C4 mix; expected status of
    every item from its construction; a 4096-item C-oracle sample."""
    from oracle import c_oracle
    from oracle import p256 as o
    n = 8 << 20
    rng = np.random.Generator(np.random.PCG64(0xC4))
    priv, xy = _keys(8)
    slots, valid = gpu_auth.register_points(xy)
    assert valid.all()
    off = xy[0].copy()
    off[63] ^= 1                                              # off-curve point
    bad_slot, bad_valid = gpu_auth.register_points(off[None, :])
    assert not bad_valid[0]
    kidx = rng.integers(0, 8, size=n).astype(np.uint32)
    e = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    r, s = gpu_auth.sign_prehashed(priv, e, kidx)
    slot = slots[kidx].copy()
    kind = rng.integers(0, 100, size=n)
    want = np.zeros(n, dtype=np.uint8)
    Nb = np.frombuffer(o.N.to_bytes(32, "big"), dtype=np.uint8)
    t = kind < 2
    e[t, 3] ^= 0x20                                           # tampered digest
    want[t] = 1
    t = (kind >= 2) & (kind < 4)
    slot[t] = slots[(kidx[t] + 1) % 8]                        # wrong key
    want[t] = 1
    t = (kind >= 4) & (kind < 5)
    r[t] = 0                                                  # r = 0
    want[t] = 1
    t = kind == 5
    s[t] = Nb                                                 # s = N
    want[t] = 1
    t = kind == 6
    r[t] = 0xFF                                               # r = 2^256 - 1
    want[t] = 1
    t = kind == 7
    slot[t] = bad_slot[0]                                     # off-curve key slot
    want[t] = 5
    t = np.nonzero(kind == 8)[0]                              # high-s: accepted
    for i in t:
        s[i] = np.frombuffer((o.N - int.from_bytes(s[i].tobytes(), "big")).to_bytes(32, "big"),
                             dtype=np.uint8)
    got = gpu_auth.verify_prehashed(e, r, s, slot)
    mism = np.nonzero(got != want)[0]
    assert mism.size == 0, [(int(i), int(kind[i]), int(got[i]), int(want[i])) for i in mism[:10]]
    idx = rng.choice(np.nonzero(kind != 7)[0], size=4096, replace=False)
    qx = np.zeros((int(slots.max()) + 1, 64), dtype=np.uint8)
    qx[slots] = xy
    ref = c_oracle.verify_prehashed_batch(qx, e[idx], r[idx], s[idx], slot[idx], nthreads=16)
    assert (ref == got[idx]).all()


def test_c4_authenticator_level_mix(lib):
    """The host-status part of the C4 mix through VerifyMessageAuthenTag
    batches: malformed DER (Go panic status), quirk-mode tamper at authen
    offset >= 32 (ACCEPTED by the reference), DER with trailing bytes
    (ignored in the ECDSA roles), against the C oracle's restatement."""
    from minbft_amd.authenticator import Authenticator, ROLE_CLIENT, der_encode_sig
    from oracle import c_oracle
    from oracle import p256 as o
    n = 65536
    rng = np.random.Generator(np.random.PCG64(0xC41))
    priv, xy = _keys(4)
    with Authenticator(0) as a:
        a.add_role(ROLE_CLIENT)
        for i in range(4):
            a.set_public_key(ROLE_CLIENT, i, xy[i].tobytes())
        ids = rng.integers(0, 4, size=n).astype(np.uint32)
        ops = rng.integers(0, 256, size=(n, 64), dtype=np.uint8)
        msgs = [o.authen_request(i + 1, ops[i].tobytes()) for i in range(n)]
        e = np.array([list(m[:32]) for m in msgs], dtype=np.uint8)
        r, s = a.sign_prehashed(priv, e, ids)
        tags = [der_encode_sig(r[i].tobytes(), s[i].tobytes()) for i in range(n)]
        kind = rng.integers(0, 100, size=n)
        for i in np.nonzero(kind < 2)[0]:
            tags[i] = tags[i][:-2]                            # malformed DER
        for i in np.nonzero((kind >= 2) & (kind < 4))[0]:
            m = bytearray(msgs[i])
            m[32 + int(rng.integers(0, 15))] ^= 1             # tamper at offset >= 32: accept
            msgs[i] = bytes(m)
        for i in np.nonzero((kind >= 4) & (kind < 6))[0]:
            m = bytearray(msgs[i])
            m[int(rng.integers(0, 32))] ^= 1                  # tamper at offset < 32: reject
            msgs[i] = bytes(m)
        for i in np.nonzero((kind >= 6) & (kind < 7))[0]:
            tags[i] = tags[i] + b"\x00\x01"                   # trailing bytes: ignored
        got = a.verify_batch([(ROLE_CLIENT, int(ids[i]), msgs[i], tags[i]) for i in range(n)])
    want = c_oracle.verify_ecdsa_role_batch(xy, ids, msgs, tags, nthreads=16)
    assert (got == want).all(), np.nonzero(got != want)[0][:10]
    assert (got[kind < 2] == 2).all()
    assert (got[(kind >= 2) & (kind < 4)] == 0).all()
    assert (got[(kind >= 4) & (kind < 6)] == 1).all()
    assert (got[kind >= 6] == 0).all()

"""Authenticator-level GPU parity: VerifyMessageAuthenTag semantics
(sample/authentication/authenticator.go:121-134, crypto.go:79-126,186-239)
replayed from the golden call sequences, one call at a time and as one
batch; plus large-batch parity against the C oracle."""
import hashlib

import numpy as np
import pytest

from golden_util import load

pytestmark = pytest.mark.gpu


def _make_auth(fx, usig=True):
    from minbft_amd.authenticator import Authenticator
    a = Authenticator(0)
    for role, m in fx["keystore"].items():
        a.add_role(int(role))
        for id_, pk in m.items():
            a.set_public_key(int(role), int(id_), bytes.fromhex(pk))
    a.enable_usig(usig)
    return a


@pytest.mark.parametrize("name", ["authen.json", "usig_epoch.json"])
def test_sequences_one_call_at_a_time(lib, name):
    fx = load(name)
    for seq in fx["sequences"]:
        a = _make_auth(fx)
        try:
            got = [a.verify_status(c["role"], c["id"], bytes.fromhex(c["msg"]), bytes.fromhex(c["tag"]))
                   for c in seq]
        finally:
            a.close()
        want = [c["expect"] for c in seq]
        bad = [(c["note"], g, w) for c, g, w in zip(seq, got, want) if g != w]
        assert not bad, bad[:10]


@pytest.mark.parametrize("name", ["authen.json", "usig_epoch.json"])
def test_sequences_as_one_batch(lib, name):
    fx = load(name)
    for seq in fx["sequences"]:
        a = _make_auth(fx)
        try:
            st = a.verify_batch([(c["role"], c["id"], bytes.fromhex(c["msg"]), bytes.fromhex(c["tag"]))
                                 for c in seq])
        finally:
            a.close()
        want = [c["expect"] for c in seq]
        bad = [(c["note"], int(g), w) for c, g, w in zip(seq, st, want) if g != w]
        assert not bad, bad[:10]


def test_go_error_kinds(lib):
    """VerifyMessageAuthenTag mirror: nil / error / panic as in Go."""
    from minbft_amd.authenticator import AuthenticationError, SignaturePanic
    fx = load("authen.json")
    a = _make_auth(fx)
    try:
        seq = fx["sequences"][0]
        for c in seq[:30]:
            args = (c["role"], c["id"], bytes.fromhex(c["msg"]), bytes.fromhex(c["tag"]))
            if c["expect"] == 0:
                assert a.VerifyMessageAuthenTag(*args) is None
            elif c["expect"] == 2 and c["role"] != 2:
                with pytest.raises(SignaturePanic):
                    a.VerifyMessageAuthenTag(*args)
            else:
                with pytest.raises(AuthenticationError):
                    a.VerifyMessageAuthenTag(*args)
    finally:
        a.close()


def test_usig_disabled_is_unknown_role(lib):
    fx = load("usig_epoch.json")
    a = _make_auth(fx, usig=False)
    try:
        c = fx["sequences"][0][2]
        assert a.verify_status(2, 0, bytes.fromhex(c["msg"]), bytes.fromhex(c["tag"])) == 10
    finally:
        a.close()


def test_off_curve_key_rejected_at_load(lib):
    from minbft_amd.authenticator import Authenticator
    a = Authenticator(0)
    try:
        a.add_role(1)
        with pytest.raises(ValueError):
            a.set_public_key(1, 0, b"\x01" * 64)
        # x >= p
        with pytest.raises(ValueError):
            a.set_public_key(1, 0, b"\xff" * 64)
        xy = np.frombuffer(b"\x01" * 64 + b"\x00" * 63 + b"\x05", dtype=np.uint8).reshape(2, 64)
        slots, valid = a.register_points(xy)
        assert list(valid) == [0, 0]
        st = a.verify_prehashed(np.zeros((1, 32), np.uint8), np.ones((1, 32), np.uint8),
                                np.ones((1, 32), np.uint8), slots[:1])
        assert st[0] == 5
        # slots past the key store -- including the range the batch pipeline
        # uses internally to carry host-decided statuses -- are BAD_KEY here
        bad = np.array([2, 1000, 0xFFFFFF00, 0xFFFFFF01, 0xFFFFFFFF], dtype=np.uint32)
        k = bad.size
        st = a.verify_prehashed(np.zeros((k, 32), np.uint8), np.ones((k, 32), np.uint8),
                                np.ones((k, 32), np.uint8), bad)
        assert list(st) == [5] * k
    finally:
        a.close()


def _keys(k):
    from oracle import p256 as o
    ds = [int.from_bytes(hashlib.sha256(b"gpu parity key %d" % i).digest(), "big") % (o.N - 1) + 1
          for i in range(k)]
    qs = [o.pubkey(d) for d in ds]
    priv = np.array([list(d.to_bytes(32, "big")) for d in ds], dtype=np.uint8)
    xy = np.array([list(q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big")) for q in qs], dtype=np.uint8)
    return priv, xy


def test_adversarial_batch_vs_c_oracle(gpu_auth):
    """C4-style mix at 131072 items, every status compared
    with the oracle's C restatement."""
    from oracle import c_oracle
    from oracle import p256 as o
    n = 131072
    rng = np.random.Generator(np.random.PCG64(0x4D696E42))
    priv, xy = _keys(8)
    slots, valid = gpu_auth.register_points(xy)
    assert valid.all()
    kidx = rng.integers(0, 8, size=n).astype(np.uint32)
    e = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    r, s = gpu_auth.sign_prehashed(priv, e, kidx)
    slot = slots[kidx].copy()
    kind = rng.integers(0, 100, size=n)
    Nb = np.frombuffer(o.N.to_bytes(32, "big"), dtype=np.uint8)
    e2, r2, s2 = e.copy(), r.copy(), s.copy()
    t = kind < 2
    e2[t, rng.integers(0, 32)] ^= 0x10                       # tampered digest
    t = (kind >= 2) & (kind < 4)
    slot[t] = slots[(kidx[t] + 1) % 8]                       # wrong key
    t = (kind >= 4) & (kind < 5)
    r2[t] = 0                                                # r = 0
    t = (kind >= 5) & (kind < 6)
    s2[t] = Nb                                               # s = N
    t = (kind >= 6) & (kind < 7)
    r2[t] = 0xFF                                             # r = 2^256-1
    t = (kind >= 7) & (kind < 8)                             # high-s: accept
    for i in np.nonzero(t)[0]:
        s2[i] = np.frombuffer((o.N - int.from_bytes(s2[i].tobytes(), "big")).to_bytes(32, "big"),
                              dtype=np.uint8)
    got = gpu_auth.verify_prehashed(e2, r2, s2, slot)
    inv = np.argsort(slots)
    qxy_by_slot = np.zeros((int(slots.max()) + 1, 64), dtype=np.uint8)
    qxy_by_slot[slots] = xy
    want = c_oracle.verify_prehashed_batch(qxy_by_slot, e2, r2, s2, slot, nthreads=16)
    assert inv is not None
    mism = np.nonzero(got != want)[0]
    assert mism.size == 0, [(int(i), int(kind[i]), int(got[i]), int(want[i])) for i in mism[:10]]
    assert (got[kind >= 8] == 0).all()
    assert (got[(kind >= 7) & (kind < 8)] == 0).all()


def test_full_size_properties(gpu_auth):
    """BASELINE size (1,048,576): sign -> verify accepts all; flipping one
    byte of e (at a random position per item) rejects all; a sample is
    cross-checked with the C oracle."""
    from oracle import c_oracle
    n = 1 << 20
    rng = np.random.Generator(np.random.PCG64(7))
    priv, xy = _keys(1)
    slots, _ = gpu_auth.register_points(xy)
    e = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    r, s = gpu_auth.sign_prehashed(priv, e)
    sl = np.full(n, slots[0], dtype=np.uint32)
    st = gpu_auth.verify_prehashed(e, r, s, sl)
    assert (st == 0).all()
    pos = rng.integers(0, 32, size=n)
    e2 = e.copy()
    e2[np.arange(n), pos] ^= 0x01
    st2 = gpu_auth.verify_prehashed(e2, r, s, sl)
    assert (st2 == 1).all()
    idx = rng.choice(n, size=2048, replace=False)
    qx = np.zeros((int(slots[0]) + 1, 64), dtype=np.uint8)
    qx[slots[0]] = xy[0]
    want = c_oracle.verify_prehashed_batch(qx, e[idx], r[idx], s[idx], sl[idx], nthreads=16)
    assert (want == 0).all()


def test_validate_message_streams(lib):
    """Batched core validators vs the oracle's sequential restatement on the
    golden MinBFT streams (every validator branch, stream stop, panic)."""
    from minbft_amd.authenticator import Authenticator
    from oracle import p256 as o
    fx = load("messages.json")
    for sq in fx["sequences"]:
        msgs = []
        for d in sq["msgs"]:
            d = dict(d)
            for k in ("op", "sig", "ui_cert", "prep_ui_cert"):
                d[k] = bytes.fromhex(d[k])
            msgs.append(o.Msg(**d))
        with Authenticator(0) as a:
            for role, m in fx["keystore"].items():
                a.add_role(int(role))
                for id_, pk in m.items():
                    a.set_public_key(int(role), int(id_), bytes.fromhex(pk))
            a.enable_usig(True)
            got = a.validate_messages(msgs, sq["n"], sq["flags"])
        bad = [(i, int(g), w) for i, (g, w) in enumerate(zip(got, sq["expect"])) if g != w]
        assert not bad, bad[:10]


def _msgs(ds):
    from oracle import p256 as o
    out = []
    for d in ds:
        d = dict(d)
        for k in ("op", "sig", "ui_cert", "prep_ui_cert"):
            d[k] = bytes.fromhex(d[k])
        out.append(o.Msg(**d))
    return out


def test_validate_replies(lib):
    """Client-side REPLY validation (client/message-handling.go:93-110,
    140-170) vs the oracle: ClientID check, ReplicaAuthen, no stream stop,
    panic on malformed DER."""
    from minbft_amd.authenticator import Authenticator
    fx = load("messages.json")
    assert fx["replies"]
    for sq in fx["replies"]:
        with Authenticator(0) as a:
            for role, m in fx["keystore"].items():
                a.add_role(int(role))
                for id_, pk in m.items():
                    a.set_public_key(int(role), int(id_), bytes.fromhex(pk))
            got = a.validate_replies(_msgs(sq["msgs"]), sq["client_id"], sq["flags"])
        bad = [(i, int(g), w) for i, (g, w) in enumerate(zip(got, sq["expect"])) if g != w]
        assert not bad, bad[:10]


def test_validate_streams_gpu_sha_stage(lib, monkeypatch):
    """Same golden streams, and the Authenticator sequences as one batch,
    with the GPU USIG digest stage forced on (k_usig_e for every USIG call;
    the message validators always build AuthenBytes and digests on the GPU,
    k_sha256_var + k_authen_e): identical results."""
    monkeypatch.setenv("MBFT_GPU_USIG_MIN_CALLS", "0")
    test_validate_message_streams(lib)
    fx = load("authen.json")
    for seq in fx["sequences"]:
        a = _make_auth(fx)
        try:
            st = a.verify_batch([(c["role"], c["id"], bytes.fromhex(c["msg"]), bytes.fromhex(c["tag"]))
                                 for c in seq])
        finally:
            a.close()
        assert [int(x) for x in st] == [c["expect"] for c in seq]


@pytest.mark.parametrize("chunk,usig_min,form", [("3000", "0", "items"), ("0", "1000000", "items"),
                                                  ("3000", "0", "pinned"), ("0", "0", "pinned")])
def test_large_batch_pipeline(lib, monkeypatch, chunk, usig_min, form):
    """mbft_verify_batch past the parallel threshold: ~20K calls (every golden
    Authenticator call of authen.json, repeated 160 times: ECDSA roles, USIG
    with epoch capture / mismatch, malformed and trailing DER, unknown
    roles and ids), in pipeline chunks of 3,000 with the GPU USIG digest
    stage, and as one chunk with host digests; and the same calls as flat
    buffers in library page-locked memory, decoded on the GPU (k_prepare),
    chunked and whole.  Expected statuses
    from the oracle's sequential restatement over the WHOLE batch (one epoch
    map), its signature checks done by the C oracle."""
    from oracle import c_oracle
    from oracle import p256 as o
    monkeypatch.setenv("MBFT_BATCH_CHUNK", chunk)
    monkeypatch.setenv("MBFT_GPU_USIG_MIN_CALLS", usig_min)
    fx = load("authen.json")
    calls = []
    for rep in range(160):
        for seq in fx["sequences"]:
            calls += [(c["role"], c["id"], bytes.fromhex(c["msg"]), bytes.fromhex(c["tag"]))
                      for c in seq]
    assert len(calls) > 20000
    ks = o.KeyStore(keys={int(r): {int(i): o.pkix_decode(bytes.fromhex(pk)) for i, pk in m.items()}
                          for r, m in fx["keystore"].items()})

    def fast_verify(q, h, r, s):
        if not (0 < r < o.N and 0 < s < o.N):
            return False
        qxy = q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big")
        e = (b"\0" * 32 + h[:32])[-32:]  # hashToInt: left-most 32 bytes, as an integer
        return c_oracle.verify(qxy, e, r.to_bytes(32, "big"), s.to_bytes(32, "big")) == 1

    monkeypatch.setattr(o, "go_ecdsa_verify", fast_verify)
    ref = o.Authenticator(ks)
    want = [ref.verify(*c) for c in calls]
    from minbft_amd.authenticator import Authenticator
    with Authenticator(0) as a:
        for role, m in ks.keys.items():
            a.add_role(role)
            for id_, q in m.items():
                a.set_public_key(role, id_, o.pkix_encode(q))
        a.enable_usig(True)
        got = a.verify_batch(calls) if form == "items" else a.verify_batch_flat(calls, pinned=True)
    bad = [(i, int(g), w) for i, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not bad, bad[:10]


@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("name", ["authen.json", "usig_epoch.json"])
def test_flat_and_two_phase_forms(lib, name, pinned):
    """mbft_verify_batch_flat == mbft_verify_batch, and the two-phase form
    (mbft_check_batch_flat over the whole sequence, then
    mbft_resolve_checked call by call in order) gives every golden
    expectation -- the integration the Go core patch uses."""
    fx = load(name)
    for seq in fx["sequences"]:
        calls = [(c["role"], c["id"], bytes.fromhex(c["msg"]), bytes.fromhex(c["tag"])) for c in seq]
        want = [c["expect"] for c in seq]
        a = _make_auth(fx)
        try:
            assert [int(x) for x in a.verify_batch_flat(calls, pinned=pinned)] == want
        finally:
            a.close()
        a = _make_auth(fx)
        try:
            pure = a.check_batch_flat(calls, pinned=pinned)
            got = [a.resolve_checked(*c, int(p)) for c, p in zip(calls, pure)]
        finally:
            a.close()
        assert got == want
        # the compact form (u8 roles, u32 offsets), with the ECDSA-role
        # messages as given and as their 32-byte e prefix (the Go binding's
        # form); and its two-phase variant
        for ecdsa_e in (False, True):
            a = _make_auth(fx)
            try:
                got = [int(x) for x in a.verify_batch_flat32(calls, pinned=pinned, ecdsa_e=ecdsa_e)]
            finally:
                a.close()
            assert got == want, ecdsa_e
        a = _make_auth(fx)
        try:
            pure = a.check_batch_flat32(calls, pinned=pinned)
            got = [a.resolve_checked(*c, int(p)) for c, p in zip(calls, pure)]
        finally:
            a.close()
        assert got == want


def test_flat_offsets_checked_where_read(lib):
    """Flat batches decoded on the GPU are not scanned by the host: a call
    whose offsets run backwards or past its chunk's bytes is caught by
    k_prepare (or, for a USIG call, by the host's own scan before it reads
    the call) -> MBFT_ERR_ARG, nothing read out of range, no epoch state
    changed; the same buffers, repaired, verify as before.  Wide and compact
    forms, single-chunk and multi-chunk batches."""
    from minbft_amd.authenticator import GpuError, flat_calls
    fx = load("authen.json")
    seq = fx["sequences"][0]
    calls = [(c["role"], c["id"], bytes.fromhex(c["msg"]), bytes.fromhex(c["tag"])) for c in seq]
    want = [c["expect"] for c in seq]
    for reps in (1, 300000 // len(calls) + 1):
        big = calls * reps
        for compact in (False, True):
            a = _make_auth(fx)
            try:
                roles, ids, mb, mo, tb, to = flat_calls(big, pinned=True, compact=compact)
                run = (a.verify_flat32_arrays if compact else a.verify_flat_arrays)
                ok = np.array(run(roles, ids, mb, mo, tb, to, pinned=True))
                assert [int(x) for x in ok[:len(calls)]] == want
                # the USIG epochs are captured now: this is what an unchanged
                # state gives from here on
                ok = np.array(run(roles, ids, mb, mo, tb, to, pinned=True))
                n = len(big)
                for k in (2, n // 2 + 1, n - 1):
                    # backwards (a call ending before it starts), crossing the
                    # next call's end (that call runs backwards), past the end
                    for arr, val in ((mo, int(mo[k - 1]) - 1), (to, int(to[k + 1]) + 1),
                                     (mo, int(mo[n]) + 10 ** 6)):
                        saved = int(arr[k])
                        assert val >= 0
                        arr[k] = val
                        with pytest.raises(GpuError):
                            run(roles, ids, mb, mo, tb, to, pinned=True)
                        arr[k] = saved
                got = np.array(run(roles, ids, mb, mo, tb, to, pinned=True))
                assert (got == ok).all()
            finally:
                a.close()


@pytest.mark.parametrize("lanes", [1, 4])
def test_coalesced_concurrent_calls(lib, lanes):
    """mbft_set_coalescing: 8 threads issue single VerifyMessageAuthenTag
    calls at once (ctypes drops the GIL), so calls from several threads share
    GPU batches -- one batch at a time, or up to 4 batches in flight on 4
    engine lanes (mbft_set_coalescing_slots).  Each thread has its own client key and its own USIG key
    (its own epoch state), and runs valid / tampered ECDSA calls and a USIG
    stream with an epoch capture, a mismatch and a tampered UI; every status
    equals the oracle's sequential result for that thread."""
    import struct
    import threading

    from minbft_amd.authenticator import Authenticator, ROLE_CLIENT, ROLE_USIG
    from oracle import p256 as o
    T, reps = 8, 6
    ks = o.KeyStore(keys={ROLE_CLIENT: {}, ROLE_USIG: {}})
    seqs = []
    for t in range(T):
        dc = int.from_bytes(hashlib.sha256(b"coalesce client %d" % t).digest(), "big") % (o.N - 1) + 1
        du = int.from_bytes(hashlib.sha256(b"coalesce usig %d" % t).digest(), "big") % (o.N - 1) + 1
        ks.keys[ROLE_CLIENT][t] = o.pubkey(dc)
        ks.keys[ROLE_USIG][t] = o.pubkey(du)
        epoch = 1000 + t
        calls = []
        for k in range(reps):
            msg = b"client %d request %d" % (t, k) + bytes(40)
            r, s = o.ecdsa_sign(dc, o.quirk_digest(msg))
            tag = o.der_encode_sig(r, s)
            calls.append((ROLE_CLIENT, t, msg, tag))
            calls.append((ROLE_CLIENT, t, b"X" + msg[1:], tag))           # tampered at offset 0
        for ctr in (1, 2, 3):
            m = b"usig %d msg %d" % (t, ctr)
            calls.append((ROLE_USIG, t, m, o.usig_create_ui(du, m, epoch, ctr)))
        m = b"usig %d other epoch" % t
        calls.append((ROLE_USIG, t, m, o.usig_create_ui(du, m, epoch + 1, 4)))   # epoch mismatch
        m = b"usig %d tampered" % t
        ui = bytearray(o.usig_create_ui(du, m, epoch, 5))
        ui[-1] ^= 1
        calls.append((ROLE_USIG, t, m, bytes(ui)))
        ref = o.Authenticator(ks)
        seqs.append([(c, ref.verify(*c)) for c in calls])
    a = Authenticator(0)
    try:
        a.add_role(ROLE_CLIENT)
        a.add_role(ROLE_USIG)
        a.enable_usig(True)
        for t in range(T):
            for role in (ROLE_CLIENT, ROLE_USIG):
                q = ks.keys[role][t]
                a.set_public_key(role, t, q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big"))
        a.set_concurrency(lanes)
        a.set_coalescing_slots(lanes)
        a.set_coalescing(True, max_wait_us=200)
        got = [[] for _ in range(T)]
        barrier = threading.Barrier(T)

        def run(t):
            barrier.wait()
            for c, _ in seqs[t]:
                got[t].append(a.verify_status(*c))

        th = [threading.Thread(target=run, args=(t,)) for t in range(T)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        for t in range(T):
            want = [w for _, w in seqs[t]]
            assert got[t] == want, (t, got[t], want)
        assert any(w == 9 for _, w in seqs[0])  # the stream does exercise EPOCH_MISMATCH
        st = a.stage_profile()
        assert st["batches"] < sum(len(s) for s in seqs), st   # calls did share batches
    finally:
        a.close()


def test_device_decode_der_edge_cases(lib, monkeypatch):
    """The GPU decode (k_prepare) and the host decode give the same status
    for every golden DER string and 6,000 mutated encodings, used as the tag
    of an ECDSA-role call (digest = a message that verifies for the valid
    encodings) and as the signature inside a USIG UI (strict DER, trailing
    bytes), plus short UIs / certs, unknown ids and roles -- one batch each
    way, in pipeline chunks of 1,000."""
    import random
    import struct

    from minbft_amd.authenticator import Authenticator, ROLE_CLIENT, ROLE_REPLICA, ROLE_USIG
    from oracle import p256 as o
    monkeypatch.setenv("MBFT_BATCH_CHUNK", "1000")
    rng = random.Random(0xDEC0)
    d = int.from_bytes(hashlib.sha256(b"device decode").digest(), "big") % (o.N - 1) + 1
    q = o.pubkey(d)
    msg = b"device decode message " + bytes(range(40))
    r, s = o.ecdsa_sign(d, o.quirk_digest(msg))
    good = o.der_encode_sig(r, s)
    sigs = [bytes.fromhex(v["sig"]) for v in load("der.json")] + [good, good + b"\0", good[:-1]]
    # tags around the decoder's LDS staging limit (25 words: 97 bytes at the
    # worst alignment) and past it: trailing bytes, long garbage
    sigs += [good + bytes(k) for k in range(48)]
    sigs += [rng.randbytes(rng.randrange(90, 160)) for _ in range(200)]
    for _ in range(6000):
        b = bytearray(good if rng.random() < 0.85 else rng.randbytes(rng.randrange(0, 80)))
        for _ in range(rng.randrange(0, 3)):
            k = rng.randrange(3)
            if k == 0 and b:
                b[rng.randrange(len(b))] = rng.randrange(256)
            elif k == 1 and b:
                del b[rng.randrange(len(b))]
            else:
                b.insert(rng.randrange(len(b) + 1), rng.randrange(256))
        sigs.append(bytes(b))
    calls = []
    for i, sig in enumerate(sigs):
        role = ROLE_CLIENT if i % 2 else ROLE_REPLICA
        # digests from messages of 0..62 bytes (e = (msg || SHA256(""))[0:32]:
        # both the byte path below 32 bytes and the blocked read above)
        calls.append((role, 5 if i % 7 else 6, msg if i % 5 else msg[:(i // 5) % 63], sig))
        ui = struct.pack(">QQ", 1 + i % 3, 77 if i % 11 else 78) + sig
        calls.append((ROLE_USIG, 5 if i % 13 else 9, msg, ui if i % 17 else ui[:rng.randrange(0, 16)]))
        if i % 101 == 0:
            calls.append((4 + i % 3, 5, msg, sig))
    got = {}
    for dev in (False, True):
        a = Authenticator(0)
        try:
            for role in (ROLE_CLIENT, ROLE_REPLICA, ROLE_USIG):
                a.add_role(role)
                a.set_public_key(role, 5, o.pkix_encode(q))
            a.enable_usig(True)
            a.set_device_prepare(dev)
            got[dev] = [int(x) for x in a.verify_batch_flat(calls, pinned=True)]
        finally:
            a.close()
    bad = [(i, calls[i][0], calls[i][3].hex(), got[False][i], got[True][i])
           for i in range(len(calls)) if got[False][i] != got[True][i]]
    assert not bad, bad[:5]
    kinds = set(got[True])
    assert {0, 1, 2, 3, 4, 6, 7, 9, 10} <= kinds, kinds   # every decode outcome is exercised


def test_device_decode_repeated_call(lib):
    """A 20K-call pinned flat batch (past the host pool's parallel
    threshold, one 128K pipeline chunk) of one valid call repeated: all
    accepted through the device decode."""
    from minbft_amd.authenticator import Authenticator, ROLE_CLIENT
    from oracle import p256 as o
    d = 0x1234567
    q = o.pubkey(d)
    msg = b"stage profile" + bytes(40)
    r, s = o.ecdsa_sign(d, o.quirk_digest(msg))
    tag = o.der_encode_sig(r, s)
    calls = [(ROLE_CLIENT, 1, msg, tag)] * 20000
    with Authenticator(0) as a:
        a.add_role(ROLE_CLIENT)
        a.set_public_key(ROLE_CLIENT, 1, o.pkix_encode(q))
        st = a.verify_batch_flat(calls, pinned=True)
        assert (np.asarray(st) == 0).all()


@pytest.mark.parametrize("lanes", [1, 4])
def test_concurrent_lanes(lib, lanes):
    """mbft_set_concurrency: 8 threads run whole batches on one context at
    once -- verify_batch_flat through library page-locked memory (the Go
    binding's arena, GPU decode), the two-phase check_batch_flat +
    resolve_checked form (Prefetch), and verify_batch_flat from ordinary
    memory (host decode) -- while a ninth thread registers new keys (the
    exclusive table lock).  Each thread owns a client key and a USIG key
    (its own epoch state); every status equals the oracle's sequential
    result of that thread's three passes."""
    import threading

    from minbft_amd.authenticator import Authenticator, ROLE_CLIENT, ROLE_USIG
    from oracle import p256 as o
    T = 8
    ks = o.KeyStore(keys={ROLE_CLIENT: {}, ROLE_USIG: {}})
    seqs, wants = [], []
    for t in range(T):
        dc = int.from_bytes(hashlib.sha256(b"lane client %d" % t).digest(), "big") % (o.N - 1) + 1
        du = int.from_bytes(hashlib.sha256(b"lane usig %d" % t).digest(), "big") % (o.N - 1) + 1
        ks.keys[ROLE_CLIENT][t] = o.pubkey(dc)
        ks.keys[ROLE_USIG][t] = o.pubkey(du)
        calls = []
        for k in range(40):
            msg = b"lane %d request %d" % (t, k) + bytes(30)
            r, s = o.ecdsa_sign(dc, o.quirk_digest(msg))
            tag = o.der_encode_sig(r, s)
            calls.append((ROLE_CLIENT, t, msg if k % 3 else b"Y" + msg[1:], tag))
        for ctr in (1, 2, 3):
            m = b"lane usig %d msg %d" % (t, ctr)
            calls.append((ROLE_USIG, t, m, o.usig_create_ui(du, m, 500 + t, ctr)))
        m = b"lane usig %d other epoch" % t
        calls.append((ROLE_USIG, t, m, o.usig_create_ui(du, m, 501 + t, 4)))
        ref = o.Authenticator(ks)
        seqs.append(calls)
        wants.append([ref.verify(*c) for c in calls * 3])
    a = Authenticator(0)
    try:
        a.add_role(ROLE_CLIENT)
        a.add_role(ROLE_USIG)
        a.enable_usig(True)
        for t in range(T):
            for role in (ROLE_CLIENT, ROLE_USIG):
                q = ks.keys[role][t]
                a.set_public_key(role, t, q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big"))
        a.set_concurrency(lanes)
        assert a.concurrency() == lanes
        got = [[] for _ in range(T)]
        errs = []
        barrier = threading.Barrier(T + 1)

        def run(t):
            try:
                barrier.wait()
                calls = seqs[t]
                got[t] += [int(x) for x in a.verify_batch_flat(calls, pinned=True)]
                pure = a.check_batch_flat(calls, pinned=True)
                got[t] += [a.resolve_checked(*c, int(p)) for c, p in zip(calls, pure)]
                got[t] += [int(x) for x in a.verify_batch_flat(calls, pinned=False)]
            except Exception as e:  # pragma: no cover - reported below
                errs.append(repr(e))

        def register():
            barrier.wait()
            for k in range(6):
                q = o.pubkey(0x51ED + k)
                a.set_public_key(ROLE_CLIENT, 1000 + k, q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big"))

        th = [threading.Thread(target=run, args=(t,)) for t in range(T)]
        th.append(threading.Thread(target=register))
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errs, errs
        for t in range(T):
            assert got[t] == wants[t], (t, [(i, g, w) for i, (g, w) in enumerate(zip(got[t], wants[t]))
                                            if g != w][:5])
        assert any(w == 9 for w in wants[0])  # EPOCH_MISMATCH is exercised
        assert a.key_slot(ROLE_CLIENT, 1005) >= 0
    finally:
        a.close()

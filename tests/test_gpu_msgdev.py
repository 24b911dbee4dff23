"""The device message layer: mbft_validate_messages_flat over library
page-locked memory (msg_kernels.hip: checks, candidate calls, content-hash
dedup, AuthenBytes digests, DER / UI decode and key lookups on the GPU, the
in-order replay on the host) against

* the golden MinBFT streams (tests/golden/messages.json, expected results
  from the oracle's sequential validators: every validator branch, stream
  stop, panic),
* the oracle's sequential validators on C3 streams (f = 1, 4, 16) with and
  without injected faults, and past 4,096 messages,
* the host message layer (mbft_validate_messages, itself pinned by the tests
  above and tests/test_gpu_configs.py) on adversarial mutations of C3
  streams: tampered and truncated certificates, malformed / trailing DER,
  unknown signers, zero counters, equal calls behind different bytes,
* and the same flat batch outside page-locked memory (the host fallback).
Argument errors (a type out of range, a field past the arena) return
MBFT_ERR_ARG without touching any result."""
import copy
import random

import numpy as np
import pytest

from test_gpu_authen import _msgs, load
from test_gpu_configs import _c3_streams, _fast_oracle

pytestmark = pytest.mark.gpu


def _auth_for(keys, window=16):
    from minbft_amd.authenticator import Authenticator
    from oracle import p256 as o
    a = Authenticator(0)
    a.set_key_window(window)
    for role, m in keys.items():
        a.add_role(role)
        for id_, q in m.items():
            a.set_public_key(role, id_, o.pkix_encode(q))
    a.enable_usig(True)
    return a


def test_flat_golden_streams(lib):
    """Every golden stream, device path and host fallback."""
    from minbft_amd.authenticator import Authenticator
    fx = load("messages.json")
    for sq in fx["sequences"]:
        msgs = _msgs(sq["msgs"])
        for pinned in (True, False):
            with Authenticator(0) as a:
                for role, m in fx["keystore"].items():
                    a.add_role(int(role))
                    for id_, pk in m.items():
                        a.set_public_key(int(role), int(id_), bytes.fromhex(pk))
                a.enable_usig(True)
                got = a.validate_messages_via_flat(msgs, sq["n"], sq["flags"], pinned=pinned)
            bad = [(i, int(g), w) for i, (g, w) in enumerate(zip(got, sq["expect"])) if g != w]
            assert not bad, (pinned, bad[:10])


@pytest.mark.parametrize("f", [1, 4, 16])
def test_flat_c3_vs_oracle(lib, monkeypatch, f):
    from oracle import p256 as o
    _fast_oracle(monkeypatch)
    rng = random.Random(0xF1A7 + f)
    for faults in (False, True):
        n, msgs, keys = _c3_streams(f, 3, rng, faults)
        ks = o.KeyStore()
        ks.keys = {role: dict(m) for role, m in keys.items()}
        want = o.validate_messages(o.Authenticator(ks), msgs, n, 0)
        a = _auth_for(keys)
        try:
            got = a.validate_messages_via_flat(msgs, n, 0)
        finally:
            a.close()
        bad = [(i, int(g), w) for i, (g, w) in enumerate(zip(got, want)) if g != w]
        assert not bad, (f, faults, bad[:10])


def test_flat_c3_large_vs_oracle_and_host(lib, monkeypatch):
    """4,118 messages at f = 16 with the faults: the pool-sized host paths
    and the device path agree with the oracle."""
    from oracle import p256 as o
    _fast_oracle(monkeypatch)
    rng = random.Random(0xF1A7B16)
    n, msgs, keys = _c3_streams(16, 121, rng, True)
    assert len(msgs) > 4096
    ks = o.KeyStore()
    ks.keys = {role: dict(m) for role, m in keys.items()}
    want = np.array(o.validate_messages(o.Authenticator(ks), msgs, n, 0))
    a = _auth_for(keys)
    try:
        got_dev = a.validate_messages_via_flat(msgs, n, 0)
        got_host = a.validate_messages(msgs, n, 0)
        got_dev2 = a.validate_messages_via_flat(msgs, n, 0)  # epochs captured now: same results
    finally:
        a.close()
    assert (got_dev == want).all(), np.nonzero(got_dev != want)[0][:10]
    assert (got_host == want).all()
    assert (got_dev2 == want).all()


def _mutate(msgs, rng):
    """Adversarial variants of C3 messages (each on a stream of its own so
    that stream stops do not hide the later ones)."""
    out = list(msgs)
    cms = [m for m in msgs if m.type == 4]
    prs = [m for m in msgs if m.type == 3]
    sid = 9000

    def add(m):
        nonlocal sid
        m.stream = sid
        sid += 1
        out.insert(rng.randrange(len(out) + 1), m)

    for _ in range(40):
        b = copy.copy(rng.choice(cms))
        kind = rng.randrange(13)
        if kind == 0:    # flipped cert byte (bad signature)
            c = bytearray(b.ui_cert)
            c[rng.randrange(len(c))] ^= 1 << rng.randrange(8)
            b.ui_cert = bytes(c)
        elif kind == 1:  # cert shorter than 8 bytes
            b.ui_cert = b.ui_cert[:rng.randrange(8)]
        elif kind == 2:  # trailing bytes after the USIG DER signature (past the LDS staging limit too)
            b.ui_cert = b.ui_cert + bytes(rng.randrange(1, 40))
        elif kind == 3:  # malformed DER in the USIG cert
            b.ui_cert = b.ui_cert[:8] + b"\x31" + b.ui_cert[9:]
        elif kind == 4:  # malformed DER in the embedded REQUEST's signature (Go panics)
            b.sig = b"\x30\x81" + b.sig[2:]
        elif kind == 5:  # unknown USIG id
            b.replica_id = 77
        elif kind == 6:  # zero COMMIT counter
            b.ui_counter = 0
        elif kind == 7:  # zero PREPARE counter
            b.prep_ui_counter = 0
        elif kind == 8:  # COMMIT from the primary
            b.replica_id = b.prep_replica_id
        elif kind == 9:  # not the primary for the view
            b.view = 1
        elif kind == 10:  # equal call content behind fresh bytes (dedup by content)
            b.ui_cert = bytes(bytearray(b.ui_cert))
            b.op = bytes(bytearray(b.op))
        elif kind == 11:  # trailing bytes after the embedded REQUEST's signature
            b.sig = b.sig + bytes(rng.randrange(1, 40))
        else:            # a REQUEST / PREPARE repeated on its own
            b = copy.copy(rng.choice(prs))
        add(b)
    r = copy.copy(rng.choice(cms))  # a REPLY in a replica's stream: the validator panics
    r.type = 2
    out.append(r)
    return out


@pytest.mark.parametrize("seed", [1, 2])
def test_flat_adversarial_vs_host_layer(lib, seed):
    """Mutated C3 streams: device path == host message layer, result by
    result (including panics and stream stops), with and without the stop
    flags; plus a REPLY in a replica's stream (panic) at the end."""
    from oracle import p256 as o
    rng = random.Random(0xADF1A7 + seed)
    n, msgs, keys = _c3_streams(4, 40, rng, True)
    msgs = _mutate(msgs, rng)
    a = _auth_for(keys)
    try:
        for flags in (0, 1, 2, 3):
            # fresh epoch state each time: both paths see the same start
            a.clear_keys()
            for role, m in keys.items():
                for id_, q in m.items():
                    a.set_public_key(role, id_, o.pkix_encode(q))
            host = a.validate_messages(msgs, n, flags)
            a.clear_keys()
            for role, m in keys.items():
                for id_, q in m.items():
                    a.set_public_key(role, id_, o.pkix_encode(q))
            dev = a.validate_messages_via_flat(msgs, n, flags)
            bad = np.nonzero(host != dev)[0]
            assert not len(bad), (flags, [(int(i), int(host[i]), int(dev[i])) for i in bad[:10]])
            assert (host != 0).sum() >= 10
    finally:
        a.close()


def test_flat_argument_errors(lib):
    """A type out of range or a field outside the arena -> MBFT_ERR_ARG on
    the device path (no byte read), and the results array untouched."""
    from minbft_amd import _lib
    from minbft_amd.authenticator import GpuError
    rng = random.Random(5)
    n, msgs, keys = _c3_streams(1, 2, rng, False)
    a = _auth_for(keys)
    try:
        arr, keep = _lib.make_messages(msgs)
        packed = np.frombuffer(arr, dtype=_lib.message_dtype(), count=len(msgs))
        recs, arena = a.pack_messages(packed, pinned=True)
        ok = a.validate_messages_flat(recs, arena, n)
        assert (ok == 0).all()
        for field, value in (("type", 9), ("sig_off", arena.nbytes), ("ui_cert_len", 1 << 20)):
            k = len(msgs) // 2
            saved = int(recs[k][field])
            recs[k][field] = value  # in place: recs must stay in page-locked memory
            out = np.full(len(msgs), 12345, dtype=np.int32)
            with pytest.raises(GpuError):
                a.validate_messages_flat(recs, arena, n, 0, out)
            assert (out == 12345).all()
            recs[k][field] = saved
        assert (a.validate_messages_flat(recs, arena, n) == 0).all()
        # past 65,536 records (8 record chunks, a two-stage verify): the error
        # is found after every chunk's kernels and the first verify stage are
        # queued; the library drains its streams before returning, so the
        # next call's uploads cannot overwrite buffers a stale kernel reads
        # (msgdev.cpp validate_flat_device)
        from minbft_amd.authenticator import host_array
        reps = -(-70000 // len(msgs))
        big = host_array(len(msgs) * reps, dtype=recs.dtype)
        for j in range(reps):
            big[j * len(msgs):(j + 1) * len(msgs)] = recs
            big["stream"][j * len(msgs):(j + 1) * len(msgs)] = recs["stream"] + 16 * j
        want = a.validate_messages_flat(big, arena, n)
        assert (want == 0).all()
        for k in (5, len(big) // 2, len(big) - 1):
            saved = int(big[k]["sig_off"])
            big[k]["sig_off"] = arena.nbytes + 4
            with pytest.raises(GpuError):
                a.validate_messages_flat(big, arena, n)
            big[k]["sig_off"] = saved
            assert (a.validate_messages_flat(big, arena, n) == want).all()
        del keep
    finally:
        a.close()


def test_flat_random_records_vs_host_layer(lib):
    """20,000 random records over a random arena -- random types (1..5),
    ids, views, counters, field offsets and lengths anywhere inside the
    arena, signatures and certs that are mostly garbage DER (with some valid
    UIs spliced in) -- through the device path and through the host layer
    (the same batch outside page-locked memory): identical results, and no
    byte outside the arena is read (the arena is sized exactly)."""
    from minbft_amd import _lib
    rng = np.random.default_rng(0x5EED)
    n, msgs, keys = _c3_streams(2, 30, random.Random(77), False)
    a = _auth_for(keys)
    try:
        arr, keep = _lib.make_messages(msgs)
        packed = np.frombuffer(arr, dtype=_lib.message_dtype(), count=len(msgs))
        recs_ok, arena_ok = a.pack_messages(packed, pinned=False)
        m = 20000
        nbytes = 1 << 20
        arena = rng.integers(0, 256, size=nbytes, dtype=np.uint8)
        arena[: arena_ok.nbytes] = arena_ok  # real messages' bytes at the front
        recs = np.zeros(m, dtype=_lib.msg_rec_dtype())
        recs["type"] = rng.integers(1, 6, size=m)
        recs["stream"] = rng.integers(0, 50, size=m)
        recs["replica_id"] = rng.integers(0, n + 2, size=m)
        recs["prep_replica_id"] = rng.integers(0, n + 2, size=m)
        recs["client_id"] = rng.choice([7, 8], size=m)
        recs["view"] = rng.integers(0, 3, size=m)
        recs["seq"] = rng.integers(0, 40, size=m)
        recs["ui_counter"] = rng.integers(0, 40, size=m)
        recs["prep_ui_counter"] = rng.integers(0, 40, size=m)
        for f in ("op", "sig", "ui_cert", "prep_ui_cert"):
            ln = rng.integers(0, 120, size=m)
            ln[rng.random(m) < 0.05] = 0
            recs[f + "_len"] = ln
            recs[f + "_off"] = rng.integers(0, nbytes - ln + 1)
        # a quarter of the records are real messages (valid calls, dedup hits)
        pick = rng.integers(0, len(recs_ok), size=m // 4)
        recs[: m // 4] = recs_ok[pick]
        rng.shuffle(recs)
        from minbft_amd.authenticator import host_array
        from oracle import p256 as o
        recs_p = host_array(m, _lib.msg_rec_dtype())
        recs_p[:] = recs
        arena_p = host_array(nbytes)
        arena_p[:] = arena

        def fresh():  # the same starting epoch state for both paths
            a.clear_keys()
            for role, mm in keys.items():
                for id_, q in mm.items():
                    a.set_public_key(role, id_, o.pkix_encode(q))

        for flags in (3, 0):
            fresh()
            host = a.validate_messages_flat(recs, arena, n, flags)  # ordinary memory: the host layer
            fresh()
            dev = a.validate_messages_flat(recs_p, arena_p, n, flags)
            bad = np.nonzero(host != dev)[0]
            assert not len(bad), (flags, [(int(i), int(host[i]), int(dev[i])) for i in bad[:10]])
            if flags == 3:  # no stream or panic stop: both outcomes plentiful
                assert (host == 0).sum() > 0 and (host != 0).sum() > m // 2
        del keep
    finally:
        a.close()


def _check_resolve(a, msgs, n, pinned=True, order=None, bulk=False):
    """mbft_check_messages_flat, then mbft_resolve_message per message in
    `order` (default: message order), or mbft_resolve_messages over all."""
    from minbft_amd import _lib
    arr, keep = _lib.make_messages(msgs)
    packed = np.frombuffer(arr, dtype=_lib.message_dtype(), count=len(msgs))
    recs, arena = a.pack_messages(packed, pinned)
    with a.check_messages_flat(recs, arena, n) as b:
        out = np.zeros(len(msgs), dtype=np.int32)
        if bulk:
            b.resolve_range(0, len(msgs), out)
        for i in ([] if bulk else range(len(msgs)) if order is None else order):
            out[i] = b.resolve(i)
    del keep
    return out


def test_check_resolve_golden_streams(lib):
    """Resolving every message in order == the one-call validation with no
    stream / panic stop (each message's own result), on every golden stream,
    from library page-locked memory and from ordinary memory (staged)."""
    from minbft_amd.authenticator import Authenticator
    from oracle import p256 as o
    fx = load("messages.json")
    for sq in fx["sequences"]:
        msgs = _msgs(sq["msgs"])
        got = {}
        for form in ("validate", "pinned", "staged", "bulk", "small"):
            with Authenticator(0) as a:
                for role, m in fx["keystore"].items():
                    a.add_role(int(role))
                    for id_, pk in m.items():
                        a.set_public_key(int(role), int(id_), bytes.fromhex(pk))
                a.enable_usig(True)
                # the device message layer, or (form "small") the small route
                # for every batch up to 64 messages
                a.set_small_check(64 if form == "small" else 0)
                if form == "validate":
                    got[form] = a.validate_messages_via_flat(
                        msgs, sq["n"], o.VF_NO_STREAM_STOP | o.VF_NO_PANIC_STOP)
                else:
                    got[form] = _check_resolve(a, msgs, sq["n"], pinned=form != "staged",
                                               bulk=form == "bulk")
        for form in ("pinned", "staged", "bulk", "small"):
            bad = [(i, int(g), int(w)) for i, (g, w) in enumerate(zip(got[form], got["validate"])) if g != w]
            assert not bad, (form, bad[:10])


@pytest.mark.parametrize("lanes", [1, 4])
def test_check_resolve_c3(lib, monkeypatch, lanes):
    """C3 streams with faults (f = 4) and past 4,096 messages (f = 16): the
    stepwise form against the oracle's validators with no stream stop, on
    the context and on concurrency lanes."""
    from oracle import p256 as o
    _fast_oracle(monkeypatch)
    for f, nreq in ((4, 3), (16, 121)):
        rng = random.Random(0xC4EC + f)
        n, msgs, keys = _c3_streams(f, nreq, rng, True)
        ks = o.KeyStore()
        ks.keys = {role: dict(m) for role, m in keys.items()}
        want = np.array(o.validate_messages(o.Authenticator(ks), msgs, n,
                                            o.VF_NO_STREAM_STOP | o.VF_NO_PANIC_STOP))
        a = _auth_for(keys)
        try:
            a.set_concurrency(lanes)
            got = _check_resolve(a, msgs, n)
        finally:
            a.close()
        assert (got == want).all(), (f, np.nonzero(got != want)[0][:10])


@pytest.mark.parametrize("small", [0, 16])
def test_unresolved_message_captures_nothing(lib, monkeypatch, small):
    """The epoch state moves only when a message is resolved: a checked but
    never-resolved COMMIT whose UI has counter 1 captures no epoch (as a
    message the reference never validates, because an earlier one failed),
    so the replica's counter-2 UI is still an epoch mismatch; once resolved,
    it captures and the counter-2 UI is accepted."""
    from oracle import p256 as o
    _fast_oracle(monkeypatch)
    rng = random.Random(0xEC0)
    n, msgs, keys = _c3_streams(1, 2, rng, False)
    commits = [m for m in msgs if m.type == o.MSG_COMMIT]
    rid = commits[0].replica_id
    first = [m for m in commits if m.replica_id == rid]
    assert [m.ui_counter for m in first] == [1, 2]
    a = _auth_for(keys)
    try:
        a.set_small_check(small)  # 0: the device message layer; 16: the small route (8 messages)
        from minbft_amd import _lib
        arr, keep = _lib.make_messages(msgs)
        packed = np.frombuffer(arr, dtype=_lib.message_dtype(), count=len(msgs))
        recs, arena = a.pack_messages(packed, True)
        i1 = msgs.index(first[0])
        ab2 = o.msg_authen_bytes(first[1])
        tag2 = o.ui_marshal(2, first[1].ui_cert)
        with a.check_messages_flat(recs, arena, n) as b:
            assert a.verify_status(o.ROLE_USIG, rid, ab2, tag2) == o.EPOCH_MISMATCH
            # resolve the messages up to that COMMIT (its PREPARE / REQUEST first)
            for i in range(i1 + 1):
                assert b.resolve(i) == 0, i
            assert a.verify_status(o.ROLE_USIG, rid, ab2, tag2) == 0
        del keep
    finally:
        a.close()


def test_check_resolve_adversarial(lib):
    """The adversarial mutations (malformed DER, panics, unknown ids, zero
    counters, trailing bytes...): stepwise == the host message layer with
    no stream / panic stop."""
    from oracle import p256 as o
    rng = random.Random(0xADF1A71)
    n, msgs, keys = _c3_streams(4, 40, rng, True)
    msgs = _mutate(msgs, rng)
    a = _auth_for(keys)
    try:
        host = a.validate_messages(msgs, n, o.VF_NO_STREAM_STOP | o.VF_NO_PANIC_STOP)
        a.clear_keys()
        for role, m in keys.items():
            for id_, q in m.items():
                a.set_public_key(role, id_, o.pkix_encode(q))
        got = _check_resolve(a, msgs, n)
    finally:
        a.close()
    bad = np.nonzero(host != got)[0]
    assert not len(bad), [(int(i), int(host[i]), int(got[i])) for i in bad[:10]]
    assert (got != 0).sum() >= 10


def test_check_resolve_chunked_and_one_wait(lib, monkeypatch):
    """Every device check form: a small batch checked with one host wait (<=
    1,365 messages: the unique-call count kept on the device, the verifier
    stopping at it), one chunk with two waits (4,114 messages), and a batch
    past 65,536 messages (8 record chunks, two verify stages) -- the C3
    streams with faults tiled 16 times (repeats are identical calls: dedup
    hits across chunks) -- each resolved in order equals the one-call
    validation with no stream / panic stop of the same batch."""
    from minbft_amd import _lib
    from oracle import p256 as o
    _fast_oracle(monkeypatch)
    rng = random.Random(0x0E1A)
    n, msgs, keys = _c3_streams(16, 121, rng, True)
    a = _auth_for(keys)
    try:
        arr, keep = _lib.make_messages(msgs)
        packed = np.frombuffer(arr, dtype=_lib.message_dtype(), count=len(msgs))
        for reps in (0, 1, 16):  # 0: the first 1,300 messages (one wait)
            if reps == 0:
                tiled = np.ascontiguousarray(packed[:1300])
            else:
                tiled = np.ascontiguousarray(np.tile(packed, reps))
            recs, arena = a.pack_messages(tiled, True)
            want = a.validate_messages_flat(recs, arena, n, o.VF_NO_STREAM_STOP | o.VF_NO_PANIC_STOP)
            with a.check_messages_flat(recs, arena, n) as b:
                got = b.resolve_range(0, tiled.shape[0])
            assert (got == want).all(), (reps, np.nonzero(got != want)[0][:10])
            assert (want == 0).any() and (reps == 0 or (want != 0).any())
        assert tiled.shape[0] > 65536
        del keep
    finally:
        a.close()

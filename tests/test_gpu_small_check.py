"""The small check route (mbft_set_small_check, msgdev.cpp check_small +
messages.cpp check_messages_small): a check of at most 512 messages (the default) builds its
checks and candidate calls on the host, deduplicates them (content hash, full
compares), hashes
the AuthenBytes digests on the host and verifies the unique calls in one
small-batch launch from zero-copy staging -- the latency path of the Go
core's one-message-at-a-time streams (core/message-handling.go:204-246,
:399).  Every result must equal the device message layer's
(mbft_set_small_check(0)) and the oracle's sequential validators:

* the golden MinBFT streams, checked in windows of 1, 3 and 16 messages and
  resolved in order, pinned and unpinned;
* C3 streams with faults (f = 1, 4) in windows of 1, 2, 5, 16, 64, 256 and 512
  (past the zero-copy and host-inverse sizes: 256 messages hold up to 768
  calls);
* the adversarial mutations (malformed / trailing DER, unknown ids, zero
  counters, REPLY in a replica stream, equal calls behind fresh bytes) in
  random windows of 1..16, against the host message layer;
* the boundary: 16 messages small, 17 through the device layer, same results;
* argument errors (type out of range, a field past the arena) -> MBFT_ERR_ARG;
* one-message checks from concurrent stream threads with check coalescing on
  (small merged passes), on 1 and 4 lanes.
"""
import random
import threading

import numpy as np
import pytest

from test_gpu_authen import _msgs, load
from test_gpu_configs import _c3_streams, _fast_oracle
from test_gpu_msgdev import _auth_for, _mutate

pytestmark = pytest.mark.gpu

NO_STOP = 3  # MBFT_VF_NO_STREAM_STOP | MBFT_VF_NO_PANIC_STOP


def _packed(a, msgs, pinned=True):
    from minbft_amd import _lib
    arr, keep = _lib.make_messages(msgs)
    packed = np.frombuffer(arr, dtype=_lib.message_dtype(), count=len(msgs))
    recs, arena = a.pack_messages(packed, pinned)
    del keep
    return recs, arena


def _windows(a, msgs, n, sizes, pinned=True):
    """Check msgs in consecutive windows (sizes cycled), resolving each
    window's messages in order before the next check: the core's loop."""
    out = np.zeros(len(msgs), dtype=np.int64)
    i = k = 0
    while i < len(msgs):
        w = sizes[k % len(sizes)]
        k += 1
        part = msgs[i:i + w]
        recs, arena = _packed(a, part, pinned)
        with a.check_messages_flat(recs, arena, n) as b:
            for j in range(len(part)):
                out[i + j] = b.resolve(j)
        i += len(part)
    return out


def _oracle_want(keys, msgs, n):
    from oracle import p256 as o
    ks = o.KeyStore()
    ks.keys = {role: dict(m) for role, m in keys.items()}
    return np.array(o.validate_messages(o.Authenticator(ks), msgs, n, NO_STOP))


def test_small_check_golden_streams(lib):
    from minbft_amd.authenticator import Authenticator
    fx = load("messages.json")
    for sq in fx["sequences"]:
        msgs = _msgs(sq["msgs"])

        def ctx():
            a = Authenticator(0)
            for role, m in fx["keystore"].items():
                a.add_role(int(role))
                for id_, pk in m.items():
                    a.set_public_key(int(role), int(id_), bytes.fromhex(pk))
            a.enable_usig(True)
            return a
        with ctx() as a:
            want = a.validate_messages_via_flat(msgs, sq["n"], NO_STOP)
        for sizes in ([1], [3], [16]):
            for pinned in (True, False):
                with ctx() as a:
                    got = _windows(a, msgs, sq["n"], sizes, pinned)
                bad = [(i, int(g), int(w)) for i, (g, w) in enumerate(zip(got, want)) if g != w]
                assert not bad, (sizes, pinned, bad[:10])


@pytest.mark.parametrize("f", [1, 4])
def test_small_check_c3_windows_vs_oracle(lib, monkeypatch, f):
    _fast_oracle(monkeypatch)
    rng = random.Random(0x5A11 + f)
    n, msgs, keys = _c3_streams(f, 4 if f == 4 else 140, rng, True)
    want = _oracle_want(keys, msgs, n)
    # 512: past 256 unique calls (the small route's verify without zero-copy)
    for sizes in ([1], [2], [5], [16], [1, 16, 3], [64], [256], [512]):
        a = _auth_for(keys)
        try:
            got = _windows(a, msgs, n, sizes)
        finally:
            a.close()
        bad = np.nonzero(got != want)[0]
        assert not len(bad), (sizes, [(int(i), int(got[i]), int(want[i])) for i in bad[:10]])
    assert (want != 0).any() and (want == 0).any()


def test_small_check_adversarial_vs_host_layer(lib):
    rng = random.Random(0x5A1AD)
    n, msgs, keys = _c3_streams(4, 12, rng, True)
    msgs = _mutate(msgs, rng)
    from oracle import p256 as o
    a = _auth_for(keys)
    try:
        host = a.validate_messages(msgs, n, NO_STOP)
        for trial in range(2):
            a.clear_keys()
            for role, m in keys.items():
                for id_, q in m.items():
                    a.set_public_key(role, id_, o.pkix_encode(q))
            sizes = [rng.randrange(1, 17) for _ in range(64)] if trial else [16]
            got = _windows(a, msgs, n, sizes)
            bad = np.nonzero(host != got)[0]
            assert not len(bad), (trial, [(int(i), int(host[i]), int(got[i])) for i in bad[:10]])
    finally:
        a.close()
    assert (host != 0).sum() >= 10


def test_small_boundary_and_device_route_agree(lib, monkeypatch):
    """At a small-route maximum of 16: 16 messages (small route), 17 (the
    device layer), the same 16 with the small route off; identical
    per-message results.  And a batch with no authenticator call at all
    (not-primary / view-change messages)."""
    from oracle import p256 as o
    _fast_oracle(monkeypatch)
    rng = random.Random(0xB0D)
    n, msgs, keys = _c3_streams(2, 4, rng, True)
    want = _oracle_want(keys, msgs, n)
    for m_, small in ((16, 16), (17, 16), (16, 0), (17, 17)):
        a = _auth_for(keys)
        try:
            a.set_small_check(small)
            got = _windows(a, msgs, n, [m_])
        finally:
            a.close()
        assert (got == want).all(), (m_, small, np.nonzero(got != want)[0][:10])
    none = [o.Msg(type=o.MSG_REQ_VIEW_CHANGE, stream=1, view=4),
            o.Msg(type=o.MSG_PREPARE, stream=2, replica_id=1, view=0, client_id=7, seq=1, op=b"x",
                  sig=b"", ui_counter=1, ui_cert=b"")]
    a = _auth_for(keys)
    try:
        got = _windows(a, none, n, [2])
    finally:
        a.close()
    assert list(got) == [o.ST_NOT_IMPLEMENTED << 8, o.ST_NOT_PRIMARY << 8]


def test_small_check_argument_errors(lib):
    from minbft_amd.authenticator import GpuError
    rng = random.Random(0xA4)
    n, msgs, keys = _c3_streams(1, 2, rng, False)
    a = _auth_for(keys)
    try:
        recs, arena = _packed(a, msgs[:6])
        for field, value, what in (("type", 9, "unknown message type"),
                                   ("sig_off", arena.nbytes, "outside the byte arena"),
                                   ("ui_cert_len", 1 << 20, "outside the byte arena")):
            saved = int(recs[3][field])
            recs[3][field] = value
            with pytest.raises(GpuError) as ei:
                a.check_messages_flat(recs, arena, n)
            assert what in str(ei.value) or "(-1)" in str(ei.value), str(ei.value)
            recs[3][field] = saved
        with a.check_messages_flat(recs, arena, n) as b:
            assert [b.resolve(i) for i in range(6)] == [0] * 6
    finally:
        a.close()


@pytest.mark.parametrize("lanes", [1, 4])
def test_small_coalesced_single_messages(lib, monkeypatch, lanes):
    """A thread per stream checks its messages one at a time (the core's
    loop at low load) with check coalescing on: concurrent single-message
    checks merge into small passes; every result equals the oracle's."""
    _fast_oracle(monkeypatch)
    rng = random.Random(0xC1 + lanes)
    n, msgs, keys = _c3_streams(2, 6, rng, False)
    want = _oracle_want(keys, msgs, n)
    streams = {}
    for i, m in enumerate(msgs):
        streams.setdefault(m.stream, []).append(i)
    a = _auth_for(keys)
    got = np.full(len(msgs), -1, dtype=np.int64)
    errs = []
    try:
        a.set_concurrency(lanes)
        a.set_check_coalescing(True)
        a.check_coalescing_stats()
        packed = {i: _packed(a, [msgs[i]]) for i in range(len(msgs))}
        gate = threading.Barrier(len(streams))

        def run(idx):
            gate.wait()
            try:
                for i in idx:
                    recs, arena = packed[i]
                    with a.check_messages_flat(recs, arena, n) as b:
                        got[i] = b.resolve(0)
            except Exception as e:  # noqa: BLE001 -- handed to the test
                errs.append(e)
        th = [threading.Thread(target=run, args=(idx,)) for idx in streams.values()]
        for t in th:
            t.start()
        for t in th:
            t.join()
        stats = a.check_coalescing_stats()
    finally:
        a.close()
    assert not errs, errs
    assert (got == want).all(), np.nonzero(got != want)[0][:10]
    assert stats["batches"] == len(msgs) and stats["messages"] == len(msgs), stats

"""Coalesced message-batch checks (mbft_set_check_coalescing): concurrent
mbft_check_messages_flat callers -- a replica's per-connection stream loops
(core/message-handling.go:250-275) -- merged into one device pass must hand
every caller exactly the batch it would have got alone:

* C3 streams with faults split into consecutive batches, checked from
  threads at once (one merged pass: the leader waits for company), then
  resolved in message order == the oracle's sequential validators with no
  stream stop; on the context and on concurrency lanes;
* a caller whose records are invalid (unknown type, a field past its arena)
  gets MBFT_ERR_ARG alone, the others their results;
* callers with different n_replicas are never merged (isPrimary reads n):
  each group against its own oracle run.
"""
import random
import threading

import numpy as np
import pytest

from test_gpu_configs import _c3_streams, _fast_oracle
from test_gpu_msgdev import _auth_for

pytestmark = pytest.mark.gpu


def _packed(a, msgs):
    from minbft_amd import _lib
    arr, keep = _lib.make_messages(msgs)
    packed = np.frombuffer(arr, dtype=_lib.message_dtype(), count=len(msgs))
    recs, arena = a.pack_messages(packed, True)
    del keep
    return recs, arena


def _check_concurrently(a, jobs):
    """jobs: [(recs, arena, n_replicas)] checked from one thread each, all
    released at once; returns [MessageBatch or the exception]."""
    out = [None] * len(jobs)
    gate = threading.Barrier(len(jobs))

    def run(k):
        recs, arena, n = jobs[k]
        gate.wait()
        try:
            out[k] = a.check_messages_flat(recs, arena, n)
        except Exception as e:  # noqa: BLE001 -- handed to the test
            out[k] = e
    th = [threading.Thread(target=run, args=(k,)) for k in range(len(jobs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    return out


def _want(keys, msgs, n):
    from oracle import p256 as o
    ks = o.KeyStore()
    ks.keys = {role: dict(m) for role, m in keys.items()}
    return np.array(o.validate_messages(o.Authenticator(ks), msgs, n,
                                        o.VF_NO_STREAM_STOP | o.VF_NO_PANIC_STOP))


@pytest.mark.parametrize("lanes", [1, 4])
def test_coalesced_c3_batches(lib, monkeypatch, lanes):
    _fast_oracle(monkeypatch)
    rng = random.Random(0xC0A1 + lanes)
    n, msgs, keys = _c3_streams(4, 40, rng, True)
    want = _want(keys, msgs, n)
    a = _auth_for(keys)
    try:
        a.set_concurrency(lanes)
        a.set_check_coalescing(True, max_wait_us=50000)
        a.check_coalescing_stats()  # reset
        K = 7
        cuts = [len(msgs) * k // K for k in range(K + 1)]
        parts = [msgs[cuts[k]:cuts[k + 1]] for k in range(K)]
        jobs = []
        for p in parts:
            recs, arena = _packed(a, p)
            jobs.append((recs, arena, n))
        batches = _check_concurrently(a, jobs)
        stats = a.check_coalescing_stats()
        got = np.zeros(len(msgs), dtype=np.int64)
        for k, b in enumerate(batches):
            assert not isinstance(b, Exception), b
            with b:
                for i in range(len(parts[k])):
                    got[cuts[k] + i] = b.resolve(i)
        bad = np.nonzero(got != want)[0]
        assert not len(bad), [(int(i), int(got[i]), int(want[i])) for i in bad[:10]]
        assert stats["batches"] == K and stats["messages"] == len(msgs), stats
        assert stats["passes"] < K, stats  # merged (the leader waited 50 ms for company)
    finally:
        a.close()


@pytest.mark.parametrize("small", [0, 256])
def test_coalesced_bad_caller_fails_alone(lib, monkeypatch, small):
    """(small: the merged pass through the device message layer, or the
    small route.)"""
    from minbft_amd.authenticator import GpuError
    _fast_oracle(monkeypatch)
    rng = random.Random(0xBAD)
    n, msgs, keys = _c3_streams(2, 12, rng, False)
    want = _want(keys, msgs, n)
    a = _auth_for(keys)
    try:
        a.set_small_check(small)
        a.set_check_coalescing(True, max_wait_us=50000)
        half = len(msgs) // 2
        r0, b0 = _packed(a, msgs[:half])
        r1, b1 = _packed(a, msgs[half:])
        rt, bt = _packed(a, msgs[:4])
        rt["type"][2] = 9                         # unknown message type
        rf, bf = _packed(a, msgs[:4])
        rf["op_off"][1] = bf.nbytes               # a field past its own arena
        rf["op_len"][1] = 1
        out = _check_concurrently(a, [(r0, b0, n), (rt, bt, n), (r1, b1, n), (rf, bf, n)])
        for e in (out[1], out[3]):  # MBFT_ERR_ARG, that caller alone
            assert isinstance(e, GpuError) and "failed (-1)" in str(e), out
        got = []
        for b in (out[0], out[2]):
            assert not isinstance(b, Exception), b
            with b:
                got += [b.resolve(i) for i in range(b.n)]
        assert (np.array(got) == want).all()
    finally:
        a.close()


@pytest.mark.parametrize("small", [0, 256])
def test_coalesced_groups_by_n_replicas(lib, monkeypatch, small):
    """The same messages checked at once under two n_replicas (isPrimary
    differs): two passes, never one; each batch, resolved alone on a fresh
    context, equals the oracle at its own n."""
    _fast_oracle(monkeypatch)
    rng = random.Random(0x2F)
    n1, msgs, keys = _c3_streams(1, 10, rng, True)
    n2 = n1 + 2
    for m in msgs:  # view 3: primary 0 at n = 3 (3 % 3), a backup at n = 5
        if m.type != 1:
            m.view = 3
    want = {n1: _want(keys, msgs, n1), n2: _want(keys, msgs, n2)}
    assert (want[n1] != want[n2]).any()  # the primary check tells them apart
    for pick in (0, 1):
        a = _auth_for(keys)
        try:
            a.set_small_check(small)
            a.set_check_coalescing(True, max_wait_us=30000)
            a.check_coalescing_stats()
            jobs = []
            for nn in (n1, n2):
                recs, arena = _packed(a, msgs)
                jobs.append((recs, arena, nn))
            out = _check_concurrently(a, jobs)
            stats = a.check_coalescing_stats()
            assert stats["passes"] == 2 and stats["batches"] == 2, stats
            for b in out:
                assert not isinstance(b, Exception), b
            nn = (n1, n2)[pick]
            with out[pick] as b:
                got = np.array([b.resolve(i) for i in range(b.n)])
            out[1 - pick].close()
            assert (got == want[nn]).all(), (nn, np.nonzero(got != want[nn])[0][:10])
        finally:
            a.close()

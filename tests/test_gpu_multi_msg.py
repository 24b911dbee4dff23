"""The message layer over every engine (mbft_ctx_add_device; VERDICT r4
missing #2): with engines on more devices, a device pass of at least
2 x shard_min messages is split into contiguous record shards, each shard's
records and only the arena bytes they reference checked on its own engine at
once, and concurrent passes lease lanes on every device.  Results must equal
the one-engine context's, message by message:

* mbft_validate_messages_flat (in-order replay on the host after the
  sharded check) on C3 streams with faults and adversarial mutations, with
  and without the stream / panic stops;
* mbft_check_messages_flat + mbft_resolve_message, on the context
  (concurrency 1) and on lanes (concurrency 2: lanes on every engine);
* coalesced passes from concurrent callers on those lanes;
* argument errors found in any shard -> MBFT_ERR_ARG.
On a one-GPU box the extra engines sit on device 0 (same code path: own
thread, streams, tables and lanes)."""
import random
import threading

import numpy as np
import pytest

from test_gpu_configs import _c3_streams, _fast_oracle
from test_gpu_msgdev import _auth_for, _mutate
from test_gpu_multi import _extra_devices

pytestmark = pytest.mark.gpu


def _multi(keys, extra=2, shard_min=64):
    a = _auth_for(keys)
    for d in _extra_devices(extra):
        a.add_device(d)
    a.set_shard_min(shard_min)
    a.set_small_check(0)  # every pass through the device layer (the sharded path)
    return a


def _fresh(a, keys):
    from oracle import p256 as o
    a.clear_keys()
    for role, m in keys.items():
        for id_, q in m.items():
            a.set_public_key(role, id_, o.pkix_encode(q))


def _packed(a, msgs):
    from minbft_amd import _lib
    arr, keep = _lib.make_messages(msgs)
    packed = np.frombuffer(arr, dtype=_lib.message_dtype(), count=len(msgs))
    recs, arena = a.pack_messages(packed, True)
    del keep
    return recs, arena


def test_sharded_validate_and_check_equal_one_engine(lib, monkeypatch):
    _fast_oracle(monkeypatch)
    rng = random.Random(0x3E61)
    n, msgs, keys = _c3_streams(4, 24, rng, True)
    msgs = _mutate(msgs, rng)
    one = _auth_for(keys)
    one.set_small_check(0)
    want = {}
    try:
        for flags in (0, 3):
            _fresh(one, keys)
            want[flags] = one.validate_messages_via_flat(msgs, n, flags)
    finally:
        one.close()
    assert (want[0] != 0).sum() >= 10 and (want[3] == 0).sum() >= 10
    for lanes in (1, 2):
        a = _multi(keys)
        try:
            a.set_concurrency(lanes)
            assert len(a.devices()) == 3
            for flags in (0, 3):
                _fresh(a, keys)
                got = a.validate_messages_via_flat(msgs, n, flags)
                bad = np.nonzero(got != want[flags])[0]
                assert not len(bad), (lanes, flags, [(int(i), int(got[i]), int(want[flags][i])) for i in bad[:10]])
            _fresh(a, keys)
            recs, arena = _packed(a, msgs)
            with a.check_messages_flat(recs, arena, n) as b:
                got = np.array([b.resolve(i) for i in range(len(msgs))])
            assert (got == want[3]).all(), (lanes, np.nonzero(got != want[3])[0][:10])
        finally:
            a.close()


def test_sharded_coalesced_passes(lib, monkeypatch):
    """Concurrent callers, lanes on three engines, coalescing on: merged
    passes are themselves split over the engines; every caller's results
    equal the oracle's."""
    from oracle import p256 as o
    _fast_oracle(monkeypatch)
    rng = random.Random(0x3E62)
    n, msgs, keys = _c3_streams(4, 30, rng, True)
    ks = o.KeyStore()
    ks.keys = {role: dict(m) for role, m in keys.items()}
    want = np.array(o.validate_messages(o.Authenticator(ks), msgs, n, 3))
    a = _multi(keys, shard_min=32)
    try:
        a.set_concurrency(2)
        a.set_check_coalescing(True, max_wait_us=20000)
        K = 6
        cuts = [len(msgs) * k // K for k in range(K + 1)]
        parts = [msgs[cuts[k]:cuts[k + 1]] for k in range(K)]
        jobs = [_packed(a, p) for p in parts]
        out = [None] * K
        gate = threading.Barrier(K)

        def run(k):
            gate.wait()
            try:
                out[k] = a.check_messages_flat(jobs[k][0], jobs[k][1], n)
            except Exception as e:  # noqa: BLE001 -- handed to the test
                out[k] = e
        th = [threading.Thread(target=run, args=(k,)) for k in range(K)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        got = np.zeros(len(msgs), dtype=np.int64)
        for k, b in enumerate(out):
            assert not isinstance(b, Exception), b
            with b:
                for i in range(len(parts[k])):
                    got[cuts[k] + i] = b.resolve(i)
    finally:
        a.close()
    assert (got == want).all(), np.nonzero(got != want)[0][:10]


def test_sharded_argument_errors(lib):
    """A bad record in the last shard (type, then a field past the arena):
    MBFT_ERR_ARG, results untouched; the batch fine again afterwards."""
    from minbft_amd.authenticator import GpuError
    rng = random.Random(0x3E63)
    n, msgs, keys = _c3_streams(2, 20, rng, False)
    a = _multi(keys, shard_min=16)
    try:
        recs, arena = _packed(a, msgs)
        assert (a.validate_messages_flat(recs, arena, n) == 0).all()
        k = len(msgs) - 3
        for field, value in (("type", 9), ("sig_off", arena.nbytes)):
            saved = int(recs[k][field])
            recs[k][field] = value
            out = np.full(len(msgs), 777, dtype=np.int32)
            with pytest.raises(GpuError):
                a.validate_messages_flat(recs, arena, n, 0, out)
            assert (out == 777).all()
            with pytest.raises(GpuError):
                a.check_messages_flat(recs, arena, n)
            recs[k][field] = saved
        assert (a.validate_messages_flat(recs, arena, n) == 0).all()
    finally:
        a.close()

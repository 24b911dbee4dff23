"""Multi-engine authenticator (mbft_ctx_add_device): host-buffer batches are
split into contiguous shards over several engines, each with its own device,
stream and replica of the comb tables, and must give exactly the
single-engine results in index order.  On a one-GPU box the extra engines
sit on device 0 (same code path: own thread, stream, tables); on a
multi-GPU node they use devices 1.. as well."""
import numpy as np
import pytest

from golden_util import load, prehashed_arrays

pytestmark = pytest.mark.gpu


def _extra_devices(k):
    from minbft_amd import _lib
    n = max(1, _lib.load().mbft_device_count())
    return [(1 + j) % n for j in range(k)]


def test_sharded_prehashed_matches_single(lib):
    from minbft_amd.authenticator import Authenticator
    xy, e, r, s, exp, labels = prehashed_arrays()
    half = len(labels) // 2
    with Authenticator(0) as one:
        one.set_key_window(8)
        slots, _ = one.register_points(xy)
        want = one.verify_prehashed(e, r, s, slots)
    with Authenticator(0) as a:
        a.set_key_window(8)
        s1, _ = a.register_points(xy[:half])          # replayed on engines added below
        for d in _extra_devices(2):
            a.add_device(d)
        assert len(a.devices()) == 3
        a.set_key_window(12)
        s2, _ = a.register_points(xy[half:])          # registered on all engines at once
        slots2 = np.concatenate([s1, s2])
        a.set_shard_min(16)
        got = a.verify_prehashed(e, r, s, slots2)
    got_ok = (got == 0).astype(np.int64)
    assert (got_ok == exp).all(), [labels[i] for i in np.nonzero(got_ok != exp)[0][:10]]
    assert ((want == 0) == (got == 0)).all()


def test_sharded_generator_window_and_large_batch(lib):
    """A batch large enough to shard at the default threshold, after a
    generator-window change that must reach every engine."""
    import hashlib
    from minbft_amd.authenticator import Authenticator
    from oracle import p256 as o
    n = 100_000
    d = int.from_bytes(hashlib.sha256(b"multi").digest(), "big") % o.N
    q = o.pubkey(d)
    xy = np.frombuffer(q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big"), dtype=np.uint8)
    rng = np.random.default_rng(3)
    e = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    with Authenticator(0, devices=_extra_devices(1)) as a:
        a.set_generator_window(20)
        slots, valid = a.register_points(xy[None, :])
        assert valid.all()
        priv = np.frombuffer(d.to_bytes(32, "big"), dtype=np.uint8)[None, :]
        r, s = a.sign_prehashed(priv, e)
        sl = np.full(n, slots[0], dtype=np.uint32)
        e2 = e.copy()
        e2[1::3, 7] ^= 0x40  # every third item tampered
        st = a.verify_prehashed(e2, r, s, sl)
    want = np.ones(n, dtype=bool)
    want[1::3] = False
    assert ((st == 0) == want).all()


@pytest.mark.parametrize("name", ["authen.json", "usig_epoch.json"])
def test_sharded_authenticator_sequences(lib, name):
    """Authenticator call sequences (USIG epoch capture included) through a
    sharded context: the epoch replay stays in call order."""
    from minbft_amd.authenticator import Authenticator
    fx = load(name)
    for seq in fx["sequences"]:
        a = Authenticator(0, devices=_extra_devices(2))
        try:
            a.set_shard_min(1)
            for role, m in fx["keystore"].items():
                a.add_role(int(role))
                for id_, pk in m.items():
                    a.set_public_key(int(role), int(id_), bytes.fromhex(pk))
            a.enable_usig(True)
            st = a.verify_batch([(c["role"], c["id"], bytes.fromhex(c["msg"]),
                                  bytes.fromhex(c["tag"])) for c in seq])
        finally:
            a.close()
        want = [c["expect"] for c in seq]
        bad = [(c["note"], int(g), w) for c, g, w in zip(seq, st, want) if g != w]
        assert not bad, bad[:10]


def test_sharded_batches_start_no_threads(lib):
    """A call-level batch on a 3-engine context (the C2 calls, flat and item
    forms, and a prehashed batch) runs its shards on one persistent host
    thread per engine: once the engines are warm, further batches start no
    host thread (mbft_debug_threads_started counts every
    thread the library starts)."""
    import hashlib
    from minbft_amd import _lib
    from minbft_amd.authenticator import Authenticator, ROLE_CLIENT
    from oracle import p256 as o
    L = _lib.load()
    d = int.from_bytes(hashlib.sha256(b"no threads").digest(), "big") % (o.N - 1) + 1
    q = o.pubkey(d)
    msgs = [b"REQUEST" + i.to_bytes(8, "big") + hashlib.sha256(b"op %d" % i).digest() for i in range(256)]
    tags = []
    for m in msgs:
        r, s = o.ecdsa_sign(d, o.quirk_digest(m))
        tags.append(o.der_encode_sig(r, s))
    calls = [(ROLE_CLIENT, 0, msgs[i % 256] if i % 5 else b"X" + msgs[i % 256][1:], tags[i % 256])
             for i in range(12288)]
    want = np.array([0 if i % 5 else 1 for i in range(12288)], dtype=np.uint8)
    with Authenticator(0, devices=_extra_devices(2)) as a:
        a.add_role(ROLE_CLIENT)
        a.set_public_key(ROLE_CLIENT, 0, q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big"))
        a.set_shard_min(1024)
        for _ in range(2):  # warm: pools and shard threads start here
            assert np.array_equal(np.asarray(a.verify_batch(calls)), want)
            assert np.array_equal(np.asarray(a.verify_batch_flat(calls)), want)
        before = L.mbft_debug_threads_started()
        for _ in range(4):
            assert np.array_equal(np.asarray(a.verify_batch(calls)), want)
            assert np.array_equal(np.asarray(a.verify_batch_flat(calls)), want)
        after = L.mbft_debug_threads_started()
    assert after == before, (before, after)

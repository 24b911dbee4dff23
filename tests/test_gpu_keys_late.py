"""Keys registered after use, and the single-live-item wave of the small-batch
kernel.

* Late registration (the Go binding's rule): the reference
  verifies any id present in keys.yaml (sample/authentication/keymanager.go:
  96-101,179-227).  A binding that registered a subset of the ids first gets
  MBFT_UNKNOWN_KEY for a call by a missing id, registers that key (here at a
  DIFFERENT comb window from the keys already in the context, whose tables
  are already built) and re-verifies.  The next batches must accept the new
  signer through every entry form: single calls, the host decode, the GPU
  decode (device (role, id) -> slot map rebuilt), the two-phase form and the
  device message layer -- and still reject ids that are still missing.
* k_verify_pairs' wave-uniform branch (kernels.hip verify_pair): a wave
  holding ONE live item inverts s with all 64 lanes (modinv_n_var_wave).
  Every golden prehashed vector is placed as the only live item of its wave
  among dead items (unknown key slot, r = 0, s = N, s = 0), at lanes other than
  0-1 and in the second / third wave of the batch, and the statuses are
  compared with the golden expectation (oracle-made, tests/golden/make_golden.py).
"""
import hashlib

import numpy as np
import pytest

from golden_util import prehashed_arrays

pytestmark = pytest.mark.gpu

ROLE_CLIENT = 3


def _client_keys(ids):
    from oracle import p256 as o
    out = {}
    for i in ids:
        d = int.from_bytes(hashlib.sha256(b"late key %d" % i).digest(), "big") % (o.N - 1) + 1
        out[i] = (d, o.pubkey(d))
    return out


def _requests(keys, per_id=3):
    """(role, id, AuthenBytes(REQUEST), DER tag) calls, signed with the
    reference's quirk digest (crypto.go:113-121)."""
    from oracle import p256 as o
    calls = []
    for i, (d, _q) in sorted(keys.items()):
        for seq in range(1, per_id + 1):
            op = hashlib.sha256(b"op %d %d" % (i, seq)).digest() * 8
            msg = o.authen_request(seq, op)
            r, s = o.ecdsa_sign(d, o.quirk_digest(msg))
            calls.append((ROLE_CLIENT, i, msg, o.der_encode_sig(r, s), op, seq))
    return calls


def _all_forms(a, calls):
    """Statuses of the calls through every entry form (they must agree)."""
    from oracle import p256 as o
    items = [c[:4] for c in calls]
    forms = {
        "single": np.array([a.verify_status(*it) for it in items], dtype=np.uint8),
        "batch": a.verify_batch(items),
        "flat_host": a.verify_batch_flat(items, pinned=False),
        "flat_gpu": a.verify_batch_flat(items, pinned=True),
        "check": a.check_batch_flat(items, pinned=True),
    }
    msgs = [o.Msg(type=o.MSG_REQUEST, stream=k, client_id=c[1], seq=c[5], op=c[4], sig=c[3])
            for k, c in enumerate(calls)]
    res = a.validate_messages_via_flat(msgs, 4, 0, pinned=True)
    # a REQUEST's result is (MBFT_ST_REQUEST_SIG << 8) | status, 0 if valid
    forms["msg_layer"] = np.array([0 if v == 0 else (int(v) & 0xFF) for v in res], dtype=np.uint8)
    assert all(int(v) == 0 or (int(v) >> 8) == o.ST_REQUEST_SIG for v in res), res
    ref = forms["single"]
    for name, st in forms.items():
        assert (np.asarray(st, dtype=np.uint8) == ref).all(), (name, list(st), list(ref))
    return ref


def test_key_registered_after_unknown_key(lib):
    from minbft_amd.authenticator import Authenticator
    from oracle import p256 as o
    first = _client_keys([5, 40])
    late = _client_keys([9, 1000])
    never = _client_keys([77])
    calls = _requests({**first, **late, **never})
    ids = np.array([c[1] for c in calls])
    with Authenticator(0) as a:
        a.add_role(ROLE_CLIENT)
        a.set_key_window(16)
        for i, (_d, q) in first.items():
            a.set_public_key(ROLE_CLIENT, i, o.pkix_encode(q))
        st = _all_forms(a, calls)
        assert (st[np.isin(ids, list(first))] == 0).all()
        assert (st[~np.isin(ids, list(first))] == 4).all()  # MBFT_UNKNOWN_KEY
        # the binding's late registration: a different window per key, the
        # existing tables untouched
        for w, (i, (_d, q)) in zip((8, 20), late.items()):
            a.set_key_window(w)
            a.set_public_key(ROLE_CLIENT, i, o.pkix_encode(q))
        st = _all_forms(a, calls)
        known = np.isin(ids, list(first) + list(late))
        assert (st[known] == 0).all(), list(st)
        assert (st[~known] == 4).all(), list(st)
        # tampered REQUESTs of the late signers are rejected, not unknown
        bad = [(r, i, m[:20] + bytes([m[20] ^ 1]) + m[21:], t, op, seq)
               for (r, i, m, t, op, seq) in calls if i in late]
        assert (a.verify_batch_flat([c[:4] for c in bad], pinned=True) == 1).all()


def _dead_rows(e, r, s, kind):
    """A dead item of each kind (never live: k_verify_pairs writes its
    status without running the comb on it)."""
    from oracle import p256 as o
    e2, r2, s2 = e.copy(), r.copy(), s.copy()
    slot_bad = False
    if kind == "bad_key":
        slot_bad = True
    elif kind == "r0":
        r2[:] = 0
    elif kind == "sN":
        s2[:] = np.frombuffer(o.N.to_bytes(32, "big"), dtype=np.uint8)
    elif kind == "s0":
        s2[:] = 0
    return e2, r2, s2, slot_bad


@pytest.mark.parametrize("form", ["pairs", "split"])
@pytest.mark.parametrize("n,live", [(2, (1,)), (3, (2,)), (33, (17, 32)), (65, (5, 40, 64))])
def test_single_live_item_per_wave(lib, n, live, form):
    """Both small-batch kernels: k_verify_pairs (its one-live-item wave
    branch) and k_verify_split (one item per 4-wave workgroup)."""
    from minbft_amd.authenticator import Authenticator
    xy, e, r, s, exp, labels = prehashed_arrays()
    kinds = ["bad_key", "r0", "sN", "s0"]
    dead_status = {"bad_key": 5, "r0": 1, "sN": 1, "s0": 1}
    with Authenticator(0) as a:
        a.set_small_batch_form(0 if form == "pairs" else 256)
        a.set_key_window(8)
        slots, valid = a.register_points(xy)
        assert valid.all()
        nv = len(labels)
        bad = []
        for v0 in range(0, nv, len(live)):
            vs = [(v0 + j) % nv for j in range(len(live))]
            E = np.zeros((n, 32), np.uint8)
            R = np.zeros((n, 32), np.uint8)
            S = np.zeros((n, 32), np.uint8)
            SL = np.zeros(n, np.uint32)
            want = np.zeros(n, np.int64)
            for p in range(n):
                src = vs[p % len(vs)]
                if p in live:
                    v = vs[live.index(p)]
                    E[p], R[p], S[p], SL[p] = e[v], r[v], s[v], slots[v]
                    want[p] = -1  # checked against the golden expectation
                    continue
                k = kinds[(p + v0) % len(kinds)]
                de, dr, ds, sb = _dead_rows(e[src], r[src], s[src], k)
                E[p], R[p], S[p] = de, dr, ds
                SL[p] = 0xFFFFFFFF if sb else slots[src]
                want[p] = dead_status[k]
            st = a.verify_prehashed(E, R, S, SL)
            for p in range(n):
                if p in live:
                    v = vs[live.index(p)]
                    if int(st[p] == 0) != int(exp[v]):
                        bad.append((labels[v], p, int(st[p]), int(exp[v])))
                elif int(st[p]) != want[p]:
                    bad.append(("dead", p, int(st[p]), int(want[p])))
        assert not bad, bad[:20]

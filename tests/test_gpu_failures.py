"""C-ABI failure paths leave the context usable (the Go binding's policy,
go/gpuauth/errors.go: a failed C call is retried once, then the call is
rejected -- never accepted -- and the replica keeps running, so the library
must come out of a failure with its key store, tables, epoch state and
streams intact).

A real failure, no injection: the device runs out of HBM while registering a
comb table (two W = 29 tables fill 258 GiB of the 288 GB card; a third
cannot fit).  The call returns MBFT_ERR_NOMEM with a message, registers
nothing, and every entry form still verifies with the keys that were there
-- and with a key registered after the failure.  The device message layer's
error path (an argument error found by the kernels after every chunk is
queued) is covered in tests/test_gpu_msgdev.py::test_flat_argument_errors."""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROLE_CLIENT = 3
MBFT_ERR_NOMEM = -3


def _key(i):
    from oracle import p256 as o
    d = int.from_bytes(hashlib.sha256(b"failure key %d" % i).digest(), "big") % (o.N - 1) + 1
    return d, o.pubkey(d)


def _calls(keys):
    from oracle import p256 as o
    out = []
    for i, (d, _q) in keys.items():
        for seq in (1, 2):
            msg = o.authen_request(seq, bytes([i, seq]) * 128)
            r, s = o.ecdsa_sign(d, o.quirk_digest(msg))
            out.append((ROLE_CLIENT, i, msg, o.der_encode_sig(r, s)))
            bad = bytearray(msg)
            bad[9] ^= 0x40
            out.append((ROLE_CLIENT, i, bytes(bad), o.der_encode_sig(r, s)))
    return out


def _expect(calls, known):
    return [0 if (c[1] in known and k % 2 == 0) else (1 if c[1] in known else 4)
            for k, c in enumerate(calls)]


def test_out_of_memory_registration_leaves_context_usable(lib):
    from minbft_amd.authenticator import Authenticator, GpuError
    from oracle import p256 as o
    keys = {i: _key(i) for i in (1, 2, 3)}
    calls = _calls(keys)
    with Authenticator(0) as a:
        a.set_generator_window(29)
        a.add_role(ROLE_CLIENT)
        a.set_key_window(29)
        a.set_public_key(ROLE_CLIENT, 1, o.pkix_encode(keys[1][1]))
        want = _expect(calls, {1})
        assert list(a.verify_batch_flat(calls, pinned=True)) == want
        # a second 129 GiB table does not fit next to the two
        with pytest.raises(GpuError) as ei:
            a.set_public_key(ROLE_CLIENT, 2, o.pkix_encode(keys[2][1]))
        assert "(%d)" % MBFT_ERR_NOMEM in str(ei.value), str(ei.value)
        assert a.key_slot(ROLE_CLIENT, 1) >= 0
        with pytest.raises(GpuError):
            a.key_slot(ROLE_CLIENT, 2)  # nothing registered
        # every form still gives the reference's statuses with the old key
        assert [a.verify_status(*c) for c in calls] == want
        assert list(a.verify_batch(calls)) == want
        assert list(a.verify_batch_flat(calls, pinned=False)) == want
        assert list(a.verify_batch_flat(calls, pinned=True)) == want
        assert list(a.check_batch_flat(calls, pinned=True)) == want
        # and a key that fits is registered and used after the failure
        a.set_key_window(8)
        a.set_public_key(ROLE_CLIENT, 3, o.pkix_encode(keys[3][1]))
        want = _expect(calls, {1, 3})
        assert list(a.verify_batch_flat(calls, pinned=True)) == want
        assert [a.verify_status(*c) for c in calls] == want

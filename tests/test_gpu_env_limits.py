"""Environment knobs cannot push a batch into a staging layout it does not
have (batch.cpp host_inv_max): MBFT_HOST_INV_MAX far above the
zero-copy batch size used to make a 5,000-call batch write its host s^-1
planes past the end of the split staging.  It is clamped to the zero-copy
batches; a subprocess (the knob is read once per process) verifies batches
of 1, 50, 64, 65, 4,096 and 5,000 calls -- tampered ones among them -- with
the knob at 100,000, every status against the construction."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import hashlib, sys
sys.path.insert(0, sys.argv[1])
import torch
torch.cuda.init()
from minbft_amd.authenticator import Authenticator, ROLE_CLIENT
from oracle import p256 as o
d = int.from_bytes(hashlib.sha256(b"env limits").digest(), "big") % o.N
calls = []
for k in range(64):
    msg = o.authen_request(k + 1, bytes([k]) * 100)
    r, s = o.ecdsa_sign(d, o.quirk_digest(msg))
    calls.append((msg, o.der_encode_sig(r, s)))
with Authenticator(0) as a:
    a.set_key_window(8)
    a.add_role(ROLE_CLIENT)
    a.set_public_key(ROLE_CLIENT, 7, o.pkix_encode(o.pubkey(d)))
    for n in (1, 50, 64, 65, 4096, 5000):
        items, want = [], []
        for i in range(n):
            msg, tag = calls[i % 64]
            if i % 7 == 3:
                msg = bytes([msg[0] ^ 1]) + msg[1:]
                want.append(1)
            else:
                want.append(0)
            items.append((ROLE_CLIENT, 7, msg, tag))
        got = [int(x) for x in a.verify_batch(items)]
        assert got == want, (n, [i for i, (g, w) in enumerate(zip(got, want)) if g != w][:10])
print("env limits ok")
"""


def test_host_inv_max_clamped(lib):
    env = dict(os.environ, MBFT_HOST_INV_MAX="100000")
    p = subprocess.run([sys.executable, "-c", SCRIPT, ROOT], env=env, capture_output=True, text=True,
                       timeout=240)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    assert "env limits ok" in p.stdout

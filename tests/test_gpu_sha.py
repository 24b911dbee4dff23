"""GPU SHA-256 stage vs hashlib (bit-exact), through the C-ABI device entry
points: REQUEST digests (messages/authen.go:33,54-56 + the Sum(m) quirk of
sample/authentication/crypto.go:121), the hashsum of arbitrary byte strings
(messages/authen.go:78-82) and the USIG signed digest
(usig/sgx/sgx-usig.go:99-101, usig/sgx/usig-enclave.go:204-214).
Edge cases: empty operations, lengths around the 55/56/64-byte padding
boundaries, ragged batch sizes (not multiples of the 64-message tile), and
both REQUEST kernels (LDS-tiled for op_len % 16 == 0, per-lane otherwise)."""
import hashlib
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _request_e(seq: int, op: bytes) -> bytes:
    authen = b"REQUEST" + struct.pack(">Q", seq) + hashlib.sha256(op).digest()
    return (authen + hashlib.sha256(b"").digest())[:32]


@pytest.mark.parametrize("op_len,n", [(256, 1), (256, 63), (256, 65), (256, 4099), (512, 200),
                                      (16, 130), (0, 70), (100, 129), (55, 64), (64, 64),
                                      (1000, 10)])
def test_request_digests(gpu_auth, op_len, n):
    import torch
    rng = np.random.default_rng(op_len * 7919 + n)
    ops = rng.integers(0, 256, size=(n, op_len), dtype=np.uint8)
    seqs = rng.integers(0, 2**63, size=n, dtype=np.int64)
    dev = torch.device("cuda", 0)
    d_ops = torch.from_numpy(ops.reshape(-1) if op_len else np.zeros(16, np.uint8)).to(dev)
    d_seq = torch.from_numpy(seqs).to(dev)
    d_e = torch.zeros((n, 32), dtype=torch.uint8, device=dev)
    gpu_auth.request_digests_device(d_seq.data_ptr(), d_ops.data_ptr(), op_len, n, d_e.data_ptr())
    torch.cuda.synchronize()
    got = d_e.cpu().numpy()
    for i in range(n):
        want = _request_e(int(seqs[i]), ops[i].tobytes())
        assert got[i].tobytes() == want, (op_len, n, i)


def test_sha256_var(gpu_auth):
    import torch
    rng = np.random.default_rng(5)
    lens = list(range(0, 200)) + [255, 256, 257, 1000, 4096]
    msgs = [rng.integers(0, 256, size=L, dtype=np.uint8).tobytes() for L in lens]
    off = np.zeros(len(msgs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    data = np.frombuffer(b"".join(msgs) + b"\0" * 16, dtype=np.uint8)
    dev = torch.device("cuda", 0)
    d_data = torch.from_numpy(data.copy()).to(dev)
    d_off = torch.from_numpy(off.astype(np.int64)).to(dev)
    d_out = torch.zeros((len(msgs), 32), dtype=torch.uint8, device=dev)
    gpu_auth.sha256_device(d_data.data_ptr(), d_off.data_ptr(), len(msgs), d_out.data_ptr())
    torch.cuda.synchronize()
    got = d_out.cpu().numpy()
    for i, m in enumerate(msgs):
        assert got[i].tobytes() == hashlib.sha256(m).digest(), lens[i]


def test_usig_digests(gpu_auth):
    import torch
    rng = np.random.default_rng(9)
    lens = [0, 1, 47, 59, 70, 23, 55, 56, 64, 200]
    msgs = [rng.integers(0, 256, size=L, dtype=np.uint8).tobytes() for L in lens]
    ep = rng.integers(0, 2**63, size=len(msgs), dtype=np.int64)
    ct = rng.integers(0, 2**63, size=len(msgs), dtype=np.int64)
    ct[0], ep[1] = 1, 0
    off = np.zeros(len(msgs) + 1, dtype=np.int64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    data = np.frombuffer(b"".join(msgs) + b"\0" * 16, dtype=np.uint8)
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d_data, d_off, d_ep, d_ct = t(data.copy()), t(off), t(ep), t(ct)
    d_e = torch.zeros((len(msgs), 32), dtype=torch.uint8, device=dev)
    gpu_auth.usig_digests_device(d_data.data_ptr(), d_off.data_ptr(), d_ep.data_ptr(),
                                 d_ct.data_ptr(), len(msgs), d_e.data_ptr())
    torch.cuda.synchronize()
    got = d_e.cpu().numpy()
    for i, m in enumerate(msgs):
        want = hashlib.sha256(hashlib.sha256(m).digest() + struct.pack("<Q", int(ep[i]))
                              + struct.pack("<Q", int(ct[i]))).digest()
        assert got[i].tobytes() == want, lens[i]


@pytest.mark.parametrize("op_len", [0, 1, 55, 56, 64, 200, 256, 1000])
def test_authen_digests_vs_oracle(gpu_auth, op_len):
    """The GPU AuthenBytes + digest stage (k_sha256_var + k_authen_e) against
    the oracle's msg_authen_bytes with the ECDSA-role quirk digest
    (REQUEST, REPLY) and the USIG chain usig_digest (PREPARE, COMMIT), on
    random fields including 64-bit extremes."""
    import random

    from oracle import p256 as o
    rng = random.Random(op_len)
    msgs, ep, ct = [], [], []
    for k in range(300):
        big = lambda b: rng.choice([0, 1, (1 << b) - 1, rng.randrange(1 << b)])  # noqa: E731
        msgs.append(o.Msg(type=o.MSG_COMMIT, replica_id=big(32), prep_replica_id=big(32), view=big(64),
                          client_id=big(32), seq=big(64), op=rng.randbytes(op_len),
                          prep_ui_counter=big(64)))
        ep.append(big(64))
        ct.append(big(64))
    for kind, typ in ((0, o.MSG_REQUEST), (1, o.MSG_REPLY), (2, o.MSG_PREPARE), (3, o.MSG_COMMIT)):
        got = gpu_auth.authen_digests(msgs, kind, ep, ct)
        for i, m in enumerate(msgs):
            ab = o.msg_authen_bytes(m, typ)
            want = o.quirk_digest(ab)[:32] if kind < 2 else o.usig_digest(ab, ep[i], ct[i])
            assert got[i].tobytes() == want, (kind, i)

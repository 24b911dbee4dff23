"""The C2 setup shared by the round-6 probes: a context with G 29 / Q 29
tables, 1M single-signer REQUESTs signed on the GPU, 3 caller streams and the
bench's step() (bench.py main, without the extra lines)."""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


class C2:
    def __init__(self, B=1 << 20, streams=3, gw=29, qw=29):
        import torch
        from minbft_amd.authenticator import Authenticator, ROLE_CLIENT, der_encode_rows
        self.torch = torch
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        self.B = B
        self.auth = auth = Authenticator(0)
        auth.set_generator_window(gw)
        d = int.from_bytes(hashlib.sha256(b"minbft-amd bench client 0").digest(), "big")
        d = d % (0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551 - 1) + 1
        self.d = d
        priv = np.frombuffer(d.to_bytes(32, "big"), dtype=np.uint8).copy()
        self.msgs = bench.make_requests(0, B)
        e = np.ascontiguousarray(self.msgs[:, :32])
        d_priv = torch.from_numpy(priv).to(dev)
        self.d_e = torch.from_numpy(e).to(dev)
        self.d_r = torch.empty((B, 32), dtype=torch.uint8, device=dev)
        self.d_s = torch.empty((B, 32), dtype=torch.uint8, device=dev)
        auth.sign_prehashed_device(d_priv.data_ptr(), 0, self.d_e.data_ptr(), B, self.d_r.data_ptr(),
                                   self.d_s.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        auth.set_key_window(qw)
        auth.add_role(ROLE_CLIENT)
        auth.set_public_key(ROLE_CLIENT, 0, bench.pubkey_bytes(d))
        slot = auth.key_slot(ROLE_CLIENT, 0)
        self.d_slot = torch.full((B,), slot, dtype=torch.int32, device=dev)
        self.streams = [torch.cuda.Stream(device=dev) for _ in range(streams)]
        self.d_sts = [torch.empty((B,), dtype=torch.uint8, device=dev) for _ in self.streams]
        self.n = 0
        for _ in self.streams:
            self.step()
        torch.cuda.synchronize()
        if min(int((x == 0).sum().item()) for x in self.d_sts) != B:
            raise SystemExit("C2 gate: valid batch not accepted")
        self.tags, self.tlen = der_encode_rows(self.d_r.cpu().numpy(), self.d_s.cpu().numpy())

    def step(self):
        k = self.n % len(self.streams)
        self.n += 1
        self.auth.verify_prehashed_device(self.d_e.data_ptr(), self.d_r.data_ptr(), self.d_s.data_ptr(),
                                          self.d_slot.data_ptr(), self.B, self.d_sts[k].data_ptr(),
                                          self.streams[k].cuda_stream)

    def close(self):
        self.auth.close()

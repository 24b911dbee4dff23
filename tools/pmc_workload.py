"""Small fixed workload for rocprofv3 PMC passes: 3 verify launches of the
bench batch (1,048,576 single-signer REQUEST items, inputs in HBM), one at
a time, and nothing else (no authenticator-level, adversarial or C3 runs).

    python3 tools/pmc_workload.py [G_WINDOW Q_WINDOW]
"""
import hashlib
import sys

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402


def main():
    g, q = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (16, 16)
    import torch

    from minbft_amd.authenticator import Authenticator, ROLE_CLIENT
    dev = torch.device("cuda", 0)
    B = 1 << 20
    with Authenticator(0) as auth:
        if g != 16:
            auth.set_generator_window(g)
        auth.set_key_window(q)
        d = int.from_bytes(hashlib.sha256(b"minbft-amd bench client 0").digest(), "big")
        d = d % (bench.N_ORDER - 1) + 1
        msgs = bench.make_requests(0, B)
        d_e = torch.from_numpy(np.ascontiguousarray(msgs[:, :32])).to(dev)
        d_priv = torch.from_numpy(np.frombuffer(d.to_bytes(32, "big"), dtype=np.uint8).copy()).to(dev)
        d_r = torch.empty((B, 32), dtype=torch.uint8, device=dev)
        d_s = torch.empty((B, 32), dtype=torch.uint8, device=dev)
        st = torch.cuda.current_stream().cuda_stream
        auth.sign_prehashed_device(d_priv.data_ptr(), 0, d_e.data_ptr(), B, d_r.data_ptr(), d_s.data_ptr(), st)
        auth.add_role(ROLE_CLIENT)
        auth.set_public_key(ROLE_CLIENT, 0, bench.pubkey_bytes(d))
        slot = auth.key_slot(ROLE_CLIENT, 0)
        d_slot = torch.full((B,), slot, dtype=torch.int32, device=dev)
        d_st = torch.empty((B,), dtype=torch.uint8, device=dev)
        for _ in range(3):
            auth.verify_prehashed_device(d_e.data_ptr(), d_r.data_ptr(), d_s.data_ptr(), d_slot.data_ptr(), B,
                                         d_st.data_ptr(), st)
            torch.cuda.synchronize()
        assert int((d_st == 0).sum().item()) == B


if __name__ == "__main__":
    main()

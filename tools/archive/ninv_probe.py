"""Batched s^-1 chain span, isolated (one 1M batch at a time, synchronized,
HIP events around the chain on its stream: mbft_profile_read's inverse_ms),
for same-box A/Bs of the inversion kernels:
    MBFT_LIB_PATH=... python tools/ninv_probe.py [n] [reps]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    import torch

    import bench
    from minbft_amd.authenticator import Authenticator
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    dev = torch.device("cuda", 0)
    d = 0x1234567
    with Authenticator(0) as a:
        e = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device=dev)
        r = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        s = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        priv = torch.from_numpy(np.frombuffer(d.to_bytes(32, "big"), dtype=np.uint8).copy()).to(dev)
        st = torch.cuda.current_stream().cuda_stream
        a.sign_prehashed_device(priv.data_ptr(), 0, e.data_ptr(), n, r.data_ptr(), s.data_ptr(), st)
        a.set_public_key(1, 0, bench.pubkey_bytes(d)) if False else None
        xy = np.frombuffer(bench.pubkey_bytes(d), dtype=np.uint8)[None, :]
        slots, _ = a.register_points(xy)
        sl = torch.full((n,), int(slots[0]), dtype=torch.int32, device=dev)
        out = torch.empty((n,), dtype=torch.uint8, device=dev)
        inv = []
        for k in range(reps + 3):
            torch.cuda.synchronize()
            a.profile(True)
            a.verify_prehashed_device(e.data_ptr(), r.data_ptr(), s.data_ptr(), sl.data_ptr(), n,
                                      out.data_ptr(), st)
            torch.cuda.synchronize()
            p = a.profile_read()
            a.profile(False)
            if k >= 3:
                inv.append(p["inverse_ms"] / max(p["batches"], 1))
        assert int((out == 0).sum().item()) == n
        print(json.dumps({"n": n, "inverse_span_ms_p50": float(np.median(inv)),
                          "min": float(min(inv))}), flush=True)


if __name__ == "__main__":
    main()

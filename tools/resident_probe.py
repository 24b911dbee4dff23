"""Single calls through the resident verifier (mbft_set_resident) against
the launch path and the coalescer: bench.py's single_calls section alone
(lone-call p50 both ways; OS-thread callers at 16 / 64 with the coalescer and
with the resident kernel), on the C2 key at the benched windows (G 29 /
Q 29).  Prints one JSON object.

    python tools/resident_probe.py [per_thread]
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    import torch
    torch.cuda.init()
    import bench
    from minbft_amd.authenticator import Authenticator, der_encode_rows
    per = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    B = 64 * per
    dev = torch.device("cuda", 0)
    d = int.from_bytes(hashlib.sha256(b"minbft-amd bench client 0").digest(), "big") % (bench.N_ORDER - 1) + 1
    msgs = bench.make_requests(0, B)
    with Authenticator(0) as a:
        a.set_generator_window(29)
        a.set_key_window(29)
        d_priv = torch.from_numpy(np.frombuffer(d.to_bytes(32, "big"), dtype=np.uint8).copy()).to(dev)
        d_e = torch.from_numpy(np.ascontiguousarray(msgs[:, :32])).to(dev)
        d_r = torch.empty((B, 32), dtype=torch.uint8, device=dev)
        d_s = torch.empty((B, 32), dtype=torch.uint8, device=dev)
        st = torch.cuda.current_stream().cuda_stream
        a.sign_prehashed_device(d_priv.data_ptr(), 0, d_e.data_ptr(), B, d_r.data_ptr(), d_s.data_ptr(), st)
        torch.cuda.synchronize()
        a.add_role(3)
        a.set_public_key(3, 0, bench.pubkey_bytes(d))
        tags, tlen = der_encode_rows(d_r.cpu().numpy(), d_s.cpu().numpy())
        out = bench.single_calls(a, msgs, tags, tlen, per_thread=per * 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

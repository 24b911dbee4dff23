"""Fixed workload for rocprofv3 PMC passes over the SHA-256 stage: 3 launches
of k_request_e_tiled over 1,048,576 REQUESTs with 256-byte operations in HBM
(the bench's sha256_stage input)."""
import sys

import numpy as np

sys.path.insert(0, ".")


def main(n=1 << 20):
    import torch
    torch.cuda.init()
    from minbft_amd.authenticator import Authenticator
    dev = torch.device("cuda", 0)
    rng = np.random.Generator(np.random.PCG64(5))
    ops = torch.from_numpy(rng.integers(0, 256, size=(n, 256), dtype=np.uint8)).to(dev)
    seq = torch.arange(1, n + 1, dtype=torch.int64, device=dev)
    out = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    with Authenticator(0) as a:
        for _ in range(3):
            a.request_digests_device(seq.data_ptr(), ops.data_ptr(), 256, n, out.data_ptr())
        torch.cuda.synchronize()
    print("ok", int(out[0, 0].item()))


if __name__ == "__main__":
    main()

"""Latency of small device batches through mbft_verify_prehashed_device (one
batch at a time, host-synchronized), under whatever small-batch form the
environment selects (kernels.hip verify(): MBFT_SPLIT_MAX, MBFT_PAIRS_PLANES,
MBFT_QUADS, MBFT_QUADS_INLINE; round 6 also MBFT_SPLIT_PLANES_MAX, since
dropped).  Every status checked (all valid, then 1 in 7 tampered).  Prints
one JSON object.

    MBFT_QUADS=0 python tools/small_batch_probe.py   # lane pairs on the planes
    python tools/small_batch_probe.py                # the default (lane quads)
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from c2_setup import C2  # noqa: E402


def main():
    sizes = [int(x) for x in os.environ.get("SMALL_SIZES", "300,512,1024,2048,4096").split(",")]
    reps = int(os.environ.get("SMALL_REPS", "100"))
    c = C2(B=max(sizes), streams=1)
    torch = c.torch
    st = c.streams[0]
    env = {k: v for k, v in os.environ.items() if k.startswith("MBFT_")}
    out = {"env": env, "sizes": {}}
    bad_e = c.d_e.clone()
    bad_e[::7, 5] ^= 1
    try:
        for n in sizes:
            d_st = c.d_sts[0]
            ts = []
            for k in range(reps + 5):
                t = time.perf_counter()
                c.auth.verify_prehashed_device(c.d_e.data_ptr(), c.d_r.data_ptr(), c.d_s.data_ptr(),
                                               c.d_slot.data_ptr(), n, d_st.data_ptr(), st.cuda_stream)
                st.synchronize()
                if k >= 5:
                    ts.append(time.perf_counter() - t)
            ok = int((d_st[:n] == 0).sum().item())
            c.auth.verify_prehashed_device(bad_e.data_ptr(), c.d_r.data_ptr(), c.d_s.data_ptr(),
                                           c.d_slot.data_ptr(), n, d_st.data_ptr(), st.cuda_stream)
            st.synchronize()
            got = d_st[:n].cpu().numpy()
            want = np.zeros(n, dtype=np.uint8)
            want[::7] = 1
            out["sizes"][str(n)] = {"p50_us": round(float(np.median(ts)) * 1e6, 1),
                                    "p90_us": round(float(np.percentile(ts, 90)) * 1e6, 1),
                                    "accepted": ok, "tamper_statuses_ok": bool((got == want).all())}
            if ok != n or not (got == want).all():
                print(json.dumps(out))
                raise SystemExit(f"status mismatch at n={n}")
    finally:
        c.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()

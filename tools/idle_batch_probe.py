"""Latency of one 1M C2 batch on an idle GPU (mbft_verify_prehashed_device,
host-synchronized, p50 of 40 after 5 warm-ups): the one-launch s^-1 form for
idle batches (env MBFT_NINV_FORM / MBFT_NINV_PER) + k_verify + the exact-path
launch -- bench.py's p50_batch_latency_device_ms.  Prints one JSON object.

    MBFT_NINV_FORM=wave MBFT_NINV_PER=16 python tools/idle_batch_probe.py
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
    c = C2(streams=1)
    st = c.streams[0]
    ts = []
    try:
        for k in range(45):
            t = time.perf_counter()
            c.step()
            st.synchronize()
            if k >= 5:
                ts.append(time.perf_counter() - t)
        ok = int((c.d_sts[0] == 0).sum().item())
    finally:
        c.close()
    print(json.dumps({"form": os.environ.get("MBFT_NINV_FORM", "block"), "per": os.environ.get("MBFT_NINV_PER", "default"),
                      "p50_ms": round(float(np.median(ts)) * 1e3, 4), "min_ms": round(min(ts) * 1e3, 4),
                      "accepted": ok, "items": c.B}))
    if ok != c.B:
        raise SystemExit("not all accepted")


if __name__ == "__main__":
    main()

"""Low-load latency probe (bench.py go_wiring_latency + c5_proxy alone): a
fresh context with the W = 29 generator table, then the one-message check
latencies of the Go core loop's C-ABI sequence.  Prints one JSON object.

    python tools/latency_probe.py [--nreq 128] [--q-window 26]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nreq", type=int, default=128)
    ap.add_argument("--q-window", type=int, default=26)
    ap.add_argument("--g-window", type=int, default=29)
    ap.add_argument("--sizes", default="2,8,16,32,64,128,256")
    ap.add_argument("--small-max", type=int, default=None)
    ap.add_argument("--f", type=int, default=1)
    ap.add_argument("--plain-only", action="store_true")
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    import bench
    from minbft_amd import build
    build.build()
    from minbft_amd.authenticator import Authenticator
    auth = Authenticator(0)
    try:
        t = time.perf_counter()
        auth.set_generator_window(a.g_window)
        g_s = time.perf_counter() - t
        kw = {}
        if a.small_max is not None:
            kw["small_max"] = a.small_max
        if a.plain_only:
            kw["configs"] = (("plain", 1, False, 0),)
        out = bench.go_wiring_latency(auth, nreq=a.nreq, f=a.f, q_window=a.q_window,
                                      sizes=tuple(int(x) for x in a.sizes.split(",")), c5=not a.plain_only, **kw)
        out["generator_table_s"] = g_s
        print(json.dumps(out, indent=1))
    finally:
        auth.close()


if __name__ == "__main__":
    main()

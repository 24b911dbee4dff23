"""The Go core loop's low-load latency alone (bench.py go_wiring_latency:
windows of 1 ... 256 messages through the C-ABI sequence the Go binding
runs, plus the C5 proxy), without the rest of the bench -- for same-box A/Bs
of the small-check route (e.g. MBFT_RESIDENT_HOST_JOIN_MAX); LOWLOAD_SIZES,
LOWLOAD_SMALL_MAX and LOWLOAD_NREQ set the windows, the route's limit and
the stream length.

    python tools/lowload_probe.py > out.json
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    import torch
    torch.cuda.init()
    import bench
    from minbft_amd.authenticator import Authenticator
    cfgs = (("go_default", 4, True, int(os.environ.get("LOWLOAD_SLOTS", "32"))),)
    if os.environ.get("LOWLOAD_ALL"):
        cfgs += (("go_default_launch", 4, True, 0),)
    with Authenticator(0) as auth:
        auth.set_generator_window(29)
        kw = {}
        if os.environ.get("LOWLOAD_SIZES"):  # e.g. "256,512,1024"
            kw["sizes"] = tuple(int(x) for x in os.environ["LOWLOAD_SIZES"].split(","))
        if os.environ.get("LOWLOAD_SMALL_MAX"):
            kw["small_max"] = int(os.environ["LOWLOAD_SMALL_MAX"])
        if os.environ.get("LOWLOAD_NREQ"):
            kw["nreq"] = int(os.environ["LOWLOAD_NREQ"])
            kw["c5"] = False
        out = bench.go_wiring_latency(auth, configs=cfgs, **kw)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

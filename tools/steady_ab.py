#!/usr/bin/env python3
"""C2 steady-state step time for the s^-1 stage's forms:
after 2 s of back-to-back steps, 500 timed steps and the driver's shape
(5 warm-up + 20 timed, after a 30-batch gate), for --streams caller streams.
The s^-1 form comes from the environment (MBFT_NINV=local | levels, read per
batch).  One JSON line."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from c2_setup import C2  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=3)
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    c = C2(streams=args.streams)
    torch = c.torch
    try:
        res = {"tag": args.tag, "streams": args.streams, "ninv": os.environ.get("MBFT_NINV")}
        t_end = time.perf_counter() + 2.0
        while time.perf_counter() < t_end:
            for _ in range(30):
                c.step()
            torch.cuda.synchronize()
        a = time.perf_counter()
        for _ in range(500):
            c.step()
        torch.cuda.synchronize()
        res["steady_ms_per_step"] = (time.perf_counter() - a) / 500 * 1e3
        win = []
        for _ in range(5):
            time.sleep(0.5)
            for _ in range(35):
                c.step()
            torch.cuda.synchronize()
            a = time.perf_counter()
            for _ in range(20):
                c.step()
            torch.cuda.synchronize()
            win.append((time.perf_counter() - a) / 20 * 1e3)
        res["driver_shape_ms_per_step"] = sorted(win)
        ok = min(int((x == 0).sum().item()) for x in c.d_sts)
        if ok != c.B:
            raise SystemExit("steady_ab gate failed")
        print(json.dumps(res), flush=True)
    finally:
        c.close()


if __name__ == "__main__":
    main()

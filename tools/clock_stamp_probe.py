#!/usr/bin/env python3
"""In-kernel clock of k_verify (a -DMBFT_CLOCK_STAMP build through
MBFT_LIB_PATH): Δs_memtime ÷ Δs_memrealtime × 100 MHz summed over every
workgroup, (a) over isolated 1M launches one at a time after idle, (b) over
the pipelined C2 loop (3 streams) after >= 2 s of back-to-back steps, (c) the
same loop with the s^-1 stage reused (MBFT_DIAG_REUSE_WINV is read by the
library at start: run the script twice for it).  One JSON line."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from c2_setup import C2  # noqa: E402


def main():
    c = C2()
    torch = c.torch
    lib = c.auth.lib
    fn = lib.mbft_debug_verify_clock
    fn.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int]
    out = (ctypes.c_double * 3)()

    def read(reset=True):
        fn(out, 1 if reset else 0)
        return {"ghz": out[0] / out[1] / 10.0 if out[1] else None, "blocks": int(out[2])}

    res = {"reuse_winv": os.environ.get("MBFT_DIAG_REUSE_WINV")}
    try:
        read()
        iso = []
        for _ in range(10):
            time.sleep(0.05)
            torch.cuda.synchronize()
            a = time.perf_counter()
            c.step()
            torch.cuda.synchronize()
            iso.append((time.perf_counter() - a) * 1e3)
        res["isolated"] = read()
        res["isolated_ms_p50"] = sorted(iso)[len(iso) // 2]
        t_end = time.perf_counter() + 2.0
        while time.perf_counter() < t_end:
            for _ in range(50):
                c.step()
            torch.cuda.synchronize()
        read()
        a = time.perf_counter()
        for _ in range(500):
            c.step()
        torch.cuda.synchronize()
        res["steady_ms_per_step"] = (time.perf_counter() - a) / 500 * 1e3
        res["steady"] = read()
        print(json.dumps(res), flush=True)
    finally:
        c.close()


if __name__ == "__main__":
    main()

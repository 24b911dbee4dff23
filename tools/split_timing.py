"""Phase timing of k_verify_split for lone calls (a timing build of the
library: bash tools/ab_build_def.sh st "-DMBFT_SPLIT_TIMING", then
MBFT_LIB_PATH=minbft_amd/libminbft_amd_st.so python tools/split_timing.py).
Windows as the bench's single calls (G 29, client key 29) unless
MBFT_PROBE_WINDOW / MBFT_PROBE_KEY_WINDOW say otherwise.

Phases (per wave, wall clock at 100 MHz): 0 start, 1 after the range / key
checks, 2 after s^-1, 3 after u1 / u2, 4 after the comb range, 5 after the
level-0 join (waves 0, 2); wave 0: 7 after the level-1 join, 8 after the
x check.
"""
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from minbft_amd import _lib  # noqa: E402
from minbft_amd.authenticator import Authenticator, ROLE_CLIENT, der_encode_rows  # noqa: E402


def main() -> None:
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    lib = _lib.load()
    f = lib.mbft_debug_split_timing
    f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    d = int.from_bytes(hashlib.sha256(b"split timing probe").digest(), "big") % (2**255) + 1
    priv = np.frombuffer(d.to_bytes(32, "big"), dtype=np.uint8).copy().reshape(1, 32)
    msgs = bench.make_requests(0, 64)
    out = (ctypes.c_ulonglong * 162)()
    rows = []
    with Authenticator(0) as a:
        a.set_generator_window(int(os.environ.get("MBFT_PROBE_WINDOW", "29")))
        a.set_key_window(int(os.environ.get("MBFT_PROBE_KEY_WINDOW", "29")))
        r, s = a.sign_prehashed(priv, np.ascontiguousarray(msgs[:, :32]))
        a.add_role(ROLE_CLIENT)
        a.set_public_key(ROLE_CLIENT, 0, bench.pubkey_bytes(d))
        tags, tlen = der_encode_rows(r, s)
        lat = []
        for k in range(n):
            i = k % 64
            m, t = bytes(msgs[i, :47]), bytes(tags[i, :int(tlen[i])])
            t0 = time.perf_counter()
            st = a.verify_status(ROLE_CLIENT, 0, m, t)
            lat.append(time.perf_counter() - t0)
            assert st == 0
            if f(out) != 0:
                raise SystemExit("mbft_debug_split_timing failed")
            v = np.array(out[:64], dtype=np.int64).reshape(4, 16)  # workgroup 0's waves (rows 5 b + wave)
            rows.append(np.where(v > 0, (v - v[0, 0]) * 10.0 / 1000.0, np.nan))  # us from wave 0's start
            clk = (out[161] - out[160]) / max((v[0, 8] - v[0, 0]) * 10.0, 1.0)  # cycles per ns
            rows[-1] = (rows[-1], clk)
        rows = rows[20:]
        med = np.nanmedian(np.stack([r for r, _ in rows]), axis=0)
        clk = float(np.median([c for _, c in rows]))
        res = {"calls": len(rows), "p50_call_us": float(np.median(lat[20:])) * 1e6,
               "shader_GHz": clk,
               "phase_us_by_wave": {f"wave{w}": [round(float(x), 2) for x in med[w][:9]] for w in range(4)},
               "phases": ["start", "checks", "s_inv", "u1u2", "comb", "join0", "-", "join1", "x_check"]}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

"""Latency of small mbft_verify_batch calls (the coalesced single calls'
batches): p50 wall time per batch of k calls, k = 1 .. 64, and the host
stage split (mbft_profile_stages), items packed once outside the timing.
Run under rocprofv3 --kernel-trace --stats for the kernels of each size.

    python tools/small_batch_probe.py [reps]
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
from minbft_amd._lib import MbftItem  # noqa: E402
from minbft_amd.authenticator import Authenticator, ROLE_CLIENT, der_encode_rows  # noqa: E402


def main() -> None:
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    d = int.from_bytes(hashlib.sha256(b"small batch probe").digest(), "big") % (2**255) + 1
    priv = np.frombuffer(d.to_bytes(32, "big"), dtype=np.uint8).copy().reshape(1, 32)
    msgs = bench.make_requests(0, 64)
    out = {}
    with Authenticator(0) as a:
        r, s = a.sign_prehashed(priv, np.ascontiguousarray(msgs[:, :32]))
        a.add_role(ROLE_CLIENT)
        a.set_public_key(ROLE_CLIENT, 0, bench.pubkey_bytes(d))
        tags, tlen = der_encode_rows(r, s)
        mb = [ctypes.create_string_buffer(bytes(msgs[i, :47]), 47) for i in range(64)]
        tb = [ctypes.create_string_buffer(bytes(tags[i, :int(tlen[i])]), int(tlen[i])) for i in range(64)]
        arr = (MbftItem * 64)()
        for i in range(64):
            arr[i].role, arr[i].id = ROLE_CLIENT, 0
            arr[i].msg, arr[i].msg_len = ctypes.cast(mb[i], ctypes.c_void_p), 47
            arr[i].tag, arr[i].tag_len = ctypes.cast(tb[i], ctypes.c_void_p), int(tlen[i])
        st = (ctypes.c_uint8 * 64)()
        for k in (1, 2, 4, 8, 16, 32, 64):
            lat = []
            for j in range(reps + 10):
                t0 = time.perf_counter()
                rc = a.lib.mbft_verify_batch(a.ctx, arr, k, st)
                dt = time.perf_counter() - t0
                if rc != 0 or any(st[i] for i in range(k)):
                    raise SystemExit(f"k={k}: rc {rc}, statuses {list(st[:k])}")
                if j == 9:
                    a.stage_profile()  # reset after the warm-up
                if j >= 10:
                    lat.append(dt)
            sp = a.stage_profile()
            out[k] = {"p50_us": float(np.median(lat)) * 1e6, "p10_us": float(np.percentile(lat, 10)) * 1e6,
                      "host_prepare_us": sp["host_prepare_ms"] * 1e3,
                      "gpu_wait_us": sp["gpu_wait_after_last_chunk_ms"] * 1e3,
                      "total_us": sp["total_ms"] * 1e3}
            print(k, json.dumps(out[k]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

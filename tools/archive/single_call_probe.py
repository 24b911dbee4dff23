"""Single VerifyMessageAuthenTag calls one at a time (the reference's
per-call API) on the GPU box: p50 latency, for a kernel / copy timeline under
rocprofv3 (tools/copy_timeline.py).

    python tools/single_call_probe.py [calls]
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from minbft_amd.authenticator import Authenticator, ROLE_CLIENT, der_encode_rows  # noqa: E402


def main() -> None:
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    d = int.from_bytes(hashlib.sha256(b"single call probe").digest(), "big") % (2**255) + 1
    priv = np.frombuffer(d.to_bytes(32, "big"), dtype=np.uint8).copy().reshape(1, 32)
    msgs = bench.make_requests(0, 64)
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
        lat = lat[20:]
        print(json.dumps({"calls": len(lat), "p50_us": float(np.median(lat)) * 1e6,
                          "min_us": min(lat) * 1e6}), flush=True)


if __name__ == "__main__":
    main()

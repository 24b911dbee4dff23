#!/usr/bin/env python3
"""tests/test_gpu_resident.py::test_resident_beside_batches as a probe: 256K
compact flat batches (GPU decode, 2 lanes) alone and beside the resident
kernel (32 slots) kept alive by single calls every 200 us from a Python
thread; off / live alternated 3 times; prints the best of each and the
ratio.  Knobs from the environment (MBFT_RESIDENT_SERVERS, ..._POLL_SLEEP)."""
import hashlib
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    torch.cuda.init()
    from minbft_amd.authenticator import Authenticator, ROLE_CLIENT, flat_calls, host_array
    from oracle import p256 as o
    d = int.from_bytes(hashlib.sha256(b"beside").digest(), "big") % (o.N - 1) + 1
    q = o.pubkey(d)
    msgs = [b"beside %d" % i + bytes(40) for i in range(64)]
    tags = [o.der_encode_sig(*o.ecdsa_sign(d, o.quirk_digest(m))) for m in msgs]
    B = 1 << 18
    batch = [(ROLE_CLIENT, 0, msgs[i % 64], tags[i % 64]) for i in range(B)]
    flat = flat_calls(batch, True, compact=True)
    a = Authenticator(0)
    alone, live = [], []
    try:
        a.add_role(ROLE_CLIENT)
        a.set_public_key(ROLE_CLIENT, 0, q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big"))
        a.set_concurrency(2)
        out = host_array(B)

        def timed(k):
            ts = []
            for _ in range(k):
                t0 = time.perf_counter()
                a.verify_flat32_arrays(*flat, out=out, pinned=True)
                ts.append(time.perf_counter() - t0)
            assert int((np.asarray(out) == 0).sum()) == B
            return ts

        timed(3)
        mode = os.environ.get("BESIDE_MODE", "resident_calls")
        for _ in range(3):
            alone += timed(6)
            if mode != "calls_only":
                a.set_resident(32)
            stop = threading.Event()

            def singles():
                if mode == "resident_idle":  # one call: the kernel up, then no posts
                    a.verify_status(ROLE_CLIENT, 0, msgs[0], tags[0])
                    return
                while not stop.is_set():
                    a.verify_status(ROLE_CLIENT, 0, msgs[0], tags[0])
                    time.sleep(0.0002)

            th = threading.Thread(target=singles)
            th.start()
            time.sleep(0.01)
            live += timed(6)
            stop.set()
            th.join()
            a.set_resident(0)
    finally:
        a.close()
    print(json.dumps({"mode": mode, "servers": os.environ.get("MBFT_RESIDENT_SERVERS"),
                      "poll_sleep": os.environ.get("MBFT_RESIDENT_POLL_SLEEP"),
                      "alone_ms": min(alone) * 1e3, "live_ms": min(live) * 1e3,
                      "ratio": min(live) / min(alone), "alone_p50": float(np.median(alone)) * 1e3,
                      "live_p50": float(np.median(live)) * 1e3}), flush=True)


if __name__ == "__main__":
    main()

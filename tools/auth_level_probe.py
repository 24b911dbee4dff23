"""Authenticator-level probe (GPU box): mbft_verify_batch on 1M C2 calls
(host items in, statuses out) with the library's stage trace on stderr
(MBFT_STAGE_TRACE), for the host-thread / chunk settings given in the
environment.  Windows 16/16 by default (small tables, quick setup; the host
part does not depend on the window), MBFT_PROBE_WINDOW=29 for the bench's.
MBFT_PROBE_FORM=pinned: the same calls through mbft_verify_batch_flat over
library page-locked buffers (the GPU decode, bench.flat_pinned_level).

    MBFT_HOST_THREADS=16 MBFT_BATCH_CHUNK=262144 MBFT_STAGE_TRACE=1 \
        python tools/auth_level_probe.py [n] [reps]
"""
from __future__ import annotations

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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    d = int.from_bytes(hashlib.sha256(b"minbft-amd bench client 0").digest(), "big") % (2**255) + 1
    priv = np.frombuffer(d.to_bytes(32, "big"), dtype=np.uint8).copy().reshape(1, 32)
    msgs = bench.make_requests(0, n)
    e = np.ascontiguousarray(msgs[:, :32])
    w = int(os.environ.get("MBFT_PROBE_WINDOW", "16"))
    with Authenticator(0) as a:
        if w != 16:
            a.set_generator_window(w)
            a.set_key_window(w)
        r, s = a.sign_prehashed(priv, e)
        a.add_role(ROLE_CLIENT)
        a.set_public_key(ROLE_CLIENT, 0, bench.pubkey_bytes(d))
        tags, tlen = der_encode_rows(r, s)
        items = Authenticator.pack_items(ROLE_CLIENT, 0, msgs, 47, tags, tlen)
        st = np.zeros(n, dtype=np.uint8)
        form = os.environ.get("MBFT_PROBE_FORM", "items")
        if form == "pinned":
            lat, stages, st = bench.flat_pinned_level(a, msgs, tags, tlen, n, reps)
            assert int((st == 0).sum()) == n, "not all accepted"
            print(json.dumps({"n": n, "form": form, "chunk": os.environ.get("MBFT_BATCH_CHUNK"),
                              "p50_ms": float(np.median(lat)) * 1e3, "min_ms": min(lat) * 1e3,
                              "stages": stages}), flush=True)
            return
        lat = []
        for k in range(3 + reps):
            t0 = time.perf_counter()
            a.verify_batch_items(items, st)
            if k >= 3:
                lat.append(time.perf_counter() - t0)
        assert int((st == 0).sum()) == n, "not all accepted"
        p50 = float(np.median(lat))
        print(json.dumps({"n": n, "threads": os.environ.get("MBFT_HOST_THREADS"),
                          "chunk": os.environ.get("MBFT_BATCH_CHUNK"), 
                          "window": w, "p50_ms": p50 * 1e3,
                          "verifies_per_s": n / p50, "min_ms": min(lat) * 1e3}), flush=True)


if __name__ == "__main__":
    main()

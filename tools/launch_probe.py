#!/usr/bin/env python3
"""Does a live resident kernel (another hardware queue, a persistent
dispatch) slow other work's kernel launches?  Per mode: 2000 tiny torch
kernels back to back on one stream (mean per launch, then synchronize), and
the same as 200 synchronized launches (round trip per launch); resident off
vs live and idle (no posts, idle exit 1 s), 1 and 16 servers."""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    torch.cuda.init()
    from minbft_amd.authenticator import Authenticator, ROLE_CLIENT
    from oracle import p256 as o
    d = 777
    q = o.pubkey(d)
    msg = b"launch probe" + bytes(30)
    tag = o.der_encode_sig(*o.ecdsa_sign(d, o.quirk_digest(msg)))
    x = torch.zeros(1024, device="cuda:0")
    st = torch.cuda.Stream()

    def probe():
        with torch.cuda.stream(st):
            for _ in range(200):
                x.add_(1)
            st.synchronize()
            a = time.perf_counter()
            for _ in range(2000):
                x.add_(1)
            st.synchronize()
            burst = (time.perf_counter() - a) / 2000 * 1e6
            rt = []
            for _ in range(200):
                a = time.perf_counter()
                x.add_(1)
                st.synchronize()
                rt.append(time.perf_counter() - a)
        rt.sort()
        return {"burst_us_per_launch": burst, "roundtrip_p50_us": rt[100] * 1e6}

    res = []
    with Authenticator(0) as auth:
        auth.add_role(ROLE_CLIENT)
        auth.set_public_key(ROLE_CLIENT, 0, q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big"))
        for rep in range(2):
            res.append({"mode": "off", **probe()})
            auth.set_resident(32)
            assert auth.verify_status(ROLE_CLIENT, 0, msg, tag) == 0
            res.append({"mode": "resident_idle", "servers": os.environ.get("MBFT_RESIDENT_SERVERS"), **probe()})
            auth.set_resident(0)
    for r in res:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()

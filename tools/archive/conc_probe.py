"""Coalesced concurrent single calls from OS threads (bench.py's
native_concurrent_calls) for chosen (threads, slots) configs (4 lanes), alone,
for a kernel trace under rocprofv3.

    python tools/conc_probe.py 64:4 16:1 ...
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from minbft_amd.authenticator import Authenticator, ROLE_CLIENT, der_encode_rows  # noqa: E402


def main() -> None:
    cfgs = [tuple(int(x) for x in a.split(":")) for a in sys.argv[1:]] or [(64, 4)]
    d = int.from_bytes(hashlib.sha256(b"conc probe").digest(), "big") % (2**255) + 1
    priv = np.frombuffer(d.to_bytes(32, "big"), dtype=np.uint8).copy().reshape(1, 32)
    n = 6400
    msgs = bench.make_requests(0, n)
    with Authenticator(0) as a:
        a.set_generator_window(29)
        a.set_key_window(29)
        r, s = a.sign_prehashed(priv, np.ascontiguousarray(msgs[:, :32]))
        a.add_role(ROLE_CLIENT)
        a.set_public_key(ROLE_CLIENT, 0, bench.pubkey_bytes(d))
        tags, tlen = der_encode_rows(r, s)
        calls = [(bytes(msgs[i, :47]), bytes(tags[i, :int(tlen[i])])) for i in range(n)]
        out = bench.native_concurrent_calls(a, calls, 16, n // 16, configs=cfgs)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

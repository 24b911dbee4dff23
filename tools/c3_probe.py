"""C3 line alone (bench.c3_line: 33 USIG keys + client, mbft_validate_messages)
with the library's stage trace (MBFT_STAGE_TRACE=1) -- host vs GPU split of
the message-level path.

    MBFT_STAGE_TRACE=1 python tools/c3_probe.py [requests]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main() -> None:
    import torch

    from minbft_amd.authenticator import Authenticator
    nreq = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    dev = torch.device("cuda", 0)
    with Authenticator(0) as auth:
        auth.set_generator_window(29)
        print(json.dumps(bench.c3_line(auth, torch, dev, nreq)), flush=True)


if __name__ == "__main__":
    main()

"""One device message-layer check pass at a time (mbft_check_messages_flat +
resolve), for a kernel / API timeline of its fixed cost under rocprofv3:
a C3 peer stream's batch of 4,096 COMMITs (what the Go core's per-stream loop
checks), then 9 streams' batches together (a coalesced pass).

    python tools/msg_pass_probe.py [reps]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main() -> None:
    from minbft_amd.authenticator import Authenticator
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    out = {}
    with Authenticator(0) as auth:
        auth.set_generator_window(int(os.environ.get("MBFT_PROBE_WINDOW", "16")))
        msgs, n, _t, keep = bench.c3_messages(auth, 4096, q_window=16)
        for name, sids in (("one_stream_4096", [1]), ("nine_streams_36864", list(range(1, 10)))):
            sub = np.ascontiguousarray(msgs[np.isin(msgs["stream"], sids)])
            recs, arena = auth.pack_messages(sub, pinned=True)
            lat = []
            for k in range(reps + 3):
                a = time.perf_counter()
                with auth.check_messages_flat(recs, arena, n) as b:
                    r = b.resolve_range(0, sub.shape[0])
                lat.append(time.perf_counter() - a)
                assert (r == 0).all()
            lat = lat[3:]
            out[name] = {"messages": int(sub.shape[0]), "p50_ms": float(np.median(lat)) * 1e3,
                         "min_ms": float(min(lat)) * 1e3}
        del keep
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""C2 ms/step in consecutive 20-step windows after an idle pause: how long the
GPU takes to reach its sustained rate from idle (the driver times 5 warm-up +
20 steps).  One JSON line per pause: {idle_s, windows: [ms/step ...]}."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from c2_setup import C2  # noqa: E402


def main():
    c = C2()
    torch = c.torch
    try:
        for idle in (0.0, 0.2, 1.0, 3.0):
            torch.cuda.synchronize()
            time.sleep(idle)
            ws = []
            for _ in range(30):
                torch.cuda.synchronize()
                a = time.perf_counter()
                for _ in range(20):
                    c.step()
                torch.cuda.synchronize()
                ws.append(round((time.perf_counter() - a) / 20 * 1e3, 4))
            print(json.dumps({"idle_s": idle, "windows_ms_per_step": ws}), flush=True)
    finally:
        c.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Resident verifier A/B probe (round 6): on the C2 setup (G 29 / Q 29, 1M
single-signer REQUESTs), one JSON line per run with

  * the lone resident call (p50 us, process CPU-us per call),
  * 16 and 64 OS-thread callers (calls/s, CPU-us per call; slots = callers),
  * the resident kernel's cost to C2 steps and to the 1M authenticator-level
    batch with 32 slots kept alive by a 200-us call trickle
    (bench.resident_interference).

Knobs come from the environment (MBFT_RESIDENT_SERVERS, MBFT_RESIDENT_SLEEP,
MBFT_LIB_PATH for another build), so one GPU call can compare several.

    python tools/resident_ab.py [--tag NAME] [--steps 200]
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--no-interference", action="store_true")
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    from minbft_amd.authenticator import Authenticator, ROLE_CLIENT, der_encode_rows
    B = args.batch
    auth = Authenticator(0)
    try:
        auth.set_generator_window(29)
        d = int.from_bytes(hashlib.sha256(b"minbft-amd bench client 0").digest(), "big")
        d = d % (0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551 - 1) + 1
        priv = np.frombuffer(d.to_bytes(32, "big"), dtype=np.uint8).copy()
        msgs = bench.make_requests(0, B)
        e = np.ascontiguousarray(msgs[:, :32])
        d_priv = torch.from_numpy(priv).to(dev)
        d_e = torch.from_numpy(e).to(dev)
        d_r = torch.empty((B, 32), dtype=torch.uint8, device=dev)
        d_s = torch.empty((B, 32), dtype=torch.uint8, device=dev)
        auth.sign_prehashed_device(d_priv.data_ptr(), 0, d_e.data_ptr(), B, d_r.data_ptr(), d_s.data_ptr(),
                                   torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        auth.set_key_window(29)
        auth.add_role(ROLE_CLIENT)
        auth.set_public_key(ROLE_CLIENT, 0, bench.pubkey_bytes(d))
        slot = auth.key_slot(ROLE_CLIENT, 0)
        d_slot = torch.full((B,), slot, dtype=torch.int32, device=dev)
        streams = [torch.cuda.Stream(device=dev) for _ in range(3)]
        d_sts = [torch.empty((B,), dtype=torch.uint8, device=dev) for _ in streams]
        n = [0]

        def step():
            k = n[0] % 3
            n[0] += 1
            auth.verify_prehashed_device(d_e.data_ptr(), d_r.data_ptr(), d_s.data_ptr(), d_slot.data_ptr(), B,
                                         d_sts[k].data_ptr(), streams[k].cuda_stream)

        for _ in range(3):
            step()
        torch.cuda.synchronize()
        if min(int((x == 0).sum().item()) for x in d_sts) != B:
            raise SystemExit("gate: valid batch not accepted")
        tags, tlen = der_encode_rows(d_r.cpu().numpy(), d_s.cpu().numpy())
        calls = [(bytes(msgs[i]), bytes(tags[i, :tlen[i]])) for i in range(16 * 400)]
        out = {"tag": args.tag, "servers_env": os.environ.get("MBFT_RESIDENT_SERVERS"),
               "sleep_env": os.environ.get("MBFT_RESIDENT_SLEEP"), "lib": os.environ.get("MBFT_LIB_PATH")}
        nat = bench.native_concurrent_calls(auth, calls, 16, 400, configs=(),
                                            resident_configs=((1, 1), (16, 16), (16, 32), (64, 64)))
        out["native"] = {k: {a: v[a] for a in ("calls_per_s", "cpu_us_per_call", "mean_call_us")}
                         for k, v in nat.items() if isinstance(v, dict) and "mean_call_us" in v}
        if not args.no_interference:
            ri = bench.resident_interference(auth, torch, step, args.steps, msgs, tags, tlen, B, 10)
            out["interference"] = {k: ri[k] for k in ("c2_ms_per_step", "c2_ratio", "auth_level_p50_ms",
                                                      "auth_level_ratio", "trickle", "c2_ms_per_step_runs")}
        print(json.dumps(out), flush=True)
    finally:
        auth.close()


if __name__ == "__main__":
    main()

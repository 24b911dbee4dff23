"""Where a k_verify comb step's cycles go: stamps in a
timing build of the library (bash tools/ab_build_def.sh stp
"-DMBFT_STEP_TIMING"; kernels.hip comb_step), per wave and step: waiting for
the gather prefetched one step earlier, reading it from LDS, issuing the next
gather, and the mixed addition.  Run with the timing build and with the
normal one (launch time only), at the benched windows (G 29 / Q 29) on the
C2 batch (1M single-signer items), 3 waves per SIMD (the default grid) or 1
(MBFT_VERIFY_BPC=1: one 256-thread block per CU, grid-stride).

    MBFT_LIB_PATH=minbft_amd/libminbft_amd_stp.so python tools/step_timing.py
    MBFT_VERIFY_BPC=1 MBFT_LIB_PATH=... python tools/step_timing.py
Prints one JSON object.
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


def main() -> None:
    import torch
    torch.cuda.init()
    import bench
    from minbft_amd import _lib
    from minbft_amd.authenticator import Authenticator
    B = int(os.environ.get("MBFT_PROBE_BATCH", str(1 << 20)))
    reps = 10
    lib = _lib.load()
    timing = hasattr(lib, "mbft_debug_step_timing")
    if timing:
        f = lib.mbft_debug_step_timing
        f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    dev = torch.device("cuda", 0)
    d = int.from_bytes(hashlib.sha256(b"minbft-amd bench client 0").digest(), "big") % (bench.N_ORDER - 1) + 1
    msgs = bench.make_requests(0, B)
    with Authenticator(0) as a:
        a.set_generator_window(29)
        a.set_key_window(29)
        d_priv = torch.from_numpy(np.frombuffer(d.to_bytes(32, "big"), dtype=np.uint8).copy()).to(dev)
        d_e = torch.from_numpy(np.ascontiguousarray(msgs[:, :32])).to(dev)
        d_r = torch.empty((B, 32), dtype=torch.uint8, device=dev)
        d_s = torch.empty((B, 32), dtype=torch.uint8, device=dev)
        st = torch.cuda.current_stream().cuda_stream
        a.sign_prehashed_device(d_priv.data_ptr(), 0, d_e.data_ptr(), B, d_r.data_ptr(), d_s.data_ptr(), st)
        a.add_role(3)
        a.set_public_key(3, 0, bench.pubkey_bytes(d))
        slot = a.key_slot(3, 0)
        d_slot = torch.full((B,), slot, dtype=torch.int32, device=dev)
        d_st = torch.empty((B,), dtype=torch.uint8, device=dev)

        def one():
            a.verify_prehashed_device(d_e.data_ptr(), d_r.data_ptr(), d_s.data_ptr(), d_slot.data_ptr(), B,
                                      d_st.data_ptr(), st)
        for _ in range(3):
            one()
        torch.cuda.synchronize()
        assert int((d_st == 0).sum().item()) == B
        out = (ctypes.c_ulonglong * 12)()
        if timing:
            f(out, 1)
        a.profile(True)
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t = time.perf_counter()
            one()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
        prof = a.profile_read()
        a.profile(False)
        res = {"lib": os.path.basename(_lib.LIB_PATH), "batch": B,
               "verify_bpc": os.environ.get("MBFT_VERIFY_BPC", "default (3 waves/SIMD)"),
               "k_verify_ms": prof["verify_ms"] / max(prof["batches"], 1),
               "p50_launch_wall_ms": float(np.median(ts)) * 1e3}
        if timing:
            f(out, 0)
            steps = max(out[4], 1)
            names = ["gather_wait", "lds_read", "gather_issue", "mixed_add"]
            per = {nm: out[k] / steps for k, nm in enumerate(names)}
            tot = sum(per.values())
            w = max(out[5], 1)
            res.update({"waves": int(out[5]), "steps": int(out[4]), "steps_per_wave": out[4] / w,
                        "cycles_per_step_per_wave": per, "cycles_per_step_total": tot,
                        "share": {k: v / tot for k, v in per.items()},
                        "in_kernel_clock_GHz": out[6] / max(out[7], 1) * 0.1,
                        "per_wave_cycles": {"comb": out[6] / w, "before_comb": out[9] / w,
                                            "verify_one_total": out[8] / w}})
        print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

"""Where a lone resident-kernel call's time goes (timing build: bash
tools/ab_build_def.sh srvt "-DMBFT_SRV_TIMING -DMBFT_SPLIT_TIMING";
MBFT_RESIDENT_FORM two / one): host part, post,
post -> done seen, host join (host clock), and the kernel's slot copy,
comb + partials and split_item's phases of slot 0 (100 MHz wall clock).
C2 calls at the benched windows (G 29 / Q 29).

    MBFT_RESIDENT_FORM=two MBFT_LIB_PATH=minbft_amd/libminbft_amd_srvt.so python tools/resident_timing.py
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
    from minbft_amd.authenticator import Authenticator, der_encode_rows
    B = 4096
    lib = _lib.load()
    rt = lib.mbft_debug_resident_timing
    rt.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int]
    sp = lib.mbft_debug_split_timing
    sp.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    dev = torch.device("cuda", 0)
    d = int.from_bytes(hashlib.sha256(b"minbft-amd bench client 0").digest(), "big") % (bench.N_ORDER - 1) + 1
    msgs = bench.make_requests(0, B)
    out = {}
    with Authenticator(0) as a:
        a.set_generator_window(29)
        a.set_key_window(29)
        d_priv = torch.from_numpy(np.frombuffer(d.to_bytes(32, "big"), dtype=np.uint8).copy()).to(dev)
        d_e = torch.from_numpy(np.ascontiguousarray(msgs[:, :32])).to(dev)
        d_r = torch.empty((B, 32), dtype=torch.uint8, device=dev)
        d_s = torch.empty((B, 32), dtype=torch.uint8, device=dev)
        a.sign_prehashed_device(d_priv.data_ptr(), 0, d_e.data_ptr(), B, d_r.data_ptr(), d_s.data_ptr(),
                                torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        a.add_role(3)
        a.set_public_key(3, 0, bench.pubkey_bytes(d))
        tags, tlen = der_encode_rows(d_r.cpu().numpy(), d_s.cpu().numpy())
        calls = [(bytes(msgs[i]), bytes(tags[i, :tlen[i]])) for i in range(B)]
        a.set_resident(1)
        for k in range(50):
            assert a.verify_status(3, 0, *calls[k]) == 0
        buf = (ctypes.c_double * 7)()
        rt(buf, 1)
        n = 2000
        lat = []
        phases = []
        st = (ctypes.c_ulonglong * 162)()
        two = os.environ.get("MBFT_RESIDENT_FORM", "two") == "two"
        for k in range(n):
            t = time.perf_counter()
            assert a.verify_status(3, 0, *calls[k % B]) == 0
            lat.append(time.perf_counter() - t)
            if k % 10 == 0:
                sp(st)
                v = np.array(st[:160], dtype=np.int64).reshape(10, 16)
                v = v[[0, 1, 2, 3, 5, 6, 7, 8]] if two else v[:4]  # rows 5 workgroup + wave
                base = v[0, 1]  # wave 0 past the input checks
                # per wave: entries in, comb done (us after wave 0's input checks)
                phases.append(np.stack([(v[:, 9] - base) / 100.0, (v[:, 4] - base) / 100.0], axis=1))
        rt(buf, 0)
        names = ["host_prepare", "post_incl_winv", "post_to_done_seen", "host_join", "kernel_slot_copy",
                 "kernel_comb_and_partials", "host_join_copy"]
        out = {"calls": n, "p50_call_us": float(np.median(lat)) * 1e6,
               "mean_us": {nm: buf[i] / n * 1e3 for i, nm in enumerate(names)},
               "per_wave_us_after_checks_slot0": {
                   "entries_in": np.median(np.array(phases), axis=0)[:, 0].round(2).tolist(),
                   "comb_done": np.median(np.array(phases), axis=0)[:, 1].round(2).tolist()}}
        a.set_resident(0)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

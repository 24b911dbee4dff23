"""Build the in-tree HIP library ``minbft_amd/libminbft_amd.so`` for gfx950.

Plain ``hipcc`` invocations (no cmake): the kernels TU is compiled for
``--offload-arch=gfx950`` only, the host TUs are ordinary C++ linked into the
same shared object.  Rebuilds only when a source is newer than the library.

    python -m minbft_amd.build [--force]
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
ROOT = os.path.dirname(HERE)
LIB = os.path.join(HERE, "libminbft_amd.so")
OBJDIR = os.path.join(HERE, "build")

ARCH = os.environ.get("MBFT_OFFLOAD_ARCH", "gfx950")

DEVICE_SOURCES = ["kernels.hip", "msg_kernels.hip"]
HOST_SOURCES = ["host.cpp", "der.cpp", "messages.cpp", "batch.cpp", "msgdev.cpp", "winv_host.cpp"]
HEADERS = ["fe29.h", "ecc.h", "modinv.h", "der_dev.h", "sha256.h", "sha256_dev.h", "authen_dev.h", "arena_dev.h",
           "kernels.h",
           "msg_dev.h", "host_internal.h"]


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm required to build minbft_amd)")


def _inputs():
    files = [os.path.join(CSRC, f) for f in DEVICE_SOURCES + HOST_SOURCES + HEADERS]
    files.append(os.path.join(ROOT, "include", "minbft_gpu.h"))
    files.append(os.path.abspath(__file__))
    return files


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(f) <= t for f in _inputs())


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and up_to_date():
        return LIB
    hipcc = _hipcc()
    os.makedirs(OBJDIR, exist_ok=True)
    common = ["-O3", "-std=c++17", "-fPIC", "-Wno-unused-result", "-I", os.path.join(ROOT, "include")]
    jobs = []
    for f in DEVICE_SOURCES:
        obj = os.path.join(OBJDIR, f + ".o")
        jobs.append(([hipcc, f"--offload-arch={ARCH}", *common, "-c", os.path.join(CSRC, f), "-o", obj], obj))
    for f in HOST_SOURCES:
        obj = os.path.join(OBJDIR, f + ".o")
        jobs.append(([hipcc, *common, "-c", os.path.join(CSRC, f), "-o", obj], obj))

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        p = subprocess.run(cmd, capture_output=True, text=True)
        if p.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{p.stdout}\n{p.stderr}")
        return p

    with ThreadPoolExecutor(max_workers=len(jobs)) as ex:
        list(ex.map(lambda j: run(j[0]), jobs))
    tmp = LIB + ".tmp"
    run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *[o for _, o in jobs]])
    os.replace(tmp, LIB)
    return LIB


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    print(build(force=a.force, verbose=a.verbose))


if __name__ == "__main__":
    sys.exit(main())

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
HOST_SOURCES = ["host.cpp", "der.cpp", "messages.cpp", "batch.cpp", "msgdev.cpp", "winv_host.cpp",
                "sha256_host.cpp", "resident.cpp", "join_host.cpp"]
HEADERS = ["fe29.h", "ecc.h", "modinv.h", "der_dev.h", "sha256.h", "sha256_dev.h", "authen_dev.h", "arena_dev.h",
           "kernels.h",
           "msg_dev.h", "host_internal.h", "join_core.inc"]


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


def _deps(src: str) -> list:
    """src, the quoted headers it includes (transitively), the public
    header and this script."""
    import re
    seen, todo = set(), [src]
    while todo:
        f = todo.pop()
        if f in seen or not os.path.exists(f):
            continue
        seen.add(f)
        with open(f, errors="replace") as fh:
            for inc in re.findall(r'^\s*#\s*include\s+"([^"]+)"', fh.read(), re.M):
                todo.append(os.path.normpath(os.path.join(os.path.dirname(f), inc)))
    return sorted(seen) + [os.path.join(ROOT, "include", "minbft_gpu.h"), os.path.abspath(__file__)]


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

    # an object is rebuilt only when its source or a header it includes
    # (transitively, quoted includes) is newer, or the build script changed
    stale = [j for j in jobs if force or not os.path.exists(j[1])
             or os.path.getmtime(j[1]) < max(os.path.getmtime(d) for d in _deps(j[0][-3]))]
    if stale:
        with ThreadPoolExecutor(max_workers=len(stale)) as ex:
            list(ex.map(lambda j: run(j[0]), stale))
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

"""Instruction histogram of the loops of one kernel in a gfx950 .s dump.

    hipcc -x hip --offload-arch=gfx950 --cuda-device-only -O3 -S kernels.hip -o k.s
    python tools/isa_hist.py k.s _Z8k_verifyILi3EEv10VerifyArgs

For every backward branch (a loop) prints the body's instruction count by
class (VALU / v_mad_u64_u32 / SALU / LDS / VMEM / other) and the most
frequent VALU mnemonics, so per-step instruction counts can be compared
across changes without a GPU.
"""
from __future__ import annotations

import collections
import re
import sys


def kernel_lines(path: str, sym: str) -> list[str]:
    out, on = [], False
    for ln in open(path):
        if ln.startswith(sym + ":"):
            on = True
            continue
        if on:
            if ln.startswith(".Lfunc_end"):
                break
            out.append(ln.rstrip("\n"))
    return out


def classify(m: str) -> str:
    if m == "v_mad_u64_u32":
        return "v_mad_u64_u32"
    if m.startswith("v_"):
        return "valu"
    if m.startswith("s_"):
        return "salu"
    if m.startswith("ds_"):
        return "lds"
    if m.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main() -> None:
    path, sym = sys.argv[1], sys.argv[2]
    lines = kernel_lines(path, sym)
    labels = {}
    for i, ln in enumerate(lines):
        m = re.match(r"^(\.LBB[\w_]+):", ln)
        if m:
            labels[m.group(1)] = i
    loops = []
    for i, ln in enumerate(lines):
        m = re.match(r"^\s+s_cbranch_\w+\s+(\.LBB[\w_]+)|^\s+s_branch\s+(\.LBB[\w_]+)", ln)
        if m:
            tgt = m.group(1) or m.group(2)
            if tgt in labels and labels[tgt] < i:
                loops.append((labels[tgt], i))
    for a, b in loops:
        cls, mn = collections.Counter(), collections.Counter()
        for ln in lines[a:b + 1]:
            t = ln.strip()
            if not t or t.startswith((";", ".")):
                continue
            op = t.split()[0]
            cls[classify(op)] += 1
            if op.startswith("v_"):
                mn[op] += 1
        valu = cls["valu"] + cls["v_mad_u64_u32"]
        if valu < int(sys.argv[3]) if len(sys.argv) > 3 else valu < 50:
            continue
        print(f"loop lines {a}-{b}: VALU {valu} (mad {cls['v_mad_u64_u32']}), "
              f"SALU {cls['salu']}, LDS {cls['lds']}, VMEM {cls['vmem']}")
        for op, c in mn.most_common(25):
            print(f"    {c:5d} {op}")


if __name__ == "__main__":
    main()

"""Drive tools/fe_debug.hip: replay the table chain d*Q for one key and find
the first wrong group operation and the first wrong intermediate in it.

    python3 tools/fe_debug.py KEYSEED_TAG D
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from oracle import p256 as o  # noqa: E402

P, N = o.P, o.N
R = 1 << 261
RINV = pow(R, -1, P)


def limbs_to_int(l):
    return sum(int(v) << (29 * i) for i, v in enumerate(l))


def mont(v):
    return v * RINV % P


def main(tag="c4 key 3", d=30855):
    lib = ctypes.CDLL(os.path.abspath("tools/libfe_debug.so"))
    rs = lib.fe_debug_rec_size()
    dk = int.from_bytes(__import__("hashlib").sha256(tag.encode()).digest(), "big") % (N - 1) + 1
    Q = o.pubkey(dk)
    xyw = np.zeros(16, dtype=np.uint32)
    for i in range(8):
        xyw[i] = (Q[0] >> (32 * i)) & 0xFFFFFFFF
        xyw[8 + i] = (Q[1] >> (32 * i)) & 0xFFFFFFFF
    buf = ctypes.create_string_buffer(64 * rs)
    n = ctypes.c_uint32(0)
    rc = lib.fe_debug_chain(xyw.ctypes.data_as(ctypes.c_void_p), d, buf, ctypes.byref(n))
    print("rc", rc, "records", n.value, "rec size", rs)
    recs = np.frombuffer(buf.raw, dtype=np.uint32).reshape(64, rs // 4)[: n.value]
    k = 1
    top = d.bit_length() - 1
    bits = [(d >> b) & 1 for b in range(top - 1, -1, -1)]
    ops = []
    for bt in bits:
        k = 2 * k
        ops.append(("dbl", k))
        if bt:
            k += 1
            ops.append(("madd", k))
    prev = None
    for j, (rec, (op, mult)) in enumerate(zip(recs, ops)):
        X = mont(limbs_to_int(rec[1:10]))
        Y = mont(limbs_to_int(rec[10:19]))
        Z = mont(limbs_to_int(rec[19:28]))
        zi = pow(Z, -1, P)
        ax, ay = X * zi * zi % P, Y * zi * zi * zi % P
        want = o.scalar_mult(mult, Q)
        ok = (ax, ay) == want
        maxl = max(int(v) for v in rec[1:28])
        print(j, op, mult, "ok" if ok else "WRONG", "max limb bits", maxl.bit_length())
        if not ok:
            if op == "madd" and prev is not None:
                x1, y1, z1 = prev
                x2, y2 = Q
                t = [mont(limbs_to_int(rec[28 + 9 * i: 37 + 9 * i])) for i in range(12)]
                raw = [limbs_to_int(rec[28 + 9 * i: 37 + 9 * i]) for i in range(12)]
                exp = {}
                exp[0] = z1 * z1 % P
                exp[1] = exp[0] * z1 % P
                exp[2] = exp[0] * x2 % P
                exp[3] = exp[1] * y2 % P
                exp[4] = (exp[2] - x1) % P
                exp[5] = (exp[3] - y1) % P
                exp[6] = exp[4] * exp[4] % P
                exp[7] = exp[6] * exp[4] % P
                exp[8] = exp[6] * x1 % P
                exp[9] = exp[5] * exp[5] % P
                x3 = (exp[9] - exp[7] - 2 * exp[8]) % P
                exp[10] = (exp[8] - x3) % P
                exp[11] = (-y1) % P
                names = ["Z1^2", "Z1^3", "U2", "S2", "H", "R", "H^2", "H^3", "X1H^2", "R^2",
                         "X1H^2-X3", "-Y1"]
                for i in range(12):
                    print("   ", names[i], "ok" if t[i] == exp[i] else "WRONG",
                          "raw bits", raw[i].bit_length(),
                          "limbs", [int(v).bit_length() for v in rec[28 + 9 * i: 37 + 9 * i]])
                y3 = (exp[5] * exp[10] - y1 * exp[7]) % P
                print("    X3", "ok" if mont(limbs_to_int(rec[1:10])) == x3 else "WRONG",
                      "Y3", "ok" if Y == y3 else "WRONG")
                print("    prev limbs X", list(prev_l[0]), "\n    Y", list(prev_l[1]),
                      "\n    Z", list(prev_l[2]))
            break
        prev = (X, Y, Z)
        prev_l = (rec[1:10], rec[10:19], rec[19:28])


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["c4 key 3"]), *([int(sys.argv[2])] if len(sys.argv) > 2 else []))

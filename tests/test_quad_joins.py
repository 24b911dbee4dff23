"""The argument behind k_verify_quads' joins (kernels.hip verify_quad): the
low and high halves of one scalar's signed-digit comb windows never meet in
a degenerate addition.  With u = a + b (a: windows [0, mid), b: [mid, S)),
a == -b (mod N) only for u == 0, and a == b (mod N) needs u = 2 a + N with a
the low part of u itself; no window size 8..29 admits one.  Pure Python over
the kernel's recoding (comb_digit), no GPU."""
import random

import pytest

N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551


def split(u, W):
    """(a, b): the comb recoding of u (kernels.hip comb_digit, top window
    unsigned) summed over the low and the high half of its windows."""
    S = (256 + W - 1) // W
    mid = (S + 1) // 2
    carry, a, b = 0, 0, 0
    for k in range(S):
        x = ((u >> (W * k)) & ((1 << W) - 1)) + carry
        neg = k + 1 < S and x > (1 << (W - 1))
        carry = 1 if neg else 0
        d = x - (1 << W) if neg else x
        if k < mid:
            a += d << (W * k)
        else:
            b += d << (W * k)
    return a, b, mid


@pytest.mark.parametrize("W", list(range(8, 30)))
def test_halves_sum_to_the_scalar(W):
    rng = random.Random(W)
    for u in [1, 2, N - 1, N - 2, (1 << 255) + 7] + [rng.randrange(1, N) for _ in range(200)]:
        a, b, mid = split(u, W)
        assert a + b == u
        assert b % (1 << (W * mid)) == 0
        assert abs(a) <= 1 << (W * mid)


@pytest.mark.parametrize("W", list(range(8, 30)))
def test_no_degenerate_half_join(W):
    S = (256 + W - 1) // W
    mid = (S + 1) // 2
    M = 1 << (W * mid)
    # a == b (mod N) <=> u = 2a + kN; a == low part of u <=> a == u == -kN (mod M)
    for k in (-1, 0, 1):
        for a in ((-k * N) % M, (-k * N) % M - M):
            u = 2 * a + k * N
            if 0 < u < N:
                got_a, got_b, _ = split(u, W)
                assert got_a != a or (got_a - got_b) % N != 0, (W, hex(u))

// The end of a resident-kernel verify on the host (declared in
// host_internal.h; resident.cpp).  k_verify_server leaves the four partial
// comb sums of an item -- u1's low and high windows times G, u2's times Q,
// Chudnovsky (X, Y, ZZ = Z^2, ZZZ = Z^3) in the device's 9 x 29-bit
// Montgomery limbs (R = 2^261) -- in host-mapped memory, and the caller's
// thread joins them and runs crypto/ecdsa.Verify's final test (the point at
// infinity rejects, else accept iff x mod N == r; Go: crypto/ecdsa
// verifyGeneric, called at sample/authentication/crypto.go:86) instead of
// one GPU wave running the three joins and the x-check one product level at
// a time (~10 us of a lone call).  Complete: equal partial sums double,
// opposite ones give infinity.  A TU of its own so the CPU tests link it
// alone (mbft_debug_host_join).
#include <stddef.h>
#include <stdint.h>
#include <string.h>

namespace mbft_host {

namespace {

using u128 = unsigned __int128;

// p = 2^256 - 2^224 + 2^192 + 2^96 - 1, 4 LE 64-bit limbs; -p^-1 = 1 mod 2^64
const uint64_t kP[4] = {0xFFFFFFFFFFFFFFFFULL, 0x00000000FFFFFFFFULL, 0x0000000000000000ULL,
                        0xFFFFFFFF00000001ULL};
struct F {
  uint64_t v[4];
};
const F kR2p = {{0x0000000000000003ULL, 0xFFFFFFFBFFFFFFFFULL, 0xFFFFFFFFFFFFFFFEULL,
                 0x00000004FFFFFFFDULL}};  // 2^512 mod p
const F kOneM = {{0x0000000000000001ULL, 0xFFFFFFFF00000000ULL, 0xFFFFFFFFFFFFFFFFULL,
                  0x00000000FFFFFFFEULL}};  // 2^256 mod p: 1 in the host's Montgomery form
// N (the group order), for the r + N < p case of the x test
const uint64_t kN[4] = {0xF3B9CAC2FC632551ULL, 0xBCE6FAADA7179E84ULL, 0xFFFFFFFFFFFFFFFFULL,
                        0xFFFFFFFF00000000ULL};

bool geq(const uint64_t a[4], const uint64_t b[4]) {
  for (int j = 3; j >= 0; j--)
    if (a[j] != b[j]) return a[j] > b[j];
  return true;
}

// a -= b (no modulus); returns the borrow
uint64_t sub4(uint64_t a[4], const uint64_t b[4]) {
  u128 br = 0;
  for (int j = 0; j < 4; j++) {
    const u128 d = (u128)a[j] - b[j] - br;
    a[j] = (uint64_t)d;
    br = (d >> 64) & 1;
  }
  return (uint64_t)br;
}

// a += b; returns the carry
uint64_t add4(uint64_t a[4], const uint64_t b[4]) {
  u128 c = 0;
  for (int j = 0; j < 4; j++) {
    c += (u128)a[j] + b[j];
    a[j] = (uint64_t)c;
    c >>= 64;
  }
  return (uint64_t)c;
}

F addm(const F& a, const F& b) {
  F r = a;
  const uint64_t c = add4(r.v, b.v);
  if (c || geq(r.v, kP)) sub4(r.v, kP);
  return r;
}

F subm(const F& a, const F& b) {
  F r = a;
  if (sub4(r.v, b.v)) add4(r.v, kP);
  return r;
}

// a b 2^-256 mod p (CIOS; m = t0 since -p^-1 = 1), inputs < p, output < p.
// (A plain product with the NIST P-256 word reduction measured 1.6x slower
// per product on this host: its signed word sums and carry loop.)
F mul(const F& a, const F& b) {
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      c += (u128)a.v[j] * b.v[i] + t[j];
      t[j] = (uint64_t)c;
      c >>= 64;
    }
    c += t[4];
    t[4] = (uint64_t)c;
    t[5] = (uint64_t)(c >> 64);
    const uint64_t m = t[0];
    c = (u128)m * kP[0] + t[0];
    c >>= 64;
    for (int j = 1; j < 4; j++) {
      c += (u128)m * kP[j] + t[j];
      t[j - 1] = (uint64_t)c;
      c >>= 64;
    }
    c += t[4];
    t[3] = (uint64_t)c;
    t[4] = t[5] + (uint64_t)(c >> 64);
  }
  F r;
  memcpy(r.v, t, sizeof(r.v));
  if (t[4] || geq(r.v, kP)) sub4(r.v, kP);
  return r;
}

bool is_zero(const F& a) { return (a.v[0] | a.v[1] | a.v[2] | a.v[3]) == 0; }
bool eq(const F& a, const F& b) { return memcmp(a.v, b.v, sizeof(a.v)) == 0; }

// The device's limbs (value = sum w[k] 2^(29 k), each w[k] < 2^32: lazy
// limbs allowed) -> the value mod p, in the host's Montgomery form (x 2^256).
// The device value is v 2^261 (its Montgomery form), so one product by
// 2^251 (< p, its own host form times 2^-5) gives v 2^256.
F from_dev(const uint32_t* w) {
  uint64_t acc[5] = {0, 0, 0, 0, 0};
  for (int k = 0; k < 9; k++) {  // add w[k] << 29k
    const int bit = 29 * k, q = bit >> 6, s = bit & 63;
    const u128 x = (u128)w[k] << s;
    u128 c = (u128)acc[q] + (uint64_t)x;
    acc[q] = (uint64_t)c;
    c = (c >> 64) + (uint64_t)(x >> 64);
    for (int j = q + 1; j < 5 && c; j++) {
      c += acc[j];
      acc[j] = (uint64_t)c;
      c >>= 64;
    }
  }
  // fold the bits from 2^256 up: 2^256 = 2^224 - 2^192 - 2^96 + 1 (mod p),
  // i.e. h 2^256 -> h (2^256 - p) = h (2^224 - 2^192 - 2^96 + 1)
  while (acc[4]) {
    const uint64_t h = acc[4];
    acc[4] = 0;
    // + h, + h 2^224; - h 2^192, - h 2^96 (h < 2^33: no wrap beyond acc[4])
    uint64_t plus[4] = {h, 0, 0, h << 32}, plus_hi = h >> 32;
    uint64_t minus[4] = {0, h << 32, 0, 0}, minus_hi = 0;
    minus[2] = h >> 32;
    minus[3] = h;
    (void)minus_hi;
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      c += (u128)acc[j] + plus[j];
      acc[j] = (uint64_t)c;
      c >>= 64;
    }
    acc[4] += (uint64_t)c + plus_hi;
    u128 br = 0;
    for (int j = 0; j < 4; j++) {
      const u128 d = (u128)acc[j] - minus[j] - br;
      acc[j] = (uint64_t)d;
      br = (d >> 64) & 1;
    }
    acc[4] -= (uint64_t)br;
  }
  F r;
  memcpy(r.v, acc, sizeof(r.v));
  while (geq(r.v, kP)) sub4(r.v, kP);
  static const F k2_251 = {{0, 0, 0, (uint64_t)1 << 59}};
  return mul(r, k2_251);
}

struct Pt {
  F X, Y, ZZ, ZZZ;
  bool inf;
  bool aff;  // ZZ = ZZZ = 1
};

// dbl-2008-s-1 (xyzz, a = -3)
Pt dbl(const Pt& a) {
  if (a.inf || is_zero(a.Y)) return Pt{{}, {}, {}, {}, true, false};
  const F U = addm(a.Y, a.Y);
  const F V = mul(U, U);
  const F W = mul(U, V);
  const F S = mul(a.X, V);
  const F M1 = mul(subm(a.X, a.ZZ), addm(a.X, a.ZZ));
  const F M = addm(addm(M1, M1), M1);
  Pt r;
  r.inf = false;
  r.aff = false;
  r.X = subm(subm(mul(M, M), S), S);
  r.Y = subm(mul(M, subm(S, r.X)), mul(W, a.Y));
  r.ZZ = mul(V, a.ZZ);
  r.ZZZ = mul(W, a.ZZZ);
  return r;
}

// add-2008-s (xyzz), complete: equal points double, opposite ones cancel;
// an affine b (ZZ = ZZZ = 1: the kernel's single-window partials) saves
// four products
Pt add(const Pt& a, const Pt& b) {
  if (a.inf) return b;
  if (b.inf) return a;
  const bool aff = b.aff;
  const F U1 = aff ? a.X : mul(a.X, b.ZZ), U2 = mul(b.X, a.ZZ);
  const F S1 = aff ? a.Y : mul(a.Y, b.ZZZ), S2 = mul(b.Y, a.ZZZ);
  const F P = subm(U2, U1), R = subm(S2, S1);
  if (is_zero(P)) {
    if (is_zero(R)) return dbl(a);
    return Pt{{}, {}, {}, {}, true, false};
  }
  const F PP = mul(P, P), PPP = mul(P, PP), Q = mul(U1, PP);
  Pt r;
  r.inf = false;
  r.aff = false;
  r.X = subm(subm(subm(mul(R, R), PPP), Q), Q);
  r.Y = subm(mul(R, subm(Q, r.X)), mul(S1, PPP));
  r.ZZ = aff ? mul(a.ZZ, PP) : mul(mul(a.ZZ, b.ZZ), PP);
  r.ZZZ = aff ? mul(a.ZZZ, PPP) : mul(mul(a.ZZZ, b.ZZZ), PPP);
  return r;
}

}  // namespace

// part: nparts partial sums, 40 words each: X, Y, ZZ, ZZZ (9 device limbs each),
// then a flags word (1: infinity -- every digit of the range was zero);
// r_be: the signature's r (32 B big-endian, 0 < r < N already checked).
// Returns 0 (accept) or 1 (reject).
uint8_t host_join_check(const uint32_t* part, int nparts, const uint8_t* r_be) {
  Pt pts[16];
  int np = 0;
  for (int w = 0; w < nparts && w < 16; w++) {
    const uint32_t* q = part + 40 * w;
    if (q[36] & 1u) continue;
    Pt& p = pts[np++];
    p.inf = false;
    p.X = from_dev(q);
    p.Y = from_dev(q + 9);
    p.ZZ = from_dev(q + 18);
    p.ZZZ = from_dev(q + 27);
    p.aff = eq(p.ZZ, kOneM) && eq(p.ZZZ, kOneM);
  }
  // the projective partials first, so the affine ones join by the cheaper form
  Pt acc{{}, {}, {}, {}, true, false};
  for (int pass = 0; pass < 2; pass++)
    for (int k = 0; k < np; k++)
      if (pts[k].aff == (pass == 1)) acc = add(acc, pts[k]);
  if (acc.inf) return 1;  // (0, 0): Go's Verify returns false
  F r;
  for (int j = 0; j < 4; j++) {
    uint64_t x = 0;
    for (int b = 0; b < 8; b++) x = (x << 8) | r_be[32 - 8 * (j + 1) + b];
    r.v[j] = x;
  }
  // x(R) = X / ZZ; accept iff x mod N == r: X == r ZZ, or (r + N < p) X == (r + N) ZZ
  // (r to the host form: times 2^512, then one Montgomery product)
  if (eq(mul(mul(r, kR2p), acc.ZZ), acc.X)) return 0;
  F rn = r;
  const uint64_t c = add4(rn.v, kN);
  if (!c && !geq(rn.v, kP) && eq(mul(mul(rn, kR2p), acc.ZZ), acc.X)) return 0;
  return 1;
}

}  // namespace mbft_host

extern "C" int mbft_debug_host_join(const uint32_t* part, int nparts, const uint8_t* r_be) {
  if (!part || !r_be || nparts < 1 || nparts > 16) return -1;
  return mbft_host::host_join_check(part, nparts, r_be);
}

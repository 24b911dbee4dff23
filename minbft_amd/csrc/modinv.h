// Variable-time modular inversion mod N (the P-256 group order) by
// Bernstein-Yang divsteps ("safegcd"), for the ONE value at the root of the
// batched s^-1 tree (kernels.hip k_ninv_top).  Verification inputs are
// public, so variable time is fine.  One lane runs it: where Fermat
// (x^(N-2): 255 squarings + ~40 multiplies, ~60K dependent VALU ops) leaves
// a single wave latency-bound for ~0.15 ms, divsteps need ~20 batches of 30
// steps on 32-bit words plus 2x2-matrix updates of 9-limb numbers (~8K ops).
//
// Representation: signed 30-bit limbs, value = sum v[i] 2^(30 i), i < 9.
// Invariants (f, g start as N, x; d, e as 0, 1): d x == f, e x == g (mod N);
// each batch applies the transition matrix of 30 divsteps to (f, g) (exact
// division by 2^30) and to (d, e) (mod N, division by 2^30 through adding
// the multiple of N that clears the low 30 bits).  g reaches 0 with
// f = +-1, and the inverse is +-d.  Host + device (tests/csrc/modinv_check.cpp
// checks it on the CPU against Python big integers).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mbft {

#define MBFT_HD __host__ __device__ __forceinline__

struct s30 {
  int32_t v[9];
};

constexpr int32_t kM30 = (int32_t)(0xFFFFFFFFu >> 2);
// N in signed 30-bit limbs, and N^-1 mod 2^30
MBFT_HD void s30_modulus(s30& m) {
  const int32_t n[9] = {0x3C632551, 0x0EE72B0B, 0x3179E84F, 0x39BEAB69, 0x3FFFFFBC,
                        0x3FFFFFFF, 0x00000FFF, 0x3FFFC000, 0x0000FFFF};
#pragma unroll
  for (int i = 0; i < 9; i++) m.v[i] = n[i];
}
constexpr uint32_t kNinv30 = 0x11FF43B1u;  // N^-1 mod 2^30

struct trans2x2 {
  int32_t u, v, q, r;
};

MBFT_HD int ctz32(uint32_t x) { return __builtin_ctz(x); }

// 30 divsteps on the low words of f (odd) and g; returns the new eta
// (eta = -delta) and the transition matrix t with
//   2^30 (f', g') = (u f + v g, q f + r g).
MBFT_HD int32_t divsteps_30_var(int32_t eta, uint32_t f0, uint32_t g0, trans2x2& t) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  uint32_t f = f0, g = g0;
  int i = 30;
  for (;;) {
    // g's zero low bits (up to i): each is one divstep that halves g
    const int zeros = ctz32(g | (0xFFFFFFFFu << i));
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    // f, g odd.  eta < 0: swap to (g, -f) (the divstep's delta > 0 branch)
    if (eta < 0) {
      uint32_t tmp;
      eta = -eta;
      tmp = f; f = g; g = 0u - tmp;
      tmp = u; u = q; q = 0u - tmp;
      tmp = v; v = r; r = 0u - tmp;
    }
    // cancel the low min(eta + 1, i, 6) bits of g with a multiple w of f:
    // f^2 == 1 (mod 8), so f (2 - f^2) == -(f (f^2 - 2)) is f^-1 mod 2^6 and
    // g + f w == g (f^2 - 1)^2 == 0 (mod 2^6) for w = f g (f^2 - 2).  Two
    // dependent multiplies instead of a full 32-bit inverse (8): the loop is
    // one lane's latency chain, and eta + 1 is rarely above 6.
    const int limit = (eta + 1) > i ? i : (eta + 1);
    const uint32_t m = (0xFFFFFFFFu >> (32 - limit)) & 63u;
    const uint32_t w = ((f * g) * (f * f - 2u)) & m;
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t.u = (int32_t)u;
  t.v = (int32_t)v;
  t.q = (int32_t)q;
  t.r = (int32_t)r;
  return eta;
}

// (d, e) <- t (d, e) / 2^30 mod N, kept in (-2N, N)
MBFT_HD void update_de_30(s30& d, s30& e, const trans2x2& t, const s30& M) {
  const int32_t u = t.u, v = t.v, q = t.q, r = t.r;
  const int32_t sd = d.v[8] >> 31, se = e.v[8] >> 31;
  int32_t md = (u & sd) + (v & se);
  int32_t me = (q & sd) + (r & se);
  int64_t cd = (int64_t)u * d.v[0] + (int64_t)v * e.v[0];
  int64_t ce = (int64_t)q * d.v[0] + (int64_t)r * e.v[0];
  md -= (int32_t)((kNinv30 * (uint32_t)cd + (uint32_t)md) & (uint32_t)kM30);
  me -= (int32_t)((kNinv30 * (uint32_t)ce + (uint32_t)me) & (uint32_t)kM30);
  cd += (int64_t)M.v[0] * md;
  ce += (int64_t)M.v[0] * me;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    cd += (int64_t)u * d.v[i] + (int64_t)v * e.v[i] + (int64_t)M.v[i] * md;
    ce += (int64_t)q * d.v[i] + (int64_t)r * e.v[i] + (int64_t)M.v[i] * me;
    d.v[i - 1] = (int32_t)cd & kM30;
    cd >>= 30;
    e.v[i - 1] = (int32_t)ce & kM30;
    ce >>= 30;
  }
  d.v[8] = (int32_t)cd;
  e.v[8] = (int32_t)ce;
}

// (f, g) <- t (f, g) / 2^30 (exact)
MBFT_HD void update_fg_30(s30& f, s30& g, const trans2x2& t) {
  const int32_t u = t.u, v = t.v, q = t.q, r = t.r;
  int64_t cf = (int64_t)u * f.v[0] + (int64_t)v * g.v[0];
  int64_t cg = (int64_t)q * f.v[0] + (int64_t)r * g.v[0];
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    cf += (int64_t)u * f.v[i] + (int64_t)v * g.v[i];
    cg += (int64_t)q * f.v[i] + (int64_t)r * g.v[i];
    f.v[i - 1] = (int32_t)cf & kM30;
    cf >>= 30;
    g.v[i - 1] = (int32_t)cg & kM30;
    cg >>= 30;
  }
  f.v[8] = (int32_t)cf;
  g.v[8] = (int32_t)cg;
}

// 8 little-endian 32-bit words (value < 2^256) <-> signed 30-bit limbs
MBFT_HD void s30_from_words(s30& a, const uint32_t w[8]) {
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const int bit = 30 * k, j = bit >> 5, sh = bit & 31;
    uint64_t x = (uint64_t)w[j] >> sh;
    if (j + 1 < 8) x |= (uint64_t)w[j + 1] << (32 - sh);
    a.v[k] = (int32_t)(x & (uint64_t)kM30);
  }
}

// value in (-2N, N) -> canonical [0, N) as 8 LE words, times sign (+-1)
MBFT_HD void s30_to_words_mod(uint32_t w[8], const s30& a, int32_t negate, const s30& M) {
  int64_t l[9];
#pragma unroll
  for (int i = 0; i < 9; i++) l[i] = negate ? -(int64_t)a.v[i] : (int64_t)a.v[i];
  // now in (-N, 2N) or (-2N, N): add N while negative, subtract while >= N
#pragma unroll
  for (int pass = 0; pass < 4; pass++) {
    // normalize to top-signed form and read the sign
    int64_t c = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      c += l[i];
      l[i] = i < 8 ? (c & kM30) : c;
      c = i < 8 ? (c >> 30) : 0;
    }
    if (l[8] < 0) {
#pragma unroll
      for (int i = 0; i < 9; i++) l[i] += M.v[i];
      continue;
    }
    // l >= N ?  (top limb first; branch-free so the limbs stay in registers)
    bool ge = true, eq = true;
#pragma unroll
    for (int i = 8; i >= 0; i--) {
      ge = (eq && l[i] > M.v[i]) || (!eq && ge);
      if (eq && l[i] < M.v[i]) ge = false;
      eq = eq && l[i] == M.v[i];
    }
    if (ge) {
#pragma unroll
      for (int i = 0; i < 9; i++) l[i] -= M.v[i];
      continue;
    }
    break;
  }
#pragma unroll
  for (int j = 0; j < 8; j++) w[j] = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const int bit = 30 * k, j = bit >> 5, sh = bit & 31;
    const uint64_t x = (uint64_t)l[k] << sh;
    w[j] |= (uint32_t)x;
    if (j + 1 < 8) w[j + 1] |= (uint32_t)(x >> 32);
  }
}

// c x^-1 mod N for 0 < x < N and 0 <= c < N (x, c, out: 8 LE words):
// (d, e) start as (0, c), so the invariants read d x == c f, e x == c g and
// the end gives +-d = c x^-1 -- the scale is free (c = R mod N hands back
// the Montgomery form x^-1 R, the host's s^-1 for k_verify_split).  Returns
// false if x is not invertible (x == 0 mod N) or the loop bound is hit
// (never for x < N).
MBFT_HD bool modinv_n_var_scaled(uint32_t out[8], const uint32_t x[8], const uint32_t c[8]) {
  s30 M, d, e, f, g;
  s30_modulus(M);
  s30_from_words(g, x);
  s30_from_words(e, c);
  f = M;
#pragma unroll
  for (int i = 0; i < 9; i++) d.v[i] = 0;
  int32_t eta = -1;
#pragma unroll 1
  for (int it = 0; it < 64; it++) {
    trans2x2 t;
    eta = divsteps_30_var(eta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
    update_de_30(d, e, t, M);
    update_fg_30(f, g, t);
    int32_t z = 0;
#pragma unroll
    for (int j = 0; j < 9; j++) z |= g.v[j];
    if (z == 0) {
      // f = +-1 (the gcd, top-signed normalized limbs); anything else means
      // x was not invertible
      int32_t lo0 = 0, lo1 = 0;
#pragma unroll
      for (int j = 1; j < 9; j++) lo0 |= f.v[j];
#pragma unroll
      for (int j = 0; j < 8; j++) lo1 |= f.v[j] ^ kM30;
      const bool one = f.v[0] == 1 && lo0 == 0;
      const bool neg = lo1 == 0 && f.v[8] == -1;
      if (!one && !neg) return false;
      s30_to_words_mod(out, d, neg ? 1 : 0, M);
      return true;
    }
  }
  return false;
}

// x^-1 mod N for 0 < x < N (x, out: 8 LE words); see modinv_n_var_scaled.
MBFT_HD bool modinv_n_var(uint32_t out[8], const uint32_t x[8]) {
  const uint32_t one[8] = {1, 0, 0, 0, 0, 0, 0, 0};
  return modinv_n_var_scaled(out, x, one);
}

}  // namespace mbft

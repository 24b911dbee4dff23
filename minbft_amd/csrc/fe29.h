// P-256 field and scalar arithmetic for gfx950, one element per lane.
//
// Representation: 9 unsaturated limbs of 29 bits (value < 2^261) in 32-bit
// VGPRs.  Products are accumulated column-wise into 64-bit accumulators with
// v_mad_u64_u32 (a*b + acc64 in ONE instruction); with 29-bit limbs a column
// of 9 products stays below 2^62, so the whole 256x256 product needs no carry
// instructions at all.  gfx950 microbenchmarks (tools/ubench_valu.hip,
// profiles/round1_ubench_valu.json) show why this shape: v_mad_u64_u32 issues
// at the same rate as any other VOP3 op (~56 lane-ops/CU/clk), while
// SGPR-carry chains (v_add_co/v_addc) need hazard wait states and run at
// half that, so a carry-free multiply beats the 8x32-bit full-radix form.
//
// Montgomery form with R = 2^261.
//  * mod p: p = 2^256 - 2^224 + 2^192 + 2^96 - 1 == -1 (mod 2^29), so the
//    per-limb Montgomery factor is m = t mod 2^29 and m*p is four shifted
//    adds (2^96 = 2^(3*29+9), 2^192 = 2^(6*29+18), 2^224 = 2^(7*29+21),
//    2^256 = 2^(8*29+24)); no multiplication by p's limbs.
//  * mod N: generic Montgomery (N has no special form), n0' = -N^-1 mod 2^29.
//
// Bounds discipline (all values non-negative, limbs normalized < 2^29):
//  * fe_mul / fe_sqr: inputs a, b with a*b < 2^518.5 (e.g. both < 2^259.2)
//    give an output < 2^258.
//  * fe_sub(a, b) = a - b + 16p then folded (fe_fold_signed, which keeps the
//    value non-negative whatever borrows the unnormalized limbs carry):
//    needs a < 2^260, b < 16p; output < 2^257 + 2^233.  fe_neg likewise.
//  * fe_add(a, b): a + b, normalized, not reduced.
//  * fe_fold: any normalized value < 2^261 -> congruent value < 2^257.
//  * fe_canon: -> the canonical residue in [0, p).
// The point formulas in ecc.h keep every stored coordinate < 2^258.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mbft {

constexpr int NL = 9;
constexpr uint32_t LMASK = (1u << 29) - 1;

struct fe {
  uint32_t v[NL];
};

#define MBFT_DEV __device__ __forceinline__

// ----------------------------------------------------------------- constants
// p and 16p in 29-bit limbs.
__device__ constexpr uint32_t kP[NL] = {0x1fffffffu, 0x1fffffffu, 0x1fffffffu,
                                        0x00001ffu,  0x0000000u,  0x0000000u,
                                        0x0040000u,  0x1fe00000u, 0x0ffffffu};
__device__ constexpr uint32_t kP16[NL] = {0x1ffffff0u, 0x1fffffffu, 0x1fffffffu,
                                          0x0001fffu,  0x0000000u,  0x0000000u,
                                          0x0400000u,  0x1e000000u, 0xfffffffu};
// p - 1 (= -1 mod p) in limbs.
__device__ constexpr uint32_t kPm1[NL] = {0x1ffffffeu, 0x1fffffffu, 0x1fffffffu,
                                          0x00001ffu,  0x0000000u,  0x0000000u,
                                          0x0040000u,  0x1fe00000u, 0x0ffffffu};
// R^2 mod p and R mod p (Montgomery one), R = 2^261.
__device__ constexpr uint32_t kR2P[NL] = {0x0000c00u,  0x0000000u,  0x1fff0000u,
                                          0x1fdfffffu, 0x1fbfffffu, 0x1fffffffu,
                                          0x1fffffffu, 0x1ffffffeu, 0x0000013u};
__device__ constexpr uint32_t kRP[NL] = {0x0000020u,  0x0000000u,  0x0000000u,
                                         0x1fffc000u, 0x1fffffffu, 0x1fffffffu,
                                         0x1f7fffffu, 0x3ffffffu,  0x0000000u};
// N (group order) in limbs, -N^-1 mod 2^29, R^2 mod N, R mod N.
__device__ constexpr uint32_t kN[NL] = {0x1c632551u, 0x1dce5617u, 0x5e7a13cu,
                                        0xdf55b4eu,  0x1ffffbceu, 0x1fffffffu,
                                        0x003ffffu,  0x1fe00000u, 0x0ffffffu};
constexpr uint32_t kNINV = 0xe00bc4fu;
__device__ constexpr uint32_t kR2N[NL] = {0x148d9ef5u, 0xf4e7f75u,  0x14c6a651u,
                                          0x3f8b765u,  0x165861f1u, 0x1256d7d8u,
                                          0x1c185b23u, 0xd4cab0fu,  0x084b655u};
__device__ constexpr uint32_t kRN[NL] = {0x139b55e0u, 0x6353d03u,  0x30bd862u,
                                         0x154963au,  0x0008632u,  0x0000000u,
                                         0x1f800000u, 0x3ffffffu,  0x0000000u};
// N and p as 8 little-endian 32-bit words (for range checks on raw inputs).
__device__ constexpr uint32_t kNw[8] = {0xFC632551u, 0xF3B9CAC2u, 0xA7179E84u,
                                        0xBCE6FAADu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                        0x00000000u, 0xFFFFFFFFu};
__device__ constexpr uint32_t kPw[8] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                        0x00000000u, 0x00000000u, 0x00000000u,
                                        0x00000001u, 0xFFFFFFFFu};
// p - N (< 2^128): r + N < p  <=>  r < p - N.
__device__ constexpr uint32_t kPmNw[8] = {0x039cdaaeu, 0x0c46353du, 0x58e8617bu,
                                          0x43190553u, 0u, 0u, 0u, 0u};

MBFT_DEV void fe_set(fe& o, const uint32_t (&c)[NL]) {
#pragma unroll
  for (int i = 0; i < NL; i++) o.v[i] = c[i];
}

MBFT_DEV void fe_zero(fe& o) {
#pragma unroll
  for (int i = 0; i < NL; i++) o.v[i] = 0;
}

// ---------------------------------------------------------- word conversion
// 8 little-endian 32-bit words (value < 2^256) -> limbs.
MBFT_DEV void fe_from_words(fe& o, const uint32_t w[8]) {
#pragma unroll
  for (int k = 0; k < NL; k++) {
    const int bit = 29 * k, j = bit >> 5, sh = bit & 31;
    uint32_t lo = w[j];
    uint32_t hi = (j + 1 < 8) ? w[j + 1] : 0u;
    uint32_t x = sh ? __builtin_amdgcn_alignbit(hi, lo, sh) : lo;
    o.v[k] = x & LMASK;
  }
}

// limbs (normalized, value < 2^256) -> 8 little-endian words.
MBFT_DEV void fe_to_words(uint32_t w[8], const fe& a) {
#pragma unroll
  for (int j = 0; j < 8; j++) {
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < NL; k++) {
      const int off = 29 * k - 32 * j;
      if (off > -29 && off < 32) x |= off >= 0 ? (a.v[k] << off) : (a.v[k] >> (-off));
    }
    w[j] = x;
  }
}

// 32 big-endian bytes (as 8 big-endian-loaded words) -> LE words.
MBFT_DEV void be_words_to_le(uint32_t w[8], const uint32_t be[8]) {
#pragma unroll
  for (int i = 0; i < 8; i++) w[7 - i] = __builtin_bswap32(be[i]);
}

// a < b for 8-word little-endian integers
MBFT_DEV bool words_lt(const uint32_t a[8], const uint32_t (&b)[8]) {
  // lexicographic from the top word; branch-free
  bool lt = false, eq = true;
#pragma unroll
  for (int i = 7; i >= 0; i--) {
    lt = lt || (eq && a[i] < b[i]);
    eq = eq && (a[i] == b[i]);
  }
  return lt;
}

MBFT_DEV bool words_is_zero(const uint32_t a[8]) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) x |= a[i];
  return x == 0;
}

// ----------------------------------------------------------- normalization
// unsigned carry propagation (all limbs non-negative, fit in 32 bits)
MBFT_DEV void fe_carry_u(fe& a) {
#pragma unroll
  for (int i = 0; i < NL - 1; i++) {
    a.v[i + 1] += a.v[i] >> 29;
    a.v[i] &= LMASK;
  }
}

// signed carry propagation (limbs are int32, total value >= 0)
MBFT_DEV void fe_carry_s(fe& a) {
#pragma unroll
  for (int i = 0; i < NL - 1; i++) {
    a.v[i + 1] = (uint32_t)((int32_t)a.v[i + 1] + ((int32_t)a.v[i] >> 29));
    a.v[i] &= LMASK;
  }
}

// Fold bits >= 2^256 using 2^256 == 2^224 - 2^192 - 2^96 + 1 (mod p).
// Input: limbs 0..7 in int32 range, top limb holding bits 232.. (unnormalized
// ok, < 2^31).  Output normalized, value < 2^257.
MBFT_DEV void fe_fold_raw(fe& a) {
  int32_t h = (int32_t)a.v[8] >> 24;
  a.v[8] &= (1u << 24) - 1;
  a.v[0] = (uint32_t)((int32_t)a.v[0] + h);
  a.v[3] = (uint32_t)((int32_t)a.v[3] - (h << 9));
  a.v[6] = (uint32_t)((int32_t)a.v[6] - (h << 18));
  a.v[7] = (uint32_t)((int32_t)a.v[7] + (h << 21));
  fe_carry_s(a);
}

MBFT_DEV void fe_fold(fe& a) { fe_fold_raw(a); }

// Fold for a value V > 0 held in UNNORMALIZED signed limbs (a + 16p - b,
// 16p - a): the low limbs may carry a net borrow of one unit of 2^232 into
// the top limb, so the top limb's quotient h = top >> 24 can exceed V's true
// multiple of 2^256 by one.  Folding h would then leave a negative value
// (seen for top == 2^28 - 2^24 exactly, e.g. 16p - y with y's top limb
// 2^24 - 1).  Folding max(h - 1, 0) multiples keeps the remainder >= 2^256 -
// 2^232 > 0 before the (non-negative) fold terms are added.
// Output: normalized, non-negative, < 2^257 + 2^233.
MBFT_DEV void fe_fold_signed(fe& a) {
  int32_t h = (int32_t)a.v[8] >> 24;
  h = h > 0 ? h - 1 : 0;
  a.v[8] = (uint32_t)((int32_t)a.v[8] - (h << 24));
  a.v[0] = (uint32_t)((int32_t)a.v[0] + h);
  a.v[3] = (uint32_t)((int32_t)a.v[3] - (h << 9));
  a.v[6] = (uint32_t)((int32_t)a.v[6] - (h << 18));
  a.v[7] = (uint32_t)((int32_t)a.v[7] + (h << 21));
  fe_carry_s(a);
}

// ------------------------------------------------------------- add / sub
MBFT_DEV void fe_add(fe& o, const fe& a, const fe& b) {
#pragma unroll
  for (int i = 0; i < NL; i++) o.v[i] = a.v[i] + b.v[i];
  fe_carry_u(o);
}

// o = a - b + 16p, folded: a < 2^260, b < 16p  ->  o < 2^257 + 2^233
MBFT_DEV void fe_sub(fe& o, const fe& a, const fe& b) {
#pragma unroll
  for (int i = 0; i < NL; i++) o.v[i] = a.v[i] + kP16[i] - b.v[i];
  // limbs are in (-2^29, 2^30) and the top limb is >= 0 (b < 16p => b.v[8] <=
  // 16p.v[8]); fold the unnormalized top limb conservatively, then one
  // signed carry pass.  The value stays congruent and positive.
  fe_fold_signed(o);
}

// o = k * a (k small, k*a < 2^261), folded to < 2^257
MBFT_DEV void fe_mulsmall(fe& o, const fe& a, uint32_t k) {
#pragma unroll
  for (int i = 0; i < NL; i++) o.v[i] = a.v[i] * k;
  fe_carry_u(o);
  fe_fold_raw(o);
}

// 5p and 2p with BORROWED limbs: every low limb in [2^29 - 1, 2^30) and the
// top limb above any normalized operand's (< 2^26; a canonical value's
// <= p's), so c_i - x_i >= 0 limb by limb with no carry pass (fe_mul_add
// operands).
__device__ constexpr uint32_t kP5B[NL] = {0x3ffffffbu, 0x3ffffffeu, 0x3ffffffeu,
                                          0x200009feu, 0x1fffffffu, 0x1fffffffu,
                                          0x2013ffffu, 0x3f5fffffu, 0x04fffffeu};
__device__ constexpr uint32_t kP2B[NL] = {0x3ffffffeu, 0x3ffffffeu, 0x3ffffffeu,
                                          0x200003feu, 0x1fffffffu, 0x1fffffffu,
                                          0x2007ffffu, 0x3fbfffffu, 0x01fffffeu};

// 48p in limbs (for fe_sub_2x)
__device__ constexpr uint32_t kP48[NL] = {0x1fffffd0u, 0x1fffffffu, 0x1fffffffu,
                                          0x0005fffu,  0x0000000u,  0x0000000u,
                                          0x0c00000u,  0x1a000000u, 0x2fffffffu};

// o = a - b - 2c + 48p, folded (one fold for the madd's X3 = R^2 - H^3 -
// 2 X1 H^2): a < 2^260, b < 2^259, c < 2^259 (so b + 2c < 48p)  ->  o < 2^257 + 2^234
MBFT_DEV void fe_sub_2x(fe& o, const fe& a, const fe& b, const fe& c) {
#pragma unroll
  for (int i = 0; i < NL; i++) o.v[i] = a.v[i] + kP48[i] - b.v[i] - (c.v[i] << 1);
  fe_fold_signed(o);
}

// 5p in limbs (for fe_sub5)
__device__ constexpr uint32_t kP5[NL] = {0x1ffffffbu, 0x1fffffffu, 0x1fffffffu,
                                         0x00009ffu,  0x0000000u,  0x0000000u,
                                         0x0140000u,  0x1f600000u, 0x4ffffffu};

// o = a - b + 5p with NO fold, one signed carry pass: a < 2^258, b < 5p
// (> 2^258.3)  ->  0 < o < 2^259.17, normalized.  For differences that only
// feed multiplications: o^2 < 2^518.4 keeps fe_mul / fe_sqr within their
// input bound.  The signed carry is exact, so the top limb ends up
// floor(o / 2^232) >= 0 whatever the intermediate borrows.
MBFT_DEV void fe_sub5(fe& o, const fe& a, const fe& b) {
#pragma unroll
  for (int i = 0; i < NL; i++) o.v[i] = a.v[i] + kP5[i] - b.v[i];
  fe_carry_s(o);
}

// negate: 16p - a, folded (a < 16p)
MBFT_DEV void fe_neg(fe& o, const fe& a) {
#pragma unroll
  for (int i = 0; i < NL; i++) o.v[i] = kP16[i] - a.v[i];
  fe_fold_signed(o);
}

// ----------------------------------------------------------- canonical
// conditional subtract of p; input normalized value < 2p
MBFT_DEV void fe_csub_p(fe& a) {
  fe d;
#pragma unroll
  for (int i = 0; i < NL; i++) d.v[i] = a.v[i] - kP[i];
  fe_carry_s(d);
  const bool neg = (int32_t)d.v[8] < 0;
#pragma unroll
  for (int i = 0; i < NL; i++) a.v[i] = neg ? a.v[i] : d.v[i];
}

// any normalized value < 2^261 -> [0, p)
MBFT_DEV void fe_canon(fe& a) {
  fe_fold_raw(a);  // < 2^256 + 2^229 < 2p
  fe_csub_p(a);
}

MBFT_DEV bool fe_is_zero_canon(const fe& a) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) x |= a.v[i];
  return x == 0;
}

MBFT_DEV bool fe_eq_canon(const fe& a, const fe& b) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) x |= a.v[i] ^ b.v[i];
  return x == 0;
}

MBFT_DEV void fe_select(fe& o, bool c, const fe& a, const fe& b) {
#pragma unroll
  for (int i = 0; i < NL; i++) o.v[i] = c ? a.v[i] : b.v[i];
}

// ---------------------------------------------------- Montgomery mod p
// Reduce the 18 column accumulators t[] (t[i] for 0 <= i < 17, t[17] = 0)
// and write the normalized result.
// LAZY (0..6): output limbs 0 .. LAZY-1 are left as the low 32 bits of
// their column, and the column's high word goes to the next column as ONE
// v_mad_u64_u32 (hi * 8 + next) -- the trick the digit loop uses -- instead
// of mask + 64-bit shift + 64-bit add: such a "lazy" limb is < 2^32, the
// value is the same.  A lazy operand may meet only a normalized one in a
// product: with at most 6 limbs below 2^32 and the rest below 2^29, a column
// stays < 6 * 2^61 + 3 * 2^58 + the reduction terms (< 2^61.05) < 2^63.9.
// fe_norm_lazy normalizes such a value.
template <bool ADD = false, int LAZY = 0>
MBFT_DEV void mont_reduce_p(fe& o, uint64_t (&t)[18], const fe* w = nullptr) {
  // m * p * 2^(29 i) with p = 2^256 - 2^224 + 2^192 + 2^96 - 1:
  //   -m at column i          : cancels t[i] mod 2^29 (carry = t[i] >> 29)
  //   +m 2^9  at column i+3   (2^96  = 2^(3*29 + 9))
  //   +m 2^18 at column i+6   (2^192 = 2^(6*29 + 18))
  //   -m 2^21 at column i+7 and +m 2^24 at column i+8 (2^224, 2^256) are
  //   re-expressed with non-negative multipliers as
  //   +m (2^29 - 2^21) at column i+7 and +m (2^24 - 1) at column i+8
  //   (the extra m 2^29 at i+7 equals m at i+8).
  // Columns 0..7 take the WHOLE low word as m (m < 2^32; m == t mod 2^29 is
  // all Montgomery needs, any m == t (mod 2^29) cancels the column): the
  // column is then exactly hi32(t) 2^32, i.e. a carry of hi32(t) * 8 -- ONE
  // v_mad_u64_u32 instead of mask + 64-bit shift + 64-bit add.  Only m_8 is
  // masked to 29 bits, so M = sum m_i 2^(29 i) < 2^261 (1 + 2^-26) and the
  // output bound moves by p 2^-26 only (a*b < 2^518.5 -> output < 2^258).
  // Every term is one v_mad_u64_u32 (m * const + t) and every column stays
  // non-negative and < 2^62.7 (fe_mul2: 18 products < 2^62.2, m terms < 2^61).
  // Opaque (SGPR) multipliers: otherwise the compiler turns the power-of-two
  // products into a 64-bit shift plus a 64-bit add (two VALU ops, not one).
  uint32_t k9 = 1u << 9, k18 = 1u << 18, k7 = (1u << 29) - (1u << 21), k8 = (1u << 24) - 1u,
           k3 = 8u;
  asm volatile("" : "+s"(k9), "+s"(k18), "+s"(k7), "+s"(k8), "+s"(k3));
#pragma unroll
  for (int i = 0; i < NL; i++) {
    const uint64_t c = t[i];
    uint32_t m;
    if (i < NL - 1) {
      m = (uint32_t)c;
      t[i + 1] += (uint64_t)(uint32_t)(c >> 32) * k3;
    } else {
      m = (uint32_t)c & LMASK;
      t[i + 1] += c >> 29;
    }
    t[i + 3] += (uint64_t)m * k9;
    t[i + 6] += (uint64_t)m * k18;
    t[i + 7] += (uint64_t)m * k7;
    t[i + 8] += (uint64_t)m * k8;
  }
  if (ADD) {
    // + w exactly: REDC(T + w R) = REDC(T) + w (w R does not change M)
    uint32_t k1 = 1u;
    asm volatile("" : "+s"(k1));
#pragma unroll
    for (int k = 0; k < NL; k++) t[NL + k] += (uint64_t)w->v[k] * k1;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
    if (k - NL < LAZY) {
      o.v[k - NL] = (uint32_t)t[k];
      t[k + 1] += (uint64_t)(uint32_t)(t[k] >> 32) * k3;
    } else {
      o.v[k - NL] = (uint32_t)t[k] & LMASK;
      t[k + 1] += t[k] >> 29;
    }
  }
  o.v[NL - 1] = (uint32_t)t[2 * NL - 1];
}

// A lazy value (mont_reduce_p<.., LAZY>: low limbs < 2^32) -> normalized
// limbs, same value (64-bit carries: a lazy limb plus a carry can pass 2^32).
MBFT_DEV void fe_norm_lazy(fe& a) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < NL - 1; i++) {
    c += a.v[i];
    a.v[i] = (uint32_t)c & LMASK;
    c >>= 29;
  }
  a.v[NL - 1] += (uint32_t)c;
}

MBFT_DEV void fe_mul(fe& o, const fe& a, const fe& b) {
  uint64_t t[18];
#pragma unroll
  for (int k = 0; k < 18; k++) t[k] = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
#pragma unroll
    for (int j = 0; j < NL; j++) t[i + j] += (uint64_t)a.v[i] * b.v[j];
  }
  mont_reduce_p(o, t);
}

// o = (a*b + c*d) R^-1 mod p with ONE reduction: 162 product mads into the
// same 17 column sums (each < 18 * 2^58 = 2^62.2 before reduction terms,
// still no carries), for formulas of the form X*Y - Z*W with -W folded into
// d by the caller.  Inputs normalized with a*b + c*d < 2^518.5 -- except
// that a's limbs may reach 2^30.6 (ec_madd_chud's V - X3 + 5p without a
// carry pass): columns then stay < 9 * 2^59.6 + 9 * 2^58 + 2^61.05 (the
// reduction terms) < 2^63.5.
MBFT_DEV void fe_mul2(fe& o, const fe& a, const fe& b, const fe& c, const fe& d) {
  uint64_t t[18];
#pragma unroll
  for (int k = 0; k < 18; k++) t[k] = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
#pragma unroll
    for (int j = 0; j < NL; j++) t[i + j] += (uint64_t)a.v[i] * b.v[j];
  }
#pragma unroll
  for (int i = 0; i < NL; i++) {
#pragma unroll
    for (int j = 0; j < NL; j++) t[i + j] += (uint64_t)c.v[i] * d.v[j];
  }
  mont_reduce_p(o, t);
}

// o = a b R^-1 + w (mod p), exactly REDC(a b) + w: the subtraction that
// follows a product folded into its reduction (no separate carry pass).
// w: non-negative limbs < 2^30 (a borrowed-limb constant minus a normalized
// value); a's limbs may be up to 2^30 when b's are normalized (columns
// < 9 * 2^59 + 2^61).  Output normalized, < a b / R + p (1 + 2^-26) + w.
// fe_mul with lazy output limbs 0 .. LAZY-1 (mont_reduce_p).
template <int LAZY>
MBFT_DEV void fe_mul_lazy(fe& o, const fe& a, const fe& b) {
  uint64_t t[18];
#pragma unroll
  for (int k = 0; k < 18; k++) t[k] = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
#pragma unroll
    for (int j = 0; j < NL; j++) t[i + j] += (uint64_t)a.v[i] * b.v[j];
  }
  mont_reduce_p<false, LAZY>(o, t);
}

// w R enters the top columns as their INITIAL values (t[9 + k] = w_k), so
// the first product mad of each column adds it for free -- instead of nine
// extra "w_k * 1" mads after the reduction (mont_reduce_p<true>, kept for
// the record and the field tests).  a may be lazy (mont_reduce_p<.., 6>) when
// b is normalized: columns < 6 * 2^61 + 3 * 2^58 + 2^61.05 + 2^30 < 2^63.9.
MBFT_DEV void fe_mul_add(fe& o, const fe& a, const fe& b, const fe& w) {
  uint64_t t[18];
#pragma unroll
  for (int k = 0; k < NL; k++) t[k] = 0;
#pragma unroll
  for (int k = 0; k < NL; k++) t[NL + k] = w.v[k];
#pragma unroll
  for (int i = 0; i < NL; i++) {
#pragma unroll
    for (int j = 0; j < NL; j++) t[i + j] += (uint64_t)a.v[i] * b.v[j];
  }
  mont_reduce_p(o, t);
}

MBFT_DEV void fe_sqr(fe& o, const fe& a) {
  uint64_t t[18];
  uint32_t d[NL];
#pragma unroll
  for (int i = 0; i < NL; i++) d[i] = a.v[i] << 1;
#pragma unroll
  for (int k = 0; k < 18; k++) t[k] = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    t[2 * i] += (uint64_t)a.v[i] * a.v[i];
#pragma unroll
    for (int j = i + 1; j < NL; j++) t[i + j] += (uint64_t)a.v[i] * d[j];
  }
  mont_reduce_p(o, t);
}

MBFT_DEV void fe_to_mont(fe& o, const fe& a) {
  fe r2;
  fe_set(r2, kR2P);
  fe_mul(o, a, r2);
}

MBFT_DEV void fe_from_mont(fe& o, const fe& a) {
  fe one;
  fe_zero(one);
  one.v[0] = 1;
  fe_mul(o, a, one);
}

MBFT_DEV void fe_one_mont(fe& o) { fe_set(o, kRP); }

// Exponents for Fermat inversion, most significant word first (read with a
// wave-uniform index -> scalar loads).
__constant__ uint32_t kExpPm2[8] = {0xFFFFFFFFu, 0x00000001u, 0x00000000u, 0x00000000u,
                                    0x00000000u, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFDu};
__constant__ uint32_t kExpNm2[8] = {0xFFFFFFFFu, 0x00000000u, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                    0xBCE6FAADu, 0xA7179E84u, 0xF3B9CAC2u, 0xFC63254Fu};

// a^(p-2) (Montgomery in, Montgomery out): square-and-multiply over the
// fixed exponent bits in a compact (non-unrolled) loop; the bit test is
// wave-uniform so the multiply is a scalar branch, not divergence.
MBFT_DEV void fe_inv(fe& o, const fe& a) {
  fe r = a;  // top exponent bit is 1
#pragma unroll 1
  for (int bit = 254; bit >= 0; bit--) {
    fe_sqr(r, r);
    if ((kExpPm2[7 - (bit >> 5)] >> (bit & 31)) & 1u) fe_mul(r, r, a);
  }
  o = r;
}

// ---------------------------------------------------- Montgomery mod N
MBFT_DEV void mont_reduce_n(fe& o, uint64_t (&t)[18]) {
#pragma unroll
  for (int i = 0; i < NL; i++) {
    const uint32_t m = ((uint32_t)t[i] * kNINV) & LMASK;
    const uint64_t c = t[i] + (uint64_t)m * kN[0];
    t[i + 1] += c >> 29;
#pragma unroll
    for (int j = 1; j < NL; j++) t[i + j] += (uint64_t)m * kN[j];
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
    o.v[k - NL] = (uint32_t)t[k] & LMASK;
    t[k + 1] += t[k] >> 29;
  }
  o.v[NL - 1] = (uint32_t)t[2 * NL - 1];
}

// a*b*R^-1 mod N, output < a*b/R + N (inputs < 2^259 -> output < 2^258)
MBFT_DEV void fn_mul(fe& o, const fe& a, const fe& b) {
  uint64_t t[18];
#pragma unroll
  for (int k = 0; k < 18; k++) t[k] = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
#pragma unroll
    for (int j = 0; j < NL; j++) t[i + j] += (uint64_t)a.v[i] * b.v[j];
  }
  mont_reduce_n(o, t);
}

// reduce a normalized value < 2^258 to [0, N): conditional subtracts of 4N..N
MBFT_DEV void fn_csub(fe& a, int k) {
  fe d;
#pragma unroll
  for (int i = 0; i < NL; i++) d.v[i] = a.v[i] - kN[i] * (uint32_t)k;
  fe_carry_s(d);
  const bool neg = (int32_t)d.v[8] < 0;
#pragma unroll
  for (int i = 0; i < NL; i++) a.v[i] = neg ? a.v[i] : d.v[i];
}

MBFT_DEV void fn_canon(fe& a) {
  // value < 2^258 < 5N  (N > 2^255.99)
  fn_csub(a, 4);
  fn_csub(a, 2);
  fn_csub(a, 1);
}

MBFT_DEV void fn_to_mont(fe& o, const fe& a) {
  fe r2;
  fe_set(r2, kR2N);
  fn_mul(o, a, r2);
}

MBFT_DEV void fn_from_mont(fe& o, const fe& a) {
  fe one;
  fe_zero(one);
  one.v[0] = 1;
  fn_mul(o, a, one);
}

// a^(N-2) mod N, Montgomery in/out (per-lane Fermat; the batched path in
// kernels.hip amortizes this across many signatures).
MBFT_DEV void fn_inv(fe& o, const fe& a) {
  fe r = a;
#pragma unroll 1
  for (int bit = 254; bit >= 0; bit--) {
    fn_mul(r, r, r);
    if ((kExpNm2[7 - (bit >> 5)] >> (bit & 31)) & 1u) fn_mul(r, r, a);
  }
  o = r;
}

}  // namespace mbft

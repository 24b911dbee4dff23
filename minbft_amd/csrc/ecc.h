// P-256 group operations in Jacobian coordinates (a = -3), one point per lane.
//
// Formulas (Hyperelliptic EFD names):
//  * ec_madd: madd-2004-hmv, Jacobian + affine, 8M + 3S.  Z3 = Z1 * H, so a
//    degenerate addition (H == 0: equal or opposite points) yields Z3 == 0,
//    and every later madd keeps Z == 0.  The verifier relies on this: a final
//    Z == 0 flags the (adversarially constructible) lanes that need the
//    complete slow path.
//  * ec_dbl: dbl-2001-b, 3M + 5S (Z3 = 2*Y1*Z1 variant).
// All inputs/outputs keep coordinates < 2^258 (see fe29.h bounds).
#pragma once
#include "fe29.h"

namespace mbft {

struct jac {
  fe X, Y, Z;
};

// o = a + (x2, y2); a is Jacobian (Z != 0), (x2, y2) affine Montgomery < p.
// Safe for o aliasing a.  ratio (optional) receives H = Z3 / Z1.
MBFT_DEV void ec_madd(jac& o, const jac& a, const fe& x2, const fe& y2, fe* ratio = nullptr) {
  fe t1, t2, t3, t4, h, r, z3;
  fe_sqr(t1, a.Z);      // Z1^2
  fe_mul(t2, t1, a.Z);  // Z1^3
  fe_mul(t1, t1, x2);   // U2 = x2 Z1^2
  fe_mul(t2, t2, y2);   // S2 = y2 Z1^3
  fe_sub(h, t1, a.X);   // H = U2 - X1
  fe_sub(r, t2, a.Y);   // R = S2 - Y1
  fe_mul(z3, a.Z, h);   // Z3 = Z1 H
  fe_sqr(t4, h);        // H^2
  fe_mul(t3, t4, h);    // H^3
  fe_mul(t4, t4, a.X);  // X1 H^2
  fe_sqr(t1, r);        // R^2
  fe_sub_2x(o.X, t1, t3, t4);  // X3 = R^2 - H^3 - 2 X1 H^2, one fold
  fe_sub(t4, t4, o.X);  // X1 H^2 - X3
  fe_neg(t1, a.Y);      // -Y1
  fe_mul2(o.Y, t4, r, t3, t1);  // Y3 = R (X1 H^2 - X3) - Y1 H^3, one reduction
  o.Z = z3;
  if (ratio) *ratio = h;
}

// The verifier's accumulator in Chudnovsky-Jacobian form: (X, Y, ZZ = Z^2,
// ZZZ = Z^3).  A mixed addition reads Z1^2 and Z1^3 directly and updates
// them as ZZ3 = ZZ1 H^2, ZZZ3 = ZZZ1 H^3, where the Jacobian form computes
// Z3 = Z1 H and squares / cubes it next step: 2S + 6M + the merged Y3
// product (9 reductions) instead of 3S + 6M + merged (10).  The x-check
// needs Z^2 only (X == r Z^2), and a degenerate addition still leaves
// ZZ == 0 (H == 0).
struct chud {
  fe X, Y, ZZ, ZZZ;
};

// The verifier's fast-path addition: madd-2004-hmv on the Chudnovsky
// accumulator with the signs of Y1 and of the comb digit folded into ONE
// per-lane select on the accumulator side.  With a.Y = s Y1 (s = +-1) and
// addend (x2, t y2) (t = +-1: a signed comb digit), c = -s t, and
//   w  = c a.Y = -t Y1                  (a.Y, or 5p - a.Y: limbs < 2^30)
//   R" = y2 Z1^3 + w = t R              (S2 = t y2 Z1^3, R = S2 - Y1)
//   R" (V - X3) + w H^3 = t Y3          -> o.Y = t Y3
// so the stored Y carries the sign of the digit just added; X3 depends on
// R"^2 only, and ZZ3 = ZZ1 H^2 (a degenerate addition still leaves
// ZZ == 0).  add_s2 = (s t == -1), per lane, no branch.  The caller tracks
// the sign (yneg = the digit's sign after the addition) and never reads it
// for the x-check (X and ZZ only).  y2 stays the canonical table value --
// which is what lets ZZZ be lazy (below) -- and w feeds the reduction of R"
// and the second product of the merged Y3 (fe_mul2 columns < 2^63.8).
// Safe for o aliasing a.
//
// LAZY: ZZ and ZZZ are kept with lazy low limbs (fe29.h mont_reduce_p<.., 6>:
// one mad per carry instead of three ops for 6 of their 9 output limbs);
// each only meets normalized operands (ZZ: the table's x2 and H^2; ZZZ: the
// table's y2 and H^3), and the caller normalizes them (fe_norm_lazy) before
// anything else reads them.
// LAST: the chain's final addition -- only X3 and ZZ3 are read afterwards
// (the x-check), so ZZZ3 and Y3 are not computed.
template <bool LAZY = false, bool LAST = false>
MBFT_DEV void ec_madd_chud(chud& o, const chud& a, const fe& x2, const fe& y2, bool add_s2) {
  constexpr bool last = LAST;
  fe t1, t2, h, r, hh, hhh;
  // H = x2 Z1^2 + (5p - X1): the subtraction folded into the reduction
#pragma unroll
  for (int i = 0; i < NL; i++) t1.v[i] = kP5B[i] - a.X.v[i];
  fe_mul_add(h, x2, a.ZZ, t1);   // H < 2^259.13
  // w = +-a.Y (5p - a.Y: kP5B's borrowed limbs dominate a.Y's, top limb
  // < 2^25.7, so no carry); R" = y2 Z1^3 + w with w folded into the reduction
#pragma unroll
  for (int i = 0; i < NL; i++) t2.v[i] = add_s2 ? a.Y.v[i] : kP5B[i] - a.Y.v[i];
  fe_mul_add(r, y2, a.ZZZ, t2);  // R" < 2^256 + 6p < 2^258.61
  fe_sqr(hh, h);           // H^2
  if (LAZY)
    fe_mul_lazy<6>(o.ZZ, a.ZZ, hh);  // ZZ3 = ZZ1 H^2
  else
    fe_mul(o.ZZ, a.ZZ, hh);
  fe_mul(hhh, h, hh);      // H^3
  if (!last) {
    if (LAZY)
      fe_mul_lazy<6>(o.ZZZ, a.ZZZ, hhh);  // ZZZ3 = ZZZ1 H^3
    else
      fe_mul(o.ZZZ, a.ZZZ, hhh);
  }
  fe_mul(t1, a.X, hh);     // V = X1 H^2
  fe_sqr(hh, r);           // R"^2 (H^2 is dead)
  fe_sub_2x(o.X, hh, hhh, t1);   // X3 = R^2 - H^3 - 2V
  if (last) return;
  // V - X3 + 5p limb by limb with NO carry pass: kP5B's borrowed limbs
  // dominate X3's (normalized, top limb < 2^25.01), so every limb lies in
  // [0, 2^30.6) and the value below 2^259.17.  fe_mul2's columns: 9 2^59.6
  // (t1 R") + 9 2^59 (w H^3, w's limbs < 2^30) + 2^61.05 < 2^63.8, and
  // Y3 < (2^259.17 2^258.61 + 2^258.32 2^258) / R + p < 2^257.7.
#pragma unroll
  for (int i = 0; i < NL; i++) t1.v[i] += kP5B[i] - o.X.v[i];
  fe_mul2(o.Y, t1, r, t2, hhh);  // R" (V - X3) + w H^3 = t Y3
}

// The verifier's first addition, two affine comb entries (Z1 = 1: U2 = x2,
// S2 = y2, Z3 = H), same sign convention (y1 holds s Y1, add_s2 = (s t ==
// -1), o.Y = -s Y3), into the Chudnovsky form: ZZ3 = H^2 and ZZZ3 = H^3 come
// for free.  H = x2 - x1 + 5p (fe_sub5, < 2^259.17, no fold): its square
// stays inside the reduction's input bound.
MBFT_DEV void ec_add_affine_chud(chud& o, const fe& x1, const fe& y1, const fe& x2, const fe& y2,
                                 bool add_s2) {
  fe t1, t4, h, r;
  fe_sub5(h, x2, x1);   // H = x2 - x1
#pragma unroll
  for (int i = 0; i < NL; i++) {
    const uint32_t m = kP5[i] - y2.v[i];
    r.v[i] = y1.v[i] + (add_s2 ? y2.v[i] : m);
  }
  fe_carry_s(r);        // R' = y1 +- y2 (+5p)
  fe_sqr(o.ZZ, h);      // H^2
  fe_mul(o.ZZZ, o.ZZ, h);  // H^3
  fe_mul(t4, o.ZZ, x1);    // V = x1 H^2
  fe_sqr(t1, r);        // R^2
  fe_sub_2x(o.X, t1, o.ZZZ, t4);  // X3 = R^2 - H^3 - 2V
  fe_sub(t4, t4, o.X);  // V - X3
  fe_mul2(o.Y, t4, r, y1, o.ZZZ);  // R' (V - X3) + y1 H^3 = -s Y3
}

// X3 and ZZ3 of a + b for two Chudnovsky points (neither at infinity), the
// x-only join of the small-batch verifier's two halves (k_verify_pairs: the
// x-check reads X and ZZ only).  a.Y holds sa Ya and b.Y holds sb Yb (sa, sb
// = +-1, same_sign = (sa == sb)); R enters only as R^2, so R = S2 -+ S1 up
// to one common sign.  add-2008-bl on the Chudnovsky form: U1 = Xa ZZb,
// U2 = Xb ZZa, H = U2 - U1, X3 = R^2 - H^3 - 2 U1 H^2, ZZ3 = ZZa ZZb H^2.
// Returns false for a degenerate addition (H == 0: equal or opposite points),
// which the caller resolves on the exact path.
MBFT_DEV bool ec_add_chud_x(fe& X3, fe& ZZ3, const chud& a, const chud& b, bool same_sign) {
  fe u1, u2, s1, s2, h, r, hh, hhh, v, t;
  fe_mul(u1, a.X, b.ZZ);
  fe_mul(u2, b.X, a.ZZ);
  fe_mul(s1, a.Y, b.ZZZ);
  fe_mul(s2, b.Y, a.ZZZ);
  fe_sub(h, u2, u1);  // < 2^257 + 2^233
  t = h;
  fe_canon(t);
  if (fe_is_zero_canon(t)) return false;
  if (same_sign)
    fe_sub(r, s2, s1);
  else
    fe_add(r, s2, s1);  // < 2^259: its square stays inside the reduction's input bound
  fe_sqr(hh, h);
  fe_mul(hhh, hh, h);
  fe_mul(v, u1, hh);
  fe_sqr(t, r);
  fe_sub_2x(X3, t, hhh, v);  // R^2 - H^3 - 2 U1 H^2
  fe_mul(t, a.ZZ, b.ZZ);
  fe_mul(ZZ3, t, hh);
  return true;
}

// o = a + b for two Chudnovsky points with their TRUE Y (no sign
// convention), both normalized and not at infinity: add-2008-bl on the
// Chudnovsky form (U1 = Xa ZZb, U2 = Xb ZZa, S1 = Ya ZZZb, S2 = Yb ZZZa,
// H = U2 - U1, R = S2 - S1, X3 = R^2 - H^3 - 2 U1 H^2, Y3 = R (U1 H^2 - X3)
// - S1 H^3 merged into one reduction, ZZ3 = ZZa ZZb H^2, ZZZ3 = ZZZa ZZZb
// H^3).  Returns false for a degenerate addition (H == 0: equal or opposite
// points), which the caller resolves on the exact path.  The small-batch
// verifier's joins of partial comb sums (k_verify_split).
MBFT_DEV bool ec_add_chud_full(chud& o, const chud& a, const chud& b) {
  fe u1, u2, s1, s2, h, r, hh, hhh, v, t, n;
  fe_mul(u1, a.X, b.ZZ);
  fe_mul(u2, b.X, a.ZZ);
  fe_mul(s1, a.Y, b.ZZZ);
  fe_mul(s2, b.Y, a.ZZZ);
  fe_sub(h, u2, u1);  // < 2^257 + 2^233
  t = h;
  fe_canon(t);
  if (fe_is_zero_canon(t)) return false;
  fe_sub(r, s2, s1);
  fe_sqr(hh, h);
  fe_mul(hhh, hh, h);
  fe_mul(v, u1, hh);
  fe_sqr(t, r);
  fe_sub_2x(o.X, t, hhh, v);  // R^2 - H^3 - 2 U1 H^2
  fe_sub(t, v, o.X);          // U1 H^2 - X3
  fe_neg(n, s1);
  fe_mul2(o.Y, t, r, n, hhh);  // R (U1 H^2 - X3) - S1 H^3
  fe_mul(t, a.ZZ, b.ZZ);
  fe_mul(o.ZZ, t, hh);
  fe_mul(t, a.ZZZ, b.ZZZ);
  fe_mul(o.ZZZ, t, hhh);
  return true;
}

// ---------------------------------------------------------------------------
// Wave-uniform forms (ONE item per wave, every lane holding the same values:
// k_verify_split).  A single wave issues one instruction every ~4-5 cycles,
// so a lone item's latency is its dependent chain of field products.  These
// forms run the independent products of each dependency level at the same
// time in different 16-lane groups of the wave -- the lanes of group q pick
// their operands with a per-lane select and execute the SAME product code --
// then hand the results to every lane (v_readlane of the group's first lane:
// the values are wave-uniform again).  Same products, operands and bounds as
// the sequential forms above, so the same results bit for bit: a mixed
// addition's 9 products in 4 levels, a full addition's 13 in 4, the affine
// first addition's 5 in 3.
MBFT_DEV int wave_group() { return (int)(__lane_id() >> 4); }

// (kept in VGPRs -- an empty asm with a VGPR operand makes the value
// divergent to the compiler: as a uniform value it would move to SGPRs and
// every linear step after it to multi-instruction 64-bit SALU code, with
// SGPR spills; measured slower)
MBFT_DEV void fe_bcast(fe& o, const fe& v, int lane) {
#pragma unroll
  for (int k = 0; k < NL; k++) {
    uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)v.v[k], lane);
    asm volatile("" : "+v"(x));
    o.v[k] = x;
  }
}

// o = a, b, c or d by lane group (0..3), as masks on the limb values (a
// select between the four references compiles to a pointer select, which
// puts the operands in scratch memory)
MBFT_DEV void fe_sel4(fe& o, int g, const fe& a, const fe& b, const fe& c, const fe& d) {
  const uint32_t m0 = 0u - (uint32_t)(g == 0), m1 = 0u - (uint32_t)(g == 1);
  const uint32_t m2 = 0u - (uint32_t)(g == 2), m3 = 0u - (uint32_t)(g == 3);
#pragma unroll
  for (int k = 0; k < NL; k++) o.v[k] = (a.v[k] & m0) | (b.v[k] & m1) | (c.v[k] & m2) | (d.v[k] & m3);
}

// ec_madd_chud<false, false> (same sign convention), uniform item.
MBFT_DEV void ec_madd_chud_wide(chud& o, const chud& a, const fe& x2, const fe& y2, bool add_s2) {
  const int g = wave_group();
  fe t1, t2, A, B, C, p, h, r, hh, rr, zz3, hhh, v, x3, w;
#pragma unroll
  for (int i = 0; i < NL; i++) t1.v[i] = kP5B[i] - a.X.v[i];
#pragma unroll
  for (int i = 0; i < NL; i++) t2.v[i] = add_s2 ? a.Y.v[i] : kP5B[i] - a.Y.v[i];
  // 1: H = x2 ZZ1 + (5p - X1) (group 0), R" = y2 ZZZ1 + w (group 1)
  fe_sel4(A, g, x2, y2, x2, x2);
  fe_sel4(B, g, a.ZZ, a.ZZZ, a.ZZ, a.ZZ);
  fe_sel4(C, g, t1, t2, t1, t1);
  fe_mul_add(p, A, B, C);
  fe_bcast(h, p, 0);
  fe_bcast(r, p, 16);
  // 2: H^2, R"^2
  fe_sel4(A, g, h, r, h, h);
  fe_sqr(p, A);
  fe_bcast(hh, p, 0);
  fe_bcast(rr, p, 16);
  // 3: ZZ3 = ZZ1 H^2, H^3, V = X1 H^2
  fe_sel4(A, g, a.ZZ, h, a.X, a.X);
  fe_mul(p, A, hh);
  fe_bcast(zz3, p, 0);
  fe_bcast(hhh, p, 16);
  fe_bcast(v, p, 32);
  fe_sub_2x(x3, rr, hhh, v);  // X3 = R"^2 - H^3 - 2V
  // 4: ZZZ3 = ZZZ1 H^3 (as a fe_mul2 with a zero second product: the same
  // columns, the same reduction), Y3 = R" (V - X3 + 5p) + w H^3
#pragma unroll
  for (int i = 0; i < NL; i++) w.v[i] = v.v[i] + kP5B[i] - x3.v[i];
  fe zero;
  fe_zero(zero);
  fe_sel4(A, g, a.ZZZ, w, a.ZZZ, a.ZZZ);
  fe_sel4(B, g, hhh, r, hhh, hhh);
  fe_sel4(C, g, zero, t2, zero, zero);
  fe_mul2(p, A, B, C, hhh);
  o.X = x3;
  o.ZZ = zz3;
  fe_bcast(o.ZZZ, p, 0);
  fe_bcast(o.Y, p, 16);
}

// ec_add_affine_chud, uniform item.
MBFT_DEV void ec_add_affine_chud_wide(chud& o, const fe& x1, const fe& y1, const fe& x2, const fe& y2,
                                      bool add_s2) {
  const int g = wave_group();
  fe h, r, A, B, p, hh, rr, zzz, v, x3, t4, y3;
  fe_sub5(h, x2, x1);
#pragma unroll
  for (int i = 0; i < NL; i++) {
    const uint32_t m = kP5[i] - y2.v[i];
    r.v[i] = y1.v[i] + (add_s2 ? y2.v[i] : m);
  }
  fe_carry_s(r);
  // 1: H^2, R'^2
  fe_sel4(A, g, h, r, h, h);
  fe_sqr(p, A);
  fe_bcast(hh, p, 0);
  fe_bcast(rr, p, 16);
  // 2: H^3 = H^2 H, V = H^2 x1
  fe_sel4(B, g, h, x1, h, h);
  fe_mul(p, hh, B);
  fe_bcast(zzz, p, 0);
  fe_bcast(v, p, 16);
  fe_sub_2x(x3, rr, zzz, v);
  fe_sub(t4, v, x3);
  fe_mul2(y3, t4, r, y1, zzz);
  o.ZZ = hh;
  o.ZZZ = zzz;
  o.X = x3;
  o.Y = y3;
}

// ec_add_chud_full, uniform item (both points normalized, TRUE Y).
MBFT_DEV bool ec_add_chud_full_wide(chud& o, const chud& a, const chud& b) {
  const int g = wave_group();
  fe A, B, C, p, u1, u2, s1, s2, h, r, t, hh, rr, hhh, v, tz, tzz, x3, t3, n;
  // 1: U1 = Xa ZZb, U2 = Xb ZZa, S1 = Ya ZZZb, S2 = Yb ZZZa
  fe_sel4(A, g, a.X, b.X, a.Y, b.Y);
  fe_sel4(B, g, b.ZZ, a.ZZ, b.ZZZ, a.ZZZ);
  fe_mul(p, A, B);
  fe_bcast(u1, p, 0);
  fe_bcast(u2, p, 16);
  fe_bcast(s1, p, 32);
  fe_bcast(s2, p, 48);
  fe_sub(h, u2, u1);
  t = h;
  fe_canon(t);
  if (fe_is_zero_canon(t)) return false;
  fe_sub(r, s2, s1);
  // 2: H^2, R^2
  fe_sel4(A, g, h, r, h, h);
  fe_sqr(p, A);
  fe_bcast(hh, p, 0);
  fe_bcast(rr, p, 16);
  // 3: H^3 = H^2 H, V = U1 H^2, ZZa ZZb, ZZZa ZZZb
  fe_sel4(A, g, hh, u1, a.ZZ, a.ZZZ);
  fe_sel4(B, g, h, hh, b.ZZ, b.ZZZ);
  fe_mul(p, A, B);
  fe_bcast(hhh, p, 0);
  fe_bcast(v, p, 16);
  fe_bcast(tz, p, 32);
  fe_bcast(tzz, p, 48);
  fe_sub_2x(x3, rr, hhh, v);  // R^2 - H^3 - 2 U1 H^2
  fe_sub(t3, v, x3);          // U1 H^2 - X3
  fe_neg(n, s1);
  // 4: Y3 = R (U1 H^2 - X3) - S1 H^3, ZZ3 = ZZa ZZb H^2, ZZZ3 = ZZZa ZZZb H^3
  // (the last two as fe_mul2 with a zero second product)
  fe zero;
  fe_zero(zero);
  fe_sel4(A, g, t3, tz, tzz, tzz);
  fe_sel4(B, g, r, hh, hhh, hhh);
  fe_sel4(C, g, n, zero, zero, zero);
  fe_mul2(p, A, B, C, hhh);
  o.X = x3;
  fe_bcast(o.Y, p, 0);
  fe_bcast(o.ZZ, p, 16);
  fe_bcast(o.ZZZ, p, 32);
  return true;
}

// o = 2a (a = -3).  Safe for o aliasing a.
MBFT_DEV void ec_dbl(jac& o, const jac& a) {
  fe delta, gamma, beta, t1, t2, alpha, b8, t;
  fe_sqr(delta, a.Z);
  fe_sqr(gamma, a.Y);
  fe_mul(beta, a.X, gamma);
  fe_sub(t1, a.X, delta);
  fe_add(t2, a.X, delta);
  fe_mul(alpha, t1, t2);
  fe_mulsmall(alpha, alpha, 3);  // 3 (X1 - delta)(X1 + delta)
  fe_mul(t, a.Y, a.Z);
  fe_mulsmall(o.Z, t, 2);        // Z3 = 2 Y1 Z1
  fe_sqr(t, alpha);
  fe_mulsmall(b8, beta, 8);
  fe_sub(o.X, t, b8);            // X3 = alpha^2 - 8 beta
  fe_mulsmall(t1, beta, 4);
  fe_sub(t1, t1, o.X);           // 4 beta - X3
  fe_mul(t1, t1, alpha);
  fe_sqr(t2, gamma);
  fe_mulsmall(t2, t2, 8);        // 8 gamma^2
  fe_sub(o.Y, t1, t2);
}

// Jacobian -> affine (canonical Montgomery); Z must be nonzero.
MBFT_DEV void ec_to_affine(fe& x, fe& y, const jac& a) {
  fe zi, zi2;
  fe_inv(zi, a.Z);
  fe_sqr(zi2, zi);
  fe_mul(x, a.X, zi2);
  fe_mul(zi2, zi2, zi);
  fe_mul(y, a.Y, zi2);
  fe_canon(x);
  fe_canon(y);
}

// Complete accumulate: (acc, inf) += (x2, y2), handling acc == +-P and
// acc == infinity exactly.  Used only on the rare slow path.
MBFT_DEV void ec_madd_complete(jac& acc, bool& inf, const fe& x2, const fe& y2) {
  if (inf) {
    acc.X = x2;
    acc.Y = y2;
    fe_one_mont(acc.Z);
    inf = false;
    return;
  }
  fe t1, t2, h, r;
  fe_sqr(t1, acc.Z);
  fe_mul(t2, t1, acc.Z);
  fe_mul(t1, t1, x2);
  fe_mul(t2, t2, y2);
  fe_sub(h, t1, acc.X);
  fe_sub(r, t2, acc.Y);
  fe_canon(h);
  fe_canon(r);
  if (fe_is_zero_canon(h)) {
    if (fe_is_zero_canon(r)) {
      ec_dbl(acc, acc);
    } else {
      inf = true;
    }
    return;
  }
  ec_madd(acc, acc, x2, y2);
}

// Load an affine table entry (16 LE words: x then y, canonical Montgomery).
MBFT_DEV void load_point(fe& x, fe& y, const uint4* p) {
  uint4 a = p[0], b = p[1], c = p[2], d = p[3];
  uint32_t wx[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  uint32_t wy[8] = {c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
  fe_from_words(x, wx);
  fe_from_words(y, wy);
}

}  // namespace mbft

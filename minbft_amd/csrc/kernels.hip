// HIP kernels for the MinBFT batch authenticator (gfx950).
//
// Hot path (replaces Go crypto/ecdsa.Verify as called from
// sample/authentication/crypto.go:86 and usig/sgx/usig-enclave.go:224):
//   k_verify   one signature per lane: range checks on r, s; w = s^-1 mod N
//              (precomputed by the batched inversion kernels, or per lane);
//              u1 = e*w, u2 = r*w; R = u1*G + u2*Q by signed-digit comb
//              tables T[i][|d|] = |d| * 2^(W i) * P (runtime W per table, up
//              to 29 bits: 16 mixed additions + 1 affine addition at 29/29,
//              no doublings), entries gathered cooperatively into LDS;
//              accept iff R != inf and x(R) mod N == r, checked
//              projectively (X == r*Z^2 or X == (r+N)*Z^2), no inversion.
// Table construction (init time, once per key; replica set is static):
//   k_check_points, k_table_pow2, k_table_fill.
// Batched scalar inversion (Montgomery's trick over strided groups):
//   k_ninv_up, k_ninv_root, k_ninv_down.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <utility>

#include "arena_dev.h"
#include "authen_dev.h"
#include "der_dev.h"
#include "ecc.h"

#include "kernels.h"
#include "modinv.h"
#include "sha256.h"
#include "sha256_dev.h"

using namespace mbft;

namespace {

// Generator and curve b as little-endian words (plain, canonical).
__constant__ uint32_t kGxw[8] = {0xD898C296u, 0xF4A13945u, 0x2DEB33A0u, 0x77037D81u,
                                 0x63A440F2u, 0xF8BCE6E5u, 0xE12C4247u, 0x6B17D1F2u};
__constant__ uint32_t kGyw[8] = {0x37BF51F5u, 0xCBB64068u, 0x6B315ECEu, 0x2BCE3357u,
                                 0x7C0F9E16u, 0x8EE7EB4Au, 0xFE1A7F9Bu, 0x4FE342E2u};
__constant__ uint32_t kBw[8] = {0x27D2604Bu, 0x3BCE3C3Eu, 0xCC53B0F6u, 0x651D06B0u,
                                0x769886BCu, 0xB3EBBD55u, 0xAA3A93E7u, 0x5AC635D8u};

MBFT_DEV void load_words8(uint32_t w[8], const uint32_t* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 a = q[0], b = q[1];
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
  w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}

MBFT_DEV void store_words8(uint32_t* p, const uint32_t w[8]) {
  uint4* q = reinterpret_cast<uint4*>(p);
  q[0] = make_uint4(w[0], w[1], w[2], w[3]);
  q[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

// 32 big-endian bytes at p -> little-endian words
MBFT_DEV void load_be256(uint32_t w[8], const uint8_t* p) {
  uint32_t be[8];
  load_words8(be, reinterpret_cast<const uint32_t*>(p));
  be_words_to_le(w, be);
}

MBFT_DEV void store_point_words(uint32_t* dst, const fe& x, const fe& y) {
  uint32_t wx[8], wy[8];
  fe_to_words(wx, x);
  fe_to_words(wy, y);
  store_words8(dst, wx);
  store_words8(dst + 8, wy);
}

}  // namespace

// ---------------------------------------------------------------------------
// Key validation: x, y < p and y^2 == x^3 - 3x + b.  xy: n x 16 LE words.
// (x509.ParsePKIXPublicKey's on-curve check, keymanager.go:357)
__global__ void k_check_points(const uint32_t* __restrict__ xy, int n,
                               uint32_t* __restrict__ ok) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t wx[8], wy[8];
  load_words8(wx, xy + 16 * i);
  load_words8(wy, xy + 16 * i + 8);
  const bool in_range = words_lt(wx, kPw) && words_lt(wy, kPw);
  fe x, y, b, t, lhs, rhs;
  fe_from_words(x, wx);
  fe_from_words(y, wy);
  fe_from_words(b, kBw);
  fe_to_mont(x, x);
  fe_to_mont(y, y);
  fe_to_mont(b, b);
  fe_sqr(lhs, y);
  fe_sqr(t, x);
  fe_mul(t, t, x);               // x^3
  fe_mulsmall(rhs, x, 3);
  fe_sub(rhs, t, rhs);           // x^3 - 3x
  fe_add(rhs, rhs, b);
  fe_canon(lhs);
  fe_canon(rhs);
  ok[i] = (in_range && fe_eq_canon(lhs, rhs)) ? 1u : 0u;
}

// Comb geometry for window W, SIGNED digits: S = ceil(256 / W) windows.  A
// scalar u < 2^256 is recoded low to high into digits d_i in
// (-2^(W-1), 2^(W-1)] (x = window bits + carry; x > 2^(W-1) -> d = x - 2^W,
// carry 1), except the last window, which holds the top L = 256 - (S-1) W
// bits plus the carry: 0 <= d <= 2^L.  A table stores |d| * 2^(W i) * P for
// |d| >= 1 only (y of a negative digit is negated at use), at index
// (i << (W-1)) + |d| - 1: 2^(W-1) entries per window, 2^L for the last --
// half the entries of an unsigned comb with the same number of windows.
MBFT_DEV int comb_steps(int W) { return (256 + W - 1) / W; }
MBFT_DEV long comb_entries(int W) {
  const int S = comb_steps(W);
  return ((long)(S - 1) << (W - 1)) + (1L << (256 - (S - 1) * W));
}

// B[pt][i] = 2^(W*i) * P_pt for i < S, affine canonical Montgomery (16 words
// each).  xy: plain affine input points (validated).  One thread per (pt, i).
__global__ void k_table_pow2(const uint32_t* __restrict__ xy, int npts, int wbits,
                             uint32_t* __restrict__ bpts) {
  const int nwin = comb_steps(wbits);
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= npts * nwin) return;
  const int pt = t / nwin, w = t % nwin;
  uint32_t wx[8], wy[8];
  load_words8(wx, xy + 16 * pt);
  load_words8(wy, xy + 16 * pt + 8);
  jac a;
  fe_from_words(a.X, wx);
  fe_from_words(a.Y, wy);
  fe_to_mont(a.X, a.X);
  fe_to_mont(a.Y, a.Y);
  fe_one_mont(a.Z);
#pragma unroll 1
  for (int j = 0; j < wbits * w; j++) ec_dbl(a, a);
  fe x, y;
  ec_to_affine(x, y, a);
  store_point_words(bpts + 16 * t, x, y);
}

// tab[pt] entry (i, d - 1) = d * B[pt][i] (signed-digit layout above); the
// tables of the npts points follow each other (comb_entries(W) entries
// each), 16 words (x, y) per entry.
//
// Run-based fill: thread t owns a run of kFillRun consecutive multiples
// d0 .. d0 + L - 1 of one window's base point B (fewer when the window is
// smaller).  P_d0 = d0 B by double-and-add, then P_d = P_(d-1) + B, one mixed
// addition each (P_2 = 2B by doubling when d0 = 1: the only degenerate
// addition, since c B = +-B needs c = +-1 mod N).  Each Jacobian (X, Y) is
// parked canonical in its own output slot and the Z ratio H_d (Z_d = Z_(d-1)
// H_d) in scratch planes; ONE inversion per run gives 1/Z_last, and the
// down pass walks back: (x, y) = (X zi^2, Y zi^3), zi <- zi H_d.  About 20
// field multiplies per entry instead of a double-and-add plus an inversion
// per entry (~700).
constexpr int kFillRun = 32;

struct FillGeom {
  int S, L0, L1;      // windows, run length for windows 0..S-2 and for the last
  long R0, R1, runs;  // runs per window (full / last), runs per point
};

MBFT_DEV FillGeom fill_geom(int W) {
  FillGeom g;
  g.S = comb_steps(W);
  const int lastbits = 256 - (g.S - 1) * W;
  const long n0 = 1L << (W - 1), n1 = 1L << lastbits;
  g.L0 = (int)min((long)kFillRun, n0);
  g.L1 = (int)min((long)kFillRun, n1);
  g.R0 = n0 / g.L0;
  g.R1 = n1 / g.L1;
  g.runs = (long)(g.S - 1) * g.R0 + g.R1;
  return g;
}

MBFT_DEV void park_xy(uint32_t* dst, const jac& a) {
  fe x = a.X, y = a.Y;
  fe_canon(x);
  fe_canon(y);
  store_point_words(dst, x, y);
}

// runs [first, first + count) of the npts points' tables; scratch: 9 x L
// planes of `count` words (H of run-local entry j, limb k at (j*9+k)*count + t)
__global__ void __launch_bounds__(256) k_table_fill(const uint32_t* __restrict__ bpts, int npts,
                                                    int wbits, long first, long count,
                                                    uint32_t* __restrict__ scratch,
                                                    uint32_t* __restrict__ tab) {
  const FillGeom g = fill_geom(wbits);
  const long tl = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long t = first + tl;
  if (tl >= count || t >= (long)npts * g.runs) return;
  const long pt = t / g.runs, rr = t - pt * g.runs;
  long win, run;
  int L;
  if (rr < (long)(g.S - 1) * g.R0) {
    win = rr / g.R0;
    run = rr - win * g.R0;
    L = g.L0;
  } else {
    win = g.S - 1;
    run = rr - (long)(g.S - 1) * g.R0;
    L = g.L1;
  }
  const long d0 = run * L + 1;  // first multiple of this run
  const long ent = comb_entries(wbits);
  uint32_t* dst = tab + 16 * (pt * ent + (win << (wbits - 1)) + (d0 - 1));
  fe bx, by;
  load_point(bx, by, reinterpret_cast<const uint4*>(bpts + 16 * (pt * g.S + win)));

  // P = d0 B (left-to-right double-and-add; partial sums c B with 1 < c < N
  // are never +-B)
  jac a;
  a.X = bx;
  a.Y = by;
  fe_one_mont(a.Z);
  const int top = 63 - __builtin_clzl((unsigned long)d0);
#pragma unroll 1
  for (int b = top - 1; b >= 0; b--) {
    ec_dbl(a, a);
    if ((d0 >> b) & 1) ec_madd(a, a, bx, by);
  }
  park_xy(dst, a);
  // chain: P_j = P_(j-1) + B, H_j parked in scratch
#pragma unroll 1
  for (int j = 1; j < L; j++) {
    fe h;
    if (d0 == 1 && j == 1) {
      ec_dbl(a, a);  // 2B from B (Z_0 = 1): the ratio is Z_1 itself
      h = a.Z;
    } else {
      ec_madd(a, a, bx, by, &h);
    }
#pragma unroll
    for (int k = 0; k < NL; k++) scratch[((long)j * NL + k) * count + tl] = h.v[k];
    park_xy(dst + 16 * j, a);
  }
  // 1/Z_(L-1), then walk back
  fe zi;
  fe_inv(zi, a.Z);
#pragma unroll 1
  for (int j = L - 1; j >= 0; j--) {
    fe X, Y, z2, z3, x, y;
    load_point(X, Y, reinterpret_cast<const uint4*>(dst + 16 * j));
    fe_sqr(z2, zi);
    fe_mul(z3, z2, zi);
    fe_mul(x, X, z2);
    fe_mul(y, Y, z3);
    fe_canon(x);
    fe_canon(y);
    store_point_words(dst + 16 * j, x, y);
    if (j > 0) {
      fe h;
#pragma unroll
      for (int k = 0; k < NL; k++) h.v[k] = scratch[((long)j * NL + k) * count + tl];
      fe_mul(zi, zi, h);  // 1/Z_(j-1)
    }
  }
}

// ---------------------------------------------------------------------------
// Batched inversion mod N (Montgomery's trick).  Values are Montgomery-form
// limbs stored as 9 planes of n uint32 (SoA, coalesced).  Level structure:
// thread g of a level with G groups owns items g, g+G, g+2G, ... (strided so
// that each step of the chain is a coalesced access); it writes the running
// prefix products over its chain in place of nothing (prefix array) and the
// chain total into the next level's input.

MBFT_DEV void plane_load(fe& a, const uint32_t* planes, long n, long i) {
#pragma unroll
  for (int k = 0; k < NL; k++) a.v[k] = planes[k * n + i];
}

MBFT_DEV void plane_store(uint32_t* planes, long n, long i, const fe& a) {
#pragma unroll
  for (int k = 0; k < NL; k++) planes[k * n + i] = a.v[k];
}

// The chain kernels run beside the previous batch's verify kernel (DESIGN.md
// §4): s_setprio(3) gives their few waves issue priority on the SIMDs they
// share with verify waves, so the latency-bound chain is not slowed 3-4x by
// round-robin issue; the verify kernel loses only the slots these waves use.
#define MBFT_CHAIN_PRIO() __builtin_amdgcn_s_setprio(3)

// s (32 BE bytes) of item i as a PLAIN value; out-of-range s -> 1 (the
// verifier rejects those items on the range check before using w).
//
// The chains run Montgomery's trick on plain values with Montgomery
// multiplies (x*y/R): prefix p_k = p_(k-1) s_k / R from p_0 = R, and the
// root hands down P^-1 R for its chain total P.  Then in the down-sweep
// r = p_k^-1 R gives mont(p_(k-1), r) = s_k^-1 R -- exactly the Montgomery
// form of w the verifier multiplies e and r by -- and mont(r, s_k) =
// p_(k-1)^-1 R for the next item.  No per-item conversion to Montgomery form.
MBFT_DEV void s_plain(fe& a, const uint8_t* s, long i) {
  uint32_t w[8];
  load_be256(w, s + 32 * i);
  const bool ok = !words_is_zero(w) && words_lt(w, kNw);
  fe_from_words(a, w);
  if (!ok) {
    fe_zero(a);
    a.v[0] = 1;
  }
}

// Level-l up-sweep.  in: x[n] (planes), or the raw s bytes at level 0;
// out: pre[n] (pre[i] = product of the chain items before i), tot[G] =
// product of each chain.  Thread g owns items g, g+G, g+2G, ... (each step
// of the chain is a coalesced access).
template <bool FROM_S>
__global__ void k_ninv_up(const uint32_t* __restrict__ x, const uint8_t* __restrict__ s, long n,
                          long G, uint32_t* __restrict__ pre, uint32_t* __restrict__ tot) {
  MBFT_CHAIN_PRIO();
  const long g = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  fe acc;
  fe_set(acc, kRN);  // Montgomery one
#pragma unroll 1
  for (long i = g; i < n; i += G) {
    plane_store(pre, n, i, acc);
    fe v;
    if (FROM_S)
      s_plain(v, s, i);
    else
      plane_load(v, x, n, i);
    fn_mul(acc, acc, v);
  }
  plane_store(tot, G, g, acc);
}

// Level 0 of the chain with TWO chains per thread (chains h and h + H, H =
// ceil(G / 2)), walked in lockstep with branch-free steps so the two
// independent products can interleave: the same outputs as k_ninv_up<true>
// with half the waves.  The idea: the chain kernels run beside the previous
// batches' verify waves (3 per SIMD, 168 VGPRs), where every chain wave
// displaces a verify wave while it lives.  Measured slower (the chain span
// grew 0.30 -> 0.355 ms, the step 1.4 %), so off by default
// (MBFT_NINV_CHAINS=2).  A chain's items: g, g + G, ... < n;
// chain h is never shorter than chain h + H.
__global__ void k_ninv_up2(const uint8_t* __restrict__ s, long n, long G, uint32_t* __restrict__ pre,
                           uint32_t* __restrict__ tot) {
  MBFT_CHAIN_PRIO();
  const long H = (G + 1) / 2;
  const long h = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= H || h >= n) return;
  const long g1 = h + H;
  const bool has1 = g1 < G && g1 < n;
  fe a0, a1;
  fe_set(a0, kRN);
  fe_set(a1, kRN);
#pragma unroll 1
  for (long i0 = h; i0 < n; i0 += G) {
    const long i1 = i0 + H;
    const bool v1 = has1 && i1 < n;
    fe x0, x1, t0, t1;
    s_plain(x0, s, i0);
    s_plain(x1, s, v1 ? i1 : i0);
    plane_store(pre, n, i0, a0);
    if (v1) plane_store(pre, n, i1, a1);
    fn_mul(t0, a0, x0);
    fn_mul(t1, a1, x1);
    a0 = t0;
#pragma unroll
    for (int k = 0; k < NL; k++) a1.v[k] = v1 ? t1.v[k] : a1.v[k];
  }
  plane_store(tot, G, h, a0);
  if (has1) plane_store(tot, G, g1, a1);
}

// Level 0's down-sweep with two chains per thread (k_ninv_up2's pairing):
// each chain walked from its last item back, in lockstep (chain h + H may be
// one item shorter: its step is then skipped).
__global__ void k_ninv_down2(const uint8_t* __restrict__ s, const uint32_t* __restrict__ pre, long n,
                             long G, const uint32_t* __restrict__ inv_tot, uint32_t* __restrict__ inv,
                             uint32_t* __restrict__ zero_word) {
  MBFT_CHAIN_PRIO();
  if (zero_word && blockIdx.x == 0 && threadIdx.x == 0) *zero_word = 0;
  const long H = (G + 1) / 2;
  const long h = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= H || h >= n) return;
  const long g1 = h + H;
  const bool has1 = g1 < G && g1 < n;
  fe r0, r1;
  plane_load(r0, inv_tot, G, h);
  if (has1) plane_load(r1, inv_tot, G, g1);
  else fe_set(r1, kRN);
  const long last0 = h + ((n - 1 - h) / G) * G;
  const long len0 = (last0 - h) / G + 1;
  const long len1 = has1 ? (n - 1 - g1) / G + 1 : 0;
  // step k: chain 0 at last0 - k G; chain 1 at its last - (k - (len0 - len1)) G
  const long skew = len0 - len1;  // 0 or 1
#pragma unroll 1
  for (long k = 0; k < len0; k++) {
    const long i0 = last0 - k * G;
    const long k1 = k - skew;
    const bool v1 = has1 && k1 >= 0;
    const long i1 = v1 ? g1 + (len1 - 1 - k1) * G : i0;
    fe p0, p1, x0, x1, t0, t1, u0, u1;
    plane_load(p0, pre, n, i0);
    plane_load(p1, pre, n, i1);
    s_plain(x0, s, i0);
    s_plain(x1, s, i1);
    fn_mul(t0, r0, p0);
    fn_mul(t1, r1, p1);
    fn_mul(u0, r0, x0);
    fn_mul(u1, r1, x1);
    plane_store(inv, n, i0, t0);
    if (v1) plane_store(inv, n, i1, t1);
    r0 = u0;
#pragma unroll
    for (int q = 0; q < NL; q++) r1.v[q] = v1 ? u1.v[q] : r1.v[q];
  }
}

// x^-1 mod N (modinv.h's divsteps) by ALL 64 lanes of a wave together, on
// ONE value (every lane passes the same x; the roots of the batched s^-1).
// The two halves of each 30-divstep batch run where they are cheap:
//  * the 30 divsteps themselves on the SCALAR unit: f0, g0 and eta are
//    wave-uniform (v_readlane), so divsteps_30_var compiles to single
//    32-bit SALU instructions (s_ff1, shifts, s_mul) and uniform branches;
//  * the 2x2 matrix applied to the four 9-limb numbers on the VALU, split
//    over every quad of lanes: lane L = lane & 3 computes d' (0), e' (1)
//    (mod N) or f' (2), g' (3) (exact), and DPP quad broadcasts hand each
//    lane its next two operands ((d, e) on lanes 0, 1, (f, g) on 2, 3), so
//    the numbers stay in VGPRs.
// (Round 2's form gathered the four outputs to every lane with 36
// v_readlane per batch, which put the whole update on the scalar unit as
// multi-instruction 64-bit SALU arithmetic: ~840 SALU + 390 VALU per batch,
// ~43 us per inversion; tools/isa_hist.py.)  Returns the same as
// modinv_n_var.
MBFT_DEV int32_t quad_bcast(int32_t v, int sel) {
  // sel 0: lanes (0,0,2,2) of the quad, sel 1: lanes (1,1,3,3)
  return sel == 0 ? __builtin_amdgcn_mov_dpp(v, 0xA0, 0xF, 0xF, true)
                  : __builtin_amdgcn_mov_dpp(v, 0xF5, 0xF, 0xF, true);
}

MBFT_DEV bool modinv_n_var_wave(uint32_t out[8], const uint32_t x[8]) {
  const int L = __lane_id() & 3;
  const bool modn = L < 2;
  s30 M, xs;
  s30_modulus(M);
  s30_from_words(xs, x);
  // this lane's operands: (d, e) = (0, 1) on lanes 0, 1; (f, g) = (N, x) on 2, 3
  int32_t a[9], b[9];
#pragma unroll
  for (int i = 0; i < 9; i++) {
    a[i] = modn ? 0 : M.v[i];
    b[i] = modn ? (i == 0 ? 1 : 0) : xs.v[i];
  }
  int32_t eta = -1;
#pragma unroll 1
  for (int it = 0; it < 64; it++) {
    trans2x2 t;
    const uint32_t f0 = (uint32_t)__builtin_amdgcn_readlane(a[0], 2);
    const uint32_t g0 = (uint32_t)__builtin_amdgcn_readlane(b[0], 2);
    eta = divsteps_30_var(eta, f0, g0, t);
    // this lane's output: L = 0 -> d', 1 -> e' (mod N), 2 -> f', 3 -> g'
    const int32_t c1 = (L & 1) ? t.q : t.u, c2 = (L & 1) ? t.r : t.v;
    int64_t c = (int64_t)c1 * a[0] + (int64_t)c2 * b[0];
    int32_t m = (c1 & (a[8] >> 31)) + (c2 & (b[8] >> 31));
    m -= (int32_t)((kNinv30 * (uint32_t)c + (uint32_t)m) & (uint32_t)kM30);
    m = modn ? m : 0;  // f, g: exact division, no multiple of N
    c += (int64_t)M.v[0] * m;
    c >>= 30;
    int32_t o[9];
#pragma unroll
    for (int i = 1; i < 9; i++) {
      c += (int64_t)c1 * a[i] + (int64_t)c2 * b[i] + (int64_t)M.v[i] * m;
      o[i - 1] = (int32_t)c & kM30;
      c >>= 30;
    }
    o[8] = (int32_t)c;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      a[i] = quad_bcast(o[i], 0);
      b[i] = quad_bcast(o[i], 1);
    }
    int32_t z = 0;
#pragma unroll
    for (int j = 0; j < 9; j++) z |= b[j];
    if (__builtin_amdgcn_readlane(z, 2) == 0) {  // g == 0 (lane 2's b)
      s30 f, d;
#pragma unroll
      for (int j = 0; j < 9; j++) {
        f.v[j] = __builtin_amdgcn_readlane(a[j], 2);
        d.v[j] = __builtin_amdgcn_readlane(a[j], 0);
      }
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

// The root of the tree: the m <= kTopMax chain totals x_k of the top level
// (planes, stride m) -> x_k^-1 R mod N, in place (what the down-sweeps hand
// down).  ONE workgroup: 4 values per thread as a chain (p_0 = R, p_j =
// mont(p_(j-1), v_j)), a product tree of the 1024 thread totals in LDS, one
// inversion at the root on lane 0 (divsteps, modinv.h: ~8K dependent ops
// where Fermat needs ~60K), then the tree and the chains walked back:
// inv(a) = mont(inv(a b / R), b) at every node, exactly as in the down-sweeps.
constexpr int kTopThreads = 256, kTopPer = 16;
constexpr long kTopMax = (long)kTopThreads * kTopPer;

// 256 threads (one wave per SIMD of one CU) so that the kernel fits beside
// the previous batch's verify waves (3 per SIMD, 168 VGPRs each): a
// 1024-thread block needs a nearly empty CU and waited for the verify
// kernel's tail.  Prefixes go to `pre` (kTopMax planes), not registers.
// The product tree of the 256 values node[256 + t] (t = thread) and back:
// node[1] = their product, inverted by wave 0 (x^-1 R), then every node
// replaced by the inverse of its value: inv(a) = mont(inv(a b / R), b).  On
// return node[256 + t] = (value of thread t)^-1 R.  All 256 threads call it.
MBFT_DEV void lds_tree_invert(uint32_t (&node)[NL][512], int t) {
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if (t < w) {
      const int i = w + t;
      fe a, b, c;
#pragma unroll
      for (int k = 0; k < NL; k++) {
        a.v[k] = node[k][2 * i];
        b.v[k] = node[k][2 * i + 1];
      }
      fn_mul(c, a, b);
#pragma unroll
      for (int k = 0; k < NL; k++) node[k][i] = c.v[k];
    }
    __syncthreads();
  }
  // The root inversion runs on ALL lanes of wave 0, each on the same value,
  // passed through an empty asm with VGPR operands so the compiler treats it
  // as divergent: the code is then VALU (one v_mad per 32x32+64 product).
  // Uniform (lane 0 alone, or a uniform LDS read) it is scalarized into
  // multi-instruction SALU 64-bit arithmetic (tools/ubench_inv.hip).
  if (t < 64) {
    fe r;
#pragma unroll
    for (int k = 0; k < NL; k++) r.v[k] = node[k][1];
    fn_canon(r);
    uint32_t w[8], iw[8];
    fe_to_words(w, r);
#pragma unroll
    for (int k = 0; k < 8; k++) asm volatile("" : "+v"(w[k]));  // divergent to the compiler
    if (!modinv_n_var_wave(iw, w)) {
      // not reachable: every leaf is a product of values in [1, N)
#pragma unroll
      for (int k = 0; k < 8; k++) iw[k] = 0;
    }
    fe_from_words(r, iw);
    fn_to_mont(r, r);  // x^-1 R
    if (t == 0) {
#pragma unroll
      for (int k = 0; k < NL; k++) node[k][1] = r.v[k];
    }
  }
  __syncthreads();
  for (int w = 1; w < 256; w <<= 1) {
    if (t < w) {
      const int i = w + t;
      fe a, b, r, ia, ib;
#pragma unroll
      for (int k = 0; k < NL; k++) {
        a.v[k] = node[k][2 * i];
        b.v[k] = node[k][2 * i + 1];
        r.v[k] = node[k][i];
      }
      fn_mul(ia, r, b);
      fn_mul(ib, r, a);
#pragma unroll
      for (int k = 0; k < NL; k++) {
        node[k][2 * i] = ia.v[k];
        node[k][2 * i + 1] = ib.v[k];
      }
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256) k_ninv_top(uint32_t* __restrict__ x, long m,
                                                  uint32_t* __restrict__ pre) {
  MBFT_CHAIN_PRIO();
  __shared__ uint32_t node[NL][2 * kTopThreads];  // node i (1 = root, leaves 256..511), SoA
  const int t = threadIdx.x;
  fe acc;
  fe_set(acc, kRN);  // Montgomery one
#pragma unroll 1
  for (int j = 0; j < kTopPer; j++) {
    const long idx = (long)j * kTopThreads + t;  // strided: coalesced planes
    plane_store(pre, kTopMax, idx, acc);
    if (idx < m) {
      fe v;
      plane_load(v, x, m, idx);
      fn_mul(acc, acc, v);
    }
  }
#pragma unroll
  for (int k = 0; k < NL; k++) node[k][kTopThreads + t] = acc.v[k];
  lds_tree_invert(node, t);
  fe r;
#pragma unroll
  for (int k = 0; k < NL; k++) r.v[k] = node[k][kTopThreads + t];
#pragma unroll 1
  for (int j = kTopPer - 1; j >= 0; j--) {
    const long idx = (long)j * kTopThreads + t;
    if (idx >= m) continue;
    fe v, p, o;
    plane_load(v, x, m, idx);
    plane_load(p, pre, kTopMax, idx);
    fn_mul(o, p, r);  // x_idx^-1 R
    fn_mul(r, r, v);
    plane_store(x, m, idx, o);
  }
}

// The chains of the one-launch batched s^-1 (k_ninv_local, k_ninv_block):
// thread-local Montgomery's trick over PER items b0, b0 + STRIDE, ... (each
// step a coalesced access).  The prefixes go to the w planes themselves
// (each is read back once, on the way down, just before the inverse
// overwrites it), and the raw bytes of the next item -- and of the next
// prefix on the way down -- are loaded one step ahead: the chain is a
// dependent multiply chain, and a load issued at its own step would stall it
// for the memory latency at every step.  Items past the batch (and
// out-of-range s, which the verifier rejects anyway) take the value 1;
// Montgomery's trick is consistent for it and nothing is stored.
template <int STRIDE>
MBFT_DEV void ninv_load_raw(const uint8_t* s, long n, long b0, int k, uint32_t* w) {
  const long i = b0 + (long)STRIDE * k;
  load_be256(w, s + 32 * (i < n ? i : 0));
}
template <int STRIDE>
MBFT_DEV void ninv_to_plain(long n, long b0, int k, const uint32_t* w, fe& v) {
  const long i = b0 + (long)STRIDE * k;
  const bool ok = i < n && !words_is_zero(w) && words_lt(w, kNw);
  fe_from_words(v, w);
  if (!ok) {
    fe_zero(v);
    v.v[0] = 1;
  }
}
// acc (Montgomery one on entry) -> the chain's product; prefix k to the planes
template <int PER, int STRIDE>
MBFT_DEV void ninv_chain_up(const uint8_t* s, long n, long b0, uint32_t* winv, fe& acc) {
  uint32_t nxt[8];
  ninv_load_raw<STRIDE>(s, n, b0, 0, nxt);
#pragma unroll 1
  for (int k = 0; k < PER; k++) {
    const long i = b0 + (long)STRIDE * k;
    uint32_t cur[8];
#pragma unroll
    for (int j = 0; j < 8; j++) cur[j] = nxt[j];
    if (k + 1 < PER) ninv_load_raw<STRIDE>(s, n, b0, k + 1, nxt);
    fe v;
    ninv_to_plain<STRIDE>(n, b0, k, cur, v);
    if (i < n) plane_store(winv, n, i, acc);  // prefix before item k
    fn_mul(acc, acc, v);
  }
}
// r = (the chain's product)^-1 R -> every item's s^-1 R in the planes
template <int PER, int STRIDE>
MBFT_DEV void ninv_chain_down(const uint8_t* s, long n, long b0, uint32_t* winv, fe& r) {
  uint32_t nxt[8];
  fe pn;
  {
    const long i = b0 + (long)STRIDE * (PER - 1);
    if (i < n) plane_load(pn, winv, n, i);
  }
  ninv_load_raw<STRIDE>(s, n, b0, PER - 1, nxt);
#pragma unroll 1
  for (int k = PER - 1; k >= 0; k--) {
    const long i = b0 + (long)STRIDE * k;
    const fe p = pn;
    uint32_t cur[8];
#pragma unroll
    for (int j = 0; j < 8; j++) cur[j] = nxt[j];
    if (k > 0) {
      const long ip = i - STRIDE;
      if (ip < n) plane_load(pn, winv, n, ip);
      if (k > 1) ninv_load_raw<STRIDE>(s, n, b0, k - 1, nxt);
    }
    fe o;
    fn_mul(o, p, r);  // s_i^-1 R
    if (k > 0) {
      fe v;
      ninv_to_plain<STRIDE>(n, b0, k, cur, v);
      fn_mul(r, r, v);
    }
    if (i < n) plane_store(winv, n, i, o);
  }
}

// Batched s^-1 of a batch issued while the GPU is idle (one batch at a time:
// its latency is what counts): ONE launch, every WAVE independent (no LDS,
// no barrier).  Wave v owns items [64 PER v, 64 PER (v + 1)); lane l the
// strided chain l, l + 64, ... (PER items, coalesced, prefixes in
// registers).  The 64 chain totals meet in a butterfly over the lanes
// (__shfl_xor at distance 1, 2, .., 32: after it every lane holds the
// wave's product, and sib[j] the product of the block it met at level j),
// the whole wave inverts that product together (modinv_n_var_wave), and the
// butterfly and the chain are walked back: inv(a) = mont(inv(a b / R), b),
// w = s^-1 R written to the planes -- the arithmetic of the level chain
// (k_ninv_up / k_ninv_top / k_ninv_down), so the same w.  fn_mul is
// symmetric bit for bit (the same products in the same columns), so both
// partners of a level compute the same value and all lanes pass the same
// root.  One inversion per 64 PER items.  The pipelined C2 loop's form
// (PER 16, batch_inverse_s_pipelined): with no barrier its waves interleave
// with the previous batch's verify waves (host.cpp verify_device).  Block 0
// also zeroes the exact-path queue counter the verify kernel that follows
// on the same stream appends to (saves a memset launch on the critical path).
// PROBE (tools/ubench_ninv.hip only): lane 0 of each wave writes
// s_memrealtime stamps after each phase to probe[6 wave ..].
template <int PER, bool PROBE = false>
__global__ void __launch_bounds__(256) k_ninv_local(const uint8_t* __restrict__ s, long n,
                                                    uint32_t* __restrict__ winv,
                                                    uint32_t* __restrict__ zero_word,
                                                    uint64_t* __restrict__ probe = nullptr,
                                                    const uint32_t* __restrict__ ndev = nullptr) {
  if (zero_word && blockIdx.x == 0 && threadIdx.x == 0) *zero_word = 0;
  uint64_t stamp[6];
  auto mark = [&](int k, const fe& dep) {
    if (PROBE) {
      asm volatile("s_nop 0" ::"v"(dep.v[0]), "v"(dep.v[8]) : "memory");
      stamp[k] = __builtin_amdgcn_s_memrealtime();
    }
  };
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long b0 = wave * 64 * PER + __lane_id();
  if (wave * 64 * PER >= n) return;  // wave-uniform
  // (ndev: n is an upper bound -- the planes' stride -- and the item count is
  // on the device; items past it in a live wave are garbage, harmless to
  // Montgomery's trick, and never read)
  if (ndev && wave * 64 * PER >= (long)*ndev) return;
  fe acc;
  fe_set(acc, kRN);  // Montgomery one
  mark(0, acc);
  ninv_chain_up<PER, 64>(s, n, b0, winv, acc);
  mark(1, acc);
  fe sib[6];
#pragma unroll
  for (int j = 0; j < 6; j++) {
#pragma unroll
    for (int k = 0; k < NL; k++) sib[j].v[k] = __shfl_xor(acc.v[k], 1 << j);
    fn_mul(acc, acc, sib[j]);
  }
  mark(2, acc);
  // the wave's product (the same on every lane) -> its inverse x^-1 R
  fe r = acc;
  fn_canon(r);
  uint32_t w[8], iw[8];
  fe_to_words(w, r);
  if (!modinv_n_var_wave(iw, w)) {
    // not reachable: every leaf is a value in [1, N)
#pragma unroll
    for (int k = 0; k < 8; k++) iw[k] = 0;
  }
  fe_from_words(r, iw);
  fn_to_mont(r, r);
  mark(3, r);
#pragma unroll
  for (int j = 5; j >= 0; j--) fn_mul(r, r, sib[j]);  // inverse of this lane's block at level j
  mark(4, r);
  ninv_chain_down<PER, 64>(s, n, b0, winv, r);
  mark(5, r);
  if (PROBE && __lane_id() == 0)
    for (int k = 0; k < 6; k++) probe[6 * wave + k] = stamp[k];
}

// The same one-launch s^-1 with ONE inversion per WORKGROUP (256 threads x
// PER items) instead of per wave: the 256 chain products meet in
// k_ninv_top's LDS product tree (lds_tree_invert: 8 levels up, the root
// inverted by wave 0, 8 levels down; a wave butterfly + 4-leaf tree instead
// had to hold 6 sibling products across the inversion and spilled: slower,
// tools/ubench_ninv.hip).  The chains issue their loads all at
// once (ninv_block_chains), so a launch waits on memory twice, not once per
// chain step -- the per-wave form's chains (k_ninv_local) stall on a load at
// every step and took ~2/3 of its launch.  PER = 8 (249 VGPRs, no spills):
// one inversion per 2,048 items, 2 blocks per CU, all resident at once for a
// 1M batch.  Block 0 zeroes the verify's queue counter.
// (The steps are expanded over an index sequence, so every array index is a
// compile-time constant and the arrays live in registers: a `#pragma unroll`
// loop left them in scratch.)  Prefixes go to the w planes on the way up (as
// in ninv_chain_up) and come back all at once, with the raw values, before the
// way down: two memory waits per launch instead of one per step.
template <int PER, bool PROBE, size_t... K>
MBFT_DEV void ninv_block_chains(const uint8_t* s, long n, long b0, uint32_t* winv,
                                uint32_t (&node)[NL][2 * kTopThreads], int t, uint64_t* probe,
                                std::index_sequence<K...>) {
  uint64_t stamp[5];
  auto mark = [&](int k, const fe& dep) {
    if (PROBE) {
      asm volatile("s_nop 0" ::"v"(dep.v[0]), "v"(dep.v[8]) : "memory");
      stamp[k] = __builtin_amdgcn_s_memrealtime();
    }
  };
  fe acc;
  fe_set(acc, kRN);
  mark(0, acc);
  {
    uint32_t raw[PER][8];
    (ninv_load_raw<256>(s, n, b0, (int)K, raw[K]), ...);  // every load in flight at once
    auto up = [&](auto kc) {
      constexpr int k = decltype(kc)::value;
      const long i = b0 + 256L * k;
      if (i < n) plane_store(winv, n, i, acc);  // the product of the items before k
      fe v;
      ninv_to_plain<256>(n, b0, k, raw[k], v);
      fn_mul(acc, acc, v);
    };
    (up(std::integral_constant<int, (int)K>{}), ...);
  }
  mark(1, acc);
#pragma unroll
  for (int j = 0; j < NL; j++) node[j][kTopThreads + t] = acc.v[j];
  lds_tree_invert(node, t);
  fe r;
#pragma unroll
  for (int j = 0; j < NL; j++) r.v[j] = node[j][kTopThreads + t];
  mark(2, r);
  uint32_t raw[PER][8];
  fe pre[PER];
  auto fetch = [&](auto kc) {
    constexpr int k = decltype(kc)::value;
    const long i = b0 + 256L * k;
    if (i < n) plane_load(pre[k], winv, n, i);
    if (k > 0) ninv_load_raw<256>(s, n, b0, k, raw[k]);
  };
  (fetch(std::integral_constant<int, (int)K>{}), ...);
  mark(3, pre[PER - 1]);
  auto down = [&](auto kc) {
    constexpr int k = PER - 1 - decltype(kc)::value;
    fe o;
    fn_mul(o, pre[k], r);  // s_k^-1 R
    if (k > 0) {
      fe v;
      ninv_to_plain<256>(n, b0, k, raw[k], v);
      fn_mul(r, r, v);  // (the product of the items before k)^-1 R
    }
    const long i = b0 + 256L * k;
    if (i < n) plane_store(winv, n, i, o);
  };
  (down(std::integral_constant<int, (int)K>{}), ...);
  mark(4, r);
  if (PROBE && t == 0)
    for (int k = 0; k < 5; k++) probe[5 * blockIdx.x + k] = stamp[k];
}

// PROBE (tools/ubench_ninv.hip only): thread 0 of each block writes
// s_memrealtime stamps after each phase to probe[5 block ..].
template <int PER, bool PROBE = false>
__global__ void __launch_bounds__(256, (PER >= 16 ? 1 : 16 / PER))
    k_ninv_block(const uint8_t* __restrict__ s, long n, uint32_t* __restrict__ winv,
                 uint32_t* __restrict__ zero_word, uint64_t* __restrict__ probe = nullptr) {
  __shared__ uint32_t node[NL][2 * kTopThreads];  // node i (1 = root, leaves 256..511), SoA
  if (zero_word && blockIdx.x == 0 && threadIdx.x == 0) *zero_word = 0;
  const int t = threadIdx.x;
  const long b0 = (long)blockIdx.x * 256 * PER + t;  // the grid covers n: every block has items
  ninv_block_chains<PER, PROBE>(s, n, b0, winv, node, t, probe, std::make_index_sequence<PER>{});
}

// Level-l down-sweep.  in: x[n] (or s bytes at level 0, recomputed: one
// multiply instead of storing and re-reading 36 B per item), pre[n],
// inv_tot[G]; out: inv[n] = x_i^-1, written straight into its final buffer.
// zero_word (level 0, optional): zeroed by block 0 -- the exact-path queue
// counter of the verify that waits for this chain (no memset launch on the
// verify's stream, where it would queue behind other batches' kernels).
template <bool FROM_S>
__global__ void k_ninv_down(const uint32_t* __restrict__ x, const uint8_t* __restrict__ s,
                            const uint32_t* __restrict__ pre, long n, long G,
                            const uint32_t* __restrict__ inv_tot, uint32_t* __restrict__ inv,
                            uint32_t* __restrict__ zero_word) {
  MBFT_CHAIN_PRIO();
  if (zero_word && blockIdx.x == 0 && threadIdx.x == 0) *zero_word = 0;
  const long g = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G || g >= n) return;
  fe r;
  plane_load(r, inv_tot, G, g);  // (prod of chain)^-1
  const long last = g + ((n - 1 - g) / G) * G;
#pragma unroll 1
  for (long i = last; i >= g; i -= G) {
    fe p, v, t;
    plane_load(p, pre, n, i);
    if (FROM_S)
      s_plain(v, s, i);
    else
      plane_load(v, x, n, i);
    fn_mul(t, r, p);   // x_i^-1 = (prefix_i) * (prod through i)^-1
    fn_mul(r, r, v);   // (prod through i-1)^-1
    plane_store(inv, n, i, t);
  }
}

// ---------------------------------------------------------------------------
// The verifier.
struct VerifyArgs {
  const uint8_t* e;        // n x 32 B big-endian digest integer (hashToInt)
  const uint8_t* r;        // n x 32 B big-endian
  const uint8_t* s;        // n x 32 B big-endian
  const uint32_t* slot;    // n key slots
  const uint32_t* winv;    // optional: s^-1 * R mod N, 9 planes of n (or null)
  const uint32_t* tabG;    // generator comb table (window wg)
  const KeyDesc* keys;     // nslots key descriptors (comb table, window, valid)
  uint32_t nslots;
  int wg;
  long n;
  uint8_t* status;
  uint32_t* slowq;         // exact-path queue: item indices (n entries)
  uint32_t* slown;         // its length (zeroed before k_verify)
  uint32_t host_status;    // slots >= kHostSlot carry the host's status (batch pipeline)
  uint32_t* scr;           // per-thread spill of the rare comb steps: 36 planes of sstride words
  uint32_t sstride;        // = threads in the grid
  const uint32_t* ndev;    // optional (small-batch kernels): the item count on the device, <= n
  const uint32_t* uhost = nullptr;  // optional (k_verify_split): u1, u2 per item, 16 LE words (host)
};

constexpr uint8_t ST_ACCEPT = 0, ST_REJECT = 1, ST_BAD_KEY = 5;

// Shift an 8-word scalar right by W bits (0 < W < 32).
MBFT_DEV void shr_words(uint32_t (&U)[8], int W) {
#pragma unroll
  for (int j = 0; j < 7; j++) U[j] = __builtin_amdgcn_alignbit(U[j + 1], U[j], W);
  U[7] >>= W;
}

MBFT_DEV const uint4* comb_entry(const uint32_t* tab, int W, int step, uint32_t idx) {
  return reinterpret_cast<const uint4*>(tab + ((((size_t)step) << (W - 1)) + idx) * 16u);
}

// Signed recoding of the current window (layout above, k_table_fill): `u` =
// the scalar's low word after the previous shifts, `carry` in/out.  Returns
// the table index of |d| (0 for d == 0, an entry that exists; `zero` flags
// the digit), `neg` = d < 0.
MBFT_DEV uint32_t comb_digit(uint32_t u, uint32_t& carry, int W, bool top, bool& neg,
                             bool& zero) {
  const uint32_t x = (u & ((1u << W) - 1u)) + carry;
  neg = !top && x > (1u << (W - 1));
  carry = neg ? 1u : 0u;
  const uint32_t mag = neg ? (1u << W) - x : x;
  zero = mag == 0u;
  return zero ? 0u : mag - 1u;
}

// y -> -y (p - y) where `neg`; y canonical < p
MBFT_DEV void fe_cneg(fe& y, bool neg) {
  fe t;
  fe_neg(t, y);
  fe_select(y, neg, t, y);
}

// acc += sum_i d_i * T[i][d_i] over the S = ceil(256/W) windows of scalar U
// (low window first): unchecked mixed additions, next entry prefetched one
// step ahead.  A degenerate addition (acc == +-entry) leaves Z == 0 for good,
// which the caller detects.  W is a runtime value (per table): the digit
// arithmetic is a handful of scalar-shift ops against ~1,800 VALU ops of the
// mixed addition, so one kernel serves every window size.
MBFT_DEV void comb_fast(jac& acc, bool& inf, uint32_t (&U)[8], const uint32_t* tab, int W) {
  const int S = (256 + W - 1) / W;
  uint32_t carry = 0;
  bool neg, zero;
  uint32_t idx = comb_digit(U[0], carry, W, S == 1, neg, zero);
  const uint4* p = comb_entry(tab, W, 0, idx);
  uint4 c0 = p[0], c1 = p[1], c2 = p[2], c3 = p[3];
#pragma unroll 1
  for (int step = 0; step < S; step++) {
    shr_words(U, W);
    bool nneg, nzero;
    const uint32_t in = comb_digit(U[0], carry, W, step + 2 >= S, nneg, nzero);
    const uint4* pn = comb_entry(tab, W, step + 1 < S ? step + 1 : step, in);
    const uint4 n0 = pn[0], n1 = pn[1], n2 = pn[2], n3 = pn[3];
    fe px, py;
    {
      uint32_t wx[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
      uint32_t wy[8] = {c2.x, c2.y, c2.z, c2.w, c3.x, c3.y, c3.z, c3.w};
      fe_from_words(px, wx);
      fe_from_words(py, wy);
    }
    fe_cneg(py, neg);
    // Branches, not selects: a zero digit has probability 2^-(W-1) and `inf`
    // is wave-uniform after the first nonzero digit, so the common path is
    // the in-place mixed addition with no extra live registers.
    if (!zero) {
      if (inf) {
        acc.X = px;
        acc.Y = py;
        fe_one_mont(acc.Z);
        inf = false;
      } else {
        ec_madd(acc, acc, px, py);
      }
    }
    neg = nneg;
    zero = nzero;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
  }
}

// Table gathers of the verifier fast path go straight into LDS (gfx950
// global_load_lds_dwordx4: lane l's 16 B land at base + 16 l), so the entry
// prefetched one step ahead holds no VGPRs across the mixed addition; the
// lane reads its 64 B back when the step starts.  Per wave a 4 KB buffer:
// 4 slots of 64 x 16 B.
//
// COOP (cooperative gather): every step each lane needs one random 64-B
// entry.  Loaded lane by lane, each of the 4 load instructions touches 64
// unrelated table pages: 256 address translations and cache-line requests
// per wave per step, which at 258 GiB of tables miss the per-CU TLB 86 % of
// the time (PMC TCP_UTCL1_TRANSLATION_MISS).  Cooperatively,
// load k fetches 16-B chunk (lane & 3) of the entries of lanes 16k .. 16k+15
// (their addresses come in by ds_bpermute): 16 entries per instruction, 64
// translations and requests per step.  Needs all 64 lanes of the wave in
// the loop with valid addresses (verify_one).  Without COOP, load k fetches
// chunk k of the lane's own entry.
#ifndef MBFT_GATHER_CPOL
#define MBFT_GATHER_CPOL 2  // table gathers non-temporal (nt): +1 % same-box, A/B builds
#endif
constexpr unsigned kWaitVm0 = 0x0F70;    // s_waitcnt vmcnt(0)
constexpr unsigned kWaitLgkm0 = 0xC07F;  // s_waitcnt lgkmcnt(0)

template <bool COOP>
MBFT_DEV void gather_issue(const uint4* mine, uint4* buf) {
  const int lane = __lane_id();
  __builtin_amdgcn_s_waitcnt(kWaitLgkm0);  // the previous reads of buf are done
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint4* src;
    if (COOP) {
      const uint64_t a = reinterpret_cast<uint64_t>(mine);
      const int from = (16 * k + (lane >> 2)) << 2;
      const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(from, (int)(uint32_t)a);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(from, (int)(uint32_t)(a >> 32));
      src = reinterpret_cast<const uint4*>(((uint64_t)hi << 32) | lo) + (lane & 3);
    } else {
      src = mine + k;
    }
    __builtin_amdgcn_global_load_lds(src, buf + 64 * k, 16, 0, MBFT_GATHER_CPOL);
  }
}

// This lane's entry from the buffer (waits for the gathers).  COOP: slot
// 64k + l holds chunk (l & 3) of the entry of lane 16k + (l >> 2), so the
// lane's 4 chunks are slots 4 lane .. 4 lane + 3.
template <bool COOP>
MBFT_DEV void gather_read(fe& px, fe& py, const uint4* buf) {
  const int lane = __lane_id();
  __builtin_amdgcn_s_waitcnt(kWaitVm0);
  uint4 c[4];
#pragma unroll
  for (int k = 0; k < 4; k++) c[k] = COOP ? buf[4 * lane + k] : buf[64 * k + lane];
  uint32_t wx[8] = {c[0].x, c[0].y, c[0].z, c[0].w, c[1].x, c[1].y, c[1].z, c[1].w};
  uint32_t wy[8] = {c[2].x, c[2].y, c[2].z, c[2].w, c[3].x, c[3].y, c[3].z, c[3].w};
  fe_from_words(px, wx);
  fe_from_words(py, wy);
}

#ifdef MBFT_STEP_TIMING
// Comb-step stamps (timing builds only: tools/step_timing.py, built with
// -DMBFT_STEP_TIMING): per wave, shader-clock cycles (s_memtime) summed over
// its cooperative comb steps in k_verify: [0] waiting for the entry
// prefetched one step earlier (vmcnt), [1] reading it from LDS, [2] issuing
// the next gather (address exchange by ds_bpermute, 4 LDS-DMA loads), [3]
// the mixed addition (its VALU issue, dependency stalls, and the cycles the
// SIMD gives the other waves); [4] steps, [5] waves; [6] / [7] the comb's
// span in shader cycles / in 100 MHz wall-clock ticks (their ratio: the
// in-kernel clock), [8] the whole verify_one in shader cycles, [9] its part
// before the comb.  The stamps themselves cost cycles (each waits for the
// LDS / SMEM queue); compare the timing build's step with the normal one.
__device__ unsigned long long g_step_clk[12];
struct StepClock {
  unsigned long long s[4] = {0, 0, 0, 0};
  unsigned long long steps = 0;
};
extern "C" int mbft_debug_step_timing(unsigned long long out[12], int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_step_clk), sizeof(g_step_clk)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_step_clk), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#else
struct StepClock {};
#endif

// Rare comb steps (a zero digit, or an accumulator still at infinity) are
// resolved around the unconditional in-place mixed addition without holding
// any extra registers across it: before it, a zero-digit lane spills its
// accumulator and an infinity lane its entry to per-thread scratch
// (coalesced planes, A.scr); after it, the zero-digit lane reloads the
// accumulator (the addition is skipped, its Y sign unflipped) and the
// infinity lane becomes the entry (Z = 1).  Both are wave-uniform branches
// that honest inputs take with probability ~2^-(W-1) per window.
// Addresses are 32-bit word offsets from the (uniform) scratch base, made
// opaque where they are used: otherwise the compiler hoists the 36 per-lane
// 64-bit addresses out of the comb loop and spills them.
struct Spill {
  uint32_t* base;   // A.scr (wave-uniform)
  uint32_t tid;     // this thread's column
  uint32_t stride;  // words per plane
  MBFT_DEV void put(int k, const fe& a) const {
    uint32_t t = tid;
    asm volatile("" : "+v"(t));
#pragma unroll
    for (int j = 0; j < NL; j++) base[t + (uint32_t)(k * NL + j) * stride] = a.v[j];
  }
  MBFT_DEV void get(int k, fe& a) const {
    uint32_t t = tid;
    asm volatile("" : "+v"(t));
#pragma unroll
    for (int j = 0; j < NL; j++) a.v[j] = base[t + (uint32_t)(k * NL + j) * stride];
  }
};

// One comb step (the body of comb_run's loop, below; LAST: the peeled final
// step of a LAST_XZ run, whose addition skips ZZZ and Y).
template <bool COOP, bool LAST>
MBFT_DEV void comb_step(chud& acc, bool& inf, bool& yneg, bool& neg, bool& zero, uint32_t (&U)[8],
                        const uint32_t* tab, int W, int S, int step, uint32_t& carry, uint4* buf,
                        const Spill& sp, bool live, StepClock& sc) {
  fe px, py;
#ifdef MBFT_STEP_TIMING
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_s_waitcnt(kWaitVm0);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
#endif
  gather_read<COOP>(px, py, buf);
#ifdef MBFT_STEP_TIMING
  __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
  const unsigned long long t2 = __builtin_amdgcn_s_memtime();
#endif
  shr_words(U, W);
  bool nneg, nzero;
  const uint32_t in = comb_digit(U[0], carry, W, step + 2 >= S, nneg, nzero);
  gather_issue<COOP>(comb_entry(tab, W, step + 1 < S ? step + 1 : step, in), buf);
#ifdef MBFT_STEP_TIMING
  const unsigned long long t3 = __builtin_amdgcn_s_memtime();
#endif
  // dead lanes (zero scalars, results discarded) never count as rare
  const bool rare = __ballot(live && (zero || inf)) != 0;
  if (rare && live) {
    if (zero) {
      sp.put(0, acc.X);
      sp.put(1, acc.Y);
      sp.put(2, acc.ZZ);
      sp.put(3, acc.ZZZ);
    } else if (inf) {
      sp.put(0, px);
      sp.put(1, py);
    }
  }
  ec_madd_chud<true, LAST>(acc, acc, px, py, yneg != neg);  // Y takes the digit's sign (ecc.h)
  const bool yold = yneg;
  yneg = neg;
  if (rare && live) {
    if (zero) {  // d = 0: nothing added
      sp.get(0, acc.X);
      sp.get(1, acc.Y);
      sp.get(2, acc.ZZ);
      sp.get(3, acc.ZZZ);
      yneg = yold;
    } else if (inf) {  // infinity + entry = entry (Z = 1); acc.Y holds t y2
      sp.get(0, acc.X);
      sp.get(1, acc.Y);
      fe_one_mont(acc.ZZ);
      fe_one_mont(acc.ZZZ);
      yneg = neg;
      inf = false;
    }
  }
  neg = nneg;
  zero = nzero;
#ifdef MBFT_STEP_TIMING
  const unsigned long long t4 = __builtin_amdgcn_s_memtime();
  sc.s[0] += t1 - t0;
  sc.s[1] += t2 - t1;
  sc.s[2] += t3 - t2;
  sc.s[3] += t4 - t3;
  sc.steps += 1;
#else
  (void)sc;
#endif
}

// Verifier fast path: acc (a Chudnovsky point, or `inf`) += the signed-digit
// entries of windows step0 .. S-1 of U (`carry` = the recoding carry into
// window step0).  Every step is the in-place mixed addition, so the common
// loop carries no control-flow merge and no register copies; the next entry
// is in flight one step ahead.  Zero digits and infinity are exact (the rare
// branches above: an attacker who picks s controls u1 or u2 and can force
// them, so they are not sent to the slow path).  `yneg`: acc.Y holds -Y
// (ec_madd_chud: after an addition, the sign of the digit it added); a
// negative digit's -y is folded into the same per-lane select.  A degenerate
// addition (acc == +-entry) leaves ZZ == 0 for good, which the caller
// detects.  COOP: cooperative gathers (W and the loop wave-uniform); else
// per lane.  acc.ZZ and acc.ZZZ are kept lazy (ecc.h ec_madd_chud<true>):
// the caller normalizes them (fe_norm_lazy) before any other use.  LAST_XZ
// (with COOP: S is wave-uniform): this run ends the
// chain and only X, ZZ are read afterwards (the x-check): the final step is
// peeled and its addition skips ZZZ and Y.
// (end_ >= 0: stop before window end_ -- a range's low part, k_verify_quads;
// the entry gathered ahead for window end_ goes unused)
template <bool COOP, bool LAST_XZ = false>
MBFT_DEV void comb_run(chud& acc, bool& inf, bool& yneg, uint32_t (&U)[8], const uint32_t* tab,
                       int W, int step0, uint32_t carry, uint4* buf, const Spill& sp, bool live,
                       StepClock& sc, int end_ = -1) {
  static_assert(COOP || !LAST_XZ, "the peeled last step needs a wave-uniform window");
  const int S = (256 + W - 1) / W;
  bool neg, zero;
  const uint32_t idx = comb_digit(U[0], carry, W, step0 + 1 >= S, neg, zero);
  gather_issue<COOP>(comb_entry(tab, W, step0, idx), buf);
  const int end = end_ >= 0 ? end_ : (LAST_XZ ? S - 1 : S);
#pragma unroll 1
  for (int step = step0; step < end; step++)
    comb_step<COOP, false>(acc, inf, yneg, neg, zero, U, tab, W, S, step, carry, buf, sp, live, sc);
  if (LAST_XZ && S - 1 >= step0)
    comb_step<COOP, true>(acc, inf, yneg, neg, zero, U, tab, W, S, S - 1, carry, buf, sp, live, sc);
  __builtin_amdgcn_s_waitcnt(kWaitVm0);  // the last (unused) gather is done with buf
}

// acc = u1 G + u2 Q over the comb tables, fast path: the first two G windows
// are one affine + affine addition, all later windows are mixed additions.
// Returns true if the sum is the point at infinity (Go's Verify: (0, 0),
// reject).  A degenerate addition (only constructible with the key's
// discrete log) leaves ZZ == 0: the caller sends that lane to the exact path.
// The G phase (one table, one window) always gathers cooperatively; the Q
// phase when QCOOP (the wave's key windows agree).
template <bool QCOOP>
MBFT_DEV bool comb_verify_fast(chud& acc, uint32_t (&U1)[8], uint32_t (&U2)[8],
                               const uint32_t* tabG, int wg, const uint32_t* tabQ, int wq,
                               uint4* buf, const Spill& sp, bool live, StepClock& sc) {
  uint32_t carry = 0;
  bool neg0, zero0, neg1, zero1;
  const uint32_t i0 = comb_digit(U1[0], carry, wg, false, neg0, zero0);
  shr_words(U1, wg);
  const uint32_t i1 = comb_digit(U1[0], carry, wg, false, neg1, zero1);
  shr_words(U1, wg);
  {
    // the first two G windows: affine + affine.  acc.Y holds +-Y (only X and
    // Z are read afterwards): a negative first digit just starts the lane
    // with Y negated.
    fe x0, y0, x1, y1;
    gather_issue<true>(comb_entry(tabG, wg, 0, i0), buf);
    gather_read<true>(x0, y0, buf);
    gather_issue<true>(comb_entry(tabG, wg, 1, i1), buf);
    gather_read<true>(x1, y1, buf);
    ec_add_affine_chud(acc, x0, y0, x1, y1, neg0 != neg1);
  }
  bool yneg = !neg0, inf = false;
  if (__ballot(live && (zero0 || zero1)) != 0) {
    // a zero digit among the first two: the sum is the other entry (Z = 1,
    // reloaded per lane), or infinity if both are zero
    if (zero0 && zero1) {
      inf = true;
    } else if (zero0 || zero1) {
      load_point(acc.X, acc.Y, comb_entry(tabG, wg, zero0 ? 1 : 0, zero0 ? i1 : i0));
      fe_one_mont(acc.ZZ);
      fe_one_mont(acc.ZZZ);
      yneg = zero0 ? neg1 : neg0;
    }
  }
  // never degenerate in the G phase: |partial sum| < |next addend| as
  // integers, and partial + addend == u1 != 0 at the top
  comb_run<true>(acc, inf, yneg, U1, tabG, wg, 2, carry, buf, sp, live, sc);
  comb_run<QCOOP, QCOOP>(acc, inf, yneg, U2, tabQ, wq, 0, 0u, buf, sp, live, sc);
  fe_norm_lazy(acc.ZZ);
  return inf;
}

constexpr unsigned kWaitVm4 = 0x0F74;  // s_waitcnt vmcnt(4): all but the youngest gather (4 loads)

// This lane's entry from a cooperative gather slot whose LDS-DMA the caller
// has waited for.  The LDS reads are inline asm (with their own lgkmcnt(0)):
// the compiler tracks LDS-DMA writes by LDS object and, unable to tell two
// slots of one array apart, would turn the caller's vmcnt(4) into vmcnt(0),
// i.e. wait for the younger gather too.  The outputs are early-clobber: a
// destination sharing the address VGPR would let a fast first read land
// before a later read of the block has sent its address.
MBFT_DEV void slot_read(fe& px, fe& py, const uint4* buf) {
  const uint32_t a = (uint32_t)(uintptr_t)(buf + 4 * __lane_id());  // low half of a flat LDS address = the offset
  uint4 c0, c1, c2, c3;
  asm volatile(
      "ds_read_b128 %0, %4\n\t"
      "ds_read_b128 %1, %4 offset:16\n\t"
      "ds_read_b128 %2, %4 offset:32\n\t"
      "ds_read_b128 %3, %4 offset:48\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(c0), "=&v"(c1), "=&v"(c2), "=&v"(c3)
      : "v"(a)
      : "memory");
  uint32_t wx[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
  uint32_t wy[8] = {c2.x, c2.y, c2.z, c2.w, c3.x, c3.y, c3.z, c3.w};
  fe_from_words(px, wx);
  fe_from_words(py, wy);
}

// The issue side of comb_verify_fast2: the stream of entries after the first
// two G windows -- G windows gk .. SG-1, then Q windows qk .. SQ-1 -- with
// each scalar's recoding carry; next() gathers the next entry into `buf`
// (its digit's sign and zero flag out).
struct CombStream {
  const uint32_t* tabG;
  const uint32_t* tabQ;
  int wg, wq, SG, SQ, gk, qk;
  uint32_t carry, qcarry;
};

MBFT_DEV void comb_stream_next(CombStream& cs, uint32_t (&U1)[8], uint32_t (&U2)[8], uint4* buf, bool& n,
                               bool& z) {
  const uint4* e;
  if (cs.gk < cs.SG) {  // wave-uniform
    const uint32_t idx = comb_digit(U1[0], cs.carry, cs.wg, cs.gk + 1 >= cs.SG, n, z);
    e = comb_entry(cs.tabG, cs.wg, cs.gk, idx);
    shr_words(U1, cs.wg);
    cs.gk++;
  } else {
    const uint32_t idx = comb_digit(U2[0], cs.qcarry, cs.wq, cs.qk + 1 >= cs.SQ, n, z);
    e = comb_entry(cs.tabQ, cs.wq, cs.qk, idx);
    shr_words(U2, cs.wq);
    cs.qk++;
  }
  gather_issue<true>(e, buf);
}

// One step of comb_verify_fast2: the entry of step k (slot A for even k, its
// digit flags na / za, else B), the slot refilled at once with step k + 2,
// then the mixed addition with comb_step's rare branches.  T: the steps.
template <bool LAST>
MBFT_DEV void comb_step2(chud& acc, bool& inf, bool& yneg, bool& na, bool& za, bool& nb, bool& zb,
                         uint32_t (&U1)[8], uint32_t (&U2)[8], CombStream& cs, int k, int T, uint4* bufA,
                         uint4* bufB, const Spill& sp, bool live, StepClock& sc) {
  const bool odd = (k & 1) != 0;
  uint4* buf = odd ? bufB : bufA;
  fe px, py;
#ifdef MBFT_STEP_TIMING
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
  if (k + 1 < T)  // wave-uniform: the other slot's gather stays in flight
    __builtin_amdgcn_s_waitcnt(kWaitVm4);
  else
    __builtin_amdgcn_s_waitcnt(kWaitVm0);
#ifdef MBFT_STEP_TIMING
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
#endif
  slot_read(px, py, buf);
#ifdef MBFT_STEP_TIMING
  const unsigned long long t2 = __builtin_amdgcn_s_memtime();
#endif
  const bool neg = odd ? nb : na, zero = odd ? zb : za;
  if (k + 2 < T) {
    bool n2, z2;
    comb_stream_next(cs, U1, U2, buf, n2, z2);
    if (odd) {
      nb = n2;
      zb = z2;
    } else {
      na = n2;
      za = z2;
    }
  }
#ifdef MBFT_STEP_TIMING
  const unsigned long long t3 = __builtin_amdgcn_s_memtime();
#endif
  // dead lanes (zero scalars, results discarded) never count as rare
  const bool rare = __ballot(live && (zero || inf)) != 0;
  if (rare && live) {
    if (zero) {
      sp.put(0, acc.X);
      sp.put(1, acc.Y);
      sp.put(2, acc.ZZ);
      sp.put(3, acc.ZZZ);
    } else if (inf) {
      sp.put(0, px);
      sp.put(1, py);
    }
  }
  ec_madd_chud<true, LAST>(acc, acc, px, py, yneg != neg);  // Y takes the digit's sign (ecc.h)
  const bool yold = yneg;
  yneg = neg;
  if (rare && live) {
    if (zero) {  // d = 0: nothing added
      sp.get(0, acc.X);
      sp.get(1, acc.Y);
      sp.get(2, acc.ZZ);
      sp.get(3, acc.ZZZ);
      yneg = yold;
    } else if (inf) {  // infinity + entry = entry (Z = 1); acc.Y holds t y2
      sp.get(0, acc.X);
      sp.get(1, acc.Y);
      fe_one_mont(acc.ZZ);
      fe_one_mont(acc.ZZZ);
      yneg = neg;
      inf = false;
    }
  }
#ifdef MBFT_STEP_TIMING
  const unsigned long long t4 = __builtin_amdgcn_s_memtime();
  sc.s[0] += t1 - t0;
  sc.s[1] += t2 - t1;
  sc.s[2] += t3 - t2;
  sc.s[3] += t4 - t3;
  sc.steps += 1;
#else
  (void)sc;
#endif
}

// comb_verify_fast<true> with TWO gathers in flight (k_verify, every lane's
// key window the same): each wave has two LDS slots; the entry of step k is
// read from its slot (waiting only for that gather: vmcnt(4) leaves the
// younger one in flight), the slot is refilled at once with the entry of step
// k + 2, then the mixed addition runs -- a gather has two additions to land
// instead of one (at one wave per SIMD the one-step prefetch left 17 % of
// each step waiting for it, tools/step_timing.py).  The G windows 2 .. SG-1
// and the Q windows 0 .. SQ-1 are one stream of steps, so the first Q entries
// are in flight during the last G additions, and the first two G entries are
// fetched at once.  Same additions, same rare branches, same results as
// comb_verify_fast.
MBFT_DEV bool comb_verify_fast2(chud& acc, uint32_t (&U1)[8], uint32_t (&U2)[8], const uint32_t* tabG,
                                int wg, const uint32_t* tabQ, int wq, uint4* bufA, uint4* bufB,
                                const Spill& sp, bool live, StepClock& sc) {
  CombStream cs{tabG, tabQ, wg, wq, (256 + wg - 1) / wg, (256 + wq - 1) / wq, 2, 0, 0u, 0u};
  const int T = cs.SG - 2 + cs.SQ;  // mixed additions
  bool neg0, zero0, neg1, zero1;
  const uint32_t i0 = comb_digit(U1[0], cs.carry, wg, false, neg0, zero0);
  shr_words(U1, wg);
  const uint32_t i1 = comb_digit(U1[0], cs.carry, wg, false, neg1, zero1);
  shr_words(U1, wg);
  gather_issue<true>(comb_entry(tabG, wg, 0, i0), bufA);
  gather_issue<true>(comb_entry(tabG, wg, 1, i1), bufB);
  bool na, za, nb, zb;  // the digit flags of the entries in slots A and B
  {
    // the first two G windows: affine + affine.  acc.Y holds +-Y (only X and
    // Z are read afterwards): a negative first digit just starts the lane
    // with Y negated.
    fe x0, y0, x1, y1;
    __builtin_amdgcn_s_waitcnt(kWaitVm4);
    slot_read(x0, y0, bufA);
    comb_stream_next(cs, U1, U2, bufA, na, za);
    __builtin_amdgcn_s_waitcnt(kWaitVm4);
    slot_read(x1, y1, bufB);
    comb_stream_next(cs, U1, U2, bufB, nb, zb);
    ec_add_affine_chud(acc, x0, y0, x1, y1, neg0 != neg1);
  }
  bool yneg = !neg0, inf = false;
  if (__ballot(live && (zero0 || zero1)) != 0) {
    // a zero digit among the first two: the sum is the other entry (Z = 1,
    // reloaded per lane), or infinity if both are zero
    if (zero0 && zero1) {
      inf = true;
    } else if (zero0 || zero1) {
      load_point(acc.X, acc.Y, comb_entry(tabG, wg, zero0 ? 1 : 0, zero0 ? i1 : i0));
      fe_one_mont(acc.ZZ);
      fe_one_mont(acc.ZZZ);
      yneg = zero0 ? neg1 : neg0;
    }
  }
#pragma unroll 1
  for (int k = 0; k < T - 1; k++)
    comb_step2<false>(acc, inf, yneg, na, za, nb, zb, U1, U2, cs, k, T, bufA, bufB, sp, live, sc);
  // the chain's last addition: X and ZZ only (the x-check)
  comb_step2<true>(acc, inf, yneg, na, za, nb, zb, U1, U2, cs, T - 1, T, bufA, bufB, sp, live, sc);
  fe_norm_lazy(acc.ZZ);
  return inf;
}

// Same sum with exact handling of doubling / opposite points / infinity.
MBFT_DEV void comb_complete(jac& acc, bool& inf, uint32_t (&U)[8], const uint32_t* tab, int W) {
  const int S = (256 + W - 1) / W;
  uint32_t carry = 0;
#pragma unroll 1
  for (int step = 0; step < S; step++) {
    bool neg, zero;
    const uint32_t idx = comb_digit(U[0], carry, W, step + 1 >= S, neg, zero);
    shr_words(U, W);
    if (zero) continue;
    fe px, py;
    load_point(px, py, comb_entry(tab, W, step, idx));
    fe_cneg(py, neg);
    ec_madd_complete(acc, inf, px, py);
  }
}

// u1 = e w, u2 = r w (mod N, canonical) as little-endian words.  One
// conditional subtraction makes them canonical: e, r < 2^256 and every w the
// s^-1 kernels produce is < 2^258 (an fn_mul output: < a b / R + N), so
// fn_mul's output is < 2^256 2^258 / 2^261 + N < 2N.
MBFT_DEV void scalars(uint32_t (&U1)[8], uint32_t (&U2)[8], const fe& e, const fe& r,
                      const fe& w) {
  fe u;
  fn_mul(u, e, w);
  fn_csub(u, 1);
  fe_to_words(U1, u);
  fn_mul(u, r, w);
  fn_csub(u, 1);
  fe_to_words(U2, u);
}

// Load e, r, s^-1 of item i and compute u1, u2 words.  LANE_INV: s^-1 by
// this lane (small batches, k_verify_pairs, A.winv null); else from the
// batched planes.  A template, so the large-batch kernel carries no
// inversion code (it would cost registers there).
template <bool LANE_INV>
MBFT_DEV void load_scalars(const VerifyArgs& A, long i, uint32_t (&U1)[8], uint32_t (&U2)[8],
                          const fe* wpre = nullptr) {
  uint32_t ew[8], rw[8];
  load_be256(ew, A.e + 32 * i);
  load_be256(rw, A.r + 32 * i);
  fe w, e, r;
  if (!LANE_INV) {
    plane_load(w, A.winv, A.n, i);
  } else if (wpre) {
    w = *wpre;  // inverted by the whole wave (verify_pair: one item in the wave)
  } else {
    // small batches (verify_device): this lane's own s^-1 by variable-time
    // divsteps (modinv.h; s is public and in [1, N) for a live lane), VALU
    // code (per-lane data), ~38 us for a wave -- instead of the batched
    // chain's five launches and ~100 us of dependent latency
    uint32_t sw[8], iw[8];
    load_be256(sw, A.s + 32 * i);
    if (!modinv_n_var(iw, sw)) {
#pragma unroll
      for (int k = 0; k < 8; k++) iw[k] = 0;  // not reachable: 0 < s < N
    }
    fe_from_words(w, iw);
    fn_to_mont(w, w);  // s^-1 R
  }
  fe_from_words(e, ew);
  fe_from_words(r, rw);
  scalars(U1, U2, e, r, w);
}

// x(R) mod N == r  <=>  X == r Z^2  or (r + N < p and X == (r + N) Z^2).
// With ZZ = Z^2 R and X = x R (Montgomery), one merged product gives
// (r ZZ + X (p - 1)) / R == r Z^2 - x (mod p): zero iff accepted.
MBFT_DEV void verify_finish(const VerifyArgs& A, long i, const fe& X, const fe& ZZ,
                           const uint32_t* rw_in = nullptr) {
  uint32_t rw[8];
  fe r, pm1, d;
  if (rw_in) {
#pragma unroll
    for (int k = 0; k < 8; k++) rw[k] = rw_in[k];
  } else {
    load_be256(rw, A.r + 32 * i);
  }
  fe_from_words(r, rw);
  fe_set(pm1, kPm1);
  fe_mul2(d, r, ZZ, X, pm1);
  fe_canon(d);
  bool ok = fe_is_zero_canon(d);
  if (!ok && words_lt(rw, kPmNw)) {
    fe nn;
    fe_set(nn, kN);
    fe_add(r, r, nn);
    fe_mul2(d, r, ZZ, X, pm1);
    fe_canon(d);
    ok = fe_is_zero_canon(d);
  }
  A.status[i] = ok ? ST_ACCEPT : ST_REJECT;
}

// The exact path for item i: both phases recomputed with complete additions
// (doubling, infinity).  A final infinity rejects, as Go's (0, 0) does.
MBFT_DEV void verify_exact(const VerifyArgs& A, long i) {
  KeyDesc kd = A.keys[A.slot[i]];
  uint32_t U1[8], U2[8];
  if (A.winv)
    load_scalars<false>(A, i, U1, U2);
  else
    load_scalars<true>(A, i, U1, U2);
  bool inf = true;
  jac j;
  comb_complete(j, inf, U1, A.tabG, A.wg);
  comb_complete(j, inf, U2, kd.tab, (int)kd.wbits);
  if (inf) {
    A.status[i] = ST_REJECT;  // (x, y) = (0, 0) -> false
    return;
  }
  fe ZZ;
  fe_sqr(ZZ, j.Z);
  verify_finish(A, i, j.X, ZZ);
}

// One item per thread.  Every lane of the wave runs the comb loop (the
// cooperative gather needs all 64): lanes past the end of the batch, with an
// unknown / invalid key, or with r or s out of range are "dead" -- they run
// the loop on zero scalars over a valid table and write only their status.
MBFT_DEV void verify_one(const VerifyArgs& A, long i, bool in_batch, uint4* buf, uint4* buf2) {
#ifdef MBFT_STEP_TIMING
  const unsigned long long tv0 = __builtin_amdgcn_s_memtime();
#endif
  const long ii = in_batch ? i : 0;  // lanes past the end read item 0
  uint32_t rw[8], sw[8];
  load_be256(rw, A.r + 32 * ii);
  load_be256(sw, A.s + 32 * ii);
  const uint32_t slot = A.slot[ii];

  // crypto/ecdsa.Verify: r <= 0 || s <= 0 || r >= N || s >= N -> false
  const bool range_ok = !words_is_zero(rw) && words_lt(rw, kNw) &&
                        !words_is_zero(sw) && words_lt(sw, kNw);
  KeyDesc kd{A.tabG, (uint32_t)A.wg, 0u};
  if (slot < A.nslots) kd = A.keys[slot];
  const bool key_ok = slot < A.nslots && kd.valid;
  // slots >= kHostSlot carry a status the host decided (batch pipeline):
  // written as is, so the statuses the host reads back are final
  const uint8_t dead_status =
      key_ok ? ST_REJECT : (A.host_status && slot >= kHostSlot ? (uint8_t)slot : ST_BAD_KEY);
  const bool live = in_batch && key_ok && range_ok;

  // w = s^-1 (Montgomery form), u1 = e w, u2 = r w (plain, canonical < N).
  // e, r, w are not kept live across the comb (register pressure): the rare
  // slow path and the final check reload them.
  uint32_t U1[8], U2[8];
#pragma unroll
  for (int j = 0; j < 8; j++) U1[j] = U2[j] = 0u;
  if (live) load_scalars<false>(A, ii, U1, U2);
  const uint32_t* tq = kd.tab;
  int wq = (int)kd.wbits;

  // Dead lanes adopt the first live lane's key table; the Q phase gathers
  // cooperatively when every lane then has the same key window.
  const uint64_t lm = __ballot(live);
  if (lm == 0) {
    if (in_batch) A.status[i] = dead_status;
    return;
  }
  const int first = __ffsll((unsigned long long)lm) - 1;
  const uint64_t tq64 = reinterpret_cast<uint64_t>(tq);
  const uint32_t tlo = __builtin_amdgcn_readlane((uint32_t)tq64, first);
  const uint32_t thi = __builtin_amdgcn_readlane((uint32_t)(tq64 >> 32), first);
  const int wq_u = __builtin_amdgcn_readlane(wq, first);
  if (!live) {
    tq = reinterpret_cast<const uint32_t*>(((uint64_t)thi << 32) | tlo);
    wq = wq_u;
  }
  const bool quni = __ballot(wq != wq_u) == 0;

  chud acc;
  const Spill sp{A.scr, blockIdx.x * blockDim.x + threadIdx.x, A.sstride};
  StepClock sc;
#ifdef MBFT_STEP_TIMING
  const unsigned long long tc0 = __builtin_amdgcn_s_memtime(), rc0 = __builtin_amdgcn_s_memrealtime();
#endif
  // The two-step-ahead gathers (comb_verify_fast2) measured no faster than
  // the one-step prefetch (round 5, same box: isolated 1.072-1.094 against
  // 1.063-1.065 ms, C2 1,015 against 1,014-1,021 M/s): the wait they remove is
  // not what leaves the SIMD idle.  Kept for A/B builds.
  static constexpr bool kTwoDeep =
#ifdef MBFT_TWO_DEEP_GATHER
      true;
#else
      false;
#endif
  const bool inf = !quni    ? comb_verify_fast<false>(acc, U1, U2, A.tabG, A.wg, tq, wq, buf, sp, live, sc)
                   : kTwoDeep ? comb_verify_fast2(acc, U1, U2, A.tabG, A.wg, tq, wq, buf, buf2, sp, live, sc)
                              : comb_verify_fast<true>(acc, U1, U2, A.tabG, A.wg, tq, wq, buf, sp, live, sc);
#ifdef MBFT_STEP_TIMING
  const unsigned long long tc1 = __builtin_amdgcn_s_memtime(), rc1 = __builtin_amdgcn_s_memrealtime();
  if (__lane_id() == 0) {
    for (int k = 0; k < 4; k++) atomicAdd(&g_step_clk[k], sc.s[k]);
    atomicAdd(&g_step_clk[4], sc.steps);
    atomicAdd(&g_step_clk[5], 1ull);
    atomicAdd(&g_step_clk[6], tc1 - tc0);
    atomicAdd(&g_step_clk[7], rc1 - rc0);
    atomicAdd(&g_step_clk[9], tc0 - tv0);
  }
  struct End {
    unsigned long long t0;
    __device__ ~End() {
      if (__lane_id() == 0) atomicAdd(&g_step_clk[8], __builtin_amdgcn_s_memtime() - t0);
    }
  } end_stamp{tv0};
#endif
  if (!live) {
    if (in_batch) A.status[i] = dead_status;
    return;
  }
  if (inf) {
    A.status[i] = ST_REJECT;  // u1 G + u2 Q = infinity: (x, y) = (0, 0) -> false
    return;
  }

  fe zc = acc.ZZ;
  fe_canon(zc);
  if (fe_is_zero_canon(zc)) {
    // The exact path (a degenerate addition: acc == +-entry in the Q phase,
    // constructible only with the key's discrete log) is deferred to
    // k_verify_slow over a compacted queue, so that a crafted item costs its
    // own exact recomputation only -- not a stall of the 63 other lanes of
    // its wave.  One atomic per wave.
    const uint64_t qm = __ballot(true);
    const int nq = __popcll(qm);
    const int rank = __popcll(qm & ((1ull << __lane_id()) - 1ull));
    const int leader = __ffsll((unsigned long long)qm) - 1;
    uint32_t base = 0;
    if (__lane_id() == leader) base = atomicAdd(A.slown, (uint32_t)nq);
    base = __shfl(base, leader);
    A.slowq[base + rank] = (uint32_t)i;
    return;
  }
  verify_finish(A, i, acc.X, acc.ZZ);
}

// Small batches (verify_device, n <= MBFT_LANE_INV_MAX): one item per LANE
// PAIR.  The even lane sums the G windows, the odd lane the Q windows, at the
// same time (the same comb loop with per-lane table, window and first step;
// per-lane gathers, as the halves read different tables), and one x-only
// Chudnovsky addition joins them on the even lane: an item's latency is the
// longer half (9 of the 17 additions at W = 29) plus one addition, not the
// whole chain.  Each half is a single-scalar comb, never degenerate (the
// G-phase argument); a degenerate join (u1 G == +-u2 Q) goes to
// the exact path inline.  s^-1 per lane (divsteps), no queue.
template <bool LANE_INV>
MBFT_DEV void verify_pair(const VerifyArgs& A, long i, int half, bool in_batch, uint4* buf,
                          const Spill& sp) {
  const long ii = in_batch ? i : 0;
  uint32_t rw[8], sw[8];
  load_be256(rw, A.r + 32 * ii);
  load_be256(sw, A.s + 32 * ii);
  const uint32_t slot = A.slot[ii];
  const bool range_ok = !words_is_zero(rw) && words_lt(rw, kNw) &&
                        !words_is_zero(sw) && words_lt(sw, kNw);
  KeyDesc kd{A.tabG, (uint32_t)A.wg, 0u};
  if (slot < A.nslots) kd = A.keys[slot];
  const bool key_ok = slot < A.nslots && kd.valid;
  const uint8_t dead_status =
      key_ok ? ST_REJECT : (A.host_status && slot >= kHostSlot ? (uint8_t)slot : ST_BAD_KEY);
  const bool live = in_batch && key_ok && range_ok;
  uint32_t U1[8], U2[8];
#pragma unroll
  for (int j = 0; j < 8; j++) U1[j] = U2[j] = 0u;
  if (LANE_INV) {
    // A wave holding ONE live item (a single VerifyMessageAuthenTag call):
    // its s^-1 by all 64 lanes together (modinv_n_var_wave, ~24 us) instead
    // of the pair's own per-lane divsteps (~38 us).  Wave-uniform: live
    // lanes come in pairs, so <= 2 live lanes is one item.
    const uint64_t lm = __ballot(live);
    if (lm != 0 && __popcll(lm) <= 2) {
      const int leader = __ffsll((unsigned long long)lm) - 1;
      uint32_t xs[8], iw[8];
#pragma unroll
      for (int j = 0; j < 8; j++) xs[j] = (uint32_t)__builtin_amdgcn_readlane((int)sw[j], leader);
      if (!modinv_n_var_wave(iw, xs)) {
#pragma unroll
        for (int k = 0; k < 8; k++) iw[k] = 0;  // not reachable: 0 < s < N for a live item
      }
      fe wv;
      fe_from_words(wv, iw);
      fn_to_mont(wv, wv);  // s^-1 R
      if (live) load_scalars<LANE_INV>(A, ii, U1, U2, &wv);
    } else if (live) {
      load_scalars<LANE_INV>(A, ii, U1, U2);
    }
  } else if (live) {
    load_scalars<LANE_INV>(A, ii, U1, U2);
  }
  // this lane's half (dead lanes sum zero scalars over the generator table)
  const bool qh = half != 0;
  const uint32_t* tab = qh && live ? kd.tab : A.tabG;
  const int W = qh && live ? (int)kd.wbits : A.wg;
  uint32_t U[8];
#pragma unroll
  for (int j = 0; j < 8; j++) U[j] = qh ? U2[j] : U1[j];
  chud acc;
  fe_zero(acc.X);
  fe_zero(acc.Y);
  fe_one_mont(acc.ZZ);
  fe_one_mont(acc.ZZZ);
  bool inf = true, yneg = false;
  uint32_t carry = 0;
  int step0 = 0;
  if (!qh) {
    // the first two G windows: affine + affine (zero digits exact, as in
    // comb_verify_fast)
    bool neg0, zero0, neg1, zero1;
    const uint32_t i0 = comb_digit(U[0], carry, W, false, neg0, zero0);
    shr_words(U, W);
    const uint32_t i1 = comb_digit(U[0], carry, W, false, neg1, zero1);
    shr_words(U, W);
    fe x0, y0, x1, y1;
    load_point(x0, y0, comb_entry(tab, W, 0, i0));
    load_point(x1, y1, comb_entry(tab, W, 1, i1));
    ec_add_affine_chud(acc, x0, y0, x1, y1, neg0 != neg1);
    yneg = !neg0;
    inf = zero0 && zero1;
    if (zero0 != zero1) {
      acc.X = zero0 ? x1 : x0;
      acc.Y = zero0 ? y1 : y0;
      fe_one_mont(acc.ZZ);
      fe_one_mont(acc.ZZZ);
      yneg = zero0 ? neg1 : neg0;
    }
    step0 = 2;
  }
  StepClock sc;
  comb_run<false>(acc, inf, yneg, U, tab, W, step0, carry, buf, sp, live, sc);
  fe_norm_lazy(acc.ZZ);
  fe_norm_lazy(acc.ZZZ);
  // the odd lane's half to the even lane
  chud o;
#pragma unroll
  for (int k = 0; k < NL; k++) {
    o.X.v[k] = __shfl_xor(acc.X.v[k], 1);
    o.Y.v[k] = __shfl_xor(acc.Y.v[k], 1);
    o.ZZ.v[k] = __shfl_xor(acc.ZZ.v[k], 1);
    o.ZZZ.v[k] = __shfl_xor(acc.ZZZ.v[k], 1);
  }
  const bool oinf = __shfl_xor(inf ? 1 : 0, 1) != 0;
  const bool oyneg = __shfl_xor(yneg ? 1 : 0, 1) != 0;
  if (qh) return;
  if (!live) {
    if (in_batch) A.status[i] = dead_status;
    return;
  }
  fe X, ZZ;
  if (inf && oinf) {
    A.status[i] = ST_REJECT;  // infinity: (x, y) = (0, 0) -> false
    return;
  }
  if (inf || oinf) {
    X = inf ? o.X : acc.X;
    ZZ = inf ? o.ZZ : acc.ZZ;
  } else if (!ec_add_chud_x(X, ZZ, acc, o, yneg == oyneg)) {
    verify_exact(A, i);  // u1 G == +-u2 Q
    return;
  }
  fe zc = ZZ;
  fe_canon(zc);
  if (fe_is_zero_canon(zc)) {
    verify_exact(A, i);
    return;
  }
  verify_finish(A, i, X, ZZ);
}

// Mid-size batches (k_verify_quads): one item per lane QUAD, s^-1 from the
// batched planes.  Lane q of the quad sums one half of one scalar's comb
// windows: q = 0 G windows [0, mid) (the first two affine + affine), 1 G
// [mid, S), 2 Q [0, mid), 3 Q [mid, S) -- per-lane table, window and range,
// per-lane gathers -- so an item's latency is ~half a scalar's additions
// (4 of 9 at W = 29) plus two joins, against 8 additions plus one join per
// lane pair (verify_pair).  The halves of one scalar join by a full
// Chudnovsky addition on lanes 0 and 2 (never degenerate: with u = a + b the
// low and high parts of a scalar in [1, N), a == -b mod N is u == 0, and a ==
// b mod N needs u = 2 a + N with a the low part of u itself, which no window
// size admits -- tests/test_gpu_parity.py checks it for W = 8..29; a zero part
// is infinity, flagged), then G and Q by the x-only addition on lane 0 (u1 G
// == +-u2 Q takes the exact path, as in verify_pair).  Neither half of a range
// degenerates: every partial sum of a range is a multiple of 2^(W lo), smaller
// in magnitude than the next addend (verify_pair's argument).
// INLINE: s^-1 by the wave itself instead of the planes -- k_ninv_local's
// arithmetic with chains of one item over the wave's 16 quads (a butterfly at
// lane distances 4 .. 32, ONE wave-cooperative inversion, the butterfly back),
// so no separate launch and no planes round trip.
template <bool INLINE>
MBFT_DEV void verify_quad(const VerifyArgs& A, long i, int q, bool in_batch, uint4* buf, const Spill& sp) {
  const long ii = in_batch ? i : 0;
  uint32_t rw[8], sw[8];
  load_be256(rw, A.r + 32 * ii);
  load_be256(sw, A.s + 32 * ii);
  const uint32_t slot = A.slot[ii];
  const bool range_ok = !words_is_zero(rw) && words_lt(rw, kNw) &&
                        !words_is_zero(sw) && words_lt(sw, kNw);
  KeyDesc kd{A.tabG, (uint32_t)A.wg, 0u};
  if (slot < A.nslots) kd = A.keys[slot];
  const bool key_ok = slot < A.nslots && kd.valid;
  const uint8_t dead_status =
      key_ok ? ST_REJECT : (A.host_status && slot >= kHostSlot ? (uint8_t)slot : ST_BAD_KEY);
  const bool live = in_batch && key_ok && range_ok;
  uint32_t U1[8], U2[8];
#pragma unroll
  for (int j = 0; j < 8; j++) U1[j] = U2[j] = 0u;
  if (INLINE) {
    // every lane of the wave (dead ones carry 1: Montgomery's trick stays
    // consistent and nothing of theirs is used)
    fe v;
    fe_from_words(v, sw);
    if (!live) {
      fe_zero(v);
      v.v[0] = 1;
    }
    fe acc;
    fe_set(acc, kRN);  // Montgomery one
    fn_mul(acc, acc, v);
    fe sib[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
#pragma unroll
      for (int k = 0; k < NL; k++) sib[j].v[k] = __shfl_xor(acc.v[k], 4 << j);
      fn_mul(acc, acc, sib[j]);
    }
    fe r = acc;
    fn_canon(r);
    uint32_t w[8], iw[8];
    fe_to_words(w, r);
    if (!modinv_n_var_wave(iw, w)) {
#pragma unroll
      for (int k = 0; k < 8; k++) iw[k] = 0;  // not reachable: every value is in [1, N)
    }
    fe_from_words(r, iw);
    fn_to_mont(r, r);
#pragma unroll
    for (int j = 3; j >= 0; j--) fn_mul(r, r, sib[j]);  // this quad's s^-1 R
    if (live) load_scalars<true>(A, ii, U1, U2, &r);
  } else if (live) {
    load_scalars<false>(A, ii, U1, U2);
  }
  const bool qh = q >= 2, high = (q & 1) != 0;
  const uint32_t* tab = qh && live ? kd.tab : A.tabG;
  const int W = qh && live ? (int)kd.wbits : A.wg;
  const int S = (256 + W - 1) / W, mid = (S + 1) / 2;
  uint32_t U[8];
#pragma unroll
  for (int j = 0; j < 8; j++) U[j] = qh ? U2[j] : U1[j];
  chud acc;
  fe_zero(acc.X);
  fe_zero(acc.Y);
  fe_one_mont(acc.ZZ);
  fe_one_mont(acc.ZZZ);
  bool inf = true, yneg = false;
  uint32_t carry = 0;
  int step0 = 0;
  if (high) {
    // the recoding carry into window mid, U shifted to it
#pragma unroll 1
    for (int k = 0; k < mid; k++) {
      bool ng, zr;
      (void)comb_digit(U[0], carry, W, k + 1 >= S, ng, zr);
      shr_words(U, W);
    }
    step0 = mid;
  } else if (!qh) {
    // G's first two windows: affine + affine (as verify_pair)
    bool neg0, zero0, neg1, zero1;
    const uint32_t i0 = comb_digit(U[0], carry, W, false, neg0, zero0);
    shr_words(U, W);
    const uint32_t i1 = comb_digit(U[0], carry, W, false, neg1, zero1);
    shr_words(U, W);
    fe x0, y0, x1, y1;
    load_point(x0, y0, comb_entry(tab, W, 0, i0));
    load_point(x1, y1, comb_entry(tab, W, 1, i1));
    ec_add_affine_chud(acc, x0, y0, x1, y1, neg0 != neg1);
    yneg = !neg0;
    inf = zero0 && zero1;
    if (zero0 != zero1) {
      acc.X = zero0 ? x1 : x0;
      acc.Y = zero0 ? y1 : y0;
      fe_one_mont(acc.ZZ);
      fe_one_mont(acc.ZZZ);
      yneg = zero0 ? neg1 : neg0;
    }
    step0 = 2;
  }
  StepClock sc;
  comb_run<false>(acc, inf, yneg, U, tab, W, step0, carry, buf, sp, live, sc, high ? -1 : mid);
  fe_norm_lazy(acc.ZZ);
  fe_norm_lazy(acc.ZZZ);
  if (!inf && yneg) fe_neg(acc.Y, acc.Y);  // the true Y from here on
  // level 1: lanes 0 / 2 take the high half from lanes 1 / 3
  chud o;
#pragma unroll
  for (int k = 0; k < NL; k++) {
    o.X.v[k] = __shfl_xor(acc.X.v[k], 1);
    o.Y.v[k] = __shfl_xor(acc.Y.v[k], 1);
    o.ZZ.v[k] = __shfl_xor(acc.ZZ.v[k], 1);
    o.ZZZ.v[k] = __shfl_xor(acc.ZZZ.v[k], 1);
  }
  const bool oinf = __shfl_xor(inf ? 1 : 0, 1) != 0;
  if (high) return;
  bool degen = false;
  if (!oinf) {
    if (inf) {
      acc = o;
      inf = false;
    } else {
      chud t;
      if (ec_add_chud_full(t, acc, o))
        acc = t;
      else
        degen = true;  // not reachable (above); the exact path if it were
    }
  }
  // level 2: lane 0 takes Q's sum from lane 2
#pragma unroll
  for (int k = 0; k < NL; k++) {
    o.X.v[k] = __shfl_xor(acc.X.v[k], 2);
    o.Y.v[k] = __shfl_xor(acc.Y.v[k], 2);
    o.ZZ.v[k] = __shfl_xor(acc.ZZ.v[k], 2);
    o.ZZZ.v[k] = __shfl_xor(acc.ZZZ.v[k], 2);
  }
  const bool qinf = __shfl_xor(inf ? 1 : 0, 2) != 0;
  const bool qdegen = __shfl_xor(degen ? 1 : 0, 2) != 0;
  if (qh) return;
  if (!live) {
    if (in_batch) A.status[i] = dead_status;
    return;
  }
  if (degen || qdegen) {
    verify_exact(A, i);
    return;
  }
  fe X, ZZ;
  if (inf && qinf) {
    A.status[i] = ST_REJECT;  // infinity: (x, y) = (0, 0) -> false
    return;
  }
  if (inf || qinf) {
    X = inf ? o.X : acc.X;
    ZZ = inf ? o.ZZ : acc.ZZ;
  } else if (!ec_add_chud_x(X, ZZ, acc, o, true)) {
    verify_exact(A, i);  // u1 G == +-u2 Q
    return;
  }
  fe zc = ZZ;
  fe_canon(zc);
  if (fe_is_zero_canon(zc)) {
    verify_exact(A, i);
    return;
  }
  verify_finish(A, i, X, ZZ);
}

// The signed-digit comb sum of windows [lo, hi) of one scalar (U: its
// words shifted right by W lo, carry: the recoding carry into window lo),
// for k_verify_split: ONE item per wave (every lane holds the same values),
// so zero digits and infinity are plain (wave-uniform) branches.  The first
// two windows of the range are one affine + affine addition, the rest mixed
// additions on the Chudnovsky accumulator (ecc.h sign convention, fixed at
// the end: acc.Y is the TRUE Y).  A degenerate addition leaves ZZ == 0 (the
// caller checks).
// The range's table entries (up to kSplitPre windows) are fetched first, all
// at once -- lane 4 j + q loads quarter q of window lo + j's 64-B entry into
// the wave's LDS slice `pre` -- so the HBM (and TLB) latency of the random
// 64-B reads is paid once instead of once per addition; windows past
// kSplitPre (key windows below 16) load as they go.
#ifdef MBFT_SPLIT_TIMING
// Phase timestamps of the last split / resident item of workgroups 0 and 1
// (timing builds only, tools/split_timing.py, tools/resident_timing.py):
// [5 workgroup + wave][phase] wall clock (100 MHz), plus the shader clock at
// phases 0 and 7 of wave 0.  Phase 9: a wave's table entries are in
// (comb_range_uniform).
__device__ unsigned long long g_split_t[10][16];
__device__ unsigned long long g_split_clk[2];
#endif
constexpr int kSplitPre = 16;
// WIDE: the lane-group parallel additions (ecc.h ec_*_wide: the same results).
// extra (the resident kernel's one-scalar form): a range of 3 or more
// windows leaves its last window's entry out of the sum and returns it as a
// point of its own (affine, ZZ = ZZZ = 1, the digit's sign applied; *extra_inf
// if the digit is zero) for the host to join -- no mixed addition after the
// first pair.
template <bool WIDE>
MBFT_DEV void comb_range_uniform(chud& acc, bool& inf, uint32_t (&U)[8], uint32_t carry,
                                 const uint32_t* tab, int W, int S, int lo, int hi, uint4* pre,
                                 chud* extra = nullptr, bool* extra_inf = nullptr) {
  {
    uint32_t V[8];
#pragma unroll
    for (int j = 0; j < 8; j++) V[j] = U[j];
    uint32_t cy = carry;
    const int slot = (int)(__lane_id() >> 2);
    const uint4* src = nullptr;
#pragma unroll 1
    for (int k = lo; k < hi && k < lo + kSplitPre; k++) {
      bool neg, zero;
      const uint32_t idx = comb_digit(V[0], cy, W, k + 1 >= S, neg, zero);
      shr_words(V, W);
      if (slot == k - lo && !zero) src = comb_entry(tab, W, k, idx) + (__lane_id() & 3);
    }
    if (src) pre[__lane_id()] = *src;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#ifdef MBFT_SPLIT_TIMING
    if (__lane_id() == 0 && blockIdx.x < 2) g_split_t[5 * blockIdx.x + (threadIdx.x >> 6)][9] = wall_clock64();
#endif
  }
  auto entry = [&](int k, uint32_t idx) -> const uint4* {
    return k - lo < kSplitPre ? pre + 4 * (k - lo) : comb_entry(tab, W, k, idx);
  };
  inf = true;
  bool yneg = false;
  int k = lo;
  const int last = hi;
  if (extra) {
    *extra_inf = true;
    if (hi - lo >= 3) hi--;  // the last window goes out on its own
  }
  if (hi - lo >= 2) {
    bool neg0, zero0, neg1, zero1;
    const uint32_t i0 = comb_digit(U[0], carry, W, lo + 1 >= S, neg0, zero0);
    shr_words(U, W);
    const uint32_t i1 = comb_digit(U[0], carry, W, lo + 2 >= S, neg1, zero1);
    shr_words(U, W);
    fe x0, y0, x1, y1;
    load_point(x0, y0, entry(lo, i0));
    load_point(x1, y1, entry(lo + 1, i1));
    if (!zero0 && !zero1) {
      if (WIDE)
        ec_add_affine_chud_wide(acc, x0, y0, x1, y1, neg0 != neg1);
      else
        ec_add_affine_chud(acc, x0, y0, x1, y1, neg0 != neg1);
      yneg = !neg0;
      inf = false;
    } else if (zero0 != zero1) {
      acc.X = zero0 ? x1 : x0;
      acc.Y = zero0 ? y1 : y0;
      fe_one_mont(acc.ZZ);
      fe_one_mont(acc.ZZZ);
      yneg = zero0 ? neg1 : neg0;
      inf = false;
    }
    k = lo + 2;
  }
#pragma unroll 1
  for (; k < hi; k++) {
    bool neg, zero;
    const uint32_t idx = comb_digit(U[0], carry, W, k + 1 >= S, neg, zero);
    shr_words(U, W);
    if (zero) continue;
    fe px, py;
    load_point(px, py, entry(k, idx));
    if (inf) {
      acc.X = px;
      acc.Y = py;
      fe_one_mont(acc.ZZ);
      fe_one_mont(acc.ZZZ);
      yneg = neg;
      inf = false;
    } else {
      if (WIDE)
        ec_madd_chud_wide(acc, acc, px, py, yneg != neg);
      else
        ec_madd_chud<false, false>(acc, acc, px, py, yneg != neg);
      yneg = neg;
    }
  }
  if (!inf && yneg) fe_neg(acc.Y, acc.Y);
  if (extra && hi < last) {
    bool neg, zero;
    const uint32_t idx = comb_digit(U[0], carry, W, hi + 1 >= S, neg, zero);
    if (!zero) {
      fe px, py;
      load_point(px, py, entry(hi, idx));
      extra->X = px;
      extra->Y = py;
      if (neg) fe_neg(extra->Y, extra->Y);
      fe_one_mont(extra->ZZ);
      fe_one_mont(extra->ZZZ);
      *extra_inf = false;
    }
  }
}

// Small batches at the lowest latency (mbft_launch::verify, n <=
// MBFT_SPLIT_MAX, default 256 -- single calls, coalesced groups): ONE item
// per 256-thread workgroup, its 2 S comb windows split over the 4 waves
// (one per SIMD): wave 0 sums the low half of the G windows, wave 1 the high
// half, waves 2 and 3 the same for Q, at the same time; waves 0 and 2 then
// join the halves (full Chudnovsky additions) and wave 0 the two sums
// (x-only).  An item's latency is s^-1 (every wave inverts s itself with all
// its lanes, modinv_n_var_wave: no barrier) + ceil(S / 2) additions + two
// joins, instead of S additions + a join (k_verify_pairs) or 2 S.
// Degenerate additions or joins (u1 G == +-u2 Q, or crafted partial sums)
// take the exact path (verify_exact).  s^-1 per item (A.winv null), or
// the host's s^-1 R planes (A.winv: the lone calls' host inversion,
// batch.cpp host_winv -- ~2 us on the CPU against ~19 us for one wave).
#ifdef MBFT_SPLIT_TIMING
// Phase timestamps of the last k_verify_split item (timing builds only,
// tools/split_timing.py): [wave][phase] wall clock (100 MHz), plus the shader
// clock at phases 0 and 7 of wave 0.
#define SPLIT_T(ph)                                                   \
  do {                                                                \
    if (lane == 0 && blockIdx.x < 2) g_split_t[5 * blockIdx.x + wave][ph] = wall_clock64(); \
  } while (0)
extern "C" int mbft_debug_split_timing(unsigned long long out[162]) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_split_t), sizeof(g_split_t)) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out + 160, HIP_SYMBOL(g_split_clk), sizeof(g_split_clk)) != hipSuccess) return -1;
  return 0;
}
#else
#define SPLIT_T(ph) \
  do {              \
  } while (0)
#endif

// Item i of A on the whole 256-thread workgroup (k_verify_split, and the
// resident k_verify_server between mailbox posts): part / pre are the
// workgroup's LDS.  Every wave returns when its share is done; the status is
// written by wave 0 (or, for inputs rejected up front, thread 0).
// half (the resident kernel's two-workgroup form): -1 = both scalars here
// (waves 0, 1: G's windows in two ranges, waves 2, 3: Q's); 0 / 1 = only G
// (u1) / only Q (u2), its windows in four ranges, one a wave -- the other
// workgroup of the item does the other scalar on another CU (its own table
// walks).  pout: the partial sums go there for the host to join, no joins
// here.
// uin (the resident kernel, and k_verify_split's host-staged batches: the
// host computed them): u1, u2 as 16 LE words, loaded with the other inputs,
// so the waves skip s^-1 and the two mod-N products (~3 us of a lone call's
// critical path on one wave).
template <bool WIDE, int NP = 4>
MBFT_DEV void split_item(const VerifyArgs& A, long i, uint32_t (&part)[NP][4 * NL + 1],
                         uint4 (&pre)[4][4 * kSplitPre], uint32_t* pout = nullptr, int half = -1,
                         const uint32_t* uin = nullptr) {
  constexpr int NW = 4;  // waves
  static_assert(NP == 4 || NP == 8, "partial sums: 4 (both scalars), 8 (one scalar, extras)");
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool qh = half < 0 ? wave >= 2 : half == 1;  // this wave's scalar: u2 (Q) or u1 (G)
  // every input load issued at once (zero-copy staging: one PCIe round trip)
  uint32_t ew[8], rw[8], sw[8], U[8];
  load_be256(ew, A.e + 32 * i);
  load_be256(rw, A.r + 32 * i);
  load_be256(sw, A.s + 32 * i);
  if (uin) {
#pragma unroll
    for (int j = 0; j < 8; j++) U[j] = uin[(qh ? 8 : 0) + j];
  }
  const uint32_t slot = A.slot[i];
  fe wv;
  if (A.winv && !uin) plane_load(wv, A.winv, A.n, i);  // s^-1 R from the host (lone calls)
  const bool range_ok = !words_is_zero(rw) && words_lt(rw, kNw) && !words_is_zero(sw) && words_lt(sw, kNw);
  KeyDesc kd{A.tabG, (uint32_t)A.wg, 0u};
  if (slot < A.nslots) kd = A.keys[slot];
  const bool key_ok = slot < A.nslots && kd.valid;
  if (!(key_ok && range_ok)) {  // block-uniform: the whole workgroup returns
    // the status last, after every wave has read the inputs: the host may
    // reuse zero-copy staging as soon as it sees it (batch.cpp spin_statuses)
    __syncthreads();
    if (threadIdx.x == 0)
      A.status[i] = key_ok ? ST_REJECT : (A.host_status && slot >= kHostSlot ? (uint8_t)slot : ST_BAD_KEY);
    return;
  }
  SPLIT_T(1);
  if (!uin) {
    if (!A.winv) {
      uint32_t iw[8];
      if (!modinv_n_var_wave(iw, sw)) {
#pragma unroll
        for (int k = 0; k < 8; k++) iw[k] = 0;  // not reachable: 0 < s < N
      }
      fe_from_words(wv, iw);
      fn_to_mont(wv, wv);  // s^-1 R
    }
    SPLIT_T(2);
    uint32_t U1[8], U2[8];
    {
      fe e, r;
      fe_from_words(e, ew);
      fe_from_words(r, rw);
      scalars(U1, U2, e, r, wv);
    }
#pragma unroll
    for (int j = 0; j < 8; j++) U[j] = qh ? U2[j] : U1[j];
  }
  SPLIT_T(3);
  const uint32_t* tab = qh ? kd.tab : A.tabG;
  const int W = qh ? (int)kd.wbits : A.wg;
  const int S = (256 + W - 1) / W, mid = (S + 1) / 2;
  // this wave's range of the scalar's windows
  const int lo = half < 0 ? ((wave & 1) ? mid : 0) : wave * S / NW;
  const int hi = half < 0 ? ((wave & 1) ? S : mid) : (wave + 1) * S / NW;
  uint32_t carry = 0;
#pragma unroll 1
  for (int k = 0; k < lo; k++) {
    bool ng, zr;
    (void)comb_digit(U[0], carry, W, k + 1 >= S, ng, zr);
    shr_words(U, W);
  }
  chud acc, ex;
  bool inf, exinf = true;
  comb_range_uniform<WIDE>(acc, inf, U, carry, tab, W, S, lo, hi, pre[wave], NP == 8 ? &ex : nullptr,
                           &exinf);
  SPLIT_T(4);
  bool degen = false;
  if (!inf) {
    fe zc = acc.ZZ;
    fe_canon(zc);
    degen = fe_is_zero_canon(zc);
  }
  auto put = [&](int slot_, const chud& p, uint32_t flags) {
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < NL; k++) {
        part[slot_][k] = p.X.v[k];
        part[slot_][NL + k] = p.Y.v[k];
        part[slot_][2 * NL + k] = p.ZZ.v[k];
        part[slot_][3 * NL + k] = p.ZZZ.v[k];
      }
      part[slot_][4 * NL] = flags;
    }
  };
  auto get = [&](int slot_, chud& p) -> uint32_t {
#pragma unroll
    for (int k = 0; k < NL; k++) {
      p.X.v[k] = part[slot_][k];
      p.Y.v[k] = part[slot_][NL + k];
      p.ZZ.v[k] = part[slot_][2 * NL + k];
      p.ZZZ.v[k] = part[slot_][3 * NL + k];
    }
    return part[slot_][4 * NL];
  };
  // flags: 1 = infinity, 2 = degenerate (the exact path decides)
  put(wave, acc, (inf ? 1u : 0u) | (degen ? 2u : 0u));
  if constexpr (NP == 8) put(NW + wave, ex, exinf ? 1u : 0u);  // (affine: never degenerate)
  __syncthreads();
  if (pout) {  // the resident kernel: the host joins the NW sums (join_host.cpp)
    if (wave != 0) return;
    uint32_t fl = 0;
#pragma unroll
    for (int w = 0; w < NP; w++) fl |= part[w][4 * NL];
    if (fl & 2u) {
      verify_exact(A, i);
      return;
    }
    for (int k = lane; k < NP * 40; k += 64) {
      const int w = k / 40, j = k - 40 * w;
      pout[k] = j <= 4 * NL ? part[w][j] : 0u;
    }
    // (thread 0 -- this wave's lane 0 -- stores the done word after
    // sys_release, which waits for these stores and writes them back)
    if (lane == 0) A.status[i] = kSrvPartials;
    return;
  }
  // The joins as a two-level tree -- level 0: waves 0 and 2 add the halves
  // (G: slots 0 + 1, Q: 2 + 3), level 1: wave 0 adds the two sums -- in ONE
  // loop body, so the second level runs the first's instructions from a warm
  // instruction cache (a lone item's cold straight-line code costs ~2x:
  // tools/split_timing.py measured 9 us for a cold x-only join against
  // 3.6 us warm).  The full join's Y3 / ZZZ3 at level 1 are not needed
  // (the x-check reads X and ZZ) but cost less than cold code.
  if constexpr (NP != 4) return;  // (the one-scalar form always has pout)
#pragma unroll 1
  for (int lvl = 0; lvl < 2; lvl++) {
    const int step = 1 << lvl;
    if ((wave & (2 * step - 1)) == 0) {
      chud a, b, o;
      const uint32_t fa = get(wave, a), fb = get(wave + step, b);
      uint32_t fo = 0;
      if ((fa | fb) & 2u) {
        fo = 2u;
      } else if (fa & 1u) {
        o = b;
        fo = fb;
      } else if (fb & 1u) {
        o = a;
      } else if (!(WIDE ? ec_add_chud_full_wide(o, a, b) : ec_add_chud_full(o, a, b))) {
        fo = 2u;  // H == 0: equal or opposite partial sums
      }
      put(wave, o, fo);
    }
    if (lvl == 0) SPLIT_T(5);
    __syncthreads();
  }
  if (wave != 0) return;
  SPLIT_T(7);
  chud g;
  const uint32_t fg = get(0, g);
  if (fg & 2u) {
    verify_exact(A, i);
    return;
  }
  if (fg & 1u) {
    if (lane == 0) A.status[i] = ST_REJECT;  // u1 G + u2 Q = infinity: (0, 0) -> false
    return;
  }
  fe zc = g.ZZ;
  fe_canon(zc);
  if (fe_is_zero_canon(zc)) {
    verify_exact(A, i);
    return;
  }
  verify_finish(A, i, g.X, g.ZZ, rw);
  SPLIT_T(8);
#ifdef MBFT_SPLIT_TIMING
  if (threadIdx.x == 0 && blockIdx.x == 0) g_split_clk[1] = clock64();
#endif
}

template <bool WIDE>
__global__ void __launch_bounds__(256) k_verify_split(VerifyArgs A) {
  __shared__ uint32_t part[4][4 * NL + 1];
  __shared__ uint4 pre[4][4 * kSplitPre];  // each wave's prefetched table entries
#ifdef MBFT_SPLIT_TIMING
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (threadIdx.x == 0 && blockIdx.x == 0) g_split_clk[0] = clock64();
  SPLIT_T(0);
#endif
  const long i = blockIdx.x;
  if (A.ndev && i >= (long)*A.ndev) return;  // past the device count: block-uniform
  split_item<WIDE>(A, i, part, pre, nullptr, -1, A.uhost ? A.uhost + 16 * i : nullptr);
}

// The resident single-call verifier (kernels.h SrvSlot; host side in
// resident.cpp): a POOL of server workgroups for the mailbox slots.  A post
// is 1 or 2 jobs (TWO: one per scalar, u1 G and u2 Q, each on its own
// workgroup and CU; else the whole item).  Wave 0 of every idle server
// polls the doorbell line (one 64-B system-scope read over PCIe: slot b's
// post tag in byte b) and the claim words (device memory, agent scope); a
// job is open when slot b's tag is the successor of its claim (tags step
// 1..255 per post, so a stale read of either never re-opens a job), and the
// server takes it with one compare-and-swap of the claim.  It then copies
// the 256-B slot into LDS (one round trip, after a system-scope acquire: the
// host writes the slot, then its seq, then its tag), runs the job with
// split_item from that copy, and writes (seq << 8) | status to the job's
// done word (system-scope release).  A server count below 2 x slots keeps
// the resident kernel's VGPRs off most CUs: C2 batches beside it lost 16 %
// with one workgroup pair per slot at 32 slots.  Every
// workgroup leaves its loop when the host posts stop_gen == gen, when
// workgroup 0 has told this generation to exit (dexit[0] == gen: no post
// for idle_ticks, or life_ticks since its start; it also writes exited_gen
// so the host relaunches on the next call), or -- a workgroup whose
// workgroup 0 was never scheduled -- past life_ticks plus a grace; so every
// wave reaches an exit.  A claimed job is always finished first.
constexpr uint64_t kSrvGraceTicks = 10000000ull;  // 100 ms at 100 MHz

MBFT_DEV uint32_t sys_load(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Release at system scope, spelled out: this wave's stores done, the L2
// written back, and the write-back itself waited for.  The compiler's own
// release before a store (__ATOMIC_RELEASE, system scope) emits the L2
// write-back but drops the wait after it when no store of the wave is
// outstanding at that point (the waitcnt pass does not count the write-back):
// with the partial sums' stores already waited for by the barrier before
// thread 0's done word, the done word could reach the host ahead of them --
// measured as 1-7 wrong statuses in 2000 resident calls (tools/resident_probe.py
// gate), none with this sequence.  A vector-memory write-back (no scalar
// cache operation).
MBFT_DEV void sys_release() {
  asm volatile("s_waitcnt vmcnt(0)\n\tbuffer_wbl2 sc0 sc1\n\ts_waitcnt vmcnt(0)" ::: "memory");
}

// A word the host polls (done, exited_gen), after sys_release.
MBFT_DEV void sys_store(uint32_t* p, uint32_t v) {
  sys_release();
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The post tag after t (tags 1..255 in turn; kernels.h srv_tag).
MBFT_DEV uint32_t srv_next_tag(uint32_t t) { return t % 255u + 1u; }

// TWO: jobs are scalars (half 0: u1 G, half 1: u2 Q), four waves over the
// scalar's windows, a range of three leaving its last entry as a partial of
// its own (so at G / key windows >= 26 no mixed addition runs: one affine +
// affine addition per wave), done word done[b][8 half] and 8 partial sums
// (part[b][320 half ..]); else one job per item, both scalars, four partial
// sums.
// The server's VGPRs are capped for 3 waves per SIMD (168; ~108 B of
// scratch per lane), so a CU holding a server workgroup still holds two
// k_verify workgroups beside it: uncapped (205 VGPRs) it held one, and 16
// servers cost a C2 batch stream ~2/3 of 16 CUs instead of ~1/3
// (tools/resident_ab.py; build flag -DMBFT_SRV_WAVES=0: uncapped).
#if !defined(MBFT_SRV_WAVES) || MBFT_SRV_WAVES == 3
#define MBFT_SRV_ATTR __attribute__((amdgpu_waves_per_eu(3)))
#else
#define MBFT_SRV_ATTR
#endif
template <bool WIDE, bool TWO>
__global__ void __launch_bounds__(256) MBFT_SRV_ATTR k_verify_server(ServerArgs S) {
  constexpr int NP = TWO ? 8 : 4;
  __shared__ uint32_t part[NP][4 * NL + 1];
  __shared__ uint4 pre[4][4 * kSplitPre];
  __shared__ uint4 item4[sizeof(SrvSlot) / 16];  // the job's slot, copied from the mailbox
  __shared__ uint32_t cmd[3];
  __shared__ uint8_t st_lds[4];  // the item's status (split_item writes it through A.status)
  uint32_t* item = reinterpret_cast<uint32_t*>(item4);
  uint64_t* act = reinterpret_cast<uint64_t*>(S.dexit + 2);
  const uint64_t t0 = wall_clock64();
  const uint32_t lane = threadIdx.x & 63u;
  // idle servers seeing one post take different halves first
  const uint32_t pref = TWO ? (blockIdx.x & 1u) : 0u;
  uint32_t iter = 0;
#pragma unroll 1
  for (;;) {
    if (threadIdx.x < 64) {
      uint32_t c = 0, jb = 0, jh = 0;
#pragma unroll 1
      for (;;) {
        const bool mine = lane < S.nslots;
        const uint32_t w = sys_load(&S.ctl->tag32[lane >> 2]);
        const uint32_t c0 = mine ? __hip_atomic_load(&S.claim[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                 : 0u;
        const uint32_t c1 = TWO && mine ? __hip_atomic_load(&S.claim[kSrvMaxSlots + lane], __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT)
                                        : 0u;
        const uint32_t tg = (w >> (8u * (lane & 3u))) & 0xFFu;
        const bool open0 = mine && tg != 0u && tg == srv_next_tag(c0);
        const bool open1 = TWO && mine && tg != 0u && tg == srv_next_tag(c1);
        const uint64_t m0 = __ballot(open0), m1 = TWO ? __ballot(open1) : 0ull;
        bool got = false;
        if (m0 | m1) {
#pragma unroll 1
          for (uint32_t k = 0; k < (TWO ? 2u : 1u) && !got; k++) {
            const uint32_t h = TWO ? (k == 0 ? pref : 1u - pref) : 0u;
            uint64_t mm = h ? m1 : m0;
#pragma unroll 1
            while (mm && !got) {
              const uint32_t b = (uint32_t)__builtin_ctzll(mm);
              mm &= mm - 1;
              uint32_t ok = 0;
              if (lane == b) {
                uint32_t exp = h ? c1 : c0;
                ok = __hip_atomic_compare_exchange_strong(&S.claim[h * kSrvMaxSlots + b], &exp, tg,
                                                          __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT)
                         ? 1u
                         : 0u;
              }
              if (__builtin_amdgcn_readlane(ok, b)) {
                got = true;
                jb = b;
                jh = h;
              }
            }
          }
        }
        if (got) {
          c = 1;
          break;
        }
        // the stop and exit words and the clock (s_memrealtime: microseconds
        // of latency; read before every poll it cost ~5 us a call) every 8th
        // poll, so a poll is one PCIe read
        if ((++iter & 7u) != 0) {
#pragma unroll 1
          for (uint32_t z = 0; z < S.poll_sleep; z++) __builtin_amdgcn_s_sleep(8);
          continue;
        }
        if (sys_load(&S.ctl->stop_gen) == S.gen ||
            __hip_atomic_load(&S.dexit[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == S.gen) {
          c = 2;
          break;
        }
        const uint64_t now = wall_clock64();
        if (blockIdx.x == 0) {
          const uint64_t a = __hip_atomic_load(act, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const uint64_t since = a > t0 ? a : t0;
          if (now - since > S.idle_ticks || now - t0 > S.life_ticks) {
            if (lane == 0) {
              __hip_atomic_store(&S.dexit[0], S.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              sys_store(&S.ctl->exited_gen, S.gen);
            }
            c = 2;
            break;
          }
        } else if (now - t0 > S.life_ticks + kSrvGraceTicks) {
          c = 2;
          break;
        }
#pragma unroll 1
        for (uint32_t z = 0; z < S.poll_sleep; z++) __builtin_amdgcn_s_sleep(8);
      }
      if (lane == 0) {
        cmd[0] = c;
        cmd[1] = jb;
        cmd[2] = jh;
      }
    }
    __syncthreads();
    const uint32_t c = cmd[0], b = cmd[1], h = cmd[2];
    if (c == 2) break;  // workgroup-uniform
#ifdef MBFT_SRV_TIMING
    const uint64_t ts0 = wall_clock64();
#endif
    // The slot, one word a lane, read only after its tag was seen: the host
    // writes the fields and the seq before the tag, and a read issued after
    // the tag's read completed sees them.
    if (threadIdx.x < 64) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope
      item[threadIdx.x] = reinterpret_cast<const uint32_t*>(S.slots + b)[threadIdx.x];
    }
    __syncthreads();
#ifdef MBFT_SRV_TIMING
    const uint64_t ts1 = wall_clock64();
#endif
    const SrvSlot* it = reinterpret_cast<const SrvSlot*>(item4);
    const uint32_t q = it->seq & 0xFFFFFFu;
    const int dw = TWO ? 8 * (int)h : 0;  // this job's done word in the slot's line
    VerifyArgs A{it->e, it->r, it->s, &it->key0, it->winv, it->tabG, &it->kd, 1u, (int)it->wg, 1,
                 st_lds, nullptr, nullptr, 0u, nullptr, 0u, nullptr};
    if (it->gjoin) {
      // the whole item on its first job, joins and x test included
      // (k_verify_split's path): a final status, no partials -- for posts of
      // many items at once, whose joins would queue on the caller's one
      // thread; the second job only answers
      if (!TWO || h == 0)
        split_item<WIDE, 4>(A, 0, *reinterpret_cast<uint32_t(*)[4][4 * NL + 1]>(&part[0][0]), pre, nullptr, -1,
                            it->ugiven ? it->u : nullptr);
      else if (threadIdx.x == 0)
        st_lds[0] = kSrvPartials;
    } else {
      split_item<WIDE, NP>(A, 0, part, pre, S.ctl->part[b] + (TWO ? 40 * NP * h : 0), TWO ? (int)h : -1,
                           it->ugiven ? it->u : nullptr);
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // the status came from wave 0, this thread's own wave
      const uint32_t st = *static_cast<volatile uint8_t*>(st_lds);
#ifdef MBFT_SRV_TIMING
      // (the done word's cache line has room)
      const uint64_t ts2 = wall_clock64();
      uint32_t* tw = &S.ctl->done[b][dw + 1];
      tw[0] = (uint32_t)(ts1 - ts0);
      tw[1] = (uint32_t)(ts2 - ts1);
#endif
      sys_store(&S.ctl->done[b][dw], (q << 8) | st);
      __hip_atomic_store(act, wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();  // cmd and the LDS item are reused by the next poll
  }
}

// LANE_INV false: s^-1 R from the batched planes (A.winv, stride A.n).
template <bool LANE_INV>
__global__ void __launch_bounds__(256, 2) k_verify_pairs(VerifyArgs A) {
  __shared__ uint4 coop[4][256];  // per wave: 64 lanes x 64 B (per-lane gathers)
  uint4* buf = coop[threadIdx.x >> 6];
  const Spill sp{A.scr, blockIdx.x * blockDim.x + threadIdx.x, A.sstride};
  const long stride = (long)gridDim.x * blockDim.x;
  // the item count: n, or the device's (<= n) when the caller sized the grid
  // for an upper bound; a wave wholly past it leaves (per-wave buffers, no
  // block barrier in verify_pair)
  long n = A.n;
  if (A.ndev && (long)*A.ndev < n) n = (long)*A.ndev;
  const long wave0 = (long)(threadIdx.x & ~63u);
#pragma unroll 1
  for (long base = (long)blockIdx.x * blockDim.x; base < 2 * n; base += stride) {
    if (base + wave0 >= 2 * n) break;
    const long t = base + threadIdx.x;
    verify_pair<LANE_INV>(A, t >> 1, (int)(t & 1), (t >> 1) < n, buf, sp);
  }
}

// One item per lane quad (verify_quad), s^-1 from the batched planes
// (A.winv) or, INLINE, by each wave; the item count n, or the device's when
// the grid was sized for an upper bound.
template <bool INLINE>
__global__ void __launch_bounds__(256, 2) k_verify_quads(VerifyArgs A) {
  __shared__ uint4 coop[4][256];  // per wave: 64 lanes x 64 B (per-lane gathers)
  uint4* buf = coop[threadIdx.x >> 6];
  const Spill sp{A.scr, blockIdx.x * blockDim.x + threadIdx.x, A.sstride};
  const long stride = (long)gridDim.x * blockDim.x;
  long n = A.n;
  if (A.ndev && (long)*A.ndev < n) n = (long)*A.ndev;
  const long wave0 = (long)(threadIdx.x & ~63u);
#pragma unroll 1
  for (long base = (long)blockIdx.x * blockDim.x; base < 4 * n; base += stride) {
    if (base + wave0 >= 4 * n) break;
    const long t = base + threadIdx.x;
    verify_quad<INLINE>(A, t >> 2, (int)(t & 3), (t >> 2) < n, buf, sp);
  }
}

// Grid-stride over items: the default grid has one 256-item block per 256
// items; a capped grid (MBFT_VERIFY_BPC blocks per CU) leaves wave slots
// free so the next batch's s^-1 kernels run concurrently.
// The exact path for the items k_verify queued: both phases recomputed with
// complete additions (doubling, infinity), one item per thread, grid-stride
// over the queue (its length is known only on the device).  A final
// infinity rejects, as Go's (0, 0) does.
//
// The queued items run as G / Q lane pairs (verify_pair): a degenerate
// addition can only happen where the two single-scalar sums meet, so the
// fast mixed addition serves both halves and only a degenerate join takes
// the complete formulas (verify_exact).  s^-1 from the batched planes.
__global__ void __launch_bounds__(256, 2) k_verify_slow(VerifyArgs A) {
  __shared__ uint4 coop[4][256];  // per wave: 64 lanes x 64 B (per-lane gathers)
  uint4* buf = coop[threadIdx.x >> 6];
  const Spill sp{A.scr, blockIdx.x * blockDim.x + threadIdx.x, A.sstride};
  const long nq = (long)*A.slown;
  const long stride = (long)gridDim.x * blockDim.x;
#pragma unroll 1
  for (long base = (long)blockIdx.x * blockDim.x; base < 2 * nq; base += stride) {
    const long t = base + threadIdx.x, q = t >> 1;
    const bool in = q < nq;
    verify_pair<false>(A, in ? (long)A.slowq[q] : 0, (int)(t & 1), in, buf, sp);
  }
}

#ifdef MBFT_CLOCK_STAMP
// Clock builds only (tools/ab_build_def.sh clk "-DMBFT_CLOCK_STAMP"): per
// k_verify workgroup, shader cycles (s_memtime) and 100 MHz wall ticks
// (s_memrealtime) from its start to its end, summed: their ratio x 100 MHz is
// the in-kernel clock over the launches since the last reset
// (tools/clock_stamp_probe.py).  Stamps go to this buffer alone.
__device__ unsigned long long g_vclk[3];
extern "C" int mbft_debug_verify_clock(double out[3], int reset) {
  unsigned long long h[3];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_vclk), sizeof(h)) != hipSuccess) return -1;
  for (int k = 0; k < 3; k++) out[k] = (double)h[k];
  if (reset) {
    const unsigned long long z[3] = {0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_vclk), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

template <int MINW>
__global__ void __launch_bounds__(256, MINW) k_verify(VerifyArgs A) {
#ifdef MBFT_CLOCK_STAMP
  unsigned long long clk0 = 0, rt0 = 0;
  if (threadIdx.x == 0) {
    clk0 = __builtin_amdgcn_s_memtime();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
#endif
#ifdef MBFT_TWO_DEEP_GATHER
  __shared__ uint4 coop[2][4][256];  // per wave: two slots of 64 entries x 64 B (gather_issue)
  uint4* buf2 = coop[1][threadIdx.x >> 6];
#else
  __shared__ uint4 coop[1][4][256];  // per wave: one slot of 64 entries x 64 B (gather_issue)
  uint4* buf2 = nullptr;
#endif
  uint4* buf = coop[0][threadIdx.x >> 6];
  const long stride = (long)gridDim.x * blockDim.x;
  // block-uniform loop: all lanes of a wave take part in every step
#pragma unroll 1
  for (long base = (long)blockIdx.x * blockDim.x; base < A.n; base += stride) {
    const long i = base + threadIdx.x;
    verify_one(A, i, i < A.n, buf, buf2);
  }
#ifdef MBFT_CLOCK_STAMP
  if (threadIdx.x == 0) {
    const unsigned long long clk1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
    atomicAdd(&g_vclk[0], clk1 - clk0);
    atomicAdd(&g_vclk[1], rt1 - rt0);
    atomicAdd(&g_vclk[2], 1ull);
  }
#endif
}

// ---------------------------------------------------------------------------
// Bulk ECDSA signing (generation side: GenerateMessageAuthenTag for the
// ECDSA roles, crypto.go:63-76, and synthetic load generation).  R = k*G by
// the same 8-bit comb over the G table (no degenerate cases possible: the
// partial sums are distinct multiples < N of G).  Deterministic nonce
// k = SHA256(d || e || ctr) mod N.
struct SignArgs {
  const uint8_t* priv;      // nkeys x 32 B big-endian
  const uint32_t* key_idx;  // n (or null: key 0)
  const uint8_t* e;         // n x 32 B big-endian
  long n;
  const uint32_t* tabG;
  int wg;
  uint8_t* r_out;           // n x 32 B big-endian
  uint8_t* s_out;
  const uint8_t* k_in;      // optional n x 32 B big-endian nonces (crafted load)
};

MBFT_DEV void store_be256(uint8_t* p, const uint32_t w[8]) {
  uint32_t be[8];
#pragma unroll
  for (int i = 0; i < 8; i++) be[i] = __builtin_bswap32(w[7 - i]);
  store_words8(reinterpret_cast<uint32_t*>(p), be);
}

__global__ void __launch_bounds__(256) k_sign(SignArgs A) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= A.n) return;
  const uint32_t kid = A.key_idx ? A.key_idx[i] : 0u;
  uint32_t dbe[8], ebe[8], dw[8], ew[8];
  load_words8(dbe, reinterpret_cast<const uint32_t*>(A.priv + 32 * (size_t)kid));
  load_words8(ebe, reinterpret_cast<const uint32_t*>(A.e + 32 * i));
  // byte-order: sha256 consumes big-endian words == the raw bytes loaded
  // little-endian then byte-swapped
  uint32_t dm[8], em[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    dm[j] = __builtin_bswap32(dbe[j]);
    em[j] = __builtin_bswap32(ebe[j]);
  }
  be_words_to_le(dw, dbe);
  be_words_to_le(ew, ebe);
  fe d, e, dm_n;
  fe_from_words(d, dw);
  fe_from_words(e, ew);
  fn_to_mont(dm_n, d);
  uint32_t rw_out[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sw_out[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll 1
  for (uint32_t ctr = 0; ctr < 4; ctr++) {
    uint32_t h[8], m[16];
    uint32_t kw[8];
    if (A.k_in) {
      // a given nonce (generation of crafted inputs): one attempt
      uint32_t kbe[8];
      load_words8(kbe, reinterpret_cast<const uint32_t*>(A.k_in + 32 * i));
      be_words_to_le(kw, kbe);
      ctr = 3;
    } else {
      sha256_init(h);
#pragma unroll
      for (int j = 0; j < 8; j++) { m[j] = dm[j]; m[8 + j] = em[j]; }
      sha256_block(h, m);
#pragma unroll
      for (int j = 0; j < 16; j++) m[j] = 0;
      m[0] = ctr;
      m[1] = 0x80000000u;
      m[15] = 68u * 8u;
      sha256_block(h, m);
#pragma unroll
      for (int j = 0; j < 8; j++) kw[7 - j] = h[j];
    }
    fe k;
    fe_from_words(k, kw);
    fn_canon(k);
    uint32_t kc[8];
    fe_to_words(kc, k);
    if (words_is_zero(kc)) continue;
    // R = k G
    uint32_t U[8];
#pragma unroll
    for (int j = 0; j < 8; j++) U[j] = kc[j];
    jac acc;
    fe_zero(acc.X); fe_zero(acc.Y); fe_zero(acc.Z);
    bool inf = true;
    comb_fast(acc, inf, U, A.tabG, A.wg);
    fe zi, x;
    fe_inv(zi, acc.Z);
    fe_sqr(zi, zi);
    fe_mul(x, acc.X, zi);
    fe_from_mont(x, x);
    fe_canon(x);
    fn_canon(x);  // r = x mod N (x < p < 2N)
    uint32_t rw[8];
    fe_to_words(rw, x);
    if (words_is_zero(rw)) continue;
    // s = k^-1 (e + r d) mod N
    fe kinv, t, rd;
    fn_to_mont(kinv, k);
    fn_inv(kinv, kinv);
    fn_mul(rd, x, dm_n);   // r d (plain)
    fe_add(t, e, rd);
    fn_canon(t);
    fn_mul(t, t, kinv);
    fn_canon(t);
    uint32_t sw[8];
    fe_to_words(sw, t);
    if (words_is_zero(sw)) continue;
#pragma unroll
    for (int j = 0; j < 8; j++) { rw_out[j] = rw[j]; sw_out[j] = sw[j]; }
    break;
  }
  store_be256(A.r_out + 32 * i, rw_out);
  store_be256(A.s_out + 32 * i, sw_out);
}


// ---------------------------------------------------------------------------
// SHA-256 stage (messages/authen.go:78-82 hashsum; the USIG digest chain
// usig/sgx/sgx-usig.go:99-101 + usig-enclave.go:204-214).  One message per
// lane; digests are written as 32 big-endian bytes.

MBFT_DEV void store_digest(uint8_t* dst, const uint32_t h[8]) {
  uint32_t w[8];
#pragma unroll
  for (int j = 0; j < 8; j++) w[j] = __builtin_bswap32(h[j]);
  store_words8(reinterpret_cast<uint32_t*>(dst), w);
}

// out[i] = SHA256(data[off[i] .. off[i+1]))
__global__ void k_sha256_var(const uint8_t* __restrict__ data, const uint64_t* __restrict__ off,
                             long n, uint8_t* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t a = off[i], b = off[i + 1];
  uint32_t h[8];
  sha256_msg(h, data + a, (uint32_t)(b - a));
  store_digest(out + 32 * i, h);
}

// e[dst_i] = SHA256(SHA256(m_i) || epoch_le || counter_le), dst_i = idx[i]
// (or i when idx is null: the batch path scatters into its item-indexed e)
__global__ void k_usig_e(const uint8_t* __restrict__ data, const uint64_t* __restrict__ off,
                         const uint64_t* __restrict__ epoch, const uint64_t* __restrict__ counter,
                         const uint32_t* __restrict__ idx, long n, uint8_t* __restrict__ e) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t a = off[i], b = off[i + 1];
  uint32_t d[8], h[8];
  sha256_msg(d, data + a, (uint32_t)(b - a));
  sha256_usig_chain(h, d, epoch[i], counter[i]);
  store_digest(e + 32 * (idx ? (long)idx[i] : i), h);
}

// REQUEST pipeline front end: AuthenBytes = "REQUEST" || seq_be64 ||
// SHA256(op) (messages/authen.go:33,54-56), and the ECDSA-role digest input
// e = (AuthenBytes || SHA256(""))[0:32] = "REQUEST" || seq || SHA256(op)[0:17]
// (sample/authentication/crypto.go:121).  ops: n x op_len bytes.
__global__ void k_request_e(const uint64_t* __restrict__ seq, const uint8_t* __restrict__ ops,
                            uint32_t op_len, long n, uint8_t* __restrict__ e) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t h[8];
  sha256_msg(h, ops + (size_t)op_len * i, op_len);
  const uint64_t q = seq[i];
  uint32_t W[8];
  W[0] = 0x52455155u;                                   // "REQU"
  W[1] = 0x45535400u | (uint32_t)(q >> 56);             // "EST" seq0
  W[2] = (uint32_t)(q >> 24);                           // seq1..4
  W[3] = ((uint32_t)q << 8) | (h[0] >> 24);             // seq5..7 H0
#pragma unroll
  for (int k = 1; k <= 4; k++) W[3 + k] = (h[k - 1] << 8) | (h[k] >> 24);
  store_digest(e + 32 * i, W);
}

// Same digest for fixed-length operations (op_len % 16 == 0, ops 16-byte
// aligned, op_len <= kReqTileMax): one wave per 64 messages.  The wave's
// 64 x op_len contiguous bytes are loaded with fully coalesced dwordx4 loads
// (each wave-instruction reads 1 KiB in one piece) into an LDS tile whose rows
// are padded to an odd word stride (conflict-free row-per-lane reads), then
// each lane hashes its row from LDS with the state in VGPRs.
constexpr int kReqTileMax = 512;

__global__ void __launch_bounds__(64) k_request_e_tiled(const uint64_t* __restrict__ seq,
                                                        const uint8_t* __restrict__ ops,
                                                        uint32_t op_len, long n,
                                                        uint8_t* __restrict__ e) {
  extern __shared__ uint32_t tile[];
  const int lane = threadIdx.x;
  const long base = (long)blockIdx.x * 64;
  const int cnt = n - base < 64 ? (int)(n - base) : 64;
  const uint32_t wpr = op_len / 4, stride = wpr + 1, cpr = op_len / 16;
  const uint4* src = reinterpret_cast<const uint4*>(ops + (size_t)base * op_len);
  const uint32_t nchunks = (uint32_t)cnt * cpr;
#pragma unroll 4
  for (uint32_t c = lane; c < nchunks; c += 64) {
    const uint4 v = src[c];
    const uint32_t msg = c / cpr, w = (c - msg * cpr) * 4;
    uint32_t* row = tile + msg * stride + w;
    row[0] = v.x; row[1] = v.y; row[2] = v.z; row[3] = v.w;
  }
  __syncthreads();
  if (lane >= cnt) return;
  const uint32_t* row = tile + lane * stride;
  uint32_t h[8];
  sha256_init(h);
  const uint32_t nblk = (op_len + 9 + 63) / 64;
  const uint64_t bits = (uint64_t)op_len * 8u;
#pragma unroll 1
  for (uint32_t b = 0; b < nblk; b++) {
    uint32_t m[16];
    const bool last = b + 1 == nblk;
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint32_t wi = 16 * b + j;
      m[j] = wi < wpr ? __builtin_bswap32(row[wi]) : (wi == wpr ? 0x80000000u : 0u);
    }
    if (last) {
      m[14] = (uint32_t)(bits >> 32);
      m[15] = (uint32_t)bits;
    }
    sha256_block(h, m);
  }
  const uint64_t q = seq[base + lane];
  uint32_t W[8];
  W[0] = 0x52455155u;
  W[1] = 0x45535400u | (uint32_t)(q >> 56);
  W[2] = (uint32_t)(q >> 24);
  W[3] = ((uint32_t)q << 8) | (h[0] >> 24);
#pragma unroll
  for (int k = 1; k <= 4; k++) W[3 + k] = (h[k - 1] << 8) | (h[k] >> 24);
  store_digest(e + 32 * (base + lane), W);
}

// AuthenBytes + digest input e of every PREPARE / COMMIT / REPLY call from
// the message's raw fields and H(op) (authen_dev.h; H(op) computed by
// k_sha256_var over the operations).  One call per thread.
__global__ void k_authen_e(const uint8_t* __restrict__ H, const AuthenDesc* __restrict__ D, long n,
                           uint8_t* __restrict__ e) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const AuthenDesc d = D[i];
  uint32_t hw[8], hb[8];
  load_words8(hb, reinterpret_cast<const uint32_t*>(H + 32 * (size_t)d.msg));
#pragma unroll
  for (int k = 0; k < 8; k++) hw[k] = __builtin_bswap32(hb[k]);  // big-endian-numeric words
  uint32_t out[8];
  authen_digest(out, d.kind, hw, d.seq, d.client, d.view, d.primary, d.prep_ctr, d.epoch, d.counter);
  store_digest(e + 32 * (size_t)d.item, out);
}

// ---------------------------------------------------------------------------
// Device-side decode of raw VerifyMessageAuthenTag calls (k_prepare): the
// byte-level part of batch.cpp's prepare_item, one call per lane, in the
// reference's check order (sample/authentication/authenticator.go:121-134,
// keymanager.go:100, crypto.go:79-89 for the ECDSA roles, crypto.go:186-239
// + usig.go:75-80 + sgx-usig.go:159-168 + usig-enclave.go:217-222 for USIG).
// The USIG epoch step stays on the host (it is ordered state); a USIG call
// whose DER fails, or has trailing bytes, is left to it (kHostSlot |
// MBFT_BAD_KEY, the host's kDeadSlot).
__constant__ uint8_t kEmptySha[32] = {0xe3, 0xb0, 0xc4, 0x42, 0x98, 0xfc, 0x1c, 0x14,
                                      0x9a, 0xfb, 0xf4, 0xc8, 0x99, 0x6f, 0xb9, 0x24,
                                      0x27, 0xae, 0x41, 0xe4, 0x64, 0x9b, 0x93, 0x4c,
                                      0xa4, 0x95, 0x99, 0x1b, 0x78, 0x52, 0xb8, 0x55};

namespace {
constexpr uint32_t kStMalformedDer = 2, kStUnknownKey = 4, kStBadKey = 5, kStBadUi = 6,
                   kStBadCert = 7, kStUnknownRole = 10;
constexpr uint32_t kRoleReplica = 1, kRoleUsig = 2, kRoleClient = 3;

MBFT_DEV uint64_t load_be64_bytes(const uint8_t* p) {
  uint64_t v = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) v = (v << 8) | p[k];
  return v;
}
}  // namespace

__global__ void __launch_bounds__(256) k_prepare(PrepArgs A) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= A.n) return;
  uint32_t role = A.roles8 ? (uint32_t)A.roles8[i] : A.roles[i];
  const uint32_t id = A.ids[i];
  const uint64_t ma = A.moff32 ? A.moff32[i] : A.moff[i], mz = A.moff32 ? A.moff32[i + 1] : A.moff[i + 1];
  const uint64_t ta = A.toff32 ? A.toff32[i] : A.toff[i], tz = A.toff32 ? A.toff32[i + 1] : A.toff[i + 1];
  // the call's fields must lie in its chunk's byte ranges, in order (the
  // host checks no call of a device-decoded batch): else flag the batch
  // (MBFT_ERR_ARG) and read nothing
  const bool in_range = A.mlo <= ma && ma <= mz && mz <= A.mhi && A.tlo <= ta && ta <= tz && tz <= A.thi;
  if (!in_range) {
    atomicOr(A.bad, 1u);
    role = ~0u;  // decided without reading a byte (an unknown role)
  }
  const uint64_t m0 = in_range ? ma - A.mbase : 0, t0 = in_range ? ta - A.tbase : 0;
  const uint32_t mlen = in_range ? (uint32_t)(mz - ma) : 0u;
  const uint32_t tlen = in_range ? (uint32_t)(tz - ta) : 0u;
  const uint8_t* msg = A.msgs + m0;
  uint32_t st = 0xFFu, sl = 0;
  uint32_t ew[8], rw[8], sw[8];
#pragma unroll
  for (int j = 0; j < 8; j++) ew[j] = rw[j] = sw[j] = 0;
  // the tag's covering words staged in this lane's LDS slot (one batch of
  // loads; DER is parsed byte by byte at LDS latency), arena_dev.h
  __shared__ uint32_t tagbuf[256 * kTagWords];
  uint32_t* tw = tagbuf + threadIdx.x * kTagWords;
  const bool staged = stage_field(tw, A.tags, t0, tlen);
  if (role > 3u || ((A.map.role_ok >> role) & 1u) == 0) {
    st = kStUnknownRole;
  } else {
    const uint64_t key = ((uint64_t)role << 32) | id;
    bool known = false;
    for (uint32_t h = keymap_hash(key) & A.map.mask, probe = 0; probe <= A.map.mask;
         probe++, h = (h + 1) & A.map.mask) {
      const uint64_t k = A.map.keys[h];
      if (k == key) {
        known = true;
        sl = A.map.slots[h];
        break;
      }
      if (k == ~0ull) break;
    }
    const bool valid = known && sl < A.nslots && A.keys[sl].valid != 0;
    auto parse = [&](const uint8_t* tag) __attribute__((always_inline)) {
      if (role != kRoleUsig) {
        // DER first: Go panics on a decode error before looking at the key
        uint32_t used;
        if (!der_sig(tag, tlen, rw, sw, used)) {
          st = kStMalformedDer;
        } else if (!known) {
          st = kStUnknownKey;
        } else if (!valid) {
          st = kStBadKey;
        } else if (mlen >= 32) {
          // md = msg || SHA256("") (crypto.go:121): e = md[0:32]
          const ArenaField f = arena_field(A.msgs, m0, 32);
          arena_block(f, 0, ew);
        } else {
#pragma unroll
          for (int k = 0; k < 32; k++) {
            const uint32_t b = (uint32_t)k < mlen ? (uint32_t)msg[k] : (uint32_t)kEmptySha[k - mlen];
            ew[k >> 2] |= b << (8 * (k & 3));
          }
        }
      } else if (tlen < 8) {
        st = kStBadUi;
      } else if (!known) {
        st = kStUnknownKey;
      } else if (!valid) {
        st = kStBadKey;
      } else if (tlen - 8 < 8) {
        st = kStBadCert;
      } else {
        const uint64_t counter = load_be64_bytes(tag), epoch = load_be64_bytes(tag + 8);
        uint32_t used;
        if (!der_sig(tag + 16, tlen - 16, rw, sw, used) || used != tlen - 16) {
          st = kStBadKey;  // the host's epoch step decides (MALFORMED_DER / DER_TRAILING)
        } else {
          uint32_t d[8], h[8];
          sha256_arena(d, A.msgs, m0, mlen);
          sha256_usig_chain(h, d, epoch, counter);
#pragma unroll
          for (int j = 0; j < 8; j++) ew[j] = __builtin_bswap32(h[j]);
        }
      }
    };
    if (staged)
      parse(reinterpret_cast<const uint8_t*>(tw) + (t0 & 3u));
    else
      parse(A.tags + t0);
  }
  store_words8(reinterpret_cast<uint32_t*>(A.e + 32 * i), ew);
  store_words8(reinterpret_cast<uint32_t*>(A.r + 32 * i), rw);
  store_words8(reinterpret_cast<uint32_t*>(A.s + 32 * i), sw);
  A.slot[i] = st == 0xFFu ? sl : (kHostSlot | st);
}

// ---------------------------------------------------------------------------
// host-side launchers (declared in kernels.h)
namespace mbft_launch {

hipError_t sha256_var(const uint8_t* data, const uint64_t* off, long n, uint8_t* out,
                      hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_sha256_var, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, data, off,
                     n, out);
  return hipGetLastError();
}

hipError_t usig_e(const uint8_t* data, const uint64_t* off, const uint64_t* epoch,
                  const uint64_t* counter, const uint32_t* idx, long n, uint8_t* e,
                  hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_usig_e, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, data, off,
                     epoch, counter, idx, n, e);
  return hipGetLastError();
}

hipError_t request_e(const uint64_t* seq, const uint8_t* ops, uint32_t op_len, long n, uint8_t* e,
                     hipStream_t st) {
  if (n <= 0) return hipSuccess;
  static const bool tiled = [] {
    const char* v = getenv("MBFT_REQUEST_TILED");
    return !(v && atoi(v) == 0);
  }();
  if (tiled && op_len > 0 && op_len % 16 == 0 && op_len <= (uint32_t)kReqTileMax &&
      ((uintptr_t)ops & 15u) == 0) {
    const size_t lds = (size_t)64 * (op_len / 4 + 1) * 4;
    hipLaunchKernelGGL(k_request_e_tiled, dim3((unsigned)((n + 63) / 64)), dim3(64), lds, st, seq,
                       ops, op_len, n, e);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_request_e, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, seq, ops,
                     op_len, n, e);
  return hipGetLastError();
}

hipError_t prepare_calls(const PrepArgs& a, hipStream_t st) {
  if (a.n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_prepare, dim3((unsigned)((a.n + 255) / 256)), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t authen_e(const uint8_t* H, const AuthenDesc* d, long n, uint8_t* e, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_authen_e, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, H, d, n, e);
  return hipGetLastError();
}

hipError_t check_points(const uint32_t* xy, int n, uint32_t* ok, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_check_points, dim3((n + 63) / 64), dim3(64), 0, st, xy, n, ok);
  return hipGetLastError();
}

size_t table_entries(int wbits) {
  const int S = (256 + wbits - 1) / wbits;
  return ((size_t)(S - 1) << (wbits - 1)) + ((size_t)1 << (256 - (S - 1) * wbits));
}
size_t table_words(int wbits) { return table_entries(wbits) * 16u; }
int table_steps(int wbits) { return (256 + wbits - 1) / wbits; }

hipError_t build_tables(const uint32_t* xy, int npts, int wbits, uint32_t* bpts, uint32_t* tab,
                        hipStream_t st) {
  if (npts <= 0) return hipSuccess;
  if (wbits < kMinWindow || wbits > kMaxWindow) return hipErrorInvalidValue;
  const int t1 = npts * table_steps(wbits);
  hipLaunchKernelGGL(k_table_pow2, dim3((t1 + 63) / 64), dim3(64), 0, st, xy, npts, wbits, bpts);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // runs (k_table_fill) in launches of at most 2^19 threads, each with its
  // own H scratch (9 x kFillRun words per thread)
  const int S = table_steps(wbits);
  const int lastbits = 256 - (S - 1) * wbits;
  const long n0 = 1L << (wbits - 1), n1 = 1L << lastbits;
  const long L0 = n0 < kFillRun ? n0 : kFillRun, L1 = n1 < kFillRun ? n1 : kFillRun;
  const long runs = (long)(S - 1) * (n0 / L0) + n1 / L1;
  const long total = (long)npts * runs;
  const long chunk = total < (1L << 19) ? total : (1L << 19);
  uint32_t* scratch = nullptr;
  e = hipMalloc(reinterpret_cast<void**>(&scratch), (size_t)chunk * NL * kFillRun * 4);
  if (e != hipSuccess) return e;
  for (long first = 0; first < total; first += chunk) {
    const long cnt = total - first < chunk ? total - first : chunk;
    hipLaunchKernelGGL(k_table_fill, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, st,
                       bpts, npts, wbits, first, cnt, scratch, tab);
    e = hipGetLastError();
    if (e != hipSuccess) break;
  }
  // the launches read the scratch until they finish
  const hipError_t es = hipStreamSynchronize(st);
  const hipError_t ef = hipFree(scratch);
  return e != hipSuccess ? e : (es != hipSuccess ? es : ef);
}

hipError_t generator_xy(uint32_t* xy16, hipStream_t st) {
  uint32_t h[16];
  hipError_t e = hipMemcpyFromSymbol(h, HIP_SYMBOL(kGxw), 32, 0, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return e;
  e = hipMemcpyFromSymbol(h + 8, HIP_SYMBOL(kGyw), 32, 0, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return e;
  return hipMemcpyAsync(xy16, h, 64, hipMemcpyHostToDevice, st);
}

// Batched s^-1 (Montgomery's trick) as a tree of strided chains of 16:
// n -> ceil(n/16) -> ... until <= kTopMax (4096) totals, which k_ninv_top
// inverts with one workgroup and one divsteps inversion.
// Workspace per level l with m_l inputs and G_l chains: pre (m_l planes),
// tot (G_l planes) and, below the top level, inv_tot (G_l planes).
namespace {
constexpr long kChain = 16, kMaxRoots = kTopMax;
// Level 0 (the batch itself) may use longer chains (env MBFT_NINV_CHAIN0):
// fewer, longer-lived waves beside the previous batch's verify kernel.
long chain0() {
  static const long c = [] {
    const char* v = getenv("MBFT_NINV_CHAIN0");
    return v && atol(v) > 0 ? atol(v) : kChain;
  }();
  return c;
}
long ninv_groups(long m, bool level0) {
  const long c = level0 ? chain0() : kChain;
  return (m + c - 1) / c;
}
}  // namespace

size_t ninv_workspace_words(long n) {
  size_t words = (size_t)NL * kTopMax;  // k_ninv_top's prefixes
  long m = n;
  bool l0 = true;
  do {
    const long G = ninv_groups(m, l0);
    l0 = false;
    words += (size_t)NL * (m + 2 * G);
    m = G;
  } while (m > kMaxRoots);
  return words + 64;
}

// w planes (9 x n) <- (s_i)^-1 * R mod N for each item (invalid s -> 1^-1)
hipError_t batch_inverse_s(const uint8_t* s, long n, uint32_t* ws, uint32_t* winv,
                           uint32_t* zero_word, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  struct Level { long m, G; uint32_t *pre, *tot, *itot; };
  Level lv[16];
  int nl = 0;
  uint32_t* top_pre = ws;
  uint32_t* wp = ws + (size_t)NL * kTopMax;
  long m = n;
  do {
    Level L;
    L.m = m;
    L.G = ninv_groups(m, nl == 0);
    L.pre = wp;  wp += (size_t)NL * L.m;
    L.tot = wp;  wp += (size_t)NL * L.G;
    L.itot = wp; wp += (size_t)NL * L.G;
    lv[nl++] = L;
    m = L.G;
  } while (m > kMaxRoots && nl < 16);
  // up-sweeps: level 0 reads s directly, level l > 0 reads level l-1's totals
  // level 0 with one chain per thread; env MBFT_NINV_CHAINS=2: two
  // (k_ninv_up2 / k_ninv_down2) -- measured 1.4 % SLOWER in the pipelined
  // C2 loop (the chain span 0.30 -> 0.355 ms, profiles/round4_chains_ab.txt)
  static const bool two = [] {
    const char* v = getenv("MBFT_NINV_CHAINS");
    return v && atoi(v) == 2;
  }();
  for (int l = 0; l < nl; l++) {
    const Level& L = lv[l];
    const dim3 grid((unsigned)((L.G + 255) / 256)), block(256);
    if (l == 0 && two)
      hipLaunchKernelGGL(k_ninv_up2, dim3((unsigned)(((L.G + 1) / 2 + 255) / 256)), block, 0, st, s, L.m, L.G,
                         L.pre, L.tot);
    else if (l == 0)
      hipLaunchKernelGGL(k_ninv_up<true>, grid, block, 0, st, nullptr, s, L.m, L.G, L.pre, L.tot);
    else
      hipLaunchKernelGGL(k_ninv_up<false>, grid, block, 0, st, lv[l - 1].tot, nullptr, L.m, L.G,
                         L.pre, L.tot);
  }
  // the top level's totals (<= kTopMax), inverted in place by one workgroup
  // (they are its inv_tot)
  Level& top = lv[nl - 1];
  hipLaunchKernelGGL(k_ninv_top, dim3(1), dim3(kTopThreads), 0, st, top.tot, top.G, top_pre);
  top.itot = top.tot;
  // down-sweeps: level l writes the inverses of its inputs, i.e. level
  // l-1's inv_tot (or winv at level 0)
  for (int l = nl - 1; l >= 0; l--) {
    const Level& L = lv[l];
    const dim3 grid((unsigned)((L.G + 255) / 256)), block(256);
    if (l == 0 && two)
      hipLaunchKernelGGL(k_ninv_down2, dim3((unsigned)(((L.G + 1) / 2 + 255) / 256)), block, 0, st, s, L.pre,
                         L.m, L.G, L.itot, winv, zero_word);
    else if (l == 0)
      hipLaunchKernelGGL(k_ninv_down<true>, grid, block, 0, st, nullptr, s, L.pre, L.m, L.G,
                         L.itot, winv, zero_word);
    else
      hipLaunchKernelGGL(k_ninv_down<false>, grid, block, 0, st, lv[l - 1].tot, nullptr, L.pre,
                         L.m, L.G, L.itot, lv[l - 1].itot, nullptr);
  }
  return hipGetLastError();
}

// The one-launch form (k_ninv_local) for a batch on an idle GPU.
template <int PER>
hipError_t launch_ninv_local(const uint8_t* s, long n, uint32_t* winv, uint32_t* zero_word,
                             hipStream_t st, const uint32_t* ndev = nullptr) {
  const long per_block = 256L * PER;
  hipLaunchKernelGGL(k_ninv_local<PER>, dim3((unsigned)((n + per_block - 1) / per_block)), dim3(256),
                     0, st, s, n, winv, zero_word, nullptr, ndev);
  return hipGetLastError();
}

template <int PER>
hipError_t launch_ninv_block(const uint8_t* s, long n, uint32_t* winv, uint32_t* zero_word,
                             hipStream_t st) {
  const long per_block = 256L * PER;
  hipLaunchKernelGGL(k_ninv_block<PER>, dim3((unsigned)((n + per_block - 1) / per_block)), dim3(256),
                     0, st, s, n, winv, zero_word);
  return hipGetLastError();
}

// Env MBFT_NINV_PER: the chain length (per-block form: 2, 4, 8 default;
// per-wave form k_ninv_local with MBFT_NINV_FORM=wave: 2, 4, 8, 16 default).
hipError_t batch_inverse_s_local(const uint8_t* s, long n, uint32_t* winv, uint32_t* zero_word,
                                 hipStream_t st) {
  if (n <= 0) return hipSuccess;
  static const bool wave = [] {
    const char* v = getenv("MBFT_NINV_FORM");
    return v && strcmp(v, "wave") == 0;
  }();
  static const int per = [] {
    const char* v = getenv("MBFT_NINV_PER");
    return v ? atoi(v) : (wave ? 16 : 8);
  }();
  if (!wave) {
    if (per == 2) return launch_ninv_block<2>(s, n, winv, zero_word, st);
    if (per == 4) return launch_ninv_block<4>(s, n, winv, zero_word, st);
    return launch_ninv_block<8>(s, n, winv, zero_word, st);
  }
  if (per == 2) return launch_ninv_local<2>(s, n, winv, zero_word, st, nullptr);
  if (per == 8) return launch_ninv_local<8>(s, n, winv, zero_word, st, nullptr);
  if (per == 16) return launch_ninv_local<16>(s, n, winv, zero_word, st, nullptr);
  return launch_ninv_local<4>(s, n, winv, zero_word, st, nullptr);
}

// The s^-1 of a batch issued while earlier batches are in flight (the
// pipelined C2 loop): the per-wave one-launch form, chains of 16, on the
// caller's stream -- no barrier, so its waves interleave with the previous
// batch's verify waves wave by wave.  Same-box A/B in the C2 loop (3 caller
// streams, tools/steady_ab.py, profiles/round6_ninv_forms.jsonl): 0.954 ms a
// step against 0.969 (per-block form) and 1.048 (the level chain on the
// high-priority stream, round 5's default).  Env MBFT_NINV_PIPE_FORM = block |
// wave and MBFT_NINV_PIPE_PER override.
hipError_t batch_inverse_s_pipelined(const uint8_t* s, long n, uint32_t* winv, uint32_t* zero_word,
                                     hipStream_t st) {
  if (n <= 0) return hipSuccess;
  static const bool block = [] {
    const char* v = getenv("MBFT_NINV_PIPE_FORM");
    return v && strcmp(v, "block") == 0;
  }();
  static const int per = [] {
    const char* v = getenv("MBFT_NINV_PIPE_PER");
    return v ? atoi(v) : (block ? 8 : 16);
  }();
  if (block) {
    if (per == 4) return launch_ninv_block<4>(s, n, winv, zero_word, st);
    return launch_ninv_block<8>(s, n, winv, zero_word, st);
  }
  if (per == 4) return launch_ninv_local<4>(s, n, winv, zero_word, st, nullptr);
  if (per == 8) return launch_ninv_local<8>(s, n, winv, zero_word, st, nullptr);
  if (per == 32) return launch_ninv_local<32>(s, n, winv, zero_word, st, nullptr);
  return launch_ninv_local<16>(s, n, winv, zero_word, st, nullptr);
}

hipError_t sign(const uint8_t* priv, const uint32_t* key_idx, const uint8_t* e, const uint8_t* k_in,
                long n, const uint32_t* tabG, int wg, uint8_t* r_out, uint8_t* s_out,
                hipStream_t st) {
  if (n <= 0) return hipSuccess;
  SignArgs A{priv, key_idx, e, n, tabG, wg, r_out, s_out, k_in};
  hipLaunchKernelGGL(k_sign, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, A);
  return hipGetLastError();
}

// The verifier's queue + scratch buffer: the exact-path queue (n words), its
// length, then (64-word aligned) 36 planes of one word per grid thread for
// the rare comb steps' spills (comb_run).
size_t verify_scratch_offset(long n) { return ((size_t)n + 1 + 63) & ~(size_t)63; }
size_t verify_words(long n, bool pairs) {
  // (small batches: room for k_verify_quads' 4 threads an item)
  const size_t threads = (size_t)(pairs ? 4 * n : n);
  return verify_scratch_offset(n) + (size_t)4 * NL * ((threads + 255) & ~(size_t)255);
}

// k_verify_split's additions: lane-group parallel (default) or sequential
// (env MBFT_SPLIT_WIDE=0)
static bool split_wide() {
  static const bool w = [] {
    const char* v = getenv("MBFT_SPLIT_WIDE");
    return !(v && atoi(v) == 0);
  }();
  return w;
}

hipError_t verify_server(const ServerArgs& a, int servers, bool two, hipStream_t st) {
  if (a.nslots == 0 || a.nslots > (uint32_t)kSrvMaxSlots || servers <= 0 || servers > 2 * kSrvMaxSlots)
    return hipErrorInvalidValue;
  const dim3 grid((unsigned)servers), block(256);
  if (two) {
    if (split_wide())
      hipLaunchKernelGGL((k_verify_server<true, true>), grid, block, 0, st, a);
    else
      hipLaunchKernelGGL((k_verify_server<false, true>), grid, block, 0, st, a);
  } else {
    if (split_wide())
      hipLaunchKernelGGL((k_verify_server<true, false>), grid, block, 0, st, a);
    else
      hipLaunchKernelGGL((k_verify_server<false, false>), grid, block, 0, st, a);
  }
  return hipGetLastError();
}

hipError_t verify(const uint8_t* e, const uint8_t* r, const uint8_t* s, const uint32_t* slot,
                  const uint32_t* winv, const uint32_t* tabG, int wg, const KeyDesc* keys,
                  uint32_t nslots, long n, uint8_t* status, uint32_t* slowq, hipStream_t st,
                  bool host_status, bool queue_zeroed, long split_max, bool split_winv,
                  const uint32_t* ndev, uint32_t* planes_ws, int small_form) {
  if (n <= 0) return hipSuccess;
  // slowq: n + 1 words (the queue, then its length)
  VerifyArgs A{e, r, s, slot, winv, tabG, keys, nslots, wg, n, status, slowq, slowq + n,
               host_status ? 1u : 0u, slowq + verify_scratch_offset(n), 0u, ndev};
  // the smallest batches: one item per 4-wave workgroup (k_verify_split);
  // split_max < 0: env MBFT_SPLIT_MAX, default 256 (at most one wave per
  // SIMD); 0 disables (mbft_set_small_batch_form)
  static const long split_env = [] {
    const char* v = getenv("MBFT_SPLIT_MAX");
    return v ? atol(v) : 256L;
  }();
  if (split_max < 0) split_max = split_env;
  // The small batches' form past the split kernel's: small_form
  // (mbft_set_small_batch_inverse;
  // -1: env MBFT_PAIRS_PLANES, MBFT_QUADS, MBFT_QUADS_INLINE, default 2):
  // 0 one item per lane pair inverting s per lane (a wave's ~38 us of
  // divsteps on the critical path); 1 the batched per-wave s^-1 into
  // planes_ws first, then the lane pairs (same box, one batch at a time,
  // 300-4,096 items: 87-91 us against 98-101, profiles/round6_planes_ab.json);
  // 3 the planes, then one item per lane quad (k_verify_quads: 82-84 us at
  // 768-4,096 items, profiles/round6_quads_ab.json); 2 the lane quads with
  // the s^-1 by each wave inside the kernel (no separate launch, no planes:
  // 76-77 us, profiles/round6_quads_inline_ab.json)
  static const int pp_env = [] {
    const char* v = getenv("MBFT_PAIRS_PLANES");
    const char* q = getenv("MBFT_QUADS");
    const char* qi = getenv("MBFT_QUADS_INLINE");
    const int planes = v ? (atoi(v) != 0 ? 1 : 0) : 1;
    if (!planes || (q && atoi(q) == 0)) return planes;
    return qi && atoi(qi) == 0 ? 3 : 2;
  }();
  const int form = small_form < 0 ? pp_env : small_form;
  if (split_winv) {  // host s^-1 R planes (winv): the split kernel's, else unused
    // (the host stages u1, u2 after the 9 planes: 16 words an item, batch.cpp
    // host_winv_u)
    A.uhost = winv + 9 * n;
    if (n <= split_max) {
      if (split_wide())
        hipLaunchKernelGGL(k_verify_split<true>, dim3((unsigned)n), dim3(256), 0, st, A);
      else
        hipLaunchKernelGGL(k_verify_split<false>, dim3((unsigned)n), dim3(256), 0, st, A);
      return hipGetLastError();
    }
    if (form >= 2) {  // past it (MBFT_HOST_INV_MAX > split_max): the lane quads on the host's planes
      A.uhost = nullptr;
      const long qblocks = (4 * n + 255) / 256;
      A.sstride = (uint32_t)(qblocks * 256);
      hipLaunchKernelGGL(k_verify_quads<false>, dim3((unsigned)qblocks), dim3(256), 0, st, A);
      return hipGetLastError();
    }
    winv = nullptr;
    A.winv = nullptr;
    A.uhost = nullptr;
  }
  // small batches (winv null) run the exact path inline: no queue to reset
  if (winv && !queue_zeroed) {
    hipError_t me = hipMemsetAsync(slowq + n, 0, 4, st);
    if (me != hipSuccess) return me;
  }
  static const int bpc = [] {
    const char* v = getenv("MBFT_VERIFY_BPC");
    return v ? atoi(v) : 0;
  }();
  static const int ncu = [] {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return cus;
  }();
  if (!winv && n <= split_max) {
    if (split_wide())
      hipLaunchKernelGGL(k_verify_split<true>, dim3((unsigned)n), dim3(256), 0, st, A);
    else
      hipLaunchKernelGGL(k_verify_split<false>, dim3((unsigned)n), dim3(256), 0, st, A);
    return hipGetLastError();
  }
  if (!winv || ndev) {  // (a device count: the small-batch kernels only)
    // small batch, exact path inline (form: above)
    const long pblocks = (2 * n + 255) / 256;
    A.sstride = (uint32_t)(pblocks * 256);  // <= verify_words(n, true)'s threads
    if (!winv && planes_ws && form != 0) {
      if (form == 2) {
        const long qblocks = (4 * n + 255) / 256;
        A.sstride = (uint32_t)(qblocks * 256);
        A.winv = nullptr;
        hipLaunchKernelGGL(k_verify_quads<true>, dim3((unsigned)qblocks), dim3(256), 0, st, A);
        return hipGetLastError();
      }
      hipError_t e0 = launch_ninv_local<1>(s, n, planes_ws, nullptr, st, ndev);
      if (e0 != hipSuccess) return e0;
      A.winv = planes_ws;
      if (form == 3) {
        const long qblocks = (4 * n + 255) / 256;
        A.sstride = (uint32_t)(qblocks * 256);
        hipLaunchKernelGGL(k_verify_quads<false>, dim3((unsigned)qblocks), dim3(256), 0, st, A);
        return hipGetLastError();
      }
      hipLaunchKernelGGL(k_verify_pairs<false>, dim3((unsigned)pblocks), dim3(256), 0, st, A);
      return hipGetLastError();
    }
    A.winv = nullptr;
    hipLaunchKernelGGL(k_verify_pairs<true>, dim3((unsigned)pblocks), dim3(256), 0, st, A);
    return hipGetLastError();
  }
  long blocks = (n + 255) / 256;
  if (bpc > 0 && blocks > (long)bpc * ncu) blocks = (long)bpc * ncu;
  const dim3 grid((unsigned)blocks), block(256);
  A.sstride = (uint32_t)(blocks * 256);  // <= verify_words' 256-rounded n
  // MBFT_VERIFY_WAVES=4 selects the 128-VGPR build (4 waves/SIMD, spills a
  // little), =2 the 256-VGPR build (2 waves/SIMD: a 1M grid is exactly 8
  // rounds of resident blocks, no partial last round); default 3 waves/SIMD
  // (no spills).
  static const int minw = [] {
    const char* v = getenv("MBFT_VERIFY_WAVES");
    const int w = v ? atoi(v) : 3;
    return (w == 2 || w == 4) ? w : 3;
  }();
  if (minw == 3)
    hipLaunchKernelGGL((k_verify<3>), grid, block, 0, st, A);
  else if (minw == 2)
    hipLaunchKernelGGL((k_verify<2>), grid, block, 0, st, A);
  else
    hipLaunchKernelGGL((k_verify<4>), grid, block, 0, st, A);
  // the queued items: a grid of up to `sbpc` blocks per CU (env
  // MBFT_SLOW_BPC, default 4 = one wave per SIMD) that exits at once when
  // the queue is empty
  static const int sbpc = [] {
    const char* v = getenv("MBFT_SLOW_BPC");
    return v && atoi(v) > 0 ? atoi(v) : 4;
  }();
  long sblocks = (n + 255) / 256 < (long)ncu * sbpc ? (n + 255) / 256 : (long)ncu * sbpc;
  if (sblocks > blocks) sblocks = blocks;  // its threads index the same spill planes (A.sstride)
  if (winv) hipLaunchKernelGGL(k_verify_slow, dim3((unsigned)sblocks), dim3(256), 0, st, A);
  return hipGetLastError();
}

}  // namespace mbft_launch

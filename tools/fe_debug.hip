// Debug harness (not part of the library): runs the comb-table
// double-and-add chain for d * P exactly as k_table_fill does and records
// the Jacobian state (Montgomery limbs) after every group operation, and the
// intermediate values of every mixed addition, for host-side checking.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/libfe_debug.so tools/fe_debug.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../minbft_amd/csrc/ecc.h"

using namespace mbft;

struct Rec {
  uint32_t op;          // 1 = dbl, 2 = madd
  uint32_t X[9], Y[9], Z[9];
  uint32_t t[12][9];    // madd intermediates
};

__device__ void put(uint32_t* d, const fe& a) {
  for (int i = 0; i < NL; i++) d[i] = a.v[i];
}

// ec_madd with every intermediate recorded (same sequence as ecc.h)
__device__ void madd_rec(jac& o, const jac& a, const fe& x2, const fe& y2, Rec& R) {
  fe t1, t2, t3, t4, h, r, z3;
  fe_sqr(t1, a.Z);      put(R.t[0], t1);
  fe_mul(t2, t1, a.Z);  put(R.t[1], t2);
  fe_mul(t1, t1, x2);   put(R.t[2], t1);
  fe_mul(t2, t2, y2);   put(R.t[3], t2);
  fe_sub(h, t1, a.X);   put(R.t[4], h);
  fe_sub(r, t2, a.Y);   put(R.t[5], r);
  fe_mul(z3, a.Z, h);
  fe_sqr(t4, h);        put(R.t[6], t4);
  fe_mul(t3, t4, h);    put(R.t[7], t3);
  fe_mul(t4, t4, a.X);  put(R.t[8], t4);
  fe_sqr(t1, r);        put(R.t[9], t1);
  fe_sub(t1, t1, t3);
  fe_add(t2, t4, t4);
  fe_sub(o.X, t1, t2);
  fe_sub(t4, t4, o.X);  put(R.t[10], t4);
  fe_neg(t1, a.Y);      put(R.t[11], t1);
  fe_mul2(o.Y, t4, r, t3, t1);
  o.Z = z3;
}

__global__ void k_chain(const uint32_t* xy, uint32_t d, Rec* out, uint32_t* nrec) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint32_t wx[8], wy[8];
  for (int i = 0; i < 8; i++) { wx[i] = xy[i]; wy[i] = xy[8 + i]; }
  fe bx, by;
  fe_from_words(bx, wx);
  fe_from_words(by, wy);
  fe_to_mont(bx, bx);
  fe_to_mont(by, by);
  jac a;
  a.X = bx; a.Y = by;
  fe_one_mont(a.Z);
  uint32_t k = 0;
  const int top = 31 - __builtin_clz(d);
  for (int b = top - 1; b >= 0; b--) {
    ec_dbl(a, a);
    out[k].op = 1; put(out[k].X, a.X); put(out[k].Y, a.Y); put(out[k].Z, a.Z); k++;
    if ((d >> b) & 1) {
      madd_rec(a, a, bx, by, out[k]);
      out[k].op = 2; put(out[k].X, a.X); put(out[k].Y, a.Y); put(out[k].Z, a.Z); k++;
    }
  }
  *nrec = k;
}

// one ec_madd on given Jacobian (Montgomery limbs) + affine (Montgomery limbs)
__global__ void k_madd1(const uint32_t* in, Rec* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  jac a;
  fe x2, y2;
  for (int i = 0; i < NL; i++) {
    a.X.v[i] = in[i]; a.Y.v[i] = in[9 + i]; a.Z.v[i] = in[18 + i];
    x2.v[i] = in[27 + i]; y2.v[i] = in[36 + i];
  }
  jac o;
  madd_rec(o, a, x2, y2, out[0]);
  out[0].op = 2; put(out[0].X, o.X); put(out[0].Y, o.Y); put(out[0].Z, o.Z);
}

extern "C" int fe_debug_chain(const uint32_t* h_xy, uint32_t d, void* h_out, uint32_t* h_n) {
  uint32_t *dxy, *dn;
  Rec* dout;
  hipMalloc(&dxy, 64);
  hipMalloc(&dn, 4);
  hipMalloc(&dout, 64 * sizeof(Rec));
  hipMemcpy(dxy, h_xy, 64, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, 0, dxy, d, dout, dn);
  hipMemcpy(h_n, dn, 4, hipMemcpyDeviceToHost);
  hipMemcpy(h_out, dout, 64 * sizeof(Rec), hipMemcpyDeviceToHost);
  hipFree(dxy); hipFree(dn); hipFree(dout);
  return (int)hipGetLastError();
}

extern "C" int fe_debug_madd(const uint32_t* h_in, void* h_out) {
  uint32_t* din;
  Rec* dout;
  hipMalloc(&din, 45 * 4);
  hipMalloc(&dout, sizeof(Rec));
  hipMemcpy(din, h_in, 45 * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_madd1, dim3(1), dim3(64), 0, 0, din, dout);
  hipMemcpy(h_out, dout, sizeof(Rec), hipMemcpyDeviceToHost);
  hipFree(din); hipFree(dout);
  return (int)hipGetLastError();
}

extern "C" int fe_debug_rec_size() { return (int)sizeof(Rec); }

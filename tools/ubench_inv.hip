// Microbenchmark: latency of ONE modular inversion mod N on the GPU (the
// root of the batched s^-1 tree), in the forms k_ninv_top could use:
//   divsteps_salu  modinv.h on wave-uniform data (the compiler keeps it in
//                  SGPRs / the scalar ALU)
//   divsteps_valu  modinv.h on one lane's VGPR data
//   fermat_valu    x^(N-2) by fe29.h Montgomery squarings (fn_inv)
// Cycles by s_memtime around the call (one wave, idle chip); prints JSON.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../minbft_amd/csrc/fe29.h"
#include "../minbft_amd/csrc/modinv.h"

using namespace mbft;

__global__ void k_salu(const uint32_t* x, uint32_t* o, unsigned long long* cyc) {
  uint32_t w[8], r[8];
  for (int i = 0; i < 8; i++) w[i] = x[i];  // uniform address: scalar loads
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const bool ok = modinv_n_var(r, w);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    for (int i = 0; i < 8; i++) o[i] = r[i] ^ (ok ? 0u : 1u);
    cyc[0] = t1 - t0;
  }
}

__global__ void k_valu(const uint32_t* x, uint32_t* o, unsigned long long* cyc) {
  uint32_t w[8], r[8];
  for (int i = 0; i < 8; i++) w[i] = x[8 * threadIdx.x + i];  // per-lane: VGPRs
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const bool ok = modinv_n_var(r, w);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 8; i++) o[8 + i] = r[i] ^ (ok ? 0u : 1u);
  cyc[1] = t1 - t0;
}

// The same inversion on ALL 64 lanes of the wave (per-lane loaded data the
// compiler cannot prove uniform): VALU code (v_mad_i64_i32 etc.) instead of
// the scalar unit's multi-instruction 64-bit arithmetic.
__global__ void k_valu64(const uint32_t* x, uint32_t* o, unsigned long long* cyc) {
  uint32_t w[8], r[8];
  __shared__ uint32_t sh[8];
  if (threadIdx.x < 8) sh[threadIdx.x] = x[threadIdx.x];
  __syncthreads();
  for (int i = 0; i < 8; i++) {
    w[i] = sh[i];
    asm volatile("" : "+v"(w[i]));  // divergent to the compiler (k_ninv_top's form)
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const bool ok = modinv_n_var(r, w);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    for (int i = 0; i < 8; i++) o[240 + i] = r[i] ^ (ok ? 0u : 1u);
    cyc[8] = t1 - t0;
  }
}

__global__ void k_fermat(const uint32_t* x, uint32_t* o, unsigned long long* cyc) {
  uint32_t w[8];
  for (int i = 0; i < 8; i++) w[i] = x[8 * threadIdx.x + i];
  if (threadIdx.x != 0) return;
  fe a, r;
  fe_from_words(a, w);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  fn_to_mont(a, a);
  fn_inv(r, a);
  fn_from_mont(r, r);
  fn_canon(r);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  uint32_t rw[8];
  fe_to_words(rw, r);
  for (int i = 0; i < 8; i++) o[16 + i] = rw[i];
  cyc[2] = t1 - t0;
}

// Latency of 64 dependent mod-N Montgomery multiplies on one wave (the
// chains of the batched inverse), and of 64 back-to-back dependent global
// loads (pointer chase), in s_memtime and s_memrealtime (100 MHz) ticks.
__global__ void k_mul(const uint32_t* x, uint32_t* o, unsigned long long* cyc) {
  fe a, r;
  uint32_t w[8];
  for (int i = 0; i < 8; i++) w[i] = x[8 * threadIdx.x + i];
  fe_from_words(a, w);
  r = a;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
  for (int k = 0; k < 64; k++) fn_mul(r, r, a);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t acc = 0;
  for (int i = 0; i < NL; i++) acc ^= r.v[i];
  o[24 + threadIdx.x] = acc;
  if (threadIdx.x == 0) {
    cyc[3] = t1 - t0;
    cyc[4] = r1 - r0;
  }
}

// The two parts of one divsteps batch, timed apart: 16 x divsteps_30_var on
// a running (f, g), and 16 x the (d, e) + (f, g) matrix updates.
__global__ void k_parts(const uint32_t* x, uint32_t* o, unsigned long long* cyc) {
  uint32_t w[8];
  for (int i = 0; i < 8; i++) w[i] = x[8 * threadIdx.x + i];
  if (threadIdx.x != 0) return;
  s30 M, d, e, f, g;
  s30_modulus(M);
  s30_from_words(g, w);
  f = M;
  for (int i = 0; i < 9; i++) d.v[i] = e.v[i] = 0;
  e.v[0] = 1;
  trans2x2 t{1, 0, 0, 1};
  int32_t eta = -1;
  uint32_t f0 = (uint32_t)f.v[0], g0 = (uint32_t)g.v[0];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int it = 0; it < 16; it++) {
    eta = divsteps_30_var(eta, f0 | 1u, g0, t);
    f0 = (uint32_t)t.u * 2654435761u + (uint32_t)t.q;
    g0 = (uint32_t)t.v * 40503u + (uint32_t)t.r;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int it = 0; it < 16; it++) {
    update_de_30(d, e, t, M);
    update_fg_30(f, g, t);
  }
  const unsigned long long t2 = __builtin_amdgcn_s_memtime();
  uint32_t acc = (uint32_t)eta;
  for (int i = 0; i < 9; i++) acc ^= (uint32_t)(d.v[i] ^ e.v[i] ^ f.v[i] ^ g.v[i]);
  o[200] = acc;
  cyc[6] = t1 - t0;
  cyc[7] = t2 - t1;
}

__global__ void k_chase(const uint32_t* nxt, uint32_t* o, unsigned long long* cyc) {
  uint32_t i = threadIdx.x;
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
  for (int k = 0; k < 64; k++) i = nxt[i];
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  o[100 + threadIdx.x] = i;
  if (threadIdx.x == 0) cyc[5] = r1 - r0;
}

int main() {
  // x = 0x1234...: any value in [1, N)
  uint32_t hx[64 * 8];
  for (int i = 0; i < 64 * 8; i++) hx[i] = 0x9E3779B9u * (uint32_t)(i % 8 + 1);
  hx[7] &= 0x7FFFFFFFu;
  uint32_t *dx, *dout;
  unsigned long long* dc;
  hipMalloc(&dx, sizeof(hx));
  hipMalloc(&dout, 256 * 4);
  hipMalloc(&dc, 8 * 9);
  // pointer chase over 64 MiB with a large stride (HBM, not cache)
  const size_t nchase = (size_t)16 << 20;
  uint32_t* dn;
  hipMalloc(&dn, nchase * 4);
  {
    uint32_t* hn = (uint32_t*)malloc(nchase * 4);
    for (size_t i = 0; i < nchase; i++) hn[i] = (uint32_t)((i + 1048583u * 64u + 64u) % nchase);
    hipMemcpy(dn, hn, nchase * 4, hipMemcpyHostToDevice);
    free(hn);
  }
  hipMemcpy(dx, hx, sizeof(hx), hipMemcpyHostToDevice);
  for (int rep = 0; rep < 3; rep++) {
    hipLaunchKernelGGL(k_salu, dim3(1), dim3(64), 0, 0, dx, dout, dc);
    hipLaunchKernelGGL(k_valu, dim3(1), dim3(64), 0, 0, dx, dout, dc);
    hipLaunchKernelGGL(k_valu64, dim3(1), dim3(64), 0, 0, dx, dout, dc);
    hipLaunchKernelGGL(k_fermat, dim3(1), dim3(64), 0, 0, dx, dout, dc);
    hipLaunchKernelGGL(k_mul, dim3(1), dim3(64), 0, 0, dx, dout, dc);
    hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, 0, dn, dout, dc);
    hipLaunchKernelGGL(k_parts, dim3(1), dim3(64), 0, 0, dx, dout, dc);
  }
  hipDeviceSynchronize();
  unsigned long long c[9];
  uint32_t o[248];
  hipMemcpy(c, dc, sizeof(c), hipMemcpyDeviceToHost);
  hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost);
  int agree = 1;
  for (int i = 0; i < 8; i++) agree &= o[i] == o[8 + i] && o[i] == o[16 + i] && o[i] == o[240 + i];
  printf("{\"divsteps_salu_cycles\": %llu, \"divsteps_valu_cycles\": %llu, \"fermat_valu_cycles\": %llu, "
         "\"results_agree\": %d, \"fn_mul_x64_memtime\": %llu, \"fn_mul_x64_realtime_100MHz\": %llu, "
         "\"load_chase_x64_realtime_100MHz\": %llu, \"divsteps30_x16_memtime\": %llu, "
         "\"updates_x16_memtime\": %llu, \"divsteps_valu64_cycles\": %llu}\n",
         c[0], c[1], c[2], agree, c[3], c[4], c[5], c[6], c[7], c[8]);
  return agree ? 0 : 1;
}

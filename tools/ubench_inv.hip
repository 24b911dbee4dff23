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

int main() {
  // x = 0x1234...: any value in [1, N)
  uint32_t hx[64 * 8];
  for (int i = 0; i < 64 * 8; i++) hx[i] = 0x9E3779B9u * (uint32_t)(i % 8 + 1);
  hx[7] &= 0x7FFFFFFFu;
  uint32_t *dx, *dout;
  unsigned long long* dc;
  hipMalloc(&dx, sizeof(hx));
  hipMalloc(&dout, 24 * 4);
  hipMalloc(&dc, 3 * 8);
  hipMemcpy(dx, hx, sizeof(hx), hipMemcpyHostToDevice);
  for (int rep = 0; rep < 3; rep++) {
    hipLaunchKernelGGL(k_salu, dim3(1), dim3(64), 0, 0, dx, dout, dc);
    hipLaunchKernelGGL(k_valu, dim3(1), dim3(64), 0, 0, dx, dout, dc);
    hipLaunchKernelGGL(k_fermat, dim3(1), dim3(64), 0, 0, dx, dout, dc);
  }
  hipDeviceSynchronize();
  unsigned long long c[3];
  uint32_t o[24];
  hipMemcpy(c, dc, sizeof(c), hipMemcpyDeviceToHost);
  hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost);
  int agree = 1;
  for (int i = 0; i < 8; i++) agree &= o[i] == o[8 + i] && o[i] == o[16 + i];
  printf("{\"divsteps_salu_cycles\": %llu, \"divsteps_valu_cycles\": %llu, \"fermat_valu_cycles\": %llu, "
         "\"results_agree\": %d}\n", c[0], c[1], c[2], agree);
  return agree ? 0 : 1;
}

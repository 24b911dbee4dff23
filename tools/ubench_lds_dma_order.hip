// Does s_waitcnt vmcnt(N > 0) order a ds_read behind an older
// global_load_lds_dwordx4 when a younger one is still in flight?  Each wave
// keeps two LDS slots and two cooperative-style gathers of random 64-B table
// entries in flight (the k_verify two-deep pipeline, kernels.hip
// comb_verify_fast2), reads the older slot after vmcnt(4) (or vmcnt(0)), and
// counts 16-B chunks whose content is not the expected function of the entry
// index.  Diagnostic only (round 5).
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_lds_dma_order tools/ubench_lds_dma_order.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

constexpr unsigned kWaitVm4 = 0x0F74, kWaitVm0 = 0x0F70, kWaitLgkm0 = 0xC07F;

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

template <bool PARTIAL>
__global__ void __launch_bounds__(256) k(const uint4* __restrict__ tab, uint32_t nent, int steps,
                                         unsigned long long* bad) {
  __shared__ uint4 slot[2][4][256];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint4* s0 = slot[0][w];
  uint4* s1 = slot[1][w];
  uint32_t seed = mix(blockIdx.x * 256 + threadIdx.x);
  uint32_t idx[2];
  auto issue = [&](uint4* buf, uint32_t e) __attribute__((always_inline)) {
    __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
    const uint64_t a = reinterpret_cast<uint64_t>(tab + 4ull * e);
    for (int q = 0; q < 4; q++) {
      const int from = (16 * q + (lane >> 2)) << 2;
      const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(from, (int)(uint32_t)a);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(from, (int)(uint32_t)(a >> 32));
      const uint4* src = reinterpret_cast<const uint4*>(((uint64_t)hi << 32) | lo) + (lane & 3);
      __builtin_amdgcn_global_load_lds(src, buf + 64 * q, 16, 0, 2);
    }
  };
  idx[0] = (seed = mix(seed)) % nent;
  issue(s0, idx[0]);
  idx[1] = (seed = mix(seed)) % nent;
  issue(s1, idx[1]);
  unsigned long long nbad = 0;
  uint32_t acc = 0;
  for (int k = 0; k < steps; k++) {
    uint4* buf = (k & 1) ? s1 : s0;
    if (PARTIAL)
      __builtin_amdgcn_s_waitcnt(kWaitVm4);
    else
      __builtin_amdgcn_s_waitcnt(kWaitVm0);
    const uint32_t a = (uint32_t)(uintptr_t)(buf + 4 * lane);
    uint4 c0, c1, c2, c3;
    asm volatile(
        "ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\tds_read_b128 %2, %4 offset:32\n\t"
        "ds_read_b128 %3, %4 offset:48\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(c0), "=&v"(c1), "=&v"(c2), "=&v"(c3) : "v"(a) : "memory");
    const uint32_t e = idx[k & 1];
    const uint4 c[4] = {c0, c1, c2, c3};
    for (int q = 0; q < 4; q++) {
      const uint32_t want = mix(e * 4 + q);
      nbad += (c[q].x != want || c[q].y != (want ^ 1u) || c[q].z != (want ^ 2u) || c[q].w != (want ^ 3u));
      acc += c[q].x;
    }
    idx[k & 1] = (seed = mix(seed ^ acc)) % nent;
    issue(buf, idx[k & 1]);
    // some VALU work between steps (the mixed addition's role)
    for (int j = 0; j < 200; j++) acc = acc * 1664525u + 1013904223u;
    seed ^= acc & 1u;
  }
  __builtin_amdgcn_s_waitcnt(kWaitVm0);
  if (nbad) atomicAdd(bad, nbad);
}

__global__ void fill(uint4* tab, size_t nent) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nent * 4; i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t v = mix((uint32_t)i);
    tab[i] = make_uint4(v, v ^ 1u, v ^ 2u, v ^ 3u);
  }
}

int main(int argc, char** argv) {
  const size_t nent = argc > 1 ? strtoull(argv[1], 0, 10) : (size_t)1 << 26;  // 64M entries = 4 GiB
  uint4* tab;
  unsigned long long* bad;
  if (hipMalloc(&tab, nent * 64) != hipSuccess || hipMalloc(&bad, 16) != hipSuccess) return 1;
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, tab, nent);
  for (int partial = 1; partial >= 0; partial--) {
    unsigned long long tot = 0, reads = 0;
    for (int rep = 0; rep < 20; rep++) {
      hipMemset(bad, 0, 8);
      if (partial)
        hipLaunchKernelGGL((k<true>), dim3(4096), dim3(256), 0, 0, tab, (uint32_t)nent, 64, bad);
      else
        hipLaunchKernelGGL((k<false>), dim3(4096), dim3(256), 0, 0, tab, (uint32_t)nent, 64, bad);
      unsigned long long h = 0;
      hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
      tot += h;
      reads += 4096ull * 256 * 64 * 4;
    }
    printf("%s: %llu stale 16-B chunks of %llu read\n", partial ? "vmcnt(4)" : "vmcnt(0)", tot, reads);
  }
  return 0;
}

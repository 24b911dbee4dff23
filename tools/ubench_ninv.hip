// Latency of the one-launch batched s^-1 (kernels.hip k_ninv_local) on
// n = 1M random s values, for chains of PER = 2, 4, 8 items per lane
// (HIP events around each launch, idle GPU).  JSON lines.  (A phase probe
// with s_memrealtime stamps put the wave inversion at ~43 us of ~90 us at
// PER = 8, chain up ~20 us, chain down ~15 us: profiles/round3_ubench_ninv.jsonl.)
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -o tools/ubench_ninv tools/ubench_ninv.hip
#include "../minbft_amd/csrc/kernels.hip"

#include <algorithm>
#include <random>
#include <vector>

using namespace mbft;

// The wave-cooperative root inversion alone: every wave inverts one value
// (its index-dependent x, the same on every lane).
__global__ void __launch_bounds__(256) k_inv_only(const uint8_t* s, uint32_t* out, long waves) {
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (wave >= waves) return;
  uint32_t w[8], iw[8];
  load_be256(w, s + 32 * wave);
  w[7] &= 0x7fffffffu;
  const bool ok = modinv_n_var_wave(iw, w);
  if (__lane_id() == 0)
    for (int k = 0; k < 8; k++) out[8 * wave + k] = iw[k] ^ (ok ? 0u : 1u);
}

int main() {
  const long n = 1 << 20;
  std::mt19937_64 rng(7);
  std::vector<uint8_t> hs(32 * n);
  for (auto& b : hs) b = (uint8_t)rng();
  for (long i = 0; i < n; i++) hs[32 * i] &= 0x7f;  // < N
  uint8_t* ds;
  uint32_t *winv, *zw;
  uint64_t* st;
  const long waves = n / (64 * 2);
  hipMalloc(&ds, 32 * n);
  hipMalloc(&winv, 36 * n);
  hipMalloc(&zw, 4);
  hipMalloc(&st, 8 * 6 * waves);
  hipMemcpy(ds, hs.data(), 32 * n, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (long waves : {1L, 256L, 1024L, 2048L}) {
    for (int rep = 0; rep < 3; rep++) {
      float ms = 0;
      hipEventRecord(a, 0);
      hipLaunchKernelGGL(k_inv_only, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, 0, ds, winv, waves);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      hipEventElapsedTime(&ms, a, b);
      if (rep == 2) printf("{\"kernel\": \"inversion only\", \"waves\": %ld, \"event_us\": %.1f}\n", waves, ms * 1e3);
    }
  }
  for (int per : {8, 16}) {
    const long pw = n / (64 * per);
    for (int rep = 0; rep < 3; rep++) {
      float ms = 0;
      hipEventRecord(a, 0);
      if (per == 8)
        hipLaunchKernelGGL((k_ninv_local<8, true>), dim3((unsigned)(n / 2048)), dim3(256), 0, 0, ds, n, winv, zw, st);
      else
        hipLaunchKernelGGL((k_ninv_local<16, true>), dim3((unsigned)(n / 4096)), dim3(256), 0, 0, ds, n, winv, zw, st);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      hipEventElapsedTime(&ms, a, b);
      if (rep < 2) continue;
      std::vector<uint64_t> h(6 * pw);
      hipMemcpy(h.data(), st, 8 * 6 * pw, hipMemcpyDeviceToHost);
      std::vector<double> ph[5];
      uint64_t t0 = ~0ull, t5 = 0;
      for (long w = 0; w < pw; w++) {
        t0 = std::min(t0, h[6 * w]);
        t5 = std::max(t5, h[6 * w + 5]);
        for (int k = 0; k < 5; k++) ph[k].push_back((h[6 * w + k + 1] - h[6 * w + k]) * 0.01);
      }
      printf("{\"kernel\": \"probe PER=%d\", \"event_us\": %.1f, \"span_us\": %.1f", per, ms * 1e3, (t5 - t0) * 0.01);
      const char* nm[5] = {"chain_up", "butterfly_up", "inversion", "butterfly_down", "chain_down"};
      for (int k = 0; k < 5; k++) {
        std::sort(ph[k].begin(), ph[k].end());
        printf(", \"%s_p50\": %.2f, \"%s_max\": %.2f", nm[k], ph[k][pw / 2], nm[k], ph[k].back());
      }
      printf("}\n");
    }
  }
  // the per-workgroup form (k_ninv_block): phases from thread 0 of each block
  for (int per : {4, 8}) {
    const long blocks = n / (256 * per);
    for (int rep = 0; rep < 3; rep++) {
      float ms = 0;
      hipEventRecord(a, 0);
      if (per == 4)
        hipLaunchKernelGGL((k_ninv_block<4, true>), dim3((unsigned)blocks), dim3(256), 0, 0, ds, n, winv, zw, st);
      else
        hipLaunchKernelGGL((k_ninv_block<8, true>), dim3((unsigned)blocks), dim3(256), 0, 0, ds, n, winv, zw, st);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      hipEventElapsedTime(&ms, a, b);
      if (rep < 2) continue;
      std::vector<uint64_t> h(5 * blocks);
      hipMemcpy(h.data(), st, 8 * 5 * blocks, hipMemcpyDeviceToHost);
      std::vector<double> ph[4];
      uint64_t t0 = ~0ull, t4 = 0;
      for (long w = 0; w < blocks; w++) {
        t0 = std::min(t0, h[5 * w]);
        t4 = std::max(t4, h[5 * w + 4]);
        for (int k = 0; k < 4; k++) ph[k].push_back((h[5 * w + k + 1] - h[5 * w + k]) * 0.01);
      }
      printf("{\"kernel\": \"probe k_ninv_block<%d>\", \"event_us\": %.1f, \"span_us\": %.1f", per, ms * 1e3,
             (t4 - t0) * 0.01);
      const char* nm[4] = {"loads_chain_up", "tree_inversion_tree", "fetch", "chain_down"};
      for (int k = 0; k < 4; k++) {
        std::sort(ph[k].begin(), ph[k].end());
        printf(", \"%s_p50\": %.2f, \"%s_max\": %.2f", nm[k], ph[k][blocks / 2], nm[k], ph[k].back());
      }
      // start skew: when blocks begin relative to the first
      std::vector<double> st0;
      for (long w = 0; w < blocks; w++) st0.push_back((h[5 * w] - t0) * 0.01);
      std::sort(st0.begin(), st0.end());
      printf(", \"start_p50\": %.2f, \"start_max\": %.2f}\n", st0[blocks / 2], st0.back());
    }
  }
  for (int rep = 0; rep < 3; rep++) {
    float ms = 0;
    hipEventRecord(a, 0);
    mbft_launch::launch_ninv_local<2>(ds, n, winv, zw, 0);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("{\"kernel\": \"k_ninv_local<2>\", \"n\": %ld, \"event_us\": %.1f}\n", n, ms * 1e3);
    hipEventRecord(a, 0);
    mbft_launch::launch_ninv_local<4>(ds, n, winv, zw, 0);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("{\"kernel\": \"k_ninv_local<4>\", \"n\": %ld, \"event_us\": %.1f}\n", n, ms * 1e3);
    hipEventRecord(a, 0);
    mbft_launch::launch_ninv_local<8>(ds, n, winv, zw, 0);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("{\"kernel\": \"k_ninv_local<8>\", \"n\": %ld, \"event_us\": %.1f}\n", n, ms * 1e3);
    hipEventRecord(a, 0);
    mbft_launch::launch_ninv_local<16>(ds, n, winv, zw, 0);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("{\"kernel\": \"k_ninv_local<16>\", \"n\": %ld, \"event_us\": %.1f}\n", n, ms * 1e3);
  }
  return 0;
}

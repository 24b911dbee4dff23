// Host-side microbenchmark of the batch pipeline's per-call work (DER decode
// of the tag, digest prefix copy, staging writes) over 1M C2-shaped calls,
// at 1..T threads, into pageable and into hipHostMalloc'd staging.  Prints
// one JSON line per configuration.  Build: hipcc -O3 -o tools/host_prepare_bench
// tools/host_prepare_bench.cpp minbft_amd/csrc/der.cpp
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../include/minbft_gpu.h"

int main(int argc, char** argv) {
  const size_t n = 1 << 20;
  std::vector<uint8_t> msgs(n * 47), tags(n * 72);
  std::vector<mbft_item> items(n);
  for (size_t i = 0; i < n; i++) {
    uint8_t* t = &tags[72 * i];
    t[0] = 0x30; t[1] = 68; t[2] = 2; t[3] = 32;
    for (int k = 0; k < 32; k++) t[4 + k] = (uint8_t)((i * 7 + k + 1) & 0x7f);
    t[36] = 2; t[37] = 32;
    for (int k = 0; k < 32; k++) t[38 + k] = (uint8_t)((i * 3 + k + 1) & 0x7f);
    items[i] = mbft_item{3, 0, &msgs[47 * i], 47, t, 70};
  }
  uint8_t* pin = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(&pin), 100 * n, hipHostMallocDefault) != hipSuccess) return 1;
  std::vector<uint8_t> page(100 * n);
  for (int pinned = 0; pinned < 2; pinned++) {
    uint8_t* base = pinned ? pin : page.data();
    memset(base, 0, 100 * n);
    for (int T : {1, 2, 4, 8, 16, 32}) {
      double best = 1e30;
      for (int rep = 0; rep < 3; rep++) {
        auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> th;
        for (int t = 0; t < T; t++)
          th.emplace_back([&, t] {
            const size_t a = n * t / T, b = n * (t + 1) / T;
            for (size_t i = a; i < b; i++) {
              size_t c = 0;
              uint8_t* e = base + 32 * i;
              mbft_der_parse_sig(items[i].tag, items[i].tag_len, base + 32 * (n + i),
                                 base + 32 * (2 * n + i), &c);
              memcpy(e, items[i].msg, 32);
              reinterpret_cast<uint32_t*>(base + 96 * n)[i] = 0;
            }
          });
        for (auto& x : th) x.join();
        const double ms =
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (ms < best) best = ms;
      }
      printf("{\"pinned\": %d, \"threads\": %d, \"ms_per_1M\": %.3f}\n", pinned, T, best);
    }
  }
  (void)hipHostFree(pin);
  return 0;
}

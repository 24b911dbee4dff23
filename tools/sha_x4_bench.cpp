// Host SHA-256 throughput: one stream at a time (sha256) against four
// interleaved (sha256_many) on the small route's digest shapes -- 256-byte
// operations, 59 / 70-byte PREPARE / COMMIT AuthenBytes, the 48-byte USIG
// chain input -- and a check that both agree.
//   g++ -O2 -std=c++17 -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ tools/sha_x4_bench.cpp \
//       minbft_amd/csrc/sha256_host.cpp -o /tmp/sha_x4_bench
#include <chrono>
#include <cstdio>
#include <vector>

#include "../minbft_amd/csrc/host_internal.h"

int main() {
  for (size_t len : {48, 59, 70, 256}) {
    const size_t m = 4096;
    std::vector<uint8_t> data(m * len), o1(32 * m), o4(32 * m);
    for (size_t i = 0; i < data.size(); i++) data[i] = (uint8_t)(i * 131 + (i >> 7));
    std::vector<const uint8_t*> p(m);
    std::vector<size_t> n(m, len);
    std::vector<uint8_t*> o(m);
    for (size_t i = 0; i < m; i++) {
      p[i] = data.data() + i * len;
      o[i] = o4.data() + 32 * i;
    }
    double best1 = 1e9, best4 = 1e9;
    for (int r = 0; r < 20; r++) {
      auto a = std::chrono::steady_clock::now();
      for (size_t i = 0; i < m; i++) mbft_host::sha256(p[i], len, o1.data() + 32 * i);
      auto b = std::chrono::steady_clock::now();
      mbft_host::sha256_many(m, p.data(), n.data(), o.data());
      auto c = std::chrono::steady_clock::now();
      best1 = std::min(best1, std::chrono::duration<double, std::nano>(b - a).count() / m);
      best4 = std::min(best4, std::chrono::duration<double, std::nano>(c - b).count() / m);
    }
    printf("{\"bytes\": %zu, \"one_ns\": %.1f, \"x4_ns\": %.1f, \"equal\": %s}\n", len, best1, best4,
           o1 == o4 ? "true" : "false");
  }
}

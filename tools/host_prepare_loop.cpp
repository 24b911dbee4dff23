// CPU-only timing of the batch pipeline's host part as the library runs it:
// mbft_host::prepare_item over 1M C2-shaped calls (ClientAuthen, 47-B
// message, 70-B DER tag) on the library's worker pool, writing the same
// staging layout.  No GPU needed (the context is built by hand, no HIP call
// is made).  Build (from the repo root):
//   hipcc -O3 -std=c++17 -Iinclude -o tools/host_prepare_loop tools/host_prepare_loop.cpp \
//     minbft_amd/csrc/batch.cpp minbft_amd/csrc/der.cpp minbft_amd/csrc/host.cpp \
//     minbft_amd/csrc/messages.cpp
#include <sched.h>

#include <chrono>
#include <cstdio>
#include <vector>

#include "../minbft_amd/csrc/host_internal.h"

using namespace mbft_host;

int main(int argc, char** argv) {
  cpu_set_t cs;
  if (sched_getaffinity(0, sizeof cs, &cs) == 0) printf("{\"affinity_cpus\": %d}\n", CPU_COUNT(&cs));
  const size_t n = argc > 1 ? (size_t)atol(argv[1]) : (size_t)1 << 20;
  std::vector<uint8_t> msgs(n * 47), tags(n * 72);
  std::vector<mbft_item> items(n);
  for (size_t i = 0; i < n; i++) {
    uint8_t* t = &tags[72 * i];
    t[0] = 0x30; t[1] = 68; t[2] = 2; t[3] = 32;
    for (int k = 0; k < 32; k++) t[4 + k] = (uint8_t)((i * 7 + k + 1) & 0x7f);
    t[36] = 2; t[37] = 32;
    for (int k = 0; k < 32; k++) t[38 + k] = (uint8_t)((i * 3 + k + 1) & 0x7f);
    for (int k = 0; k < 47; k++) msgs[47 * i + k] = (uint8_t)(i + k);
    items[i] = mbft_item{MBFT_ROLE_CLIENT, 0, &msgs[47 * i], 47, t, 70};
  }
  mbft_ctx* c = new mbft_ctx();
  SlotInfo si{};
  si.valid = true;
  c->slots.push_back(si);
  c->roles[MBFT_ROLE_CLIENT][0] = KeyEntry{0};
  std::vector<uint8_t> stage(100 * n);
  std::vector<CallInfo> info(n);
  {
    // floor: the DER decode and the digest copy alone, one thread
    double best = 1e30;
    for (int rep = 0; rep < 5; rep++) {
      const auto t0 = std::chrono::steady_clock::now();
      uint8_t* e = stage.data();
      uint8_t* r = e + 32 * n;
      uint8_t* s = r + 32 * n;
      uint32_t* sl = reinterpret_cast<uint32_t*>(s + 32 * n);
      for (size_t i = 0; i < n; i++) {
        size_t cons = 0;
        mbft_der_parse_sig(items[i].tag, items[i].tag_len, r + 32 * i, s + 32 * i, &cons);
        memcpy(e + 32 * i, items[i].msg, 32);
        sl[i] = 0;
      }
      const double ms =
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (ms < best) best = ms;
    }
    printf("{\"floor_threads\": 1, \"ms_per_%zu\": %.3f}\n", n, best);
  }
  for (int T : {1, 2, 4, 8, 16, 24, 32}) {
    Pool pool(T - 1);
    double best = 1e30;
    for (int rep = 0; rep < 5; rep++) {
      const auto t0 = std::chrono::steady_clock::now();
      pool.run(T, [&](int t) {
        Lookup lk;
        const size_t a = n * t / T, b = n * (t + 1) / T;
        uint8_t* e = stage.data();
        uint8_t* r = e + 32 * n;
        uint8_t* s = r + 32 * n;
        uint32_t* sl = reinterpret_cast<uint32_t*>(s + 32 * n);
        for (size_t i = a; i < b; i++)
          prepare_item(c, items[i], info[i], e + 32 * i, r + 32 * i, s + 32 * i, sl + i, false, lk);
      });
      const double ms =
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (ms < best) best = ms;
    }
    printf("{\"threads\": %d, \"ms_per_%zu\": %.3f, \"ns_per_item_thread\": %.1f}\n", T, n, best,
           best * 1e6 * T / n);
  }
  return 0;
}

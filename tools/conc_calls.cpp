// Native driver for concurrent single calls (bench.py single_calls, the
// `native` leg): `threads` OS threads call mbft_verify_message_authen_tag
// (passed as a function pointer, so this file needs no link against the
// library) over their own slice of the calls, all released at once.  A Go
// replica's goroutines reach the C-ABI the same way (one cgo call per
// VerifyMessageAuthenTag, sample/authentication/authenticator.go:121); the
// Python leg of the bench measures the interpreter's lock as much as the
// library.
//
//   hipcc -O2 -std=c++17 -shared -fPIC -o tools/libconc_calls.so tools/conc_calls.cpp
#include <atomic>
#include <chrono>
#include <cstddef>
#include <cstdint>
#include <thread>
#include <vector>

typedef int (*verify_fn)(void* ctx, uint32_t role, uint32_t id, const uint8_t* msg,
                         size_t msg_len, const uint8_t* tag, size_t tag_len);

// Call i: role[i], id[i], msg bytes [msg_off[i], msg_off[i+1]), tag bytes
// [tag_off[i], tag_off[i+1]).  Thread t makes calls t*per .. (t+1)*per - 1
// one after another; rc[i] receives each return value.  Returns the seconds
// from the release of the threads to the last thread's end.
extern "C" double conc_calls_run(void* fn, void* ctx, int threads, int per,
                                 const uint32_t* role, const uint32_t* id, const uint8_t* msgs,
                                 const uint64_t* msg_off, const uint8_t* tags,
                                 const uint64_t* tag_off, int32_t* rc) {
  const verify_fn f = reinterpret_cast<verify_fn>(fn);
  std::atomic<int> ready{0};
  std::atomic<bool> go{false};
  std::vector<std::thread> th;
  th.reserve((size_t)threads);
  for (int t = 0; t < threads; t++) {
    th.emplace_back([&, t] {
      ready.fetch_add(1);
      while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
      for (int k = 0; k < per; k++) {
        const size_t i = (size_t)t * (size_t)per + (size_t)k;
        rc[i] = f(ctx, role[i], id[i], msgs + msg_off[i], msg_off[i + 1] - msg_off[i],
                  tags + tag_off[i], tag_off[i + 1] - tag_off[i]);
      }
    });
  }
  while (ready.load() < threads) std::this_thread::yield();
  const auto a = std::chrono::steady_clock::now();
  go.store(true, std::memory_order_release);
  for (auto& x : th) x.join();
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
}

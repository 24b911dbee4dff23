// Native driver for message-check latency (bench.py go_wiring_latency and
// c5_proxy): the C-ABI sequence of the Go core's batched stream loop
// (go/core/message-handling-batch.go, go/gpuauth/messages.go) -- per window
// of messages already received: mbft_check_messages_flat, then
// mbft_resolve_message for each message in order, then mbft_msg_batch_free --
// timed per window with the steady clock, from OS threads (how goroutines
// reach the C-ABI through cgo; no interpreter in the timed region).  The
// entry points are passed as function pointers, so this file needs no link
// against the library.
//
//   hipcc -O2 -std=c++17 -shared -fPIC -o tools/libmsg_latency.so tools/msg_latency.cpp
#include <sys/resource.h>

#include <atomic>
#include <chrono>
#include <cstddef>
#include <cstdint>
#include <thread>
#include <vector>

typedef int (*check_fn)(void* ctx, const void* recs, size_t n, const uint8_t* bytes, size_t nbytes,
                        uint32_t n_replicas, void** out);
typedef int (*resolve_fn)(void* ctx, void* batch, size_t i);
typedef void (*free_fn)(void* batch);

static constexpr size_t kRecBytes = 104;  // sizeof(mbft_msg_rec)

// Process CPU seconds (user + system, every thread) over the last
// msg_latency_run, release to join.
static double g_cpu_s = 0;

static double process_cpu_s() {
  struct rusage u;
  getrusage(RUSAGE_SELF, &u);
  return (double)u.ru_utime.tv_sec + 1e-6 * (double)u.ru_utime.tv_usec + (double)u.ru_stime.tv_sec +
         1e-6 * (double)u.ru_stime.tv_usec;
}

extern "C" double msg_latency_cpu_s() { return g_cpu_s; }

// Window w: records [rec_off[w], rec_off[w+1]) of `recs` (104 B each) over the
// arena bytes [byte_off[w], byte_off[w+1]) (the records' offsets are
// relative to their window's arena).  Thread t runs windows
// [first[t], first[t+1]) one after another; all threads are released at
// once.  results[i] = message i's resolve result; lat_us[w] = window w's
// check + resolves + free.  Returns the seconds from the release to the last
// thread's end, or -1 - w if window w's check failed (rc in results[rec_off[w]]).
extern "C" double msg_latency_run(void* check, void* resolve, void* bfree, void* ctx, uint32_t n_replicas,
                                  int threads, const int* first, const uint8_t* recs,
                                  const uint64_t* rec_off, const uint8_t* bytes, const uint64_t* byte_off,
                                  int32_t* results, double* lat_us) {
  const check_fn ck = reinterpret_cast<check_fn>(check);
  const resolve_fn rs = reinterpret_cast<resolve_fn>(resolve);
  const free_fn fr = reinterpret_cast<free_fn>(bfree);
  std::atomic<int> ready{0}, failed{-1};
  std::atomic<bool> go{false};
  std::vector<std::thread> th;
  for (int t = 0; t < threads; t++) {
    th.emplace_back([&, t] {
      ready.fetch_add(1);
      while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
      for (int w = first[t]; w < first[t + 1]; w++) {
        const uint64_t r0 = rec_off[w], r1 = rec_off[w + 1];
        const auto a = std::chrono::steady_clock::now();
        void* b = nullptr;
        const int rc = ck(ctx, recs + kRecBytes * r0, (size_t)(r1 - r0), bytes + byte_off[w],
                          (size_t)(byte_off[w + 1] - byte_off[w]), n_replicas, &b);
        if (rc != 0) {
          results[r0] = rc;
          failed.store(w);
          return;
        }
        for (uint64_t i = r0; i < r1; i++) results[i] = rs(ctx, b, (size_t)(i - r0));
        fr(b);
        lat_us[w] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
      }
    });
  }
  while (ready.load() < threads) std::this_thread::yield();
  const double c0 = process_cpu_s();
  const auto a = std::chrono::steady_clock::now();
  go.store(true, std::memory_order_release);
  for (auto& x : th) x.join();
  g_cpu_s = process_cpu_s() - c0;
  if (failed.load() >= 0) return -1.0 - failed.load();
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
}

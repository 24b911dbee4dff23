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
#include <sys/prctl.h>
#include <sys/resource.h>
#include <time.h>

#include <atomic>
#include <chrono>
#include <cstddef>
#include <cstdint>
#include <thread>
#include <vector>

typedef int (*verify_fn)(void* ctx, uint32_t role, uint32_t id, const uint8_t* msg,
                         size_t msg_len, const uint8_t* tag, size_t tag_len);

// Process CPU seconds (user + system, every thread: the callers, the
// library's pools) over the last conc_calls_run, release to join.
static double g_cpu_s = 0;

static double process_cpu_s() {
  struct rusage u;
  getrusage(RUSAGE_SELF, &u);
  return (double)u.ru_utime.tv_sec + 1e-6 * (double)u.ru_utime.tv_usec + (double)u.ru_stime.tv_sec +
         1e-6 * (double)u.ru_stime.tv_usec;
}

extern "C" double conc_calls_cpu_s() { return g_cpu_s; }

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
  const double c0 = process_cpu_s();
  const auto a = std::chrono::steady_clock::now();
  go.store(true, std::memory_order_release);
  for (auto& x : th) x.join();
  g_cpu_s = process_cpu_s() - c0;
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
}

// A trickle of single calls on a background OS thread (bench.py
// resident_interference): call i = (role, id, msg, tag) every period_us on
// the monotonic clock, until trickle_stop.  Keeps the resident verifier's
// kernel alive beside batch work, the way a replica's client streams keep
// calling while its peer streams verify batches
// (core/message-handling.go:204-246).
static std::thread g_tr;
static std::atomic<bool> g_tr_stop{false};
static std::vector<double> g_tr_lat;
static long g_tr_bad = 0;

extern "C" int trickle_start(void* fn, void* ctx, uint32_t role, uint32_t id, const uint8_t* msg,
                             size_t msg_len, const uint8_t* tag, size_t tag_len, int period_us) {
  if (g_tr.joinable()) return -1;
  g_tr_stop.store(false);
  g_tr_lat.clear();
  g_tr_bad = 0;
  const verify_fn f = reinterpret_cast<verify_fn>(fn);
  g_tr = std::thread([=] {
    (void)prctl(PR_SET_TIMERSLACK, 1ul, 0ul, 0ul, 0ul);
    timespec next;
    clock_gettime(CLOCK_MONOTONIC, &next);
    while (!g_tr_stop.load(std::memory_order_relaxed)) {
      const auto a = std::chrono::steady_clock::now();
      if (f(ctx, role, id, msg, msg_len, tag, tag_len) != 0) g_tr_bad++;
      g_tr_lat.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
      next.tv_nsec += (long)period_us * 1000l;
      while (next.tv_nsec >= 1000000000l) {
        next.tv_nsec -= 1000000000l;
        next.tv_sec++;
      }
      clock_nanosleep(CLOCK_MONOTONIC, TIMER_ABSTIME, &next, nullptr);
    }
  });
  return 0;
}

// Stops the trickle; returns its calls, copies up to `max` latencies (us)
// into lat and the count of non-zero statuses into *bad.
extern "C" long trickle_stop(double* lat, long max, long* bad) {
  if (!g_tr.joinable()) return -1;
  g_tr_stop.store(true);
  g_tr.join();
  const long n = (long)g_tr_lat.size();
  for (long i = 0; i < n && i < max; i++) lat[i] = g_tr_lat[(size_t)i];
  if (bad) *bad = g_tr_bad;
  return n;
}

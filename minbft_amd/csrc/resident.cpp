// The resident single-call verifier, host side (mbft_set_resident; the kernel
// is kernels.hip k_verify_server).  VerifyMessageAuthenTag one call at a time
// (api/api.go:133-144, sample/authentication/authenticator.go:121-134) costs
// a kernel launch, a stream's worth of HIP API time and, under concurrency, a
// wait for the batch in flight (the coalescer, batch.cpp).  Here a kernel
// stays on the GPU while calls keep coming: a caller takes a free mailbox
// slot, runs the call's host part (prepare_item: role dispatch, DER, digest,
// key lookup; host_winv: s^-1), writes the item into the slot in host-mapped
// memory and its sequence number last, and spins on the slot's done word.
// The slot's workgroup sees the new sequence number over PCIe, runs the
// item's comb sums (k_verify_split's code) and writes back the four partial
// sums, which the caller's thread joins and x-checks (join_host.cpp: ~2 us
// on the CPU against ~10 us of one GPU wave's dependent products).  No
// launch, no HIP call, no queue between concurrent callers: each has a
// workgroup.
//
// Lifetime: the kernel leaves after `idle_us` without a post or `life_ms`
// after its start (the generation's workgroup 0 decides and writes
// exited_gen); a caller that sees its generation gone relaunches it (under
// Resident::m), and every few spins queries the stream too, so a post that
// raced an exit is picked up by the next generation (a slot is served while
// its seq differs from its done word).  The tables stay put while an item is
// on the GPU: callers hold tab_mu shared, as batches do, and the item carries
// its own table pointers and windows.
#include <errno.h>
#include <sched.h>
#include <string.h>
#include <sys/prctl.h>
#include <time.h>

#include <chrono>
#include <map>

#include "host_internal.h"

using namespace mbft_host;

namespace mbft_host {

namespace {

constexpr size_t kCtlBytes = (sizeof(mbft::SrvCtl) + 255) & ~(size_t)255;

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

uint32_t env_u32(const char* name, uint32_t dflt) {
  const char* v = getenv(name);
  return v ? (uint32_t)strtoul(v, nullptr, 10) : dflt;
}

}  // namespace

struct Resident {
  std::mutex m;  // launches and stops
  int nslots = 0;
  uint8_t* host = nullptr;  // SrvCtl, then nslots SrvSlot (host view)
  uint8_t* dev = nullptr;   // the same, device view
  hipStream_t stream = nullptr;
  bool cu_mask = false;     // the stream was created with a CU mask (its own hardware queue)
  bool low_prio = false;    // the stream has the lowest priority (its own hardware queue)
  DevBuf d_st, d_exit, d_claim;
  int servers = 0;          // workgroups of the server pool (k_verify_server's grid)
  std::atomic<uint32_t> gen{0};
  std::atomic<bool> launched{false};
  std::atomic<uint64_t> free_mask{0};
  uint32_t seq[mbft::kSrvMaxSlots] = {};  // last posted, per slot (its holder only)
  uint32_t idle_us = 2000, life_ms = 200;
  bool two = true;  // two workgroups per item, one per scalar (MBFT_RESIDENT_FORM=one: one)
  bool host_u = true;  // u1, u2 from the host (SrvSlot::u; MBFT_RESIDENT_HOST_U=0: on the GPU)
  // posts of more items than this at once (resident_check) join on the GPU
  // (MBFT_RESIDENT_HOST_JOIN_MAX; 0: every item, single calls too)
  size_t host_join_max = 4;
  // posts of at most this many items at once (MBFT_RESIDENT_CHECK_MAX, <=
  // kResidentCheckMax); larger ones launch
  size_t check_max = kResidentCheckDefault;
  std::atomic<uint64_t> calls{0}, launches{0}, fallbacks{0}, stream_relaunches{0};
  std::atomic<int> waiting{0};  // callers spinning on done words
  // The wait (wait_slots): the caller sleeps through the items' expected GPU
  // time instead of spinning on it (MBFT_RESIDENT_SLEEP=0: spin).  Estimates
  // in ns, per post size (one item, several): post -> all done, and how late
  // a sleep wakes past its deadline.
  bool sleep = true;
  std::atomic<uint32_t> done_ns[2] = {{11000}, {16000}};
  std::atomic<uint32_t> over_ns{2000};
  std::atomic<uint64_t> sleeps{0}, sleep_late{0};
  std::atomic<uint32_t> probe{0};
  // s_sleep(8) steps (~0.25 us each) between a server's empty doorbell polls
  // (MBFT_RESIDENT_POLL_SLEEP)
  uint32_t poll_sleep = 1;

  mbft::SrvCtl* ctl() const { return reinterpret_cast<mbft::SrvCtl*>(host); }
  mbft::SrvSlot* slot(int b) const { return reinterpret_cast<mbft::SrvSlot*>(host + kCtlBytes) + b; }
};

std::mutex g_res_mu;
std::vector<Resident*> g_res_all;  // every live Resident of the process (resident_park_all)

void unregister_resident(Resident* R) {
  std::lock_guard<std::mutex> g(g_res_mu);
  for (size_t i = 0; i < g_res_all.size(); i++)
    if (g_res_all[i] == R) {
      g_res_all.erase(g_res_all.begin() + (long)i);
      break;
    }
}

namespace {

// R.m held.
// The calling thread's current device is restored afterwards (a message
// pass may reach resident_check on a lane of another device).
int launch_server(mbft_ctx* c, Resident& R) {
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (hipSetDevice(c->device) != hipSuccess) return fail(c, MBFT_ERR_HIP, "resident verifier: set device");
  struct Restore {
    int d, now;
    ~Restore() {
      if (d >= 0 && d != now) (void)hipSetDevice(d);
    }
  } restore{prev, c->device};
  uint32_t g = R.gen.load() + 1;
  if (g == 0) g = 1;
  mbft::ServerArgs a{};
  a.ctl = reinterpret_cast<mbft::SrvCtl*>(R.dev);
  a.slots = reinterpret_cast<mbft::SrvSlot*>(R.dev + kCtlBytes);
  a.st = R.d_st.as<uint8_t>();
  a.dexit = R.d_exit.as<uint32_t>();
  a.claim = R.d_claim.as<uint32_t>();
  a.gen = g;
  a.nslots = (uint32_t)R.nslots;
  a.idle_ticks = (uint64_t)R.idle_us * 100ull;      // s_memrealtime: 100 MHz
  a.life_ticks = (uint64_t)R.life_ms * 100000ull;
  a.poll_sleep = R.poll_sleep;
  // (a generation still draining runs first: same stream)
  HIPCHK(c, mbft_launch::verify_server(a, R.servers, R.two, R.stream));
  R.gen.store(g);
  R.launched.store(true);
  R.launches++;
  return MBFT_OK;
}

// Relaunch when no generation is live: never launched, the last one decided
// to exit, or (check_stream) the stream has drained.
int ensure_server(mbft_ctx* c, Resident& R, bool check_stream) {
  const volatile uint32_t* ex = &R.ctl()->exited_gen;
  if (!check_stream && R.launched.load() && *ex != R.gen.load()) return MBFT_OK;
  std::lock_guard<std::mutex> l(R.m);
  bool need = !R.launched.load() || *ex == R.gen.load();
  if (!need && check_stream) {
    const hipError_t q = hipStreamQuery(R.stream);
    if (q == hipSuccess) {
      need = true;
      R.stream_relaunches++;
    } else if (q != hipErrorNotReady) {
      return hip_fail(c, q, "resident verifier");
    }
  }
  return need ? launch_server(c, R) : MBFT_OK;
}

// R.m held, no call in flight: ends the live generation (stop_gen) and
// waits for it.
void stop_server(Resident& R) {
  if (!R.launched.load()) return;
  std::atomic_thread_fence(std::memory_order_release);
  *reinterpret_cast<volatile uint32_t*>(&R.ctl()->stop_gen) = R.gen.load();
  (void)hipStreamSynchronize(R.stream);
  R.launched.store(false);
}



int acquire_slot(Resident& R) {
  uint64_t m = R.free_mask.load(std::memory_order_relaxed);
  while (m) {
    const int b = __builtin_ctzll(m);
    if (R.free_mask.compare_exchange_weak(m, m & ~(1ull << b), std::memory_order_acquire)) return b;
  }
  return -1;
}

// The server's stream: non-blocking, at the LOWEST stream priority.  HIP
// keeps a pool of hardware queues per priority level (GPU_MAX_HW_QUEUES
// each); the library's other streams are normal or high priority, so the
// resident kernel gets a queue of its own and no batch queues behind it (on a
// shared queue a batch would wait up to the kernel's 20 ms lifetime).  It is
// non-blocking, so null-stream work of the application (a synchronous
// hipMemcpy, torch's default stream) does not wait for the live generation
// either -- round 5's CU-masked stream did both (hipExtStreamCreateWithCUMask
// takes no flags: a blocking stream) and, never destroyed, was still
// registered when rocprofv3's destructors ran after the HSA runtime's
// shutdown, which faulted at exit.  MBFT_RESIDENT_CUMASK=1:
// the round-5 CU-masked stream (one per device, lent to one context at a
// time, destroyed at exit).
std::mutex g_cu_mu;
std::map<int, std::pair<hipStream_t, bool>> g_cu_streams;  // device -> (stream, lent)

void destroy_cu_streams_at_exit() {
  std::lock_guard<std::mutex> l(g_cu_mu);
  for (auto& kv : g_cu_streams) {
    if (!kv.second.first || kv.second.second) continue;  // lent: its context is still open
    if (hipSetDevice(kv.first) == hipSuccess) {
      (void)hipStreamSynchronize(kv.second.first);
      (void)hipStreamDestroy(kv.second.first);
    }
    kv.second.first = nullptr;
  }
  (void)hipGetLastError();
}

hipError_t create_stream(mbft_ctx* c, Resident& R) {
  if (env_u32("MBFT_RESIDENT_CUMASK", 0) != 0) {
    std::lock_guard<std::mutex> l(g_cu_mu);
    static const bool registered = [] {
      return atexit(destroy_cu_streams_at_exit) == 0 || true;
    }();
    (void)registered;
    auto it = g_cu_streams.find(c->device);
    if (it == g_cu_streams.end()) {
      int cus = 0;
      hipStream_t st = nullptr;
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) == hipSuccess &&
          cus > 0) {
        std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0xFFFFFFFFu);
        if (cus % 32) mask.back() = (1u << (cus % 32)) - 1u;
        if (hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
          (void)hipGetLastError();
          st = nullptr;
        }
      }
      it = g_cu_streams.emplace(c->device, std::make_pair(st, false)).first;
    }
    if (it->second.first && !it->second.second) {
      it->second.second = true;
      R.stream = it->second.first;
      R.cu_mask = true;
      return hipSuccess;
    }
  }
  int lo = 0, hi = 0;
  if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) lo = 0;
  R.low_prio = lo != hi;
  return hipStreamCreateWithPriority(&R.stream, hipStreamNonBlocking, lo);
}

void release_stream(int device, Resident& R) {
  if (!R.stream) return;
  if (R.cu_mask) {
    std::lock_guard<std::mutex> l(g_cu_mu);
    g_cu_streams[device].second = false;
  } else {
    (void)hipStreamDestroy(R.stream);
  }
  R.stream = nullptr;
}

void free_resident(int device, Resident* R) {
  if (!R) return;
  unregister_resident(R);
  {
    std::lock_guard<std::mutex> l(R->m);
    stop_server(*R);
  }
  R->d_st.release();
  R->d_exit.release();
  R->d_claim.release();
  if (R->host) (void)hipHostFree(R->host);
  release_stream(device, *R);
  delete R;
}

}  // namespace

void resident_park(mbft_ctx* c) {
  Resident* R = c->res;
  if (!R) return;
  std::lock_guard<std::mutex> l(R->m);
  stop_server(*R);
}

// A call in flight when its generation is parked is served by the next one:
// its caller relaunches on its next stream check (<= 1 ms; wait_slots).
void resident_park_all() {
  std::lock_guard<std::mutex> g(g_res_mu);
  for (Resident* R : g_res_all) {
    std::lock_guard<std::mutex> l(R->m);
    stop_server(*R);
  }
}

void resident_destroy(mbft_ctx* c) {
  Resident* R = c->res;
  c->res = nullptr;
  c->res_on.store(false);
  if (R) {
    (void)hipSetDevice(c->device);
    free_resident(c->device, R);
  }
}

namespace {

// The posted items of one caller: slot and sequence number.
struct Post {
  int b;
  uint32_t q;
};

// The host's scalars of several items at once (pre, resident_check): the
// s^-1 planes of host_winv_u (9 planes of stride m) and u1, u2 after them.
struct PreScalars {
  const uint32_t* buf;
  size_t m, j;  // items in buf, this item's index
};

// Fill slot b (held by the caller) with one item and post it; its s^-1 and
// u1, u2 computed here, or taken from pre.
uint32_t post_slot(mbft_ctx* c, Resident& R, int b, const uint8_t* e, const uint8_t* r, const uint8_t* s,
                   uint32_t key, bool gjoin = false, const PreScalars* pre = nullptr) {
  mbft::SrvSlot& S = *R.slot(b);
  S.gjoin = gjoin ? 1u : 0u;
  memcpy(S.e, e, 32);
  memcpy(S.r, r, 32);
  memcpy(S.s, s, 32);
  if (pre) {
    for (int k = 0; k < 9; k++) S.winv[k] = pre->buf[(size_t)k * pre->m + pre->j];
    memcpy(S.u, pre->buf + 9 * pre->m + 16 * pre->j, sizeof(S.u));
    S.ugiven = 1;
  } else if (R.host_u) {
    host_scalars(e, r, s, S.winv, S.u);
    S.ugiven = 1;
  } else {
    host_winv(s, 1, S.winv);
    S.ugiven = 0;
  }
  S.kd = c->keydesc[key];
  S.key0 = 0;
  S.tabG = c->d_tabG;
  S.wg = (uint32_t)c->g_wbits;
  uint32_t q = (R.seq[b] + 1) & 0xFFFFFFu;
  if (q == 0) q = 1;
  R.seq[b] = q;
  std::atomic_thread_fence(std::memory_order_release);
  *reinterpret_cast<volatile uint32_t*>(&S.seq) = q;
  // then the doorbell: the slot's tag byte (the servers poll this one line)
  std::atomic_thread_fence(std::memory_order_release);
  reinterpret_cast<volatile uint8_t*>(R.ctl()->tag32)[b] = (uint8_t)mbft::srv_tag(q);
  return q;
}

// An item's partial sums out of the mapped control block (the GPU wrote them:
// each line a cache miss on the host) into the caller's buffer, every line's
// load issued before the copy so the misses overlap; returns the count.
int copy_parts(uint32_t* loc, const uint32_t* part, int nparts) {
  const size_t bytes = (size_t)nparts * 40 * sizeof(uint32_t);
  const char* src = reinterpret_cast<const char*>(part);
  for (size_t o = 0; o < bytes; o += 64) __builtin_prefetch(src + o);
  memcpy(loc, part, bytes);
  return nparts;
}

// The CPUs this process may run on (its affinity mask).
int usable_cpus() {
  static const int n = [] {
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof(set), &set) == 0) return CPU_COUNT(&set) > 0 ? CPU_COUNT(&set) : 1;
    return 1;
  }();
  return n;
}

int64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (int64_t)ts.tv_sec * 1000000000ll + ts.tv_nsec;
}

// Sleep until the monotonic deadline.  The thread's timer slack is set to
// 1 ns the first time (the default 50 us slack would turn a 8 us sleep into
// one of up to 58 us); it stays set for the thread -- the caller's timers
// then also fire without slack.
void sleep_until_ns(int64_t t) {
  static thread_local bool slack = false;
  if (!slack) {
    (void)prctl(PR_SET_TIMERSLACK, 1ul, 0ul, 0ul, 0ul);
    slack = true;
  }
  timespec ts{(time_t)(t / 1000000000ll), (long)(t % 1000000000ll)};
  while (clock_nanosleep(CLOCK_MONOTONIC, TIMER_ABSTIME, &ts, nullptr) == EINTR) {
  }
}

// One estimate step: x += (v - x) / 8, kept in [lo, hi].
void ewma(std::atomic<uint32_t>& x, int64_t v, int64_t lo, int64_t hi) {
  const int64_t o = x.load(std::memory_order_relaxed);
  int64_t n = o + (v - o) / 8;
  n = n < lo ? lo : n > hi ? hi : n;
  x.store((uint32_t)n, std::memory_order_relaxed);
}

// Wait until every posted item's done word carries its seq; st[j] = item j's
// status.  Relaunches a generation that left (its exit word, or the stream
// found drained) -- the next one serves every slot whose seq is not done.
//
// The CPU is the caller's (a Go replica's goroutine thread, next to gRPC and
// the consensus loop), so the wait first SLEEPS through the items' expected
// GPU time less the expected wake-up delay (both estimated per Resident from
// the calls so far: a wake that finds the items done pulls the estimate
// down, one that finds them pending re-measures it), then spins the last
// microseconds.  Past twice the expected time (a relaunch, a queue of
// callers) it sleeps in 10 us steps; while more callers wait than there are
// CPUs, each spin yields.  MBFT_RESIDENT_SLEEP=0: spin only (round 5).
int wait_slots(mbft_ctx* c, Resident& R, const Post* p, size_t m, uint8_t* st, int64_t t_post) {
  int rc = ensure_server(c, R, false);
  if (rc) return rc;
  struct Count {
    std::atomic<int>& w;
    explicit Count(std::atomic<int>& x) : w(x) { w++; }
    ~Count() { w--; }
  } count(R.waiting);
  const volatile uint32_t* ex = &R.ctl()->exited_gen;
  const double t0 = now_ms();
  double next_query = t0 + 1.0;
  size_t left = m;
  std::vector<char> got(m, 0);
  const int kind = m == 1 ? 0 : 1;
  const int64_t expect = R.done_ns[kind].load(std::memory_order_relaxed);
  bool slept = false, first_after_sleep = false;
  if (R.sleep) {
    const int64_t over = R.over_ns.load(std::memory_order_relaxed);
    int64_t target = t_post + expect - over - 500;
    // a wake-up estimate so large that no sleep fits would never be measured
    // again: every 32nd wait then sleeps half the expected time to re-measure
    if (target - mono_ns() <= 2000 && (R.probe.fetch_add(1, std::memory_order_relaxed) & 31u) == 0)
      target = t_post + expect / 2;
    if (target - mono_ns() > 2000) {
      sleep_until_ns(target);
      // one late wake (a preempted or deeply idle CPU) moves the estimate a
      // bounded step: samples are capped at 4x the estimate + 2 us
      const int64_t late = mono_ns() - target;
      ewma(R.over_ns, std::min<int64_t>(late, 4 * over + 2000), 0, 50000);
      R.sleeps++;
      slept = first_after_sleep = true;
    }
  }
  for (;;) {
    for (size_t j = 0; j < m; j++) {
      if (got[j]) continue;
      const volatile uint32_t* dl = &R.ctl()->done[p[j].b][0];
      const uint32_t d = dl[0];
      if ((d >> 8) != p[j].q) continue;
      uint8_t g = (uint8_t)(d & 0xFF);
      if (R.two) {  // both workgroups; a final status from either decides
        const uint32_t d2 = dl[8];
        if ((d2 >> 8) != p[j].q) continue;
        if (g == mbft::kSrvPartials) g = (uint8_t)(d2 & 0xFF);
      }
      st[j] = g;
      got[j] = 1;
      left--;
    }
    if (left == 0) {
      if (R.sleep) {
        if (first_after_sleep) {  // done before the wake: expect less next time
          R.sleep_late++;
          ewma(R.done_ns[kind], expect - expect / 4, 2000, 200000);
        } else {  // seen done while spinning: a fair measurement
          ewma(R.done_ns[kind], mono_ns() - t_post, 2000, 200000);
        }
      }
      break;
    }
    first_after_sleep = false;
    if (*ex == R.gen.load(std::memory_order_relaxed)) {
      rc = ensure_server(c, R, false);
      if (rc) return rc;
    }
    const double t = now_ms();
    if (R.sleep && (t - t0) * 1e6 > 2.0 * (double)expect + 20000.0) {
      sleep_until_ns(mono_ns() + 10000);
    } else if ((!R.sleep && t - t0 > 0.012) || R.waiting.load(std::memory_order_relaxed) > usable_cpus()) {
      sched_yield();
    }
    if (t > next_query) {  // a generation that left without a word (or failed)
      rc = ensure_server(c, R, true);
      if (rc) return rc;
      next_query = t + 1.0;
      if (t - t0 > 10000.0) return fail(c, MBFT_ERR_HIP, "resident verifier: no answer in 10 s");
    }
    __builtin_ia32_pause();
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  return MBFT_OK;
}

// Take m slots at once, or none.
bool acquire_slots(Resident& R, size_t m, Post* p) {
  for (size_t j = 0; j < m; j++) {
    p[j].b = acquire_slot(R);
    if (p[j].b < 0) {
      for (size_t k = 0; k < j; k++) R.free_mask.fetch_or(1ull << p[k].b, std::memory_order_release);
      return false;
    }
  }
  return true;
}

void release_slots(Resident& R, const Post* p, size_t m) {
  uint64_t bits = 0;
  for (size_t j = 0; j < m; j++) bits |= 1ull << p[j].b;
  R.free_mask.fetch_or(bits, std::memory_order_release);
}

}  // namespace

#ifdef MBFT_SRV_TIMING
// Timing builds (tools/ab_build_def.sh srvt "-DMBFT_SRV_TIMING"): per lone
// call, summed -- host part (prepare + s^-1), post -> done word seen, host
// join; the kernel's slot copy and comb (100 MHz ticks, from the slot's
// partial area); calls.
double g_srv_t[7];
std::mutex g_srv_mu;
#endif

int resident_call(mbft_ctx* c, const mbft_item& it, uint8_t* st) {
#ifdef MBFT_SRV_TIMING
  const double tt0 = now_ms();
#endif
  std::shared_lock<std::shared_mutex> tl(c->tab_mu);
  Resident* R = c->res;
  if (!R || R->nslots == 0) return kNoResident;
  Post p;
  if (!acquire_slots(*R, 1, &p)) {
    R->fallbacks++;
    return kNoResident;
  }
  // a slot whose wait failed stays taken: a stalled generation may still
  // write its done word and partial sums
  struct Give {
    Resident* R;
    Post* p;
    bool keep;
    ~Give() {
      if (!keep) release_slots(*R, p, 1);
    }
  } give{R, &p, false};
  {
    std::lock_guard<std::mutex> m(c->mu);
    sync_host_keymap(c);
  }
  CallInfo ci;
  alignas(16) uint8_t e[32], r[32], s[32];
  uint32_t key = 0;
  Lookup lk;
  prepare_item(c, it, ci, e, r, s, &key, /*defer=*/false, lk);
  uint8_t g = ci.pre;
  if (ci.pre == 0xFF && key >= kHostSlot) {
    g = (uint8_t)(key & 0xFF);  // decided on the host (the USIG epoch step below decides)
  } else if (ci.pre == 0xFF) {
    if (key >= c->keydesc.size()) return fail(c, MBFT_ERR_STATE, "resident verifier: key slot");
#ifdef MBFT_SRV_TIMING
    const double tt1 = now_ms();
#endif
    const int64_t tp = mono_ns();
    p.q = post_slot(c, *R, p.b, e, r, s, key, /*gjoin=*/R->host_join_max == 0);
#ifdef MBFT_SRV_TIMING
    const double tt2 = now_ms();
#endif
    const int rc = wait_slots(c, *R, &p, 1, &g, tp);
    if (rc) {
      give.keep = true;
      return rc;
    }
#ifdef MBFT_SRV_TIMING
    const double tt3 = now_ms();
#endif
#ifdef MBFT_SRV_TIMING
    double tt3b = tt3;
#endif
    if (g == mbft::kSrvPartials && R->host_join_max == 0)
      return fail(c, MBFT_ERR_STATE, "resident verifier: partial sums for a GPU-join item");
    if (g == mbft::kSrvPartials) {
      alignas(64) uint32_t loc[mbft::kSrvMaxParts * 40];
      const int np = copy_parts(loc, R->ctl()->part[p.b], R->two ? mbft::kSrvMaxParts : 4);
#ifdef MBFT_SRV_TIMING
      tt3b = now_ms();
#endif
      g = host_join_check(loc, np, r);
    }
#ifdef MBFT_SRV_TIMING
    const double tt4 = now_ms();
    {
      const volatile uint32_t* tw = &R->ctl()->done[p.b][1];
      std::lock_guard<std::mutex> l(g_srv_mu);
      g_srv_t[0] += tt1 - tt0;  // lock, key map, prepare_item
      g_srv_t[1] += tt2 - tt1;  // post (s^-1 and the slot writes)
      g_srv_t[2] += tt3 - tt2;  // post -> done seen
      g_srv_t[3] += tt4 - tt3;  // host join (copy + arithmetic)
      g_srv_t[6] += tt3b - tt3;  // ... of which the copy out of the mapped block
      g_srv_t[4] += (double)tw[0] * 1e-5;  // kernel: slot copy (ms)
      g_srv_t[5] += (double)tw[1] * 1e-5;  // kernel: comb + partials (ms)
    }
#endif
  }
  if (ci.usig) {
    std::lock_guard<std::mutex> m(c->mu);
    g = resolve_call(c, ci, g);
  }
  R->calls++;
  *st = g;
  return MBFT_OK;
}

int resident_check(mbft_ctx* c, const mbft_item* items, size_t n, uint8_t* gst,
                   std::vector<UsigCall>* usig) {
  Resident* R = c->res;
  if (!R || R->nslots == 0 || n == 0 || n > R->check_max) return kNoResident;
  CallInfo ci[kResidentCheckMax];
  alignas(16) uint8_t e[kResidentCheckMax][32], r[kResidentCheckMax][32], s[kResidentCheckMax][32];
  uint32_t key[kResidentCheckMax];
  size_t gpu[kResidentCheckMax];
  size_t m = 0;
  Lookup lk;
  for (size_t i = 0; i < n; i++) {
    prepare_item(c, items[i], ci[i], e[i], r[i], s[i], &key[i], /*defer=*/false, lk);
    if (ci[i].pre != 0xFF) {
      gst[i] = ci[i].pre;
    } else if (key[i] >= kHostSlot) {
      gst[i] = (uint8_t)(key[i] & 0xFF);
    } else {
      if (key[i] >= c->keydesc.size()) return fail(c, MBFT_ERR_STATE, "resident verifier: key slot");
      gpu[m++] = i;
    }
  }
  if (m) {
    Post p[kResidentCheckMax];
    if (!acquire_slots(*R, m, p)) {
      R->fallbacks += m;
      return kNoResident;
    }
    struct Give {
      Resident* R;
      Post* p;
      size_t m;
      bool keep;
      ~Give() {
        if (!keep) release_slots(*R, p, m);
      }
    } give{R, p, m, false};
    // past a few items the joins go to the GPU (one workgroup per item, a
    // final status): on the host they would run one after another on this
    // thread, ~3 us each
    const bool gjoin = m > R->host_join_max;
    // every item's s^-1 by one inversion (Montgomery's trick) and its u1, u2,
    // before the first post: ~1 us in all instead of ~1 us an item
    alignas(16) uint8_t ge[kResidentCheckMax][32], gr[kResidentCheckMax][32], gs[kResidentCheckMax][32];
    uint32_t sc[25 * kResidentCheckMax];
    const bool batch = m > 1 && R->host_u;
    if (batch) {
      for (size_t j = 0; j < m; j++) {
        memcpy(ge[j], e[gpu[j]], 32);
        memcpy(gr[j], r[gpu[j]], 32);
        memcpy(gs[j], s[gpu[j]], 32);
      }
      host_winv_u(ge[0], gr[0], gs[0], m, sc);
    }
    const int64_t tp = mono_ns();
    for (size_t j = 0; j < m; j++) {
      const size_t i = gpu[j];
      const PreScalars ps{sc, m, j};
      p[j].q = post_slot(c, *R, p[j].b, e[i], r[i], s[i], key[i], gjoin, batch ? &ps : nullptr);
    }
    uint8_t st[kResidentCheckMax];
    const int rc = wait_slots(c, *R, p, m, st, tp);
    if (rc) {
      give.keep = true;
      return rc;
    }
    for (size_t j = 0; j < m; j++)
      if (gjoin && st[j] == mbft::kSrvPartials) {
        const volatile uint32_t* dl = &R->ctl()->done[p[j].b][0];
        char msg[160];
        snprintf(msg, sizeof msg,
                 "resident verifier: partial sums for a GPU-join item (item %zu of %zu, slot %d, seq %u, "
                 "done %08x %08x, gen %u)",
                 j, m, p[j].b, p[j].q, dl[0], dl[8], R->gen.load());
        return fail(c, MBFT_ERR_STATE, msg);
      }
    for (size_t j = 0; j < m; j++)
      if (st[j] == mbft::kSrvPartials) {
        alignas(64) uint32_t loc[mbft::kSrvMaxParts * 40];
        const int np = copy_parts(loc, R->ctl()->part[p[j].b], R->two ? mbft::kSrvMaxParts : 4);
        gst[gpu[j]] = host_join_check(loc, np, r[gpu[j]]);
      } else {
        gst[gpu[j]] = st[j];
      }
    R->calls += m;
  }
  if (usig)
    for (size_t i = 0; i < n; i++)
      if (ci[i].usig) usig->push_back(UsigCall{(uint32_t)i, ci[i]});
  return MBFT_OK;
}

}  // namespace mbft_host

extern "C" {

int mbft_set_resident(mbft_ctx* c, int slots) {
  if (!c || slots < 0 || slots > mbft::kSrvMaxSlots || c->owner) return MBFT_ERR_ARG;
  KeyWriteGuard kw(c);  // no call in flight
  if (hipSetDevice(c->device) != hipSuccess) return MBFT_ERR_HIP;
  resident_destroy(c);
  if (slots == 0) return MBFT_OK;
  Resident* R = new (std::nothrow) Resident();
  if (!R) return MBFT_ERR_NOMEM;
  R->nslots = slots;
  R->idle_us = env_u32("MBFT_RESIDENT_IDLE_US", 2000);
  R->life_ms = env_u32("MBFT_RESIDENT_LIFE_MS", 200);
  // bounded: a generation never outlives 10 s, idles at most its lifetime
  R->life_ms = std::min<uint32_t>(R->life_ms, 10000u);
  R->idle_us = std::min<uint32_t>(R->idle_us, R->life_ms * 1000u);
  {
    const char* f = getenv("MBFT_RESIDENT_FORM");
    R->two = !(f && strcmp(f, "one") == 0);
    R->host_u = env_u32("MBFT_RESIDENT_HOST_U", 1) != 0;
    R->host_join_max = env_u32("MBFT_RESIDENT_HOST_JOIN_MAX", 4);
    R->sleep = env_u32("MBFT_RESIDENT_SLEEP", 1) != 0;
    R->poll_sleep = std::max<uint32_t>(1u, std::min<uint32_t>(env_u32("MBFT_RESIDENT_POLL_SLEEP", 1), 1000u));
    R->check_max = std::min<size_t>(env_u32("MBFT_RESIDENT_CHECK_MAX", (uint32_t)kResidentCheckDefault),
                                    kResidentCheckMax);
  }
  if (R->idle_us == 0) R->idle_us = 1;
  if (R->life_ms == 0) R->life_ms = 1;
  const size_t bytes = kCtlBytes + (size_t)slots * sizeof(mbft::SrvSlot);
  void* h = nullptr;
  void* d = nullptr;
  auto bail = [&](const char* what) {
    free_resident(c->device, R);
    return fail(c, MBFT_ERR_HIP, std::string("resident verifier: ") + what);
  };
  if (host_malloc_near(&h, bytes, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
    R->host = nullptr;
    return bail("mapped mailbox");
  }
  R->host = static_cast<uint8_t*>(h);
  memset(h, 0, bytes);
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || !d) return bail("device view of the mailbox");
  R->dev = static_cast<uint8_t*>(d);
  if (create_stream(c, *R) != hipSuccess) return bail("stream");
  // device scratch, initialized on the server's own stream (a null-stream
  // memset would wait for every blocking stream of the device)
  {
    std::vector<uint32_t> claim0(2 * mbft::kSrvMaxSlots, mbft::srv_tag(0));  // seq 0: nothing posted
    if (R->d_st.ensure((size_t)(2 * slots)) != hipSuccess || R->d_exit.ensure(16) != hipSuccess ||
        R->d_claim.ensure(claim0.size() * 4) != hipSuccess ||
        hipMemsetAsync(R->d_exit.p, 0, 16, R->stream) != hipSuccess ||
        hipMemcpyAsync(R->d_claim.p, claim0.data(), claim0.size() * 4, hipMemcpyHostToDevice, R->stream) !=
            hipSuccess ||
        hipStreamSynchronize(R->stream) != hipSuccess)
      return bail("device scratch");
  }
  // the server pool: 2 workgroups per slot up to MBFT_RESIDENT_SERVERS
  // (default 16: ~1.1 M calls/s of comb capacity on 16 of the 256 CUs)
  {
    const int per = R->two ? 2 : 1;
    const int cap = (int)std::max<uint32_t>(1u, std::min<uint32_t>(env_u32("MBFT_RESIDENT_SERVERS", 16),
                                                                     2u * mbft::kSrvMaxSlots));
    R->servers = std::min(per * slots, cap);
  }
  R->free_mask.store(slots == 64 ? ~0ull : (1ull << slots) - 1ull);
  {
    std::lock_guard<std::mutex> g(g_res_mu);
    g_res_all.push_back(R);
  }
  c->res = R;
  c->res_on.store(true);
  return MBFT_OK;
}

#ifdef MBFT_SRV_TIMING
int mbft_debug_resident_timing(double out[7], int reset) {
  std::lock_guard<std::mutex> l(g_srv_mu);
  for (int k = 0; k < 7; k++) {
    out[k] = g_srv_t[k];
    if (reset) g_srv_t[k] = 0;
  }
  return 0;
}
#endif

int mbft_resident_stats(mbft_ctx* c, double out[6]) {
  if (!c || !out) return MBFT_ERR_ARG;
  std::shared_lock<std::shared_mutex> tl(c->tab_mu);
  const Resident* R = c->res;
  for (int k = 0; k < 6; k++) out[k] = 0;
  if (!R) return MBFT_OK;
  out[0] = (double)R->nslots;
  out[1] = (double)R->calls.load();
  out[2] = (double)R->launches.load();
  out[3] = (double)R->fallbacks.load();
  out[4] = (double)R->stream_relaunches.load();
  out[5] = R->cu_mask || R->low_prio ? 1.0 : 0.0;
  return MBFT_OK;
}

int mbft_resident_wait_stats(mbft_ctx* c, double out[5]) {
  if (!c || !out) return MBFT_ERR_ARG;
  std::shared_lock<std::shared_mutex> tl(c->tab_mu);
  const Resident* R = c->res;
  for (int k = 0; k < 5; k++) out[k] = 0;
  if (!R) return MBFT_OK;
  out[0] = (double)R->sleeps.load();
  out[1] = (double)R->sleep_late.load();
  out[2] = (double)R->done_ns[0].load();
  out[3] = (double)R->over_ns.load();
  out[4] = R->sleep ? 1.0 : 0.0;
  return MBFT_OK;
}

}  // extern "C"

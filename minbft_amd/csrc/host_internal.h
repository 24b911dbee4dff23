// Internal declarations shared by the host translation units of
// libminbft_amd.so (host.cpp: context, key store, batch verifier, C-ABI;
// messages.cpp: AuthenBytes and the MinBFT validators).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <array>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/minbft_gpu.h"
#include "kernels.h"
#include "sha256.h"

namespace mbft_host {

constexpr int kVersion = 1;

extern const uint8_t kPkixPrefix[26];
extern const uint8_t kEmptyHash[32];  // SHA256("")

// SHA-256 on the host (sha256_host.cpp): the x86 SHA extensions when the CPU
// has them, else the portable compression; form 0 / 1 forces one (tests).
void sha256(const uint8_t* p, size_t n, uint8_t out[32]);
void sha256_form(int form, const uint8_t* p, size_t n, uint8_t out[32]);
bool cpu_has_shani();
// m messages at once (out[i] = SHA256(p[i][0 .. n[i]))): with the SHA
// extensions, four messages of equal padded length interleaved per block.
void sha256_many(size_t m, const uint8_t* const* p, const size_t* n, uint8_t* const* out);

// 32 B big-endian -> 8 LE 32-bit words
inline void be_to_words(uint32_t w[8], const uint8_t* be) {
  for (int i = 0; i < 8; i++) {
    const uint8_t* q = be + 4 * (7 - i);
    w[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
}

inline uint64_t be64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 0; i < 8; i++) v = (v << 8) | p[i];
  return v;
}

inline void put_le64(uint8_t* p, uint64_t v) {
  for (int i = 0; i < 8; i++) p[i] = (uint8_t)(v >> (8 * i));
}

inline void put_be64(uint8_t* p, uint64_t v) {
  for (int i = 0; i < 8; i++) p[i] = (uint8_t)(v >> (8 * (7 - i)));
}

inline void put_be32(uint8_t* p, uint32_t v) {
  for (int i = 0; i < 4; i++) p[i] = (uint8_t)(v >> (8 * (3 - i)));
}

// Grown on demand.  A grown buffer's old block is retired, not freed: hipFree
// synchronizes the whole device, so a free on a batch path would wait for
// every stream's work -- the resident verifier's kernel included, up to its
// idle exit.  Retired blocks go at release(); growth is
// geometric (x1.5 at least), so they total less than the live block.
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  std::vector<void*> retired;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    size_t want = bytes < 4096 ? 4096 : bytes;
    if (p) {
      retired.push_back(p);
      if (want < cap + cap / 2) want = cap + cap / 2;
    }
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, want);
    if (e != hipSuccess) {  // out of memory: the retired blocks go first
      (void)hipGetLastError();
      free_retired();
      e = hipMalloc(&p, bytes < 4096 ? 4096 : bytes);
      want = bytes < 4096 ? 4096 : bytes;
    }
    if (e == hipSuccess) cap = want;
    return e;
  }
  void free_retired() {
    for (void* q : retired) (void)hipFree(q);
    retired.clear();
  }
  void release() {
    free_retired();
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

struct KeyEntry {
  uint32_t slot;
};

struct SlotInfo {
  std::array<uint8_t, 64> xy;
  bool valid;
  uint64_t fingerprint;  // SHA256(PKIX)[0:8] (crypto.go:134-144)
  uint32_t fp_group;     // index of this fingerprint's USIG epoch entry
};

// hipHostMalloc on the NUMA node closest to the CURRENT device (every engine
// sets its device before it allocates): the engine's staging, read by its
// GPU's DMA engines, sits next to that GPU's PCIe root (host.cpp).  Plain
// hipHostMalloc on one-node hosts or when the placement is refused.
hipError_t host_malloc_near(void** p, size_t bytes, unsigned flags);

// Page-locked host staging (hipHostMalloc), grown on demand: DMA engines
// read it directly, so H2D copies run at PCIe rate and asynchronously.
// (Grown like DevBuf: hipHostFree synchronizes the device too, so an old
// block is retired until release().)
struct PinnedBuf {
  void* p = nullptr;
  size_t cap = 0;
  std::vector<void*> retired;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) retired.push_back(p);
    p = nullptr;
    cap = 0;
    size_t want = bytes < 4096 ? 4096 : bytes + bytes / 4;
    hipError_t e = host_malloc_near(&p, want, hipHostMallocDefault);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      for (void* q : retired) (void)hipHostFree(q);
      retired.clear();
      e = host_malloc_near(&p, want, hipHostMallocDefault);
    }
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    for (void* q : retired) (void)hipHostFree(q);
    retired.clear();
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

// Host threads the library has started (pools, engine workers): a batch on
// a multi-engine context starts none (mbft_debug_threads_started).
extern std::atomic<uint64_t> g_threads_started;

// One persistent host thread per engine for the shards of multi-engine
// batches (one host thread per GPU).  submit() queues a task
// and returns a ticket; wait(ticket) returns when that task has run.  Tasks
// run one at a time, in submission order (a shard task takes its engine's
// mutex anyway).  Started with its engine's first shard, joined at destroy.
class EngineWorker {
 public:
  EngineWorker() {
    g_threads_started.fetch_add(1);
    th_ = std::thread([this] { loop(); });
  }
  ~EngineWorker() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  uint64_t submit(std::function<void()> fn) {
    std::lock_guard<std::mutex> g(m_);
    q_.push_back(std::move(fn));
    const uint64_t t = ++queued_;
    cv_.notify_all();
    return t;
  }
  void wait(uint64_t ticket) {
    std::unique_lock<std::mutex> g(m_);
    done_cv_.wait(g, [&] { return done_ >= ticket; });
  }

 private:
  void loop() {
    std::unique_lock<std::mutex> g(m_);
    for (;;) {
      cv_.wait(g, [&] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;  // stop, nothing left
      std::function<void()> fn = std::move(q_.front());
      q_.pop_front();
      g.unlock();
      fn();
      g.lock();
      done_++;
      done_cv_.notify_all();
    }
  }
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  std::deque<std::function<void()>> q_;
  uint64_t queued_ = 0, done_ = 0;
  bool stop_ = false;
  std::thread th_;
};

// Persistent host worker pool for the batch pipeline's per-item work (DER
// decode, digest construction, staging writes).  run(n, fn) calls fn(t) for
// t in [0, n) on the workers and the calling thread and returns when all are
// done.  One pool per engine context; calls on one pool are serialized by
// the context mutex.
class Pool {
 public:
  explicit Pool(int nworkers) {
    for (int i = 0; i < nworkers; i++) th_.emplace_back([this] { loop(); });
    g_threads_started.fetch_add((uint64_t)(nworkers > 0 ? nworkers : 0));
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
      gen_++;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return (int)th_.size() + 1; }
  void run(int ntasks, const std::function<void(int)>& fn) {
    start(ntasks, fn);
    wait();
  }
  // Asynchronous form: the workers start on fn(0 .. ntasks) and the caller
  // goes on; wait() joins in on the remaining tasks and returns when all are
  // done.  fn must stay alive until wait() returns; one run at a time.
  void start(int ntasks, const std::function<void(int)>& fn) {
    if (ntasks <= 0) return;
    if (th_.empty() || ntasks == 1) {
      for (int t = 0; t < ntasks; t++) fn(t);
      return;
    }
    {
      std::lock_guard<std::mutex> g(m_);
      fn_ = &fn;
      ntasks_ = ntasks;
      next_.store(0);
      done_ = 0;
      gen_++;
    }
    pending_ = true;
    cv_.notify_all();
  }
  void wait() {
    if (!pending_) return;
    work();
    std::unique_lock<std::mutex> g(m_);
    done_cv_.wait(g, [&] { return done_ == ntasks_; });
    fn_ = nullptr;
    pending_ = false;
  }

 private:
  void work() {
    for (;;) {
      const int t = next_.fetch_add(1);
      if (t >= ntasks_) return;
      (*fn_)(t);
      std::lock_guard<std::mutex> g(m_);
      if (++done_ == ntasks_) done_cv_.notify_one();
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
        if (!fn_) continue;
      }
      work();
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* fn_ = nullptr;
  std::atomic<int> next_{0};
  int ntasks_ = 0, done_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
  bool pending_ = false;  // a start() not yet joined by wait()
};

// The (role, id) -> key slot map as one flat open-addressing table (the
// host's mirror of the device KeyMap): prepare_item's lookup is a hash and a
// probe or two in a few cache lines instead of two unordered_map finds.
// Valid while gen == the context's key_gen (sync_host_keymap rebuilds it).
struct HostKeyMap {
  std::vector<uint64_t> keys;  // (role << 32) | id, ~0 = empty
  std::vector<uint32_t> slots;
  uint32_t mask = 0;
  uint32_t role_ok = 0;  // bit r: role r has a scheme (Replica / Client registered; USIG and enabled)
  uint64_t gen = 0;
};

// One VerifyMessageAuthenTag call split into a pure part (everything that
// depends only on the call's own bytes, including the GPU signature check)
// and the stateful USIG epoch step, applied later in call order.  The GPU
// item of call i is item i of the batch (kDeadSlot when the host decided).
struct CallInfo {
  uint8_t pre = 0xFF;        // final status decided on the host, or 0xFF
  uint8_t usig_tail = 0xFF;  // DER outcome if the epoch matches (USIG)
  bool usig = false;
  uint32_t fpg = 0;          // the key's fingerprint group (USIG epoch entry)
  uint64_t ui_epoch = 0, counter = 0;
};
// Key slots >= kHostSlot carry a status the host decided: the kernel writes
// their low byte as the item's status (and verifies nothing).
using mbft::kHostSlot;
constexpr uint32_t kDeadSlot = kHostSlot | MBFT_BAD_KEY;  // host-decided, status ignored

// A USIG call whose status the epoch step can still change: call index and
// its host outcome (verify_batch keeps only these, not one record per call).
struct UsigCall {
  uint32_t i;
  CallInfo p;
};

struct Resident;  // the resident single-call verifier (resident.cpp)

}  // namespace mbft_host

struct mbft_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  std::mutex mu;

  // Concurrent check batches on one device (mbft_set_concurrency).  A lane
  // is an engine with its own scratch, streams, s^-1 pipeline and worker
  // pool that reads its owner's tables and key store (owner != null; it
  // owns no table).  Check / verify batches lease a free lane and hold
  // tab_mu shared for the call; every change to keys, roles, windows or
  // engines takes tab_mu exclusively (then mu), so it waits for the batches
  // in flight.  The USIG epoch step stays under mu, batch by batch.
  mbft_ctx* owner = nullptr;
  std::shared_mutex tab_mu;
  std::mutex lane_mu;
  std::condition_variable lane_cv;
  std::vector<mbft_ctx*> lanes, lane_free;
  std::map<int, int> lane_busy;  // leased lanes per device (under lane_mu)
  int concurrency = 1;
  int pool_threads = 0;  // worker threads of this engine's pool (0: host_pool_threads())
  // this engine's shard thread (multi-engine batches; started on first use)
  std::unique_ptr<mbft_host::EngineWorker> worker;
  std::mutex worker_mu;

  // Comb tables.  The generator table is built at create time
  // (and rebuilt by mbft_set_generator_window); each registration call that
  // brings new valid keys allocates one block holding their tables.  d_keys
  // mirrors `slots` on the device as KeyDesc {table, window, valid}.
  uint32_t* d_tabG = nullptr;
  int g_wbits = 16;  // generator comb window (16: 64 MiB, 26: 36 GiB)
  int q_wbits = 16;  // key comb window for keys registered from now on
  std::vector<void*> tab_blocks;
  // blocks released by mbft_clear_keys, kept for reuse (re-mapping a
  // 129 GiB allocation costs seconds); freed when the generator table needs
  // the memory, on a failed allocation, and at destroy
  std::vector<std::pair<void*, size_t>> free_blocks;
  std::vector<size_t> tab_sizes;  // bytes of each tab_blocks entry
  std::vector<mbft::KeyDesc> keydesc;
  mbft_host::DevBuf d_keys;

  // Multi-GPU in one process (mbft_ctx_add_device): peer engines on other
  // devices hold replicas of the comb tables (same slot numbering, same
  // windows); host-buffer verifies are split into contiguous shards, one host
  // thread and stream per engine, and concatenated in index order.  Roles,
  // private keys and the USIG epoch state stay in this (primary) context.
  std::vector<mbft_ctx*> peers;
  size_t shard_min = 32768;  // items per engine below which a batch is not split
  std::vector<mbft_host::SlotInfo> slots;
  std::map<std::array<uint8_t, 64>, uint32_t> slot_of_xy;

  std::unordered_map<uint32_t, std::unordered_map<uint32_t, mbft_host::KeyEntry>> roles;  // role -> id -> key
  bool usig_enabled = false;
  // USIG epoch state (crypto.go:148-154, keyed by key fingerprint): one
  // entry per distinct fingerprint, found through the slot's fp_group.
  std::unordered_map<uint64_t, uint32_t> fp_group_of;
  std::vector<uint64_t> epoch_val;
  std::vector<uint8_t> epoch_set;
  std::map<uint32_t, std::array<uint8_t, 32>> priv;

  // scratch
  mbft_host::DevBuf e, r, s, slot, status, xy, ok, bpts, priv_d;
  mbft_host::DevBuf sha_data, sha_off, sha_out, sha_ep, sha_ctr;

  // Batched-inverse pipeline: s^-1 of batch i+1 runs on `istream` while the
  // verify kernel of batch i runs on the caller's stream.  The s^-1 planes,
  // workspace and exact-path queue rotate over kPipe buffers guarded by
  // events: with three, batch i+2's inverse waits only for the verify of
  // batch i-1, long done, so it never sits between two verify kernels.
  static constexpr int kPipe = 3;
  hipStream_t istream = nullptr;
  mbft_host::DevBuf winv[kPipe], ws[kPipe], slowq[kPipe];
  hipEvent_t ev_in = nullptr, ev_inv[kPipe] = {}, ev_done[kPipe] = {};
  int pipe = 0;

  // Batch pipeline (batch.cpp): host workers fill page-locked staging chunk
  // by chunk; each chunk's H2D runs on `cstream` while the workers fill the
  // next, and its s^-1 + verify kernels and status D2H on vstream[k & 1]
  // (two streams so consecutive chunks' kernels overlap).
  std::unique_ptr<mbft_host::Pool> pool;
  hipStream_t cstream = nullptr, vstream[2] = {nullptr, nullptr};
  hipEvent_t ev_h2d = nullptr;
  // a second copy stream: with MBFT_COPY_STREAMS=2 consecutive chunks' H2D
  // copies alternate between the two (two DMA engines)
  hipStream_t cstream2 = nullptr;
  hipEvent_t ev_h2d2 = nullptr;
  // small synchronous uploads (the device key map): a non-blocking stream of
  // their own -- a null-stream hipMemcpy would wait for every blocking stream
  // of the device, the resident kernel's CU-masked one included
  hipStream_t kstream = nullptr;
  mbft_host::PinnedBuf h_e, h_r, h_s, h_slot, h_status, h_udata, h_uoff, h_uidx, h_uep, h_uctr;
  mbft_host::PinnedBuf h_small;  // small batches: e | r | s | slot contiguous (one H2D)
  // Zero-copy staging for the smallest batches (single calls): e | r | s |
  // slot | status in fine-grained host memory mapped into the device
  // (hipHostMallocCoherent, hipHostGetDevicePointer); the kernel reads its
  // inputs and writes its statuses there, so a call makes no copy at all.
  // zc_state: 0 not tried, 1 usable, -1 unavailable (the copy path is used).
  void* zc_host = nullptr;
  void* zc_dev = nullptr;
  int zc_state = 0;
  mbft_host::DevBuf b_small;
  mbft_host::DevBuf b_e, b_r, b_s, b_slot, b_status, b_udata, b_uoff, b_uidx, b_uep, b_uctr;
  // Device-side call decode (batch.cpp engine_check_dev, k_prepare): flat
  // calls in library-owned page-locked memory (mbft_host_alloc) go to the GPU
  // raw, chunk by chunk, and are decoded there; the host touches none of
  // their bytes.  The (role, id) -> slot map is mirrored on every engine,
  // rebuilt when key_gen (bumped by each change to roles, keys or USIG
  // enablement, kept in the primary) moves past kmap_gen.
  int dev_prepare = 1;  // mbft_set_device_prepare: 0 never, 1 when the buffers allow it
  // batches up to this size take k_verify_split, larger small ones k_verify_pairs
  // (mbft_set_small_batch_form; -1: env MBFT_SPLIT_MAX, default 256)
  long split_max = -1;
  // the larger small batches' form (mbft_set_small_batch_inverse): -1 env
  // MBFT_PAIRS_PLANES / MBFT_QUADS, 0 k_verify_pairs inverting per lane, 1 the
  // batched per-wave s^-1 into planes first, then k_verify_pairs, 2
  // k_verify_quads inverting per wave inside, 3 the planes and k_verify_quads
  int small_inv = -1;
  uint64_t key_gen = 1, kmap_gen = 0;
  mbft_host::HostKeyMap hkm;  // host mirror, see HostKeyMap
  uint32_t kmap_mask = 0, kmap_role_ok = 0;
  mbft_host::DevBuf d_kmap_keys, d_kmap_slots;
  mbft_host::DevBuf b_roles, b_ids, b_moff, b_toff, b_msgs, b_tags;
  mbft_host::DevBuf b_bad;     // a device-decoded call's offsets out of range (k_prepare)
  mbft_host::PinnedBuf hm_bad;
  // message layer (messages.cpp): per-call AuthenBytes descriptors
  mbft_host::PinnedBuf h_desc;
  mbft_host::DevBuf b_desc;
  // the device message layer (msgdev.cpp, msg_kernels.hip): records, arena,
  // candidates, dedup table, per-call outcomes; and what the replay reads back
  mbft_host::DevBuf m_recs, m_bytes, m_chk, m_flag, m_cand, m_chash, m_cslot, m_uniq, m_ref, m_idx,
      m_callof, m_candof, m_bounds, m_tkeys, m_treps, m_scan, m_fpg, m_info, m_epset, m_epval, m_cap, m_out;
  // the device message layer's record chunks: copied on cstream, each one's
  // candidate kernels start on `stream` once it is in (msgdev.cpp)
  // m_fpg holds the fingerprint groups of key_gen fpg_gen (fpg_n slots)
  uint64_t fpg_gen = 0;
  size_t fpg_n = 0;
  static constexpr int kMsgChunks = 8;
  hipEvent_t ev_msg[kMsgChunks] = {}, ev_cnt[kMsgChunks] = {};
  mbft_host::PinnedBuf hm_small, hm_chk, hm_callof, hm_info, hm_cap, hm_out;
  // a device check's outputs in one block each side (msgdev.cpp PackLayout)
  mbft_host::DevBuf m_pack;
  mbft_host::PinnedBuf hm_pack;
  // mbft_check_messages_flat: records / arena outside library page-locked
  // memory are staged here
  mbft_host::PinnedBuf hm_recs, hm_bytes;
  // checks of at most this many messages take the small route
  // (mbft_set_small_check; msgdev.cpp)
  std::atomic<size_t> msg_small_max{512};
  // Coalescing of concurrent single calls (mbft_set_coalescing, batch.cpp):
  // a queue of waiting calls, each led or served by the batch that takes it.
  struct Waiter {
    mbft_item it;
    int rc = 0;
    uint8_t st = 0;
    // set under Coalescer::m, read by the waiter without it (batch.cpp
    // coalesced_call); ev: the futex word bumped after each change
    std::atomic<bool> done{false}, lead{false};  // lead: holds a batch slot
    std::atomic<uint32_t> ev{0};
    bool taken = false;
  };
  struct Coalescer {
    std::mutex m;
    std::condition_variable cv_fill;
    std::vector<std::shared_ptr<Waiter>> q;
    int running = 0;  // batch slots held (collecting or running)
    int slots = 1;    // mbft_set_coalescing_slots (at most the concurrency)
    std::atomic<bool> enabled{false};
    uint32_t max_wait_us = 0, max_batch = 0;
  } co;
  // Coalescing of concurrent message-batch checks (mbft_set_check_coalescing,
  // msgdev.cpp): callers queue; the one collecting waits for an engine lane,
  // then takes the queue and runs it as ONE device pass (calls deduplicated
  // across the callers' batches), handing each caller its own batch.
  struct CheckCoalescer {
    std::mutex m;
    std::condition_variable cv;
    std::vector<struct mbft_check_req*> q;
    bool collecting = false;  // a leader is waiting for a lane (it takes the queue)
    int running = 0;          // passes holding a lane now (at most max_passes)
    // host workers of the running passes (record / arena concatenation): one
    // pool per pass slot, each a share of the host threads independent of
    // the lane count (a lane's own pool is host_threads / lanes)
    std::vector<std::unique_ptr<mbft_host::Pool>> pools;
    std::vector<char> pool_busy;
    std::atomic<bool> enabled{false};
    uint32_t max_wait_us = 0;
    size_t max_messages = (size_t)1 << 20;
    double passes = 0, requests = 0, messages = 0;  // mbft_check_coalescing_stats
  } cco;
  // The resident single-call verifier (mbft_set_resident, resident.cpp):
  // set and cleared under tab_mu held exclusively; callers read it under
  // tab_mu shared.
  mbft_host::Resident* res = nullptr;
  std::atomic<bool> res_on{false};
  // stage times of verify_batch (ms, summed; mbft_profile_stages)
  double st_prepare_ms = 0, st_gpu_ms = 0, st_resolve_ms = 0, st_total_ms = 0;
  double st_calls = 0, st_items = 0;

  // profiling (HIP events around the kernels of each batch)
  bool prof = false;
  struct Ev {
    hipEvent_t a, b, c, d;
    size_t n;
  };
  std::vector<Ev> evs;
  double prof_verify_ms = 0, prof_inv_ms = 0, prof_batches = 0, prof_items = 0;
  // device message layer (mbft_profile_msg_layer): calls, H2D ms, device ms, bytes up
  double prof_msg[4] = {0, 0, 0, 0};
  // MBFT_DIAG_REUSE_WINV (host.cpp verify_device): batch size whose w planes
  // buffer k holds
  size_t diag_winv_n[kPipe] = {};
};

namespace mbft_host {

// The context whose tables and key store engine g reads (its owner for a
// lane).
inline const mbft_ctx* tabs(const mbft_ctx* g) { return g->owner ? g->owner : g; }

// Exclusive access to the key store and tables: waits for the check
// batches in flight on lanes (tab_mu), then takes the context mutex.
struct KeyWriteGuard {
  std::unique_lock<std::shared_mutex> t;
  std::lock_guard<std::mutex> m;
  explicit KeyWriteGuard(mbft_ctx* c) : t(c->tab_mu), m(c->mu) {}
};

// Worker threads for engine g's pool.
int pool_workers(const mbft_ctx* g);

void sync_host_keymap(mbft_ctx* c);

// The engine one check / verify batch runs on.  Concurrency 1: the context
// itself, under its mutex for the whole call (the reference's one-at-a-time
// behaviour).  Otherwise a free lane, leased for the call, with tab_mu held
// shared (key changes wait for the batch) and the host key map brought up to
// date under the mutex first; the caller takes the mutex again only for the
// USIG epoch step.  With engines on more devices (mbft_ctx_add_device) every
// device has `concurrency` lanes: call-level batches lease one on the
// context's device (their large batches shard over the peer engines
// themselves), message-level passes (any_device) the free lane of the device
// with the fewest leased, the context's own on a tie -- concurrent passes
// spread over the GPUs, one caller at a time stays on one.  The caller sets
// the lane's device (g->device).
struct Lease {
  mbft_ctx* c;
  mbft_ctx* g;
  std::shared_lock<std::shared_mutex> tl;
  std::unique_lock<std::mutex> cl;
  explicit Lease(mbft_ctx* ctx, bool any_device = false) : c(ctx), g(ctx), tl(ctx->tab_mu) {
    if (c->concurrency <= 1) {
      cl = std::unique_lock<std::mutex>(c->mu);
      return;
    }
    {
      std::lock_guard<std::mutex> m(c->mu);
      sync_host_keymap(c);
    }
    std::unique_lock<std::mutex> lk(c->lane_mu);
    long k = -1;
    c->lane_cv.wait(lk, [&] {
      k = -1;
      int best = 0;
      for (size_t j = 0; j < c->lane_free.size(); j++) {
        const mbft_ctx* l = c->lane_free[j];
        if (!any_device && l->device != c->device) continue;
        const int b = 2 * c->lane_busy[l->device] + (l->device == c->device ? 0 : 1);
        if (k < 0 || b < best) {
          k = (long)j;
          best = b;
        }
      }
      return k >= 0;
    });
    g = c->lane_free[(size_t)k];
    c->lane_free.erase(c->lane_free.begin() + k);
    c->lane_busy[g->device]++;
  }
  ~Lease() {
    if (g == c) return;
    {
      std::lock_guard<std::mutex> lk(c->lane_mu);
      c->lane_free.push_back(g);
      c->lane_busy[g->device]--;
    }
    c->lane_cv.notify_all();  // waiters differ in which lanes they take
  }
  Lease(const Lease&) = delete;
  Lease& operator=(const Lease&) = delete;
};

int fail(mbft_ctx* c, int code, const std::string& what);
int hip_fail(mbft_ctx* c, hipError_t e, const char* what);

#define HIPCHK(c, x)                                                    \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess) return ::mbft_host::hip_fail(c, e_, #x);     \
  } while (0)

int register_points(mbft_ctx* c, const uint8_t* xy64, size_t n, uint32_t* out_slots,
                    uint8_t* valid_out);
int verify_device(mbft_ctx* c, const uint8_t* d_e, const uint8_t* d_r, const uint8_t* d_s,
                  const uint32_t* d_slot, size_t n, uint8_t* d_status, hipStream_t st,
                  bool host_status = false, bool latency = false,
                  const uint32_t* d_winv = nullptr, const uint32_t* d_count = nullptr);
// s^-1 R mod N of n big-endian s values into 9 planes of n 29-bit limbs (the
// k_verify_split form); zeros where s is 0 or >= N (the kernel rejects those
// before reading w).  Lone calls (batch.cpp).
void host_winv(const uint8_t* s, size_t n, uint32_t* planes);
// host_winv plus u1 = e s^-1, u2 = r s^-1 mod N after the planes (planes + 9 n,
// 16 LE words an item): the split kernel's host-staged scalars
void host_winv_u(const uint8_t* e, const uint8_t* r, const uint8_t* s, size_t n, uint32_t* planes);
// one call: host_winv(s, 1, planes) plus u1 = e s^-1, u2 = r s^-1 mod N (8 LE
// words each) for the resident kernel (SrvSlot::u)
void host_scalars(const uint8_t* e, const uint8_t* r, const uint8_t* s, uint32_t* planes, uint32_t u[16]);
int verify_host(mbft_ctx* c, const uint8_t* e, const uint8_t* r, const uint8_t* s,
                const uint32_t* slots, size_t n, uint8_t* status);

// Host worker threads per engine pool (env MBFT_HOST_THREADS, else
// OMP_NUM_THREADS, else the hardware threads, at most 32).
int host_pool_threads();
// The engine's shard thread (started on first use).
mbft_host::EngineWorker& engine_worker(mbft_ctx* e);

// Rebuild c->hkm from the key store if the keys changed (caller holds c->mu).

// A worker's memo of its last (role, id) key-store lookup: batches repeat
// signers, and the two hash-map probes cost more than the DER decode.
struct Lookup {
  uint32_t role = 0xFFFFFFFFu, id = 0xFFFFFFFFu;
  int state = -1;     // 0 unknown role, 1 no scheme, 2 unknown id, 3 known
  uint32_t slot = 0;
};

// The host (byte-level) part of one call, in the reference's check order:
// fills CallInfo and the GPU item (e, r, s, key slot; kDeadSlot when the
// host decided).  Returns true when the USIG digest e is left to the caller
// (defer): the GPU SHA stage.
bool prepare_item(const mbft_ctx* c, const mbft_item& it, CallInfo& p, uint8_t* e32, uint8_t* r32,
                  uint8_t* s32, uint32_t* slot, bool defer, Lookup& lk);

// The batch pipeline (batch.cpp): the pure part of n calls on the GPU.
// gst[i] receives call i's status (the host's where it decided, else the
// GPU's; gst must hold n bytes); resolve_call then applies the USIG epoch
// state in call order.  usig (optional) receives, ascending, the calls that
// resolve_call can still change, with their host outcome.
int check_calls(mbft_ctx* c, const mbft_item* items, size_t n, uint8_t* gst,
                std::vector<UsigCall>* usig = nullptr, mbft_ctx* g0 = nullptr);
int check_calls_flat(mbft_ctx* c, const uint32_t* roles, const uint32_t* ids, const uint8_t* msgs,
                     const uint64_t* msg_off, const uint8_t* tags, const uint64_t* tag_off,
                     size_t n, uint8_t* gst, mbft_ctx* g0 = nullptr);
uint8_t resolve_call(mbft_ctx* c, const CallInfo& ci, uint8_t g);
// n calls on engine g alone (no sharding over peer engines): the batch
// pipeline's pure part, as check_calls (the caller holds g: the context's
// lock or a lane's lease).  The small message checks.
int check_calls_on(mbft_ctx* c, mbft_ctx* g, const mbft_item* items, size_t n, uint8_t* gst,
                   std::vector<UsigCall>* usig);
int verify_batch_impl(mbft_ctx* c, const mbft_item* items, size_t n, uint8_t* out,
                      mbft_ctx* g0 = nullptr);
// One VerifyMessageAuthenTag call through the resident verifier
// (resident.cpp): kNoResident when it is off or every mailbox slot is taken
// (the caller takes the batch path), else an mbft_err with the call's status
// in *st.
constexpr int kNoResident = 1 << 20;
int resident_call(mbft_ctx* c, const mbft_item& it, uint8_t* st);
// Stops and frees it (context destroy).
void resident_destroy(mbft_ctx* c);
// Ends the live resident generation (no call may be in flight: key writes
// hold KeyWriteGuard); the next call relaunches it.  Before a device-wide
// synchronize, which would otherwise wait for the kernel's idle exit.
void resident_park(mbft_ctx* c);
// The same for every resident verifier of the process (before a free that
// synchronizes the device: mbft_host_free).
void resident_park_all();
// The end of a resident-kernel verify (join_host.cpp): the nparts partial
// comb sums (kernels.h SrvCtl::part) joined, infinity rejected, x(R) mod N
// == r tested; r_be: the item's r.  0 accept, 1 reject.
uint8_t host_join_check(const uint32_t* part, int nparts, const uint8_t* r_be);
// The small message checks' calls (check_calls_on, at most
// kResidentCheckMax) through the resident verifier, every item posted at
// once; the caller holds tab_mu shared with the host key map current (a
// lease).  kNoResident when it is off or too few slots are free.
constexpr size_t kResidentCheckMax = 32;
// the default limit (MBFT_RESIDENT_CHECK_MAX): past 16 items the launch's
// batched form measured faster (tools/lowload_probe.py: 64-message windows
// 97 us at 16, 110 at 32, 84 at 8; 16-message windows 36 us at 16, 58 at 8)
constexpr size_t kResidentCheckDefault = 16;
int resident_check(mbft_ctx* c, const mbft_item* items, size_t n, uint8_t* gst,
                   std::vector<UsigCall>* usig);
// One VerifyMessageAuthenTag call through the coalescer (mbft_set_coalescing):
// returns an mbft_err, or MBFT_OK with the call's status in *st.
int coalesced_call(mbft_ctx* c, const mbft_item& it, uint8_t* st);
int verify_batch_flat_impl(mbft_ctx* c, const uint32_t* roles, const uint32_t* ids,
                           const uint8_t* msgs, const uint64_t* msg_off, const uint8_t* tags,
                           const uint64_t* tag_off, size_t n, uint8_t* out, mbft_ctx* g0 = nullptr);
// Batches with at least this many USIG calls build their digests with the
// GPU SHA stage (k_usig_e; env MBFT_GPU_USIG_MIN_CALLS, default 4096).
size_t gpu_usig_min_calls();

// [p, p + bytes) lies in one live mbft_host_alloc allocation (batch.cpp).
bool host_owned(const void* p, size_t bytes);
// The (role, id) -> slot map of key store c on engine g's device (batch.cpp).
int sync_keymap(mbft_ctx* c, mbft_ctx* g);

// The message layer's replay input (messages.cpp): one step of a message's
// validation, and a message's steps in validator order (at most 3: a
// COMMIT's REQUEST signature, PREPARE UI and COMMIT UI).
struct Check {
  uint8_t stage;  // mbft_stage
  uint8_t kind;   // 0 = authenticator call, 1 = fail (no call), 2 = zero-counter UI,
                  // 3 = Go panic (no call)
  uint32_t call;  // unique call index (kind 0)
};
struct MsgChecks {
  uint8_t n = 0;
  Check c[3];
  void push(Check k) { c[n++] = k; }
};
// The in-order replay of a validated message batch (messages.cpp):
// short-circuit per message, stop per stream, stop all after a panic, the
// USIG epoch state evolving call by call.  info / gst: each unique call's
// host outcome and status; stream_of(i): message i's stream; role_of(k):
// unique call k's role.  Writes out[0 .. n).
int replay_messages(mbft_ctx* c, size_t n, const MsgChecks* checks, const CallInfo* info,
                    const uint8_t* gst, uint32_t flags, int32_t* out,
                    const std::function<uint32_t(size_t)>& stream_of,
                    const std::function<uint32_t(uint32_t)>& role_of);
// Its sequential part alone, from message f on: every earlier message's
// result and every capture before f are already in place (the device message
// layer's optimistic pass, msg_kernels.hip k_replay_*).
void replay_tail(mbft_ctx* c, size_t f, size_t n, const MsgChecks* checks, const CallInfo* info,
                 const uint8_t* gst, uint32_t flags, int32_t* out,
                 const std::function<uint32_t(size_t)>& stream_of,
                 const std::function<uint32_t(uint32_t)>& role_of);
// The small check of n messages on engine g (messages.cpp; msgdev.cpp
// mbft_set_small_check): checks[0 .. n), and per unique call its host
// outcome, status and role.  No state read or written.
int check_messages_small(mbft_ctx* c, mbft_ctx* g, const mbft_message* msgs, size_t n,
                         uint32_t n_replicas, MsgChecks* checks, std::vector<CallInfo>& info,
                         std::vector<uint8_t>& gst, std::vector<uint8_t>& role);

}  // namespace mbft_host

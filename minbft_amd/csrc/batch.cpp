// Batch pipeline of the authenticator: n VerifyMessageAuthenTag calls
// (api/api.go:133-144, sample/authentication/authenticator.go:121-134) with
// host buffers in and statuses out.
//
//   1. Per call, on the host worker pool (the pure, byte-level part, in the
//      reference's check order): role key set (keymanager.go:100) -> scheme
//      (authenticator.go:126-129) -> ECDSA roles: Go-exact DER decode
//      (crypto.go:81; a failure is where Go panics) -> key -> digest e =
//      (msg || SHA256(""))[0:32] (crypto.go:121); USIG role: UI / cert split
//      (usig.go:75-80, sgx-usig.go:159-168), strict DER with trailing bytes
//      rejected (usig-enclave.go:217-222), e = SHA256(SHA256(msg) || epoch_le
//      || counter_le) (sgx-usig.go:99-101, usig-enclave.go:204-214) -- on the
//      GPU (k_usig_e) when the batch has many USIG calls.  Call i's (e, r, s,
//      key slot) go to item i of page-locked staging;
//      a call decided on the host carries its status in the slot (kHostSlot
//      | status) and the kernel writes it, so the statuses that come back
//      are final and no host pass merges them.
//   2. Chunk by chunk: H2D on the copy stream while the workers fill the next
//      chunk; s^-1 + verify kernels and the status D2H on two alternating
//      compute streams, so consecutive chunks' kernels overlap.
//   3. In call order: the USIG epoch capture (crypto.go:219-236), the only
//      state, replayed on the host over the USIG calls alone.
// With engines on more GPUs (mbft_ctx_add_device), contiguous shards of the
// calls run this pipeline on every engine at once.
#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <chrono>

#include "host_internal.h"

using namespace mbft_host;

namespace mbft_host {

namespace {

double now_ms() {
  return std::chrono::duration<double, std::milli>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// Calls below this many run the host part on the calling thread only
// (env MBFT_PARALLEL_MIN, for A/Bs); below kParallelMin, one worker per
// kParallelGrain calls.  Measured slower for small checks: at 256 the pool's
// wake-ups cost more than they save (256-message windows 167 -> 218 us,
// 512: 316 -> 421 us, profiles/round5_lowload_parmin_{4096,256}.json).
constexpr size_t kParallelMin = 4096;
constexpr size_t kParallelGrain = 128;
int host_threads_for(const mbft_ctx* g, size_t n) {
  static const size_t lo = [] {
    const char* v = getenv("MBFT_PARALLEL_MIN");
    return v && atol(v) > 0 ? (size_t)atol(v) : kParallelMin;
  }();
  if (n < lo) return 1;
  const size_t t = n / kParallelGrain;
  const size_t p = (size_t)g->pool->size();
  if (n >= kParallelMin) return (int)p;
  return (int)(t < 1 ? 1 : (t < p ? t : p));
}
// Batches up to this many calls stage contiguously (one H2D copy).
constexpr size_t kSmallBatch = 4096;
// Batches up to this many calls take the zero-copy staging (mbft_ctx::zc_*):
// single calls, coalesced groups, small message checks (the small route's
// default limit, 512 messages, so none of its windows takes a copy).  201 B
// per call.
constexpr size_t kZeroCopyMax = 512;
// ... and up to this many have s inverted on the host (below).
constexpr size_t kHostInvMax = 64;

// Batches up to this many calls have s inverted on the HOST (host_winv: ~2
// us of divsteps for one call, Montgomery's trick for several -- 64 in ~10
// us on one core -- where one GPU wave needs ~19 us per item on the
// critical path) and take k_verify_split with the s^-1 R planes staged
// beside e | r | s | slot.  Env MBFT_HOST_INV_MAX (default 64; 0 disables;
// at most the zero-copy batches).
// At most kZeroCopyMax: the planes are staged only in the small batches'
// contiguous layout (e | r | s | slot | planes), which the larger pipeline
// paths do not have.
size_t host_inv_max() {
  static const size_t v = [] {
    const char* e = getenv("MBFT_HOST_INV_MAX");
    const size_t x = e ? (size_t)strtoull(e, nullptr, 10) : kHostInvMax;
    return x < kZeroCopyMax ? x : kZeroCopyMax;
  }();
  return v;
}

// The engine's zero-copy staging, allocated on first use; false when the
// platform cannot map it (then the copy path is used).  Env
// MBFT_ZERO_COPY=0 disables it.
bool zero_copy_ready(mbft_ctx* g) {
  static const bool off = [] {
    const char* v = getenv("MBFT_ZERO_COPY");
    return v && atoi(v) == 0;
  }();
  if (off) return false;
  if (g->zc_state == 0) {
    g->zc_state = -1;
    void* h = nullptr;
    void* d = nullptr;
    if (host_malloc_near(&h, 201 * kZeroCopyMax + 64, hipHostMallocCoherent | hipHostMallocMapped) ==
        hipSuccess) {
      if (hipHostGetDevicePointer(&d, h, 0) == hipSuccess && d) {
        g->zc_host = h;
        g->zc_dev = d;
        g->zc_state = 1;
      } else {
        (void)hipHostFree(h);
      }
    }
  }
  return g->zc_state == 1;
}

// The zero-copy statuses: the host waits for the kernel's status bytes in
// the mapped staging instead of the stream's completion signal (the
// synchronize's wake-up is several us of a lone call's latency).  Every item
// gets its status written once, after its inputs were read for the last
// time, so all n present means the staging is free again.  A bounded spin
// (MBFT_SPIN_US, default 300 us + 4 us a call; 0 disables): past it -- a
// long batch beside other work, or a kernel that failed -- the caller
// synchronizes the stream as before, which also reports a failure.  After a
// successful spin the stream is queried once, so an error the kernel raised
// after writing its statuses is reported by this call, not a later one.
constexpr uint8_t kStatusPending = 0xFF;
bool spin_statuses(mbft_ctx* g, const uint8_t* st, size_t n) {
  static const double spin_env = [] {
    const char* v = getenv("MBFT_SPIN_US");
    return v ? atof(v) / 1000.0 : -1.0;
  }();
  (void)g;
  const double spin_ms = spin_env >= 0 ? spin_env : 0.3 + 0.004 * (double)n;
  if (spin_ms <= 0) return false;
  const volatile uint8_t* vs = st;
  const double t0 = now_ms();
  size_t i = 0;
  for (;;) {
    while (i < n && vs[i] != kStatusPending) i++;
    if (i == n) break;
    if (now_ms() - t0 > spin_ms) return false;
    __builtin_ia32_pause();
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  return true;
}

}  // namespace

void sync_host_keymap(mbft_ctx* c) {
  HostKeyMap& m = c->hkm;
  if (m.gen == c->key_gen) return;
  size_t count = 0;
  uint32_t role_ok = 0;
  for (const auto& r : c->roles) {
    if (r.first < 1 || r.first > 3) continue;
    count += r.second.size();
    if (r.first != MBFT_ROLE_USIG || c->usig_enabled) role_ok |= 1u << r.first;
  }
  size_t cap = 16;
  while (cap < 2 * count) cap <<= 1;
  m.keys.assign(cap, ~0ull);
  m.slots.assign(cap, 0);
  for (const auto& r : c->roles) {
    if (r.first < 1 || r.first > 3) continue;
    for (const auto& kv : r.second) {
      const uint64_t k = ((uint64_t)r.first << 32) | kv.first;
      uint32_t h = mbft::keymap_hash(k) & (uint32_t)(cap - 1);
      while (m.keys[h] != ~0ull) h = (h + 1) & (uint32_t)(cap - 1);
      m.keys[h] = k;
      m.slots[h] = kv.second.slot;
    }
  }
  m.mask = (uint32_t)(cap - 1);
  m.role_ok = role_ok;
  m.gen = c->key_gen;
}

// The pure part of one call.  Writes e, r, s (32 B each) and the key slot of
// GPU item i; returns true if the USIG digest is left to the GPU (defer).
bool prepare_item(const mbft_ctx* c, const mbft_item& it, CallInfo& p, uint8_t* e32, uint8_t* r32,
                  uint8_t* s32, uint32_t* slot, bool defer, Lookup& lk) {
  p = CallInfo();
  *slot = kDeadSlot;
  if ((it.role != lk.role || it.id != lk.id || lk.state < 0) && c->hkm.gen == c->key_gen) {
    // the flat mirror (same outcome as the store below: states 0 / 1 both
    // mean UNKNOWN_ROLE)
    const HostKeyMap& m = c->hkm;
    lk.role = it.role;
    lk.id = it.id;
    if (it.role > 3 || ((m.role_ok >> it.role) & 1u) == 0) {
      lk.state = 0;
    } else {
      const uint64_t key = ((uint64_t)it.role << 32) | it.id;
      lk.state = 2;
      for (uint32_t h = mbft::keymap_hash(key) & m.mask;; h = (h + 1) & m.mask) {
        if (m.keys[h] == key) {
          lk.state = 3;
          lk.slot = m.slots[h];
          break;
        }
        if (m.keys[h] == ~0ull) break;
      }
    }
  }
  if (it.role != lk.role || it.id != lk.id || lk.state < 0) {
    lk.role = it.role;
    lk.id = it.id;
    auto rs = c->roles.find(it.role);
    const bool usig_role = it.role == MBFT_ROLE_USIG;
    if (rs == c->roles.end()) {
      lk.state = 0;
    } else if ((usig_role && !c->usig_enabled) ||
               (!usig_role && it.role != MBFT_ROLE_REPLICA && it.role != MBFT_ROLE_CLIENT)) {
      lk.state = 1;
    } else {
      auto ke = rs->second.find(it.id);
      lk.state = ke == rs->second.end() ? 2 : 3;
      lk.slot = lk.state == 3 ? ke->second.slot : 0;
    }
  }
  if (lk.state <= 1) {  // keymanager.go:100; authenticator.go:126-129 (no scheme)
    p.pre = MBFT_UNKNOWN_ROLE;
    return false;
  }
  const bool is_usig = it.role == MBFT_ROLE_USIG;
  const bool known = lk.state == 3;
  if (!is_usig) {
    // crypto.go:79-89: DER first (Go panics on error), then the pk type check
    size_t consumed = 0;
    if (!mbft_der_parse_sig(it.tag, it.tag_len, r32, s32, &consumed)) {
      p.pre = MBFT_MALFORMED_DER;
      return false;
    }
    if (!known) {
      p.pre = MBFT_UNKNOWN_KEY;
      return false;
    }
    const uint32_t sl = lk.slot;
    if (!c->slots[sl].valid) {
      p.pre = MBFT_BAD_KEY;
      return false;
    }
    // md = msg || SHA256("") (crypto.go:121); e = left-most 32 bytes
    const size_t k0 = it.msg_len < 32 ? it.msg_len : 32;
    if (k0) memcpy(e32, it.msg, k0);
    if (k0 < 32) memcpy(e32 + k0, kEmptyHash, 32 - k0);
    *slot = sl;
    return false;
  }
  // USIG: crypto.go:186-239
  if (it.tag_len < 8) {  // usig.go:75-80
    p.pre = MBFT_BAD_UI;
    return false;
  }
  if (!known) {  // makeUSIGKeyFingerprint(nil) fails
    p.pre = MBFT_UNKNOWN_KEY;
    return false;
  }
  const uint32_t sl = lk.slot;
  if (!c->slots[sl].valid) {
    p.pre = MBFT_BAD_KEY;
    return false;
  }
  p.counter = be64(it.tag);
  const uint8_t* cert = it.tag + 8;
  const size_t cert_len = it.tag_len - 8;
  if (cert_len < 8) {  // ParseCert (both the capture and the VerifyUI paths)
    p.pre = MBFT_BAD_CERT;
    return false;
  }
  p.usig = true;
  p.fpg = c->slots[sl].fp_group;
  p.ui_epoch = be64(cert);
  const uint8_t* sig = cert + 8;
  const size_t sig_len = cert_len - 8;
  size_t consumed = 0;
  if (!mbft_der_parse_sig(sig, sig_len, r32, s32, &consumed)) {
    p.usig_tail = MBFT_MALFORMED_DER;
    return false;
  }
  if (consumed != sig_len) {  // usig-enclave.go:220-221
    p.usig_tail = MBFT_DER_TRAILING;
    return false;
  }
  *slot = sl;
  // e = SHA256(SHA256(msg) || epoch_le || counter_le) with the cert's epoch
  // (only used when it equals the captured epoch)
  if (defer) return true;
  uint8_t buf[48];
  sha256(it.msg, it.msg_len, buf);
  put_le64(buf + 32, p.ui_epoch);
  put_le64(buf + 40, p.counter);
  sha256(buf, 48, e32);
  return false;
}

int host_pool_threads() {
  static const int n = [] {
    for (const char* k : {"MBFT_HOST_THREADS", "OMP_NUM_THREADS"}) {
      const char* v = getenv(k);
      if (v && atoi(v) > 0) return atoi(v) > 64 ? 64 : atoi(v);
    }
    const unsigned h = std::thread::hardware_concurrency();
    return h == 0 ? 1 : (h > 32 ? 32 : (int)h);
  }();
  return n;
}

int pool_workers(const mbft_ctx* g) {
  return g->pool_threads > 0 ? g->pool_threads - 1 : host_pool_threads() - 1;
}

namespace {

// items per pipeline chunk (env MBFT_BATCH_CHUNK, read per batch; 0 = one
// chunk).  256K: same-box sweep over 1M C2 calls (tools/auth_sweep.sh,
// profiles/round2_auth_sweep.jsonl) -- GPU decode 5.3 ms at 128K, 4.4 at
// 256K, 4.7 at 512K, 5.5 as one chunk; host decode 7.0 / 5.2 / 6.6 ms.
size_t chunk_items(size_t n) {
  const char* v = getenv("MBFT_BATCH_CHUNK");
  const size_t ck = v ? (size_t)strtoull(v, nullptr, 10) : (size_t)1 << 18;
  return ck == 0 ? n : ck;
}

// Chunk sizes of a GPU-decode batch of n calls (chunks of ck).  After the
// last copy only the last chunks' decode, s^-1 and verify remain on the
// critical path, so the batch ends in a shorter chunk.  Env MBFT_TAIL_FORM:
//   short    (default) one last chunk of ck / MBFT_TAIL_DIV (default 4);
//   geo      ck / 2, ck / 4, ... down to MBFT_TAIL_MIN (default 4096: a
//            chunk that small takes the per-lane inverse, no chain), the
//            main part's remainder first.  Measured 0.5 ms slower per 1M
//            batch than `short`: kept for the record.
// Env MBFT_TAIL_LOCAL = how many of the last chunks take the one-launch
// s^-1 on their own stream instead of the level chain (default 1: no later
// chunk to hide a five-launch chain behind; 3.95/3.82 -> 3.73/3.79 ms).
std::vector<size_t> chunk_plan(size_t n, size_t ck) {
  std::vector<size_t> out;
  if (ck >= n) {
    out.push_back(n);
    return out;
  }
  const char* form = getenv("MBFT_TAIL_FORM");
  if (!(form && strcmp(form, "geo") == 0)) {
    const char* dv = getenv("MBFT_TAIL_DIV");
    const size_t div = dv ? (size_t)strtoull(dv, nullptr, 10) : 4;
    const size_t tail = div ? ck / div : 0;
    for (size_t lo = 0, m = 0; lo < n; lo += m) {
      const size_t rem = n - lo;
      m = rem > ck + tail ? ck : (rem > 2 * tail && tail > 0 ? rem - tail : rem);
      out.push_back(m);
    }
    return out;
  }
  const char* tv = getenv("MBFT_TAIL_MIN");
  const size_t tmin = std::max<size_t>(tv ? (size_t)strtoull(tv, nullptr, 10) : 4096, 256);
  std::vector<size_t> tail;
  size_t sum = 0;
  for (size_t t = ck / 2; t >= tmin && sum + t + ck <= n; t /= 2) {
    tail.push_back(t);
    sum += t;
  }
  const size_t main = n - sum;
  if (main % ck) out.push_back(main % ck);
  for (size_t j = 0; j < main / ck; j++) out.push_back(ck);
  out.insert(out.end(), tail.begin(), tail.end());
  return out;
}

bool tail_prio() {
  const char* v = getenv("MBFT_TAIL_PRIO");
  return v && atoi(v) != 0;
}

int tail_local() {
  const char* v = getenv("MBFT_TAIL_LOCAL");
  return v ? atoi(v) : 1;
}

// copy streams the chunks' H2D copies alternate over (env MBFT_COPY_STREAMS,
// read per batch: 1 or 2)
int copy_streams() {
  const char* v = getenv("MBFT_COPY_STREAMS");
  return v && atoi(v) == 2 ? 2 : 1;
}

// A worker's deferred USIG digest (GPU SHA stage): call i, its UI fields.
struct DeferredDigest {
  uint32_t i;
  uint64_t epoch, counter;
};

struct Deferred {  // one worker's share of the current chunk
  std::vector<DeferredDigest> item;
  size_t bytes = 0;
  std::vector<UsigCall> usig;   // calls with USIG epoch state to resolve, ascending
  Lookup lk;
};

// The calls of a batch: an mbft_item array, or the flat buffers of the
// pointer-free entry points (read in place, no item array built).
struct ItemArray {
  const mbft_item* items;
  mbft_item operator[](size_t i) const { return items[i]; }
  uint32_t role(size_t i) const { return items[i].role; }
  size_t msg_len(size_t i) const { return items[i].msg_len; }
};

// Flat calls: the wide form (u32 roles, u64 offsets; mbft_verify_batch_flat)
// or the compact one (u8 roles, u32 offsets; mbft_verify_batch_flat32).
struct FlatItems {
  const uint32_t* roles = nullptr;
  const uint32_t* ids = nullptr;
  const uint8_t* msgs = nullptr;
  const uint64_t* msg_off = nullptr;
  const uint8_t* tags = nullptr;
  const uint64_t* tag_off = nullptr;
  bool dev = false;  // every buffer library-owned page-locked: decode on the GPU
  const uint8_t* roles8 = nullptr;                             // compact form
  const uint32_t* msg_off32 = nullptr, *tag_off32 = nullptr;  // compact form
  bool compact() const { return roles8 != nullptr; }
  uint64_t moff(size_t i) const { return msg_off32 ? msg_off32[i] : msg_off[i]; }
  uint64_t toff(size_t i) const { return tag_off32 ? tag_off32[i] : tag_off[i]; }
  mbft_item operator[](size_t i) const {
    const uint64_t m = moff(i), t = toff(i);
    return mbft_item{role(i), ids[i], msgs + m, (size_t)(moff(i + 1) - m), tags + t,
                     (size_t)(toff(i + 1) - t)};
  }
  uint32_t role(size_t i) const { return roles8 ? roles8[i] : roles[i]; }
  size_t msg_len(size_t i) const { return (size_t)(moff(i + 1) - moff(i)); }
  // call i's fields lie inside the batch's byte ranges, in order (the host's
  // check for a call it reads; the device checks every call it decodes)
  bool fields_ok(size_t i, size_t n) const {
    return moff(0) <= moff(i) && moff(i) <= moff(i + 1) && moff(i + 1) <= moff(n) &&
           toff(0) <= toff(i) && toff(i) <= toff(i + 1) && toff(i + 1) <= toff(n);
  }
};

// The pipeline on one engine `g` for calls [base, base + n) of `src` (key
// store of `c`).  gst[i] receives call base + i's status: the host's where
// it decided the call (carried to the kernel in the key slot, kHostSlot |
// status, so the status D2H is already final), else the GPU's.  The calls
// that still need the USIG epoch step are appended to *usig (ascending).
template <class Src>
int engine_check(mbft_ctx* c, mbft_ctx* g, const Src& src, size_t base, size_t n, uint8_t* gst,
                 bool defer, std::vector<UsigCall>* usig) {
  if (n == 0) return MBFT_OK;
  const double t_start = now_ms();
  if (!g->pool) g->pool.reset(new Pool(pool_workers(g)));
  // Small batches (<= kSmallBatch calls: coalesced single calls, short
  // streams) stage e | r | s | slot contiguously and cross PCIe in ONE copy
  // (each separate small copy costs ~8 us of API time on the critical path).
  const bool small = n <= kSmallBatch;
  // the smallest batches: no copy at all, the kernel reads and writes the
  // mapped host staging (the USIG digest stage, defer, only runs past 4,096
  // USIG calls)
  const bool zc = n <= kZeroCopyMax && !defer && zero_copy_ready(g);
  // lone calls: s^-1 R planes (9 x 4 B a call) and u1, u2 (64 B a call:
  // host_winv_u) after e | r | s | slot (the small batches' contiguous
  // staging only)
  const bool hostinv = small && n <= host_inv_max() && !defer;
  const size_t wb = hostinv ? 100 * n : 0;
  // small batches with several USIG calls: their digest chains are built
  // after the prep pass, all at once (sha256_many: equal-length messages
  // interleaved on the SHA unit), instead of one call at a time in
  // prepare_item -- the same bytes hashed, the same e
  const bool hdefer = !defer && small && n >= 4;
  if (zc) {
  } else if (small) {
    HIPCHK(g, g->h_small.ensure(100 * n + wb));
    HIPCHK(g, g->b_small.ensure(100 * n + wb));
  } else {
    HIPCHK(g, g->h_e.ensure(32 * n));
    HIPCHK(g, g->h_r.ensure(32 * n));
    HIPCHK(g, g->h_s.ensure(32 * n));
    HIPCHK(g, g->h_slot.ensure(4 * n));
  }
  HIPCHK(g, g->h_status.ensure(n));
  if (!small) {
    HIPCHK(g, g->b_e.ensure(32 * n));
    HIPCHK(g, g->b_r.ensure(32 * n));
    HIPCHK(g, g->b_s.ensure(32 * n));
    HIPCHK(g, g->b_slot.ensure(4 * n));
  }
  HIPCHK(g, g->b_status.ensure(n));
  uint8_t* he = zc ? static_cast<uint8_t*>(g->zc_host)
                  : small ? g->h_small.as<uint8_t>() : g->h_e.as<uint8_t>();
  uint8_t* hr = small ? he + 32 * n : g->h_r.as<uint8_t>();
  uint8_t* hs = small ? he + 64 * n : g->h_s.as<uint8_t>();
  uint32_t* hslot = small ? reinterpret_cast<uint32_t*>(he + 96 * n) : g->h_slot.as<uint32_t>();
  uint8_t* de = zc ? static_cast<uint8_t*>(g->zc_dev)
                  : small ? g->b_small.as<uint8_t>() : g->b_e.as<uint8_t>();
  uint8_t* dr = small ? de + 32 * n : g->b_r.as<uint8_t>();
  uint8_t* ds = small ? de + 64 * n : g->b_s.as<uint8_t>();
  uint32_t* dslot = small ? reinterpret_cast<uint32_t*>(de + 96 * n) : g->b_slot.as<uint32_t>();
  size_t ubytes = 0, ucalls = 0;
  if (defer) {
    for (size_t i = 0; i < n; i++)
      if (src.role(base + i) == MBFT_ROLE_USIG) {
        ubytes += src.msg_len(base + i);
        ucalls++;
      }
    HIPCHK(g, g->h_udata.ensure(ubytes + 1));
    HIPCHK(g, g->h_uoff.ensure(8 * (ucalls + 1)));
    HIPCHK(g, g->h_uidx.ensure(4 * ucalls + 4));
    HIPCHK(g, g->h_uep.ensure(8 * ucalls + 8));
    HIPCHK(g, g->h_uctr.ensure(8 * ucalls + 8));
    HIPCHK(g, g->b_udata.ensure(ubytes + 1));
    HIPCHK(g, g->b_uoff.ensure(8 * (ucalls + 1)));
    HIPCHK(g, g->b_uidx.ensure(4 * ucalls + 4));
    HIPCHK(g, g->b_uep.ensure(8 * ucalls + 8));
    HIPCHK(g, g->b_uctr.ensure(8 * ucalls + 8));
  }
  const int T = host_threads_for(g, n);
  // Worker state of two chunks: without deferred digests the workers prepare
  // chunk k+1 while this thread enqueues chunk k's copies and kernels.
  std::vector<Deferred> dfr2[2] = {std::vector<Deferred>(T), std::vector<Deferred>(T)};
  const bool overlap = !defer && T > 1;
  size_t ubase = 0, ucount = 0;  // running position in the deferred-digest staging
  const size_t ck = small ? n : chunk_items(n);  // a small batch is one chunk (one copy)
  const int ncs = copy_streams();
  double t_prep = 0;
  // the host part of calls [lo, lo + m) into worker state dfr2[b]
  auto prep_chunk = [&](int b, size_t lo, size_t m) {
    return std::function<void(int)>([&, b, lo, m](int t) {
      const size_t a = lo + m * t / T, e = lo + m * (t + 1) / T;
      Deferred& d = dfr2[b][t];
      d.item.clear();
      d.bytes = 0;
      for (size_t i = a; i < e; i++) {
        const mbft_item it = src[base + i];
        CallInfo p;
        if (prepare_item(c, it, p, he + 32 * i, hr + 32 * i, hs + 32 * i, hslot + i, defer || hdefer,
                         d.lk)) {
          d.item.push_back(DeferredDigest{(uint32_t)i, p.ui_epoch, p.counter});
          d.bytes += it.msg_len;
        }
        if (p.pre != 0xFF) hslot[i] = kHostSlot | p.pre;  // the kernel writes the host's status
        if (p.usig) d.usig.push_back(UsigCall{(uint32_t)(base + i), p});
      }
    });
  };
  {
    const double t0 = now_ms();
    const std::function<void(int)> f0 = prep_chunk(0, 0, n < ck ? n : ck);
    g->pool->run(T, f0);
    if (hdefer) {  // e = SHA256(SHA256(msg) || epoch_le || counter_le), usig-enclave.go:204-214
      std::vector<const uint8_t*> pp;
      std::vector<size_t> ln;
      std::vector<uint8_t*> oo;
      std::vector<uint8_t> buf;
      size_t m = 0;
      for (const Deferred& d : dfr2[0]) m += d.item.size();
      buf.resize(48 * m + 1);
      size_t j = 0;
      for (Deferred& d : dfr2[0]) {
        for (const DeferredDigest& dd : d.item) {
          const mbft_item it = src[base + dd.i];
          uint8_t* b = buf.data() + 48 * j++;
          put_le64(b + 32, dd.epoch);
          put_le64(b + 40, dd.counter);
          pp.push_back(it.msg);
          ln.push_back(it.msg_len);
          oo.push_back(b);
        }
      }
      sha256_many(m, pp.data(), ln.data(), oo.data());  // SHA256(msg) into each buffer's first 32 B
      j = 0;
      for (Deferred& d : dfr2[0]) {
        for (const DeferredDigest& dd : d.item) {
          pp[j] = buf.data() + 48 * j;
          ln[j] = 48;
          oo[j] = he + 32 * dd.i;
          j++;
        }
        d.item.clear();
        d.bytes = 0;
      }
      sha256_many(m, pp.data(), ln.data(), oo.data());
    }
    if (hostinv) host_winv_u(he, hr, hs, n, reinterpret_cast<uint32_t*>(he + 100 * n));
    t_prep += now_ms() - t0;
  }
  std::function<void(int)> fnext;
  // an early error return must not leave workers on a prep of this frame
  struct Join {
    Pool* p;
    ~Join() { p->wait(); }
  } join{g->pool.get()};
  int k = 0;
  for (size_t lo = 0; lo < n; lo += ck, k++) {
    const size_t hi = n - lo < ck ? n : lo + ck, m = hi - lo;
    const bool more = hi < n;
    const size_t mn = more ? (n - hi < ck ? n - hi : ck) : 0;
    if (overlap && more) {
      fnext = prep_chunk((k + 1) & 1, hi, mn);
      g->pool->start(T, fnext);
    }
    const double t0 = now_ms();
    std::vector<Deferred>& dfr = dfr2[k & 1];
    // ascending call order: chunk by chunk, worker by worker
    for (Deferred& d : dfr) {
      if (usig) usig->insert(usig->end(), d.usig.begin(), d.usig.end());
      d.usig.clear();
    }
    size_t nu = 0;
    if (defer) {
      // offsets of each worker's deferred messages, then copy them in
      std::vector<size_t> boff(T), coff(T);
      size_t bb = ubase, cc = ucount;
      for (int t = 0; t < T; t++) {
        boff[t] = bb;
        coff[t] = cc;
        bb += dfr[t].bytes;
        cc += dfr[t].item.size();
      }
      nu = cc - ucount;
      uint8_t* ud = g->h_udata.as<uint8_t>();
      uint64_t* uo = g->h_uoff.as<uint64_t>();
      uint32_t* ui = g->h_uidx.as<uint32_t>();
      uint64_t* ue = g->h_uep.as<uint64_t>();
      uint64_t* uc = g->h_uctr.as<uint64_t>();
      g->pool->run(T, [&](int t) {
        size_t pos = boff[t], j = coff[t];
        for (const DeferredDigest& dd : dfr[t].item) {
          const mbft_item it = src[base + dd.i];
          if (it.msg_len) memcpy(ud + pos, it.msg, it.msg_len);
          uo[j] = pos;
          ui[j] = dd.i;
          ue[j] = dd.epoch;
          uc[j] = dd.counter;
          pos += it.msg_len;
          j++;
        }
      });
      if (nu) uo[ucount + nu] = bb;  // end offset of this chunk's last message
      ubase = bb;
    }
    t_prep += now_ms() - t0;
    // H2D of this chunk on the copy stream (the workers go on with the next)
    const bool alt = ncs == 2 && (k & 1);
    // a small batch (one chunk) runs copy, kernels and statuses on ONE stream:
    // no cross-stream event, one synchronize
    hipStream_t cs = small ? g->vstream[0] : alt ? g->cstream2 : g->cstream;
    hipEvent_t evh = alt ? g->ev_h2d2 : g->ev_h2d;
    if (zc) {
      // no copy: the kernel reads e | r | s | slot from the mapped staging
    } else if (small) {  // one chunk, one copy
      HIPCHK(g, hipMemcpyAsync(de, he, 100 * n + wb, hipMemcpyHostToDevice, cs));
    } else {
      HIPCHK(g, hipMemcpyAsync(de + 32 * lo, he + 32 * lo, 32 * m, hipMemcpyHostToDevice, cs));
      HIPCHK(g, hipMemcpyAsync(dr + 32 * lo, hr + 32 * lo, 32 * m, hipMemcpyHostToDevice, cs));
      HIPCHK(g, hipMemcpyAsync(ds + 32 * lo, hs + 32 * lo, 32 * m, hipMemcpyHostToDevice, cs));
      HIPCHK(g, hipMemcpyAsync(dslot + lo, hslot + lo, 4 * m, hipMemcpyHostToDevice, cs));
    }
    if (nu) {
      const size_t b0 = g->h_uoff.as<uint64_t>()[ucount], b1 = ubase;
      HIPCHK(g, hipMemcpyAsync(g->b_udata.as<uint8_t>() + b0, g->h_udata.as<uint8_t>() + b0, b1 - b0,
                               hipMemcpyHostToDevice, cs));
      HIPCHK(g, hipMemcpyAsync(g->b_uoff.as<uint64_t>() + ucount, g->h_uoff.as<uint64_t>() + ucount,
                               8 * (nu + 1), hipMemcpyHostToDevice, cs));
      HIPCHK(g, hipMemcpyAsync(g->b_uidx.as<uint32_t>() + ucount, g->h_uidx.as<uint32_t>() + ucount,
                               4 * nu, hipMemcpyHostToDevice, cs));
      HIPCHK(g, hipMemcpyAsync(g->b_uep.as<uint64_t>() + ucount, g->h_uep.as<uint64_t>() + ucount,
                               8 * nu, hipMemcpyHostToDevice, cs));
      HIPCHK(g, hipMemcpyAsync(g->b_uctr.as<uint64_t>() + ucount, g->h_uctr.as<uint64_t>() + ucount,
                               8 * nu, hipMemcpyHostToDevice, cs));
      // the digests land in e at their items (after e's own H2D)
      HIPCHK(g, mbft_launch::usig_e(g->b_udata.as<uint8_t>(), g->b_uoff.as<uint64_t>() + ucount,
                                    g->b_uep.as<uint64_t>() + ucount,
                                    g->b_uctr.as<uint64_t>() + ucount,
                                    g->b_uidx.as<uint32_t>() + ucount, (long)nu,
                                    de, cs));
      ucount += nu;
    }
    hipStream_t vs = g->vstream[k & 1];
    if (!small) {
      HIPCHK(g, hipEventRecord(evh, cs));
      HIPCHK(g, hipStreamWaitEvent(vs, evh, 0));
    }
    // zero copy: the statuses land in the mapped staging after the inputs
    uint8_t* dst_dev = zc ? de + 100 * n + wb : g->b_status.as<uint8_t>() + lo;
    if (zc) memset(he + 100 * n + wb, kStatusPending, n);  // spin_statuses' marker
    int rc = verify_device(g, de + 32 * lo, dr + 32 * lo, ds + 32 * lo, dslot + lo, m, dst_dev, vs,
                           /*host_status=*/true, /*latency=*/false,
                           hostinv ? reinterpret_cast<const uint32_t*>(de + 100 * n) : nullptr);
    if (rc) return rc;
    if (!zc)
      HIPCHK(g, hipMemcpyAsync(g->h_status.as<uint8_t>() + lo, g->b_status.as<uint8_t>() + lo, m,
                               hipMemcpyDeviceToHost, vs));
    if (more) {
      const double t2 = now_ms();
      if (overlap) {
        g->pool->wait();
      } else {
        fnext = prep_chunk((k + 1) & 1, hi, mn);
        g->pool->run(T, fnext);
      }
      t_prep += now_ms() - t2;
    }
  }
  const double t1 = now_ms();
  if (!(zc && spin_statuses(g, he + 100 * n + wb, n))) {
    HIPCHK(g, hipStreamSynchronize(g->vstream[0]));
    if (!small) HIPCHK(g, hipStreamSynchronize(g->vstream[1]));
  } else {
    const hipError_t q = hipStreamQuery(g->vstream[0]);
    if (q != hipSuccess && q != hipErrorNotReady) return hip_fail(g, q, "verify kernel (after its statuses)");
  }
  const double t2 = now_ms();
  // the statuses are final (host-decided ones written by the kernel); the
  // USIG epoch step is left to the caller, in call order
  const uint8_t* hst = zc ? he + 100 * n + wb : g->h_status.as<uint8_t>();
  g->pool->run(T, [&](int t) {
    const size_t a = n * t / T, b = n * (t + 1) / T;
    memcpy(gst + a, hst + a, b - a);
  });
  static const bool trace = getenv("MBFT_STAGE_TRACE") != nullptr;
  if (trace)
    fprintf(stderr, "[mbft stage] n=%zu T=%d chunks=%d prep=%.3f enqueue+prep=%.3f wait=%.3f copy=%.3f ms\n",
            n, T, k, t_prep, t1 - t_start, t2 - t1, now_ms() - t2);
  if (g == c) {
    c->st_prepare_ms += t_prep + (now_ms() - t2);
    c->st_gpu_ms += t2 - t1;
  }
  return MBFT_OK;
}

// ---------------------------------------------------------------------------
// Device-side decode (k_prepare).  The host's only per-call work is the
// USIG calls' part of the epoch step (their CallInfo, prepare_item without
// the digest), found by a scan of the 4-byte roles and run on the pool while
// the GPU decodes and verifies.

}  // namespace

// The (role, id) -> slot map of key store c on engine g's device.
int sync_keymap(mbft_ctx* c, mbft_ctx* g) {
  if (g->kmap_gen == c->key_gen && g->d_kmap_keys.p) return MBFT_OK;
  size_t count = 0;
  uint32_t role_ok = 0;
  for (const auto& r : c->roles) {
    if (r.first < 1 || r.first > 3) continue;  // no scheme: UNKNOWN_ROLE on the device too
    count += r.second.size();
    if (r.first != MBFT_ROLE_USIG || c->usig_enabled) role_ok |= 1u << r.first;
  }
  size_t cap = 16;
  while (cap < 2 * count) cap <<= 1;
  std::vector<uint64_t> keys(cap, ~0ull);
  std::vector<uint32_t> slots(cap, 0);
  for (const auto& r : c->roles) {
    if (r.first < 1 || r.first > 3) continue;
    for (const auto& kv : r.second) {
      const uint64_t k = ((uint64_t)r.first << 32) | kv.first;
      uint32_t h = mbft::keymap_hash(k) & (uint32_t)(cap - 1);
      while (keys[h] != ~0ull) h = (h + 1) & (uint32_t)(cap - 1);
      keys[h] = k;
      slots[h] = kv.second.slot;
    }
  }
  HIPCHK(g, g->d_kmap_keys.ensure(8 * cap));
  HIPCHK(g, g->d_kmap_slots.ensure(4 * cap));
  HIPCHK(g, hipMemcpyAsync(g->d_kmap_keys.p, keys.data(), 8 * cap, hipMemcpyHostToDevice, g->kstream));
  HIPCHK(g, hipMemcpyAsync(g->d_kmap_slots.p, slots.data(), 4 * cap, hipMemcpyHostToDevice, g->kstream));
  HIPCHK(g, hipStreamSynchronize(g->kstream));
  g->kmap_mask = (uint32_t)(cap - 1);
  g->kmap_role_ok = role_ok;
  g->kmap_gen = c->key_gen;
  return MBFT_OK;
}

namespace {

int engine_check_dev(mbft_ctx* c, mbft_ctx* g, const FlatItems& src, size_t base, size_t n,
                     uint8_t* gst, bool gst_pinned, std::vector<UsigCall>* usig) {
  if (n == 0) return MBFT_OK;
  const double t_start = now_ms();
  if (!g->pool) g->pool.reset(new Pool(pool_workers(g)));
  const uint64_t mb0 = src.moff(base), tb0 = src.toff(base);
  const size_t mbytes = (size_t)(src.moff(base + n) - mb0);
  const size_t tbytes = (size_t)(src.toff(base + n) - tb0);
  const size_t rsz = src.compact() ? 1 : 4, osz = src.compact() ? 4 : 8;
  HIPCHK(g, g->b_e.ensure(32 * n));
  HIPCHK(g, g->b_r.ensure(32 * n));
  HIPCHK(g, g->b_s.ensure(32 * n));
  HIPCHK(g, g->b_slot.ensure(4 * n));
  HIPCHK(g, g->b_status.ensure(n));
  HIPCHK(g, g->b_roles.ensure(4 * n));
  HIPCHK(g, g->b_ids.ensure(4 * n));
  HIPCHK(g, g->b_moff.ensure(8 * (n + 1)));
  HIPCHK(g, g->b_toff.ensure(8 * (n + 1)));
  HIPCHK(g, g->b_bad.ensure(4));
  HIPCHK(g, g->hm_bad.ensure(4));
  HIPCHK(g, g->b_msgs.ensure(mbytes + 16));
  HIPCHK(g, g->b_tags.ensure(tbytes + 16));
  if (!gst_pinned) HIPCHK(g, g->h_status.ensure(n));
  int rc = sync_keymap(c, g);
  if (rc) return rc;
  // Offsets are checked where they are used, not in a host pass over every
  // call (1.3 ms per 1M calls on one thread): the chunk boundaries here, each
  // call's fields by k_prepare against its chunk's byte ranges (a bad call
  // sets b_bad and reads nothing), the USIG calls' fields by the host scan
  // below before it reads them.  Any of them -> MBFT_ERR_ARG.
  const std::vector<size_t> plan = chunk_plan(n, chunk_items(n));
  for (size_t lo = 0, k0 = 0; lo < n; lo += plan[k0], k0++) {
    const size_t hi = lo + plan[k0];
    if (src.moff(base + hi) < src.moff(base + lo) || src.moff(base + hi) > mb0 + mbytes ||
        src.toff(base + hi) < src.toff(base + lo) || src.toff(base + hi) > tb0 + tbytes ||
        src.moff(base + lo) < mb0 || src.toff(base + lo) < tb0)
      return fail(g, MBFT_ERR_ARG, "flat batch: offsets out of order");
  }
  std::atomic<bool> host_bad{false};
  // USIG calls' host part, in call order per worker, on the pool meanwhile
  const int T = host_threads_for(g, n);
  std::vector<std::vector<UsigCall>> us(T);
  const std::function<void(int)> scan = [&](int t) {
    const size_t a = n * t / T, b = n * (t + 1) / T;
    Lookup lk;
    uint8_t e[32], r[32], s[32];
    uint32_t sl;
    for (size_t i = a; i < b; i++) {
      if (src.role(base + i) != MBFT_ROLE_USIG) continue;
      if (!src.fields_ok(base + i, base + n) || src.moff(base + i) < mb0 || src.toff(base + i) < tb0) {
        host_bad = true;
        continue;
      }
      CallInfo p;
      prepare_item(c, src[base + i], p, e, r, s, &sl, /*defer=*/true, lk);
      if (p.usig) us[t].push_back(UsigCall{(uint32_t)(base + i), p});
    }
  };
  struct Join {
    Pool* p;
    ~Join() { p->wait(); }
  } join{g->pool.get()};
  if (usig) g->pool->start(T, scan);
  const int ncs = copy_streams();
  int k = 0;
  const int nlocal = tail_local();
  // The four per-call arrays (roles, ids, offsets: 24 B per call) go up whole
  // before the first chunk's bytes when the batch is chunked: each copy costs
  // the DMA engine ~10 us of setup, so 4 copies instead of 4 per chunk (env
  // MBFT_SMALL_FIRST=0: per chunk, as the bytes).
  static const bool small_first = [] {
    const char* v = getenv("MBFT_SMALL_FIRST");
    return !(v && atoi(v) == 0);
  }();
  const bool upfront = small_first && plan.size() > 1;
  bool used_prio = false;
  // device copies of the per-call arrays keep the caller's widths
  const void* roles_src = src.compact() ? (const void*)src.roles8 : (const void*)src.roles;
  const void* moff_src = src.compact() ? (const void*)src.msg_off32 : (const void*)src.msg_off;
  const void* toff_src = src.compact() ? (const void*)src.tag_off32 : (const void*)src.tag_off;
  auto copy_small = [&](size_t lo, size_t m, hipStream_t cs) -> int {
    HIPCHK(g, hipMemcpyAsync(g->b_roles.as<uint8_t>() + rsz * lo,
                             static_cast<const uint8_t*>(roles_src) + rsz * (base + lo), rsz * m,
                             hipMemcpyHostToDevice, cs));
    HIPCHK(g, hipMemcpyAsync(g->b_ids.as<uint32_t>() + lo, src.ids + base + lo, 4 * m,
                             hipMemcpyHostToDevice, cs));
    HIPCHK(g, hipMemcpyAsync(g->b_moff.as<uint8_t>() + osz * lo,
                             static_cast<const uint8_t*>(moff_src) + osz * (base + lo), osz * (m + 1),
                             hipMemcpyHostToDevice, cs));
    HIPCHK(g, hipMemcpyAsync(g->b_toff.as<uint8_t>() + osz * lo,
                             static_cast<const uint8_t*>(toff_src) + osz * (base + lo), osz * (m + 1),
                             hipMemcpyHostToDevice, cs));
    return MBFT_OK;
  };
  HIPCHK(g, hipMemsetAsync(g->b_bad.p, 0, 4, g->cstream));
  if (ncs == 2 && !upfront) {  // the second copy stream's k_prepare sets b_bad after the clear
    HIPCHK(g, hipEventRecord(g->ev_in, g->cstream));
    HIPCHK(g, hipStreamWaitEvent(g->cstream2, g->ev_in, 0));
  }
  if (upfront) {
    rc = copy_small(0, n, g->cstream);
    if (rc) return rc;
    if (ncs == 2) {  // the second copy stream's chunks read them too
      HIPCHK(g, hipEventRecord(g->ev_in, g->cstream));
      HIPCHK(g, hipStreamWaitEvent(g->cstream2, g->ev_in, 0));
    }
  }
  for (size_t lo = 0, m = 0; lo < n; lo += m, k++) {
    m = plan[k];
    const size_t hi = lo + m;
    const bool latency = (int)(plan.size() - (size_t)k) <= nlocal;
    const uint64_t ma = src.moff(base + lo) - mb0, mz = src.moff(base + hi) - mb0;
    const uint64_t ta = src.toff(base + lo) - tb0, tz = src.toff(base + hi) - tb0;
    const bool alt = ncs == 2 && (k & 1);
    hipStream_t cs = alt ? g->cstream2 : g->cstream;
    hipEvent_t evh = alt ? g->ev_h2d2 : g->ev_h2d;
    if (!upfront) {
      rc = copy_small(lo, m, cs);
      if (rc) return rc;
    }
    if (mz > ma)
      HIPCHK(g, hipMemcpyAsync(g->b_msgs.as<uint8_t>() + ma, src.msgs + mb0 + ma, mz - ma,
                               hipMemcpyHostToDevice, cs));
    if (tz > ta)
      HIPCHK(g, hipMemcpyAsync(g->b_tags.as<uint8_t>() + ta, src.tags + tb0 + ta, tz - ta,
                               hipMemcpyHostToDevice, cs));
    mbft::PrepArgs a{};
    if (src.compact()) {
      a.roles8 = g->b_roles.as<uint8_t>() + lo;
      a.moff32 = g->b_moff.as<uint32_t>() + lo;
      a.toff32 = g->b_toff.as<uint32_t>() + lo;
    } else {
      a.roles = g->b_roles.as<uint32_t>() + lo;
      a.moff = g->b_moff.as<uint64_t>() + lo;
      a.toff = g->b_toff.as<uint64_t>() + lo;
    }
    a.ids = g->b_ids.as<uint32_t>() + lo;
    a.msgs = g->b_msgs.as<uint8_t>();
    a.tags = g->b_tags.as<uint8_t>();
    a.mbase = mb0;
    a.tbase = tb0;
    a.mlo = mb0 + ma;  // this chunk's byte ranges (absolute offsets)
    a.mhi = mb0 + mz;
    a.tlo = tb0 + ta;
    a.thi = tb0 + tz;
    a.bad = g->b_bad.as<uint32_t>();
    a.n = (long)m;
    a.map = mbft::KeyMap{g->d_kmap_keys.as<uint64_t>(), g->d_kmap_slots.as<uint32_t>(),
                         g->kmap_mask, g->kmap_role_ok};
    a.keys = tabs(g)->d_keys.as<mbft::KeyDesc>();
    a.nslots = (uint32_t)tabs(g)->slots.size();
    a.e = g->b_e.as<uint8_t>() + 32 * lo;
    a.r = g->b_r.as<uint8_t>() + 32 * lo;
    a.s = g->b_s.as<uint8_t>() + 32 * lo;
    a.slot = g->b_slot.as<uint32_t>() + lo;
    // MBFT_TAIL_PRIO: the latency chunks' decode, s^-1, verify and statuses
    // on the high-priority stream, so their workgroups are dispatched ahead of
    // the previous chunk's remaining verify workgroups
    const bool prio = latency && tail_prio();
    hipStream_t vs = prio ? g->istream : g->vstream[k & 1];
    if (prio) {
      HIPCHK(g, hipEventRecord(evh, cs));
      HIPCHK(g, hipStreamWaitEvent(vs, evh, 0));
      HIPCHK(g, mbft_launch::prepare_calls(a, vs));
    } else {
      HIPCHK(g, mbft_launch::prepare_calls(a, cs));
      HIPCHK(g, hipEventRecord(evh, cs));
      HIPCHK(g, hipStreamWaitEvent(vs, evh, 0));
    }
    used_prio |= prio;
    rc = verify_device(g, a.e, a.r, a.s, a.slot, m, g->b_status.as<uint8_t>() + lo, vs,
                       /*host_status=*/true, latency);
    if (rc) return rc;
    uint8_t* dst = gst_pinned ? gst + lo : g->h_status.as<uint8_t>() + lo;
    HIPCHK(g, hipMemcpyAsync(dst, g->b_status.as<uint8_t>() + lo, m, hipMemcpyDeviceToHost, vs));
    if (lo + m == n) {  // after every chunk's k_prepare: in order on each copy stream; with
                        // two, vs also waits for the other one's last chunk
      if (ncs == 2 && k > 0) HIPCHK(g, hipStreamWaitEvent(vs, alt ? g->ev_h2d : g->ev_h2d2, 0));
      HIPCHK(g, hipMemcpyAsync(g->hm_bad.p, g->b_bad.p, 4, hipMemcpyDeviceToHost, vs));
    }
  }
  const double t1 = now_ms();
  HIPCHK(g, hipStreamSynchronize(g->vstream[0]));
  HIPCHK(g, hipStreamSynchronize(g->vstream[1]));
  if (used_prio) HIPCHK(g, hipStreamSynchronize(g->istream));
  const double t2 = now_ms();
  g->pool->wait();
  if (host_bad || *g->hm_bad.as<uint32_t>() != 0)
    return fail(g, MBFT_ERR_ARG, "flat batch: a call's offsets lie outside its byte range or out of order");
  if (usig)
    for (auto& u : us) usig->insert(usig->end(), u.begin(), u.end());
  if (!gst_pinned) {
    const uint8_t* hst = g->h_status.as<uint8_t>();
    g->pool->run(T, [&](int t) {
      const size_t a = n * t / T, b = n * (t + 1) / T;
      memcpy(gst + a, hst + a, b - a);
    });
  }
  static const bool trace = getenv("MBFT_STAGE_TRACE") != nullptr;
  if (trace)
    fprintf(stderr, "[mbft stage dev] n=%zu chunks=%d enqueue=%.3f wait=%.3f usig+copy=%.3f ms\n", n,
            k, t1 - t_start, t2 - t1, now_ms() - t2);
  if (g == c) {
    c->st_prepare_ms += (t1 - t_start) + (now_ms() - t2);
    c->st_gpu_ms += t2 - t1;
  }
  return MBFT_OK;
}

inline bool is_dev(const ItemArray&) { return false; }
inline bool is_dev(const FlatItems& f) { return f.dev; }

template <class Src>
int engine_run(mbft_ctx* c, mbft_ctx* g, const Src& src, size_t base, size_t n, uint8_t* gst,
               bool defer, bool gst_pinned, std::vector<UsigCall>* usig) {
  (void)gst_pinned;
  return engine_check(c, g, src, base, n, gst, defer, usig);
}

template <>
int engine_run<FlatItems>(mbft_ctx* c, mbft_ctx* g, const FlatItems& src, size_t base, size_t n,
                          uint8_t* gst, bool defer, bool gst_pinned, std::vector<UsigCall>* usig) {
  if (src.dev) return engine_check_dev(c, g, src, base, n, gst, gst_pinned, usig);
  return engine_check(c, g, src, base, n, gst, defer, usig);
}

// g0: the engine for the first shard (the context itself, or a leased lane).
template <class Src>
int check_calls_src(mbft_ctx* c, const Src& src, size_t n, uint8_t* gst,
                    std::vector<UsigCall>* usig, bool gst_pinned = false, mbft_ctx* g0 = nullptr) {
  if (!g0) g0 = c;
  if (n == 0) return MBFT_OK;
  sync_host_keymap(c);
  size_t nusig = 0;
  if (!is_dev(src))  // the device decode builds every digest on the GPU anyway
    for (size_t i = 0; i < n; i++) nusig += src.role(i) == MBFT_ROLE_USIG;
  const bool defer = nusig >= gpu_usig_min_calls();  // GPU SHA stage for large USIG batches
  if (c->slots.empty()) {
    // no key registered: every call is decided on the host (UNKNOWN_KEY at
    // worst); nothing for the GPU
    uint8_t e[32], r[32], s[32];
    uint32_t sl;
    Lookup lk;
    for (size_t i = 0; i < n; i++) {
      CallInfo p;
      prepare_item(c, src[i], p, e, r, s, &sl, false, lk);
      gst[i] = p.pre != 0xFF ? p.pre : MBFT_BAD_KEY;
      if (usig && p.usig) usig->push_back(UsigCall{(uint32_t)i, p});
    }
    return MBFT_OK;
  }
  const size_t engines = 1 + c->peers.size();
  size_t k = c->shard_min ? n / c->shard_min : engines;
  if (k > engines) k = engines;
  if (k <= 1) {
    const int rc = engine_run(c, g0, src, 0, n, gst, defer, gst_pinned, usig);
    return rc && g0 != c ? fail(c, rc, std::string("lane: ") + g0->err) : rc;
  }
  std::vector<int> rcs(k, MBFT_OK);
  std::vector<std::vector<UsigCall>> us(k);
  // shards 1 .. k-1 on threads of their own, shard 0 on the caller's thread
  // (it holds the context's lock or the lane's lease)
  auto shard = [=, &src, &rcs, &us](size_t j) {
    const size_t lo = n * j / k, hi = n * (j + 1) / k;
    mbft_ctx* eng = j == 0 ? g0 : c->peers[j - 1];
    std::unique_lock<std::mutex> g(eng->mu, std::defer_lock);
    if (j != 0) g.lock();
    if (hipSetDevice(eng->device) != hipSuccess) {
      rcs[j] = MBFT_ERR_HIP;
      return;
    }
    rcs[j] = engine_run(c, eng, src, lo, hi - lo, gst + lo, defer, gst_pinned, usig ? &us[j] : nullptr);
  };
  // shards 1 .. k-1 on their engines' persistent threads (no thread start
  // per batch), shard 0 here
  std::vector<uint64_t> tickets(k, 0);
  for (size_t j = 1; j < k; j++) tickets[j] = engine_worker(c->peers[j - 1]).submit([&shard, j] { shard(j); });
  shard(0);
  for (size_t j = 1; j < k; j++) engine_worker(c->peers[j - 1]).wait(tickets[j]);
  if (usig)
    for (auto& u : us) usig->insert(usig->end(), u.begin(), u.end());
  (void)hipSetDevice(c->device);
  for (size_t j = 0; j < k; j++)
    if (rcs[j]) {
      mbft_ctx* eng = j == 0 ? g0 : c->peers[j - 1];
      return eng == c ? rcs[j] : fail(c, rcs[j], std::string("engine: ") + eng->err);
    }
  return MBFT_OK;
}

// n calls in order: the pure part on the GPU, then the USIG epoch step in
// call order (the epoch map), straight into `out`.
// With a lane (g0 != c): the check runs without the context's mutex (the
// caller holds tab_mu shared and the lane's lease); the epoch step then
// takes the mutex, so concurrent batches apply theirs one batch at a time.
template <class Src>
int verify_batch_src(mbft_ctx* c, const Src& src, size_t n, uint8_t* out, bool out_pinned = false,
                     mbft_ctx* g0 = nullptr) {
  if (n == 0) return MBFT_OK;
  const double t0 = now_ms();
  std::vector<UsigCall> usig;
  int rc = check_calls_src(c, src, n, out, &usig, out_pinned, g0);
  if (rc) return rc;
  std::unique_lock<std::mutex> lk(c->mu, std::defer_lock);
  if (g0 && g0 != c) lk.lock();
  const double t1 = now_ms();
  for (const UsigCall& u : usig) out[u.i] = resolve_call(c, u.p, out[u.i]);
  const double t2 = now_ms();
  c->st_resolve_ms += t2 - t1;
  c->st_total_ms += t2 - t0;
  c->st_calls += 1;
  c->st_items += (double)n;
  return MBFT_OK;
}

}  // namespace

int check_calls(mbft_ctx* c, const mbft_item* items, size_t n, uint8_t* gst,
                std::vector<UsigCall>* usig, mbft_ctx* g0) {
  return check_calls_src(c, ItemArray{items}, n, gst, usig, false, g0);
}

int check_calls_on(mbft_ctx* c, mbft_ctx* g, const mbft_item* items, size_t n, uint8_t* gst,
                   std::vector<UsigCall>* usig) {
  if (n == 0) return MBFT_OK;
  if (c->res_on.load(std::memory_order_relaxed) && n <= kResidentCheckMax && !c->slots.empty()) {
    const int rr = resident_check(c, items, n, gst, usig);  // no launch: the resident kernel
    if (rr != kNoResident) return rr;
  }
  const int rc = engine_check(c, g, ItemArray{items}, 0, n, gst, /*defer=*/false, usig);
  return rc && g != c ? fail(c, rc, std::string("lane: ") + g->err) : rc;
}

// Library-owned page-locked host memory (mbft_host_alloc): [start, end) of
// every live allocation, process-wide (any context, any engine may DMA it).
namespace {
std::mutex g_host_mu;
std::map<uintptr_t, uintptr_t> g_host_allocs;
}  // namespace

bool host_owned(const void* p, size_t bytes) {
  if (bytes == 0) return true;
  if (!p) return false;
  const uintptr_t a = (uintptr_t)p;
  std::lock_guard<std::mutex> g(g_host_mu);
  auto it = g_host_allocs.upper_bound(a);
  if (it == g_host_allocs.begin()) return false;
  --it;
  return a >= it->first && a + bytes <= it->second;
}

namespace {

// The device decode applies when it is enabled and every buffer of the calls
// is library-owned page-locked memory (DMA straight from it, no staging).
FlatItems flat_src(mbft_ctx* c, const uint32_t* roles, const uint32_t* ids, const uint8_t* msgs,
                   const uint64_t* msg_off, const uint8_t* tags, const uint64_t* tag_off,
                   size_t n) {
  FlatItems f;
  f.roles = roles;
  f.ids = ids;
  f.msgs = msgs;
  f.msg_off = msg_off;
  f.tags = tags;
  f.tag_off = tag_off;
  f.dev = c->dev_prepare != 0 && n > 0 && host_owned(roles, 4 * n) && host_owned(ids, 4 * n) &&
          host_owned(msg_off, 8 * (n + 1)) && host_owned(tag_off, 8 * (n + 1)) &&
          msg_off[n] >= msg_off[0] && tag_off[n] >= tag_off[0] &&
          host_owned(msgs + msg_off[0], (size_t)(msg_off[n] - msg_off[0])) &&
          host_owned(tags + tag_off[0], (size_t)(tag_off[n] - tag_off[0]));
  return f;
}

FlatItems flat_src32(mbft_ctx* c, const uint8_t* roles, const uint32_t* ids, const uint8_t* msgs,
                     const uint32_t* msg_off, const uint8_t* tags, const uint32_t* tag_off,
                     size_t n) {
  FlatItems f;
  f.roles8 = roles;
  f.ids = ids;
  f.msgs = msgs;
  f.msg_off32 = msg_off;
  f.tags = tags;
  f.tag_off32 = tag_off;
  f.dev = c->dev_prepare != 0 && n > 0 && host_owned(roles, n) && host_owned(ids, 4 * n) &&
          host_owned(msg_off, 4 * (n + 1)) && host_owned(tag_off, 4 * (n + 1)) &&
          msg_off[n] >= msg_off[0] && tag_off[n] >= tag_off[0] &&
          host_owned(msgs + msg_off[0], (size_t)(msg_off[n] - msg_off[0])) &&
          host_owned(tags + tag_off[0], (size_t)(tag_off[n] - tag_off[0]));
  return f;
}
}  // namespace

namespace {

// The host pass over every call's offsets, for batches the host decodes
// (the device decode checks them where it reads them).
bool flat_offsets_ok(const FlatItems& f, size_t n) {
  bool bad = false;
  for (size_t i = 0; i < n; i++) bad |= (f.moff(i + 1) < f.moff(i)) | (f.toff(i + 1) < f.toff(i));
  return !bad;
}

}  // namespace

int check_calls_flat(mbft_ctx* c, const uint32_t* roles, const uint32_t* ids, const uint8_t* msgs,
                     const uint64_t* msg_off, const uint8_t* tags, const uint64_t* tag_off,
                     size_t n, uint8_t* gst, mbft_ctx* g0) {
  const FlatItems f = flat_src(c, roles, ids, msgs, msg_off, tags, tag_off, n);
  if (!f.dev && !flat_offsets_ok(f, n)) return fail(c, MBFT_ERR_ARG, "flat batch: offsets out of order");
  return check_calls_src(c, f, n, gst, nullptr, f.dev && host_owned(gst, n), g0);
}

int verify_batch_impl(mbft_ctx* c, const mbft_item* items, size_t n, uint8_t* out, mbft_ctx* g0) {
  return verify_batch_src(c, ItemArray{items}, n, out, false, g0);
}

int verify_batch_flat_impl(mbft_ctx* c, const uint32_t* roles, const uint32_t* ids,
                           const uint8_t* msgs, const uint64_t* msg_off, const uint8_t* tags,
                           const uint64_t* tag_off, size_t n, uint8_t* out, mbft_ctx* g0) {
  const FlatItems f = flat_src(c, roles, ids, msgs, msg_off, tags, tag_off, n);
  if (!f.dev && !flat_offsets_ok(f, n)) return fail(c, MBFT_ERR_ARG, "flat batch: offsets out of order");
  return verify_batch_src(c, f, n, out, f.dev && host_owned(out, n), g0);
}


// The compact flat form: u8 roles, u32 offsets (mbft_verify_batch_flat32).
int flat32_impl(mbft_ctx* c, const uint8_t* roles, const uint32_t* ids, const uint8_t* msgs,
                const uint32_t* msg_off, const uint8_t* tags, const uint32_t* tag_off, size_t n,
                uint8_t* out, mbft_ctx* g0, bool verify) {
  const FlatItems f = flat_src32(c, roles, ids, msgs, msg_off, tags, tag_off, n);
  if (!f.dev && !flat_offsets_ok(f, n)) return fail(c, MBFT_ERR_ARG, "flat batch: offsets out of order");
  const bool pinned = f.dev && host_owned(out, n);
  return verify ? verify_batch_src(c, f, n, out, pinned, g0)
                : check_calls_src(c, f, n, out, nullptr, pinned, g0);
}

// Apply one call's outcome in order: the USIG epoch capture is the only
// state (crypto.go:219-236).
uint8_t resolve_call(mbft_ctx* c, const CallInfo& p, uint8_t g) {
  if (p.pre != 0xFF) return p.pre;
  if (!p.usig) return g;
  uint64_t epoch;
  if (c->epoch_set[p.fpg]) {
    epoch = c->epoch_val[p.fpg];
  } else {
    epoch = p.counter == 1 ? p.ui_epoch : 0;
  }
  if (p.ui_epoch != epoch) return MBFT_EPOCH_MISMATCH;  // sgx-usig.go:92-94
  if (p.usig_tail != 0xFF) return p.usig_tail;
  if (g == MBFT_ACCEPT) {
    c->epoch_val[p.fpg] = epoch;
    c->epoch_set[p.fpg] = 1;
  }
  return g;
}

// Group commit over concurrent single calls: a call queues itself and waits
// until its status is in or it is handed a batch slot.  Up to
// mbft_set_coalescing_slots batches run at once (each on an engine lane;
// default one at a time): a call that finds a slot free leads -- optionally waits
// max_wait_us for company, takes the queue's front (in order, at most
// max_batch), runs it as one verify_batch and hands out the statuses; then
// the slot passes to the next queued call that holds none (calls that queued
// meanwhile have waited a whole batch already), or is freed.  A leader's own
// call may be taken by another batch while it waits for company; it then
// passes its slot on and waits like any other call.  Every batch applies the
// USIG epoch step in its own order under the context mutex; batches running
// at once are as unordered as the concurrent callers themselves.
//
// Wake-ups are the cost at high call rates (one per call): each waiter sleeps
// on a futex word of its own, NOT under the queue's mutex, so a caller whose
// status is in returns without touching the mutex, a handoff wakes exactly
// one thread, and a leader hands its slot on first and wakes its batch's
// callers after releasing the mutex.  The queue's front waits for its slot
// spinning (coalesce_spin_us), so no sleeping leader's wake-up sits between
// two batches.
namespace {

void futex_wait(std::atomic<uint32_t>* a, uint32_t v) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(a), FUTEX_WAIT_PRIVATE, v, nullptr, nullptr, 0);
}

void futex_wake(std::atomic<uint32_t>* a) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(a), FUTEX_WAKE_PRIVATE, 1, nullptr, nullptr, 0);
}

// after setting done or lead
void signal_waiter(mbft_ctx::Waiter& x) {
  x.ev.fetch_add(1, std::memory_order_release);
  futex_wake(&x.ev);
}

// How long the queue's front call waits for its batch slot awake (env
// MBFT_COALESCE_SPIN_US, default 200; 0: it sleeps like the others).
double coalesce_spin_us() {
  static const double v = [] {
    const char* e = getenv("MBFT_COALESCE_SPIN_US");
    return e ? atof(e) : 200.0;
  }();
  return v;
}

// until done or lead; no lock held
void wait_waiter(mbft_ctx::Waiter& w, bool spin) {
  if (spin) {
    const double t0 = now_ms(), lim = coalesce_spin_us() / 1000.0;
    while (!w.lead.load(std::memory_order_acquire) && !w.done.load(std::memory_order_acquire) &&
           now_ms() - t0 < lim)
      __builtin_ia32_pause();
  }
  for (;;) {
    const uint32_t e = w.ev.load(std::memory_order_acquire);
    if (w.done.load(std::memory_order_acquire) || w.lead.load(std::memory_order_acquire)) return;
    futex_wait(&w.ev, e);
  }
}

}  // namespace

// The batch runner: mbft_verify_batch, or a stand-in (mbft_debug_coalesce_stress).
using BatchRunner = int (*)(mbft_ctx*, const mbft_item*, size_t, uint8_t*);

int coalesced_call_with(mbft_ctx* c, const mbft_item& it, uint8_t* st, BatchRunner run_batch) {
  auto& co = c->co;
  int lanes;
  {
    std::shared_lock<std::shared_mutex> tl(c->tab_mu);
    lanes = c->concurrency;
  }
  // shared: a leader signals its callers after releasing co.m, when a caller
  // may already have seen its status and returned
  const auto wp = std::make_shared<mbft_ctx::Waiter>();
  mbft_ctx::Waiter& w = *wp;
  w.it = it;
  std::unique_lock<std::mutex> lk(co.m);
  const int cap = co.slots < lanes ? co.slots : lanes;
  // the slot this thread holds goes to the first queued call without one
  auto pass_slot = [&] {
    for (const auto& x : co.q)
      if (!x->lead.load(std::memory_order_relaxed)) {
        x->lead.store(true, std::memory_order_release);
        signal_waiter(*x);
        return;
      }
    co.running--;
  };
  // Done.  A slot handed to this call before another batch took it is
  // passed on (lead is set only while queued, so it is visible by now).
  auto result = [&] {
    if (w.lead.load(std::memory_order_acquire)) {
      if (!lk.owns_lock()) lk.lock();
      w.lead.store(false, std::memory_order_relaxed);
      pass_slot();
    }
    *st = w.st;
    return w.rc;
  };
  co.q.push_back(wp);
  if (co.max_batch && co.q.size() >= co.max_batch) co.cv_fill.notify_all();
  for (;;) {
    if (w.done.load(std::memory_order_acquire)) return result();
    if (w.taken) {  // in someone's batch: wait for it (a slot handed meanwhile goes on)
      if (w.lead.load(std::memory_order_acquire)) {
        w.lead.store(false, std::memory_order_relaxed);
        pass_slot();
      }
      lk.unlock();
      wait_waiter(w, false);
      if (w.done.load(std::memory_order_acquire)) return result();
      lk.lock();
      continue;
    }
    if (!w.lead.load(std::memory_order_acquire) && co.running >= cap) {
      const bool front = co.q.front() == wp && coalesce_spin_us() > 0;
      lk.unlock();
      wait_waiter(w, front);
      if (w.done.load(std::memory_order_acquire)) return result();
      lk.lock();
      continue;
    }
    if (!w.lead.load(std::memory_order_acquire)) co.running++;
    w.lead.store(false, std::memory_order_relaxed);
    if (co.max_wait_us)
      co.cv_fill.wait_for(lk, std::chrono::microseconds(co.max_wait_us),
                          [&] { return co.max_batch && co.q.size() >= co.max_batch; });
    if (co.q.empty()) {  // every queued call (this one too) was taken meanwhile
      pass_slot();
      continue;
    }
    // lead one batch: the queue's front calls
    const size_t take = co.max_batch && co.q.size() > co.max_batch ? co.max_batch : co.q.size();
    std::vector<std::shared_ptr<mbft_ctx::Waiter>> batch(co.q.begin(), co.q.begin() + (long)take);
    co.q.erase(co.q.begin(), co.q.begin() + (long)take);
    for (const auto& x : batch) x->taken = true;  // (one holding a handed slot passes it on when it wakes)
    lk.unlock();
    std::vector<mbft_item> items(take);
    std::vector<uint8_t> out(take, 0);
    for (size_t k = 0; k < take; k++) items[k] = batch[k]->it;
    const int rc = run_batch(c, items.data(), take, out.data());
    lk.lock();
    for (size_t k = 0; k < take; k++) {
      batch[k]->rc = rc;
      batch[k]->st = out[k];
      batch[k]->done.store(true, std::memory_order_release);
    }
    pass_slot();  // the next batch's leader runs while this one wakes its callers
    lk.unlock();
    for (const auto& x : batch)
      if (x != wp) signal_waiter(*x);
    if (w.done.load(std::memory_order_acquire)) return result();
    lk.lock();
  }
}

int coalesced_call(mbft_ctx* c, const mbft_item& it, uint8_t* st) {
  return coalesced_call_with(c, it, st, mbft_verify_batch);
}

}  // namespace mbft_host

namespace {

// Pointers and the batch's end offsets; each call's offsets are checked by
// the path that reads them (flat_offsets_ok on the host path, the device
// decode per call and per chunk).
template <class R, class O>
bool flat_args_ok(const R* roles, const uint32_t* ids, const uint8_t* msgs, const O* msg_off,
                  const uint8_t* tags, const O* tag_off, size_t n, const uint8_t* out) {
  if (n == 0) return true;
  if (!roles || !ids || !msg_off || !tag_off || !out) return false;
  if (msg_off[n] < msg_off[0] || tag_off[n] < tag_off[0]) return false;
  if ((msg_off[n] > msg_off[0] && !msgs) || (tag_off[n] > tag_off[0] && !tags)) return false;
  return true;
}

}  // namespace

extern "C" int mbft_verify_batch_flat(mbft_ctx* c, const uint32_t* roles, const uint32_t* ids,
                                      const uint8_t* msgs, const uint64_t* msg_off,
                                      const uint8_t* tags, const uint64_t* tag_off, size_t n,
                                      uint8_t* status_out) {
  if (!c || !flat_args_ok(roles, ids, msgs, msg_off, tags, tag_off, n, status_out))
    return MBFT_ERR_ARG;
  Lease ls(c);
  if (hipSetDevice(c->device) != hipSuccess) return MBFT_ERR_HIP;
  return verify_batch_flat_impl(c, roles, ids, msgs, msg_off, tags, tag_off, n, status_out, ls.g);
}

extern "C" int mbft_verify_batch_flat32(mbft_ctx* c, const uint8_t* roles, const uint32_t* ids,
                                        const uint8_t* msgs, const uint32_t* msg_off,
                                        const uint8_t* tags, const uint32_t* tag_off, size_t n,
                                        uint8_t* status_out) {
  if (!c || !flat_args_ok(roles, ids, msgs, msg_off, tags, tag_off, n, status_out))
    return MBFT_ERR_ARG;
  if (n == 0) return MBFT_OK;
  Lease ls(c);
  if (hipSetDevice(c->device) != hipSuccess) return MBFT_ERR_HIP;
  return flat32_impl(c, roles, ids, msgs, msg_off, tags, tag_off, n, status_out, ls.g, true);
}

extern "C" int mbft_check_batch_flat32(mbft_ctx* c, const uint8_t* roles, const uint32_t* ids,
                                       const uint8_t* msgs, const uint32_t* msg_off,
                                       const uint8_t* tags, const uint32_t* tag_off, size_t n,
                                       uint8_t* pure_out) {
  if (!c || !flat_args_ok(roles, ids, msgs, msg_off, tags, tag_off, n, pure_out))
    return MBFT_ERR_ARG;
  if (n == 0) return MBFT_OK;
  Lease ls(c);
  if (hipSetDevice(c->device) != hipSuccess) return MBFT_ERR_HIP;
  return flat32_impl(c, roles, ids, msgs, msg_off, tags, tag_off, n, pure_out, ls.g, false);
}

extern "C" int mbft_check_batch(mbft_ctx* c, const mbft_item* items, size_t n, uint8_t* pure_out) {
  if (!c || (n && (!items || !pure_out))) return MBFT_ERR_ARG;
  if (n == 0) return MBFT_OK;
  Lease ls(c);
  if (hipSetDevice(c->device) != hipSuccess) return MBFT_ERR_HIP;
  return check_calls(c, items, n, pure_out, nullptr, ls.g);
}

extern "C" int mbft_check_batch_flat(mbft_ctx* c, const uint32_t* roles, const uint32_t* ids,
                                     const uint8_t* msgs, const uint64_t* msg_off,
                                     const uint8_t* tags, const uint64_t* tag_off, size_t n,
                                     uint8_t* pure_out) {
  if (!c || !flat_args_ok(roles, ids, msgs, msg_off, tags, tag_off, n, pure_out))
    return MBFT_ERR_ARG;
  Lease ls(c);
  if (hipSetDevice(c->device) != hipSuccess) return MBFT_ERR_HIP;
  return check_calls_flat(c, roles, ids, msgs, msg_off, tags, tag_off, n, pure_out, ls.g);
}

extern "C" int mbft_resolve_checked(mbft_ctx* c, uint32_t role, uint32_t id, const uint8_t* msg,
                                    size_t msg_len, const uint8_t* tag, size_t tag_len,
                                    uint8_t pure) {
  if (!c || (msg_len && !msg) || (tag_len && !tag)) return MBFT_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  const mbft_item it{role, id, msg, msg_len, tag, tag_len};
  CallInfo p;
  uint8_t r[32], s[32], e[32];
  uint32_t sl;
  Lookup lk;
  // the host part only (defer: no digest is needed, the signature verdict is
  // `pure`)
  prepare_item(c, it, p, e, r, s, &sl, true, lk);
  return (int)resolve_call(c, p, p.pre != 0xFF ? p.pre : pure);
}

extern "C" int mbft_set_coalescing(mbft_ctx* c, int enabled, uint32_t max_wait_us,
                                   uint32_t max_batch) {
  if (!c) return MBFT_ERR_ARG;
  std::lock_guard<std::mutex> g(c->co.m);
  c->co.max_wait_us = max_wait_us;
  c->co.max_batch = max_batch;
  c->co.enabled = enabled != 0;
  return MBFT_OK;
}

// More slots split the callers into smaller batches that run no faster on
// the lanes: 64 callers 468 K calls/s on 1 slot, 413 K on 4, 261 K on 8
// (profiles/round4_coalesce_slots.txt), hence the default of 1.
extern "C" int mbft_set_coalescing_slots(mbft_ctx* c, int slots) {
  if (!c || slots < 1 || slots > 64) return MBFT_ERR_ARG;
  std::lock_guard<std::mutex> g(c->co.m);
  c->co.slots = slots;
  return MBFT_OK;
}

extern "C" int mbft_host_alloc(size_t bytes, void** out) {
  if (!out) return MBFT_ERR_ARG;
  *out = nullptr;
  if (bytes == 0) bytes = 1;
  void* p = nullptr;
  // portable: any engine's device may DMA from it
  if (hipHostMalloc(&p, bytes, hipHostMallocPortable) != hipSuccess || !p) return MBFT_ERR_NOMEM;
  std::lock_guard<std::mutex> g(g_host_mu);
  g_host_allocs[(uintptr_t)p] = (uintptr_t)p + bytes;
  *out = p;
  return MBFT_OK;
}

extern "C" int mbft_host_free(void* p) {
  if (!p) return MBFT_OK;
  {
    std::lock_guard<std::mutex> g(g_host_mu);
    auto it = g_host_allocs.find((uintptr_t)p);
    if (it == g_host_allocs.end()) return MBFT_ERR_ARG;
    g_host_allocs.erase(it);
  }
  // hipHostFree synchronizes the device: a live resident kernel generation
  // would hold it up to its lifetime, so the live generations end first (the
  // next resident call relaunches)
  resident_park_all();
  return hipHostFree(p) == hipSuccess ? MBFT_OK : MBFT_ERR_HIP;
}

extern "C" int mbft_set_device_prepare(mbft_ctx* c, int enabled) {
  if (!c) return MBFT_ERR_ARG;
  KeyWriteGuard g(c);
  c->dev_prepare = enabled != 0;
  for (mbft_ctx* l : c->lanes) l->dev_prepare = c->dev_prepare;
  for (mbft_ctx* p : c->peers) p->dev_prepare = c->dev_prepare;
  return MBFT_OK;
}

extern "C" int mbft_profile_stages(mbft_ctx* c, double out[6]) {
  if (!c || !out) return MBFT_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  out[0] = c->st_calls;
  out[1] = c->st_items;
  out[2] = c->st_prepare_ms;
  out[3] = c->st_gpu_ms;
  out[4] = c->st_resolve_ms;
  out[5] = c->st_total_ms;
  c->st_calls = c->st_items = c->st_prepare_ms = c->st_gpu_ms = c->st_resolve_ms = c->st_total_ms = 0;
  return MBFT_OK;
}

// Test hook (tests/test_coalesce_cpu.py; not in the public header): the
// coalescer's hand-offs without a GPU.  `threads` threads make `per` calls
// each through coalesced_call_with on a bare context with `lanes` lanes and
// `slots` batch slots; the stand-in batch runner spins `batch_us` and answers
// each call with a function of its id.  Returns the number of wrong
// statuses; stats = {batches, most batches in flight at once, seconds,
// slots still held after every call returned (0 unless a slot leaked)}.
namespace {
std::atomic<int> g_stress_inflight{0}, g_stress_max{0}, g_stress_batches{0};
uint32_t g_stress_us = 0;
int stress_batch(mbft_ctx*, const mbft_item* items, size_t n, uint8_t* out) {
  const int f = g_stress_inflight.fetch_add(1) + 1;
  int m = g_stress_max.load();
  while (f > m && !g_stress_max.compare_exchange_weak(m, f)) {
  }
  g_stress_batches.fetch_add(1);
  const double t0 = now_ms();
  while (now_ms() - t0 < g_stress_us / 1000.0) __builtin_ia32_pause();
  for (size_t k = 0; k < n; k++) out[k] = (uint8_t)((items[k].id * 2654435761u) >> 24);
  g_stress_inflight.fetch_sub(1);
  return MBFT_OK;
}
}  // namespace

extern "C" int mbft_debug_coalesce_stress(int threads, int per, int lanes, int slots,
                                          uint32_t batch_us, double* stats) {
  if (threads < 1 || per < 1 || lanes < 1 || slots < 1 || !stats) return MBFT_ERR_ARG;
  auto c = std::make_unique<mbft_ctx>();
  c->concurrency = lanes;
  c->co.slots = slots;
  c->co.enabled = true;
  g_stress_us = batch_us;
  g_stress_inflight = 0;
  g_stress_max = 0;
  g_stress_batches = 0;
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  const double t0 = now_ms();
  for (int t = 0; t < threads; t++)
    th.emplace_back([&, t] {
      for (int k = 0; k < per; k++) {
        const uint32_t id = (uint32_t)(t * per + k);
        const mbft_item it{MBFT_ROLE_CLIENT, id, nullptr, 0, nullptr, 0};
        uint8_t st = 0xEE;
        const int rc = coalesced_call_with(c.get(), it, &st, stress_batch);
        if (rc != MBFT_OK || st != (uint8_t)((id * 2654435761u) >> 24)) bad.fetch_add(1);
      }
    });
  for (auto& x : th) x.join();
  stats[0] = g_stress_batches.load();
  stats[1] = g_stress_max.load();
  stats[2] = (now_ms() - t0) / 1000.0;
  {
    std::lock_guard<std::mutex> g(c->co.m);
    stats[3] = c->co.running;
  }
  return bad.load();
}

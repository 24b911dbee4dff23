// Host runtime + C-ABI of the MI355X batch authenticator (include/minbft_gpu.h).
//
// Layering (mirrors sample/authentication):
//   mbft_ctx            = Authenticator (authenticator.go:33-38): key store,
//                         role -> scheme wiring, USIG epoch map
//                         (crypto.go:148-154), plus the per-GPU state:
//                         stream, generator comb table, per-key comb tables.
//   verify_batch        = VerifyMessageAuthenTag (authenticator.go:121-134)
//                         for n items: host does the byte-level work (role
//                         and key lookup, UI/cert split, Go-exact DER,
//                         digest construction), the GPU checks all
//                         signatures at once, then the host replays the
//                         USIG epoch capture in item order.
#include <stdlib.h>
#include <string.h>

#include <thread>

#include <sys/syscall.h>
#include <unistd.h>

#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>

#include "host_internal.h"

using namespace mbft_host;

// MBFT_SEGV_TRACE=1: a fault on the host prints the native stack (library
// offsets for addr2line) to stderr before the process ends -- diagnostics
// for a crash the Python fault handler can only place at the ctypes call.
// Each frame prints as module(+offset); the faulting address and the
// module holding the faulting PC follow (dladdr), so a fault inside another
// library's teardown names that library.
namespace {
void segv_trace(int sig, siginfo_t* si, void* uc) {
  char buf[256];
  int k = snprintf(buf, sizeof buf, "mbft segv trace: signal %d, fault address %p\n", sig,
                   si ? si->si_addr : nullptr);
  if (k > 0) (void)!write(2, buf, (size_t)k);
  void* fr[64];
  const int n = backtrace(fr, 64);
  backtrace_symbols_fd(fr, n, 2);
  for (int i = 0; i < n; i++) {
    Dl_info d;
    if (dladdr(fr[i], &d) && d.dli_fname) {
      k = snprintf(buf, sizeof buf, "  frame %d: %s +0x%lx (%s)\n", i, d.dli_fname,
                   (unsigned long)((char*)fr[i] - (char*)d.dli_fbase), d.dli_sname ? d.dli_sname : "?");
    } else {
      k = snprintf(buf, sizeof buf, "  frame %d: %p (no module)\n", i, fr[i]);
    }
    if (k > 0) (void)!write(2, buf, (size_t)k);
  }
  (void)uc;
  signal(sig, SIG_DFL);
  raise(sig);
}
struct SegvInit {
  SegvInit() {
    const char* v = getenv("MBFT_SEGV_TRACE");
    if (v && atoi(v)) {
      struct sigaction sa;
      memset(&sa, 0, sizeof sa);
      sa.sa_sigaction = segv_trace;
      sa.sa_flags = SA_SIGINFO;
      sigaction(SIGSEGV, &sa, nullptr);
      sigaction(SIGBUS, &sa, nullptr);
    }
  }
} segv_init;
}  // namespace

namespace mbft_host {

namespace {

// The host NUMA node nearest device d (hipDeviceAttributeHostNumaId), -1 when
// unknown or when the host has one node; cached per device.
int device_numa_node(int d) {
  static std::mutex mu;
  static std::map<int, int> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(d);
  if (it != cache.end()) return it->second;
  int node = -1, nodes = 0;
  for (int k = 0; k < 64; k++) {
    char path[64];
    snprintf(path, sizeof path, "/sys/devices/system/node/node%d", k);
    if (access(path, F_OK) == 0) nodes++;
  }
  if (nodes > 1 && hipDeviceGetAttribute(&node, hipDeviceAttributeHostNumaId, d) != hipSuccess) node = -1;
  if (nodes <= 1) node = -1;
  (void)hipGetLastError();
  cache[d] = node;
  return node;
}

}  // namespace

hipError_t host_malloc_near(void** p, size_t bytes, unsigned flags) {
  static const bool off = [] {
    const char* v = getenv("MBFT_NUMA_STAGING");
    return v && atoi(v) == 0;
  }();
  int dev = 0;
  const int node = off || hipGetDevice(&dev) != hipSuccess ? -1 : device_numa_node(dev);
  if (node < 0 || node >= 64) return hipHostMalloc(p, bytes, flags);
  // MPOL_PREFERRED for this thread while the pages are allocated and pinned,
  // then the previous policy back
  int old_mode = 0;
  unsigned long old_mask[16] = {0};
  const bool saved = syscall(SYS_get_mempolicy, &old_mode, old_mask, 64 * 16, nullptr, 0) == 0;
  unsigned long mask[16] = {0};
  mask[node / 64] = 1ul << (node % 64);
  const bool set = saved && syscall(SYS_set_mempolicy, 1 /* MPOL_PREFERRED */, mask, 64 * 16) == 0;
  const hipError_t e = hipHostMalloc(p, bytes, set ? flags | hipHostMallocNumaUser : flags);
  if (set) (void)syscall(SYS_set_mempolicy, old_mode, old_mode == 0 ? nullptr : old_mask, old_mode == 0 ? 0 : 64 * 16);
  return e;
}


const uint8_t kPkixPrefix[26] = {0x30, 0x59, 0x30, 0x13, 0x06, 0x07, 0x2a, 0x86, 0x48,
                                 0xce, 0x3d, 0x02, 0x01, 0x06, 0x08, 0x2a, 0x86, 0x48,
                                 0xce, 0x3d, 0x03, 0x01, 0x07, 0x03, 0x42, 0x00};
const uint8_t kEmptyHash[32] = {0xe3, 0xb0, 0xc4, 0x42, 0x98, 0xfc, 0x1c, 0x14, 0x9a, 0xfb, 0xf4,
                                0xc8, 0x99, 0x6f, 0xb9, 0x24, 0x27, 0xae, 0x41, 0xe4, 0x64, 0x9b,
                                0x93, 0x4c, 0xa4, 0x95, 0x99, 0x1b, 0x78, 0x52, 0xb8, 0x55};

}  // namespace mbft_host

namespace mbft_host {

std::atomic<uint64_t> g_threads_started{0};

EngineWorker& engine_worker(mbft_ctx* e) {
  std::lock_guard<std::mutex> g(e->worker_mu);
  if (!e->worker) e->worker.reset(new EngineWorker());
  return *e->worker;
}

int fail(mbft_ctx* c, int code, const std::string& what) {
  if (c) c->err = what;
  return code;
}

int hip_fail(mbft_ctx* c, hipError_t e, const char* what) {
  return fail(c, MBFT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

// Upload the slot descriptors (small: 16 B per slot).
int upload_keydesc(mbft_ctx* c) {
  if (c->keydesc.empty()) return MBFT_OK;
  HIPCHK(c, c->d_keys.ensure(c->keydesc.size() * sizeof(mbft::KeyDesc)));
  HIPCHK(c, hipMemcpyAsync(c->d_keys.p, c->keydesc.data(),
                           c->keydesc.size() * sizeof(mbft::KeyDesc), hipMemcpyHostToDevice,
                           c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return MBFT_OK;
}

// (Re)build the generator comb table with window w.  The old table is freed
// first so that a large window can use the memory it held.
void release_free_blocks(mbft_ctx* c) {
  for (auto& b : c->free_blocks) (void)hipFree(b.first);
  c->free_blocks.clear();
}

// A device block of at least `bytes` for key tables: a released block that
// is large enough but not wastefully so (smallest first), else a fresh
// allocation (released blocks are given back first if it fails).
hipError_t table_block(mbft_ctx* c, size_t bytes, uint32_t** out) {
  const size_t waste = bytes + ((size_t)1 << 30) > 2 * bytes ? bytes + ((size_t)1 << 30) : 2 * bytes;
  size_t best = c->free_blocks.size();
  for (size_t i = 0; i < c->free_blocks.size(); i++)
    if (c->free_blocks[i].second >= bytes && c->free_blocks[i].second <= waste &&
        (best == c->free_blocks.size() || c->free_blocks[i].second < c->free_blocks[best].second))
      best = i;
  if (best < c->free_blocks.size()) {
    *out = static_cast<uint32_t*>(c->free_blocks[best].first);
    c->tab_blocks.push_back(c->free_blocks[best].first);
    c->tab_sizes.push_back(c->free_blocks[best].second);
    c->free_blocks.erase(c->free_blocks.begin() + (long)best);
    return hipSuccess;
  }
  hipError_t e = hipMalloc(reinterpret_cast<void**>(out), bytes);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    release_free_blocks(c);
    e = hipMalloc(reinterpret_cast<void**>(out), bytes);
  }
  if (e != hipSuccess) return e;
  c->tab_blocks.push_back(*out);
  c->tab_sizes.push_back(bytes);
  return hipSuccess;
}

int build_generator(mbft_ctx* c, int w) {
  release_free_blocks(c);
  if (c->d_tabG) {
    HIPCHK(c, hipFree(c->d_tabG));
    c->d_tabG = nullptr;
  }
  if (hipMalloc(&c->d_tabG, mbft_launch::table_words(w) * 4) != hipSuccess) {
    (void)hipGetLastError();
    c->d_tabG = nullptr;
    return fail(c, MBFT_ERR_NOMEM, "generator table: out of device memory (window " +
                                       std::to_string(w) + ")");
  }
  HIPCHK(c, c->xy.ensure(64));
  HIPCHK(c, c->bpts.ensure((size_t)mbft_launch::table_steps(w) * 64));
  HIPCHK(c, mbft_launch::generator_xy(c->xy.as<uint32_t>(), c->stream));
  HIPCHK(c, mbft_launch::build_tables(c->xy.as<uint32_t>(), 1, w, c->bpts.as<uint32_t>(),
                                      c->d_tabG, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->g_wbits = w;
  return MBFT_OK;
}

uint64_t fingerprint_of(const uint8_t xy[64]) {
  uint8_t pkix[91], h[32];
  memcpy(pkix, kPkixPrefix, 26);
  pkix[26] = 0x04;
  memcpy(pkix + 27, xy, 64);
  sha256(pkix, 91, h);
  uint64_t f = 0;
  for (int i = 0; i < 8; i++) f = (f << 8) | h[i];
  return f;
}

// Register (dedup) raw points on ONE engine; validates on the GPU and builds
// comb tables.
int register_points_engine(mbft_ctx* c, const uint8_t* xy64, size_t n, uint32_t* out_slots,
                           uint8_t* valid_out) {
  std::vector<size_t> fresh;  // indices into input needing a new slot
  std::vector<uint32_t> slot_ids(n);
  std::map<std::array<uint8_t, 64>, uint32_t> pending;
  for (size_t i = 0; i < n; i++) {
    std::array<uint8_t, 64> k;
    memcpy(k.data(), xy64 + 64 * i, 64);
    auto it = c->slot_of_xy.find(k);
    if (it != c->slot_of_xy.end()) {
      slot_ids[i] = it->second;
      continue;
    }
    auto pt = pending.find(k);
    if (pt != pending.end()) {
      slot_ids[i] = pt->second;
      continue;
    }
    const uint32_t sl = (uint32_t)(c->slots.size() + fresh.size());
    pending[k] = sl;
    slot_ids[i] = sl;
    fresh.push_back(i);
  }
  if (!fresh.empty()) {
    const size_t m = fresh.size();
    const size_t base = c->slots.size();
    std::vector<uint32_t> words(16 * m);
    for (size_t j = 0; j < m; j++) {
      const uint8_t* p = xy64 + 64 * fresh[j];
      be_to_words(&words[16 * j], p);
      be_to_words(&words[16 * j + 8], p + 32);
    }
    HIPCHK(c, c->xy.ensure(words.size() * 4));
    HIPCHK(c, c->ok.ensure(m * 4));
    HIPCHK(c, hipMemcpyAsync(c->xy.p, words.data(), words.size() * 4, hipMemcpyHostToDevice,
                             c->stream));
    HIPCHK(c, mbft_launch::check_points(c->xy.as<uint32_t>(), (int)m, c->ok.as<uint32_t>(),
                                        c->stream));
    std::vector<uint32_t> ok(m);
    HIPCHK(c, hipMemcpyAsync(ok.data(), c->ok.p, m * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    // compact the valid points; their tables go into one new block
    std::vector<uint32_t> vwords;
    std::vector<uint32_t> vslots;
    for (size_t j = 0; j < m; j++) {
      SlotInfo si;
      memcpy(si.xy.data(), xy64 + 64 * fresh[j], 64);
      si.valid = ok[j] != 0;
      si.fingerprint = fingerprint_of(si.xy.data());
      auto fg = c->fp_group_of.emplace(si.fingerprint, (uint32_t)c->epoch_val.size());
      if (fg.second) {
        c->epoch_val.push_back(0);
        c->epoch_set.push_back(0);
      }
      si.fp_group = fg.first->second;
      c->slots.push_back(si);
      c->slot_of_xy[si.xy] = (uint32_t)(base + j);
      c->keydesc.push_back(mbft::KeyDesc{nullptr, (uint32_t)c->q_wbits, 0u});
      if (si.valid) {
        vwords.insert(vwords.end(), &words[16 * j], &words[16 * j] + 16);
        vslots.push_back((uint32_t)(base + j));
      }
    }
    if (!vslots.empty()) {
      const int w = c->q_wbits;
      const size_t cnt = vslots.size();
      const size_t tw = mbft_launch::table_words(w);
      uint32_t* blk = nullptr;
      hipError_t he = table_block(c, cnt * tw * sizeof(uint32_t), &blk);
      if (he != hipSuccess) {
        // keep the slots (invalid) so slot numbering stays consistent
        (void)hipGetLastError();
        return fail(c, MBFT_ERR_NOMEM, "key tables: out of device memory (window " +
                                           std::to_string(w) + ")");
      }
      HIPCHK(c, c->xy.ensure(16 * 4 * cnt));
      HIPCHK(c, c->bpts.ensure((size_t)mbft_launch::table_steps(w) * 16 * 4 * cnt));
      HIPCHK(c, hipMemcpyAsync(c->xy.p, vwords.data(), 16 * 4 * cnt, hipMemcpyHostToDevice,
                               c->stream));
      HIPCHK(c, mbft_launch::build_tables(c->xy.as<uint32_t>(), (int)cnt, w,
                                          c->bpts.as<uint32_t>(), blk, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      for (size_t j = 0; j < cnt; j++) {
        mbft::KeyDesc& kd = c->keydesc[vslots[j]];
        kd.tab = blk + j * tw;
        kd.valid = 1;
      }
    }
    int rc = upload_keydesc(c);
    if (rc) return rc;
  }
  for (size_t i = 0; i < n; i++) {
    if (out_slots) out_slots[i] = slot_ids[i];
    if (valid_out) valid_out[i] = c->slots[slot_ids[i]].valid ? 1 : 0;
  }
  return MBFT_OK;
}

// Verify n decoded items (device pointers) -> device status, on stream st.
int verify_device(mbft_ctx* c, const uint8_t* d_e, const uint8_t* d_r, const uint8_t* d_s,
                  const uint32_t* d_slot, size_t n, uint8_t* d_status, hipStream_t st,
                  bool host_status, bool latency, const uint32_t* d_winv, const uint32_t* d_count) {
  if (n == 0) return MBFT_OK;
  const mbft_ctx* tb = tabs(c);  // the tables (a lane reads its owner's)
  const int k = c->pipe;
  c->pipe = (k + 1) % mbft_ctx::kPipe;
  const size_t wwords = mbft_launch::ninv_workspace_words((long)n);
  HIPCHK(c, c->ws[k].ensure(wwords * 4));
  HIPCHK(c, c->winv[k].ensure((size_t)9 * n * 4));
  // Small batches: no batched s^-1 chain (five dependent launches, ~180 us
  // of latency); k_verify_pairs inverts s per lane (divsteps, modinv.h).
  // Env MBFT_LANE_INV_MAX (default 4096 items; 0 disables).
  static const size_t lane_inv_max = [] {
    const char* v = getenv("MBFT_LANE_INV_MAX");
    return v ? (size_t)strtoull(v, nullptr, 10) : (size_t)4096;
  }();
  // d_count: n is an upper bound, the count is on the device -- the small-batch
  // kernels, which read it (no batched chain: it is sized by n on the host)
  const bool small = n <= lane_inv_max || d_count;
  HIPCHK(c, c->slowq[k].ensure(mbft_launch::verify_words((long)n, small) * 4));
  mbft_ctx::Ev ev{};
  if (c->prof) {
    HIPCHK(c, hipEventCreate(&ev.a));
    HIPCHK(c, hipEventCreate(&ev.b));
    HIPCHK(c, hipEventCreate(&ev.c));
    HIPCHK(c, hipEventCreate(&ev.d));
    ev.n = n;
  }
  if (small || d_winv) {
    HIPCHK(c, hipStreamWaitEvent(st, c->ev_done[k], 0));  // slowq[k] reuse
    if (c->prof) {
      HIPCHK(c, hipEventRecord(ev.a, st));
      HIPCHK(c, hipEventRecord(ev.b, st));
      HIPCHK(c, hipEventRecord(ev.c, st));
    }
    HIPCHK(c, mbft_launch::verify(d_e, d_r, d_s, d_slot, d_winv, tb->d_tabG, tb->g_wbits,
                                  tb->d_keys.as<mbft::KeyDesc>(), (uint32_t)tb->slots.size(),
                                  (long)n, d_status, c->slowq[k].as<uint32_t>(), st, host_status,
                                  /*queue_zeroed=*/false, tabs(c)->split_max,
                                  /*split_winv=*/d_winv != nullptr, d_count,
                                  /*planes_ws=*/d_winv ? nullptr : c->winv[k].as<uint32_t>(),
                                  tabs(c)->small_inv));
    HIPCHK(c, hipEventRecord(c->ev_done[k], st));
    if (c->prof) {
      HIPCHK(c, hipEventRecord(ev.d, st));
      c->evs.push_back(ev);
    }
    return MBFT_OK;
  }
  // A batch issued while every earlier batch of this engine has finished
  // (one batch at a time: its latency counts) takes the one-launch s^-1
  // (k_ninv_local) on the caller's stream, no cross-stream hand-off; while
  // earlier batches are in flight the level chain runs on the high-priority
  // stream beside them, hidden, with less VALU work.  Env
  // MBFT_NINV = local | levels forces one form.  `latency` (a pipeline's
  // last chunks, nothing after them to hide a chain behind) takes the
  // one-launch form in any case, once buffer k is free.
  // Diagnostic only (never set by the bench line): MBFT_DIAG_REUSE_WINV=1
  // skips the s^-1 kernels once buffer k holds a batch's w planes, for
  // callers that verify the SAME batch again through the prehashed device
  // entry (the s^-1 stage's share of a step, tools/streams_ab.sh).
  static const bool diag_reuse = getenv("MBFT_DIAG_REUSE_WINV") != nullptr;
  if (diag_reuse && !host_status && c->diag_winv_n[k] == n) {
    HIPCHK(c, hipStreamWaitEvent(st, c->ev_done[k], 0));
    if (c->prof) {
      HIPCHK(c, hipEventRecord(ev.a, st));
      HIPCHK(c, hipEventRecord(ev.b, st));
      HIPCHK(c, hipEventRecord(ev.c, st));
    }
    HIPCHK(c, mbft_launch::verify(d_e, d_r, d_s, d_slot, c->winv[k].as<uint32_t>(), tb->d_tabG,
                                  tb->g_wbits, tb->d_keys.as<mbft::KeyDesc>(),
                                  (uint32_t)tb->slots.size(), (long)n, d_status,
                                  c->slowq[k].as<uint32_t>(), st, host_status, /*queue_zeroed=*/false));
    HIPCHK(c, hipEventRecord(c->ev_done[k], st));
    if (c->prof) {
      HIPCHK(c, hipEventRecord(ev.d, st));
      c->evs.push_back(ev);
    }
    return MBFT_OK;
  }
  if (diag_reuse && !host_status) c->diag_winv_n[k] = n;
  const char* ninv = getenv("MBFT_NINV");
  bool idle = !(ninv && strcmp(ninv, "levels") == 0);
  if (idle && !(ninv && strcmp(ninv, "local") == 0))
    for (int j = 0; j < mbft_ctx::kPipe && idle; j++) {
      const hipError_t q = hipEventQuery(c->ev_done[j]);
      if (q == hipErrorNotReady) {
        idle = false;
      } else if (q != hipSuccess) {
        return hip_fail(c, q, "hipEventQuery(ev_done)");
      }
    }
  if (latency && !idle) {
    HIPCHK(c, hipStreamWaitEvent(st, c->ev_done[k], 0));  // winv[k] / slowq[k] reuse
    idle = true;
  }
  // Split idle batch (env MBFT_SPLIT_DIV = d >= 2; off by default, and never
  // while profiling, which times whole kernels): part 0 (the first n / d
  // items) inverts and verifies on the caller's stream, part 1 inverts on the
  // library stream at the same time and verifies there as soon as its
  // inverse is done, so the larger part's s^-1 runs beside part 0's verify
  // instead of before it.  Each part has its own w planes, exact-path queue
  // and spill planes; the caller's stream joins part 1 before anything reads
  // the statuses.  Measured no better than one launch of each (two
  // concurrent verify grids lose ~40 us to their tails).
  static const long split_div = [] {
    const char* v = getenv("MBFT_SPLIT_DIV");
    return v ? atol(v) : 0L;
  }();
  if (idle && !c->prof && split_div >= 2 && n >= 65536) {
    const size_t n0 = (((size_t)n / (size_t)split_div) + 255) & ~(size_t)255, n1 = n - n0;
    const size_t q0 = mbft_launch::verify_words((long)n0, false);
    HIPCHK(c, c->slowq[k].ensure((q0 + mbft_launch::verify_words((long)n1, false)) * 4));
    uint32_t* w = c->winv[k].as<uint32_t>();
    uint32_t* q = c->slowq[k].as<uint32_t>();
    HIPCHK(c, hipEventRecord(c->ev_in, st));
    HIPCHK(c, hipStreamWaitEvent(c->istream, c->ev_in, 0));
    HIPCHK(c, mbft_launch::batch_inverse_s_local(d_s, (long)n0, w, q + n0, st));
    HIPCHK(c, mbft_launch::batch_inverse_s_local(d_s + 32 * n0, (long)n1, w + 9 * n0, q + q0 + n1,
                                                 c->istream));
    HIPCHK(c, mbft_launch::verify(d_e, d_r, d_s, d_slot, w, tb->d_tabG, tb->g_wbits,
                                  tb->d_keys.as<mbft::KeyDesc>(), (uint32_t)tb->slots.size(),
                                  (long)n0, d_status, q, st, host_status, /*queue_zeroed=*/true));
    HIPCHK(c, mbft_launch::verify(d_e + 32 * n0, d_r + 32 * n0, d_s + 32 * n0, d_slot + n0,
                                  w + 9 * n0, tb->d_tabG, tb->g_wbits,
                                  tb->d_keys.as<mbft::KeyDesc>(), (uint32_t)tb->slots.size(),
                                  (long)n1, d_status + n0, q + q0, c->istream, host_status,
                                  /*queue_zeroed=*/true));
    HIPCHK(c, hipEventRecord(c->ev_inv[k], c->istream));
    HIPCHK(c, hipStreamWaitEvent(st, c->ev_inv[k], 0));
    HIPCHK(c, hipEventRecord(c->ev_done[k], st));
    return MBFT_OK;
  }
  if (idle) {
    if (c->prof) HIPCHK(c, hipEventRecord(ev.a, st));
    // (the kernel also zeroes the verify's exact-path queue counter)
    HIPCHK(c, mbft_launch::batch_inverse_s_local(d_s, (long)n, c->winv[k].as<uint32_t>(),
                                                 c->slowq[k].as<uint32_t>() + n, st));
    if (c->prof) {
      HIPCHK(c, hipEventRecord(ev.b, st));
      HIPCHK(c, hipEventRecord(ev.c, st));
    }
    HIPCHK(c, mbft_launch::verify(d_e, d_r, d_s, d_slot, c->winv[k].as<uint32_t>(), tb->d_tabG,
                                  tb->g_wbits, tb->d_keys.as<mbft::KeyDesc>(),
                                  (uint32_t)tb->slots.size(), (long)n, d_status,
                                  c->slowq[k].as<uint32_t>(), st, host_status, /*queue_zeroed=*/true));
    HIPCHK(c, hipEventRecord(c->ev_done[k], st));
    if (c->prof) {
      HIPCHK(c, hipEventRecord(ev.d, st));
      c->evs.push_back(ev);
    }
    return MBFT_OK;
  }
  // Earlier batches in flight (the pipelined loop): the one-launch per-wave
  // s^-1 on the caller's stream, right before the verify, once buffer k is
  // free -- its waves interleave with the previous batch's verify waves
  // (0.954 against 1.048 ms a step with the level chain below, same box,
  // profiles/round6_ninv_forms.jsonl).  MBFT_NINV=levels: the level chain on
  // the high-priority stream (round 5).
  if (!(ninv && strcmp(ninv, "levels") == 0)) {
    HIPCHK(c, hipStreamWaitEvent(st, c->ev_done[k], 0));  // winv[k] / slowq[k] reuse
    if (c->prof) HIPCHK(c, hipEventRecord(ev.a, st));
    HIPCHK(c, mbft_launch::batch_inverse_s_pipelined(d_s, (long)n, c->winv[k].as<uint32_t>(),
                                                     c->slowq[k].as<uint32_t>() + n, st));
    if (c->prof) {
      HIPCHK(c, hipEventRecord(ev.b, st));
      HIPCHK(c, hipEventRecord(ev.c, st));
    }
    HIPCHK(c, mbft_launch::verify(d_e, d_r, d_s, d_slot, c->winv[k].as<uint32_t>(), tb->d_tabG,
                                  tb->g_wbits, tb->d_keys.as<mbft::KeyDesc>(),
                                  (uint32_t)tb->slots.size(), (long)n, d_status,
                                  c->slowq[k].as<uint32_t>(), st, host_status, /*queue_zeroed=*/true));
    HIPCHK(c, hipEventRecord(c->ev_done[k], st));
    if (c->prof) {
      HIPCHK(c, hipEventRecord(ev.d, st));
      c->evs.push_back(ev);
    }
    return MBFT_OK;
  }
  // inputs ready on the caller's stream; buffer k free once the verify that
  // last read it (two calls ago) has finished
  HIPCHK(c, hipEventRecord(c->ev_in, st));
  HIPCHK(c, hipStreamWaitEvent(c->istream, c->ev_in, 0));
  HIPCHK(c, hipStreamWaitEvent(c->istream, c->ev_done[k], 0));
  if (c->prof) HIPCHK(c, hipEventRecord(ev.a, c->istream));
  // (the chain's last kernel also zeroes the verify's exact-path queue counter:
  // slowq[k] is free, the chain waited for ev_done[k])
  HIPCHK(c, mbft_launch::batch_inverse_s(d_s, (long)n, c->ws[k].as<uint32_t>(),
                                         c->winv[k].as<uint32_t>(),
                                         c->slowq[k].as<uint32_t>() + n, c->istream));
  if (c->prof) HIPCHK(c, hipEventRecord(ev.b, c->istream));
  HIPCHK(c, hipEventRecord(c->ev_inv[k], c->istream));
  HIPCHK(c, hipStreamWaitEvent(st, c->ev_inv[k], 0));
  // slowq[k]: free once the verify that last used it has finished (it may
  // have run on another stream)
  HIPCHK(c, hipStreamWaitEvent(st, c->ev_done[k], 0));
  if (c->prof) HIPCHK(c, hipEventRecord(ev.c, st));
  HIPCHK(c, mbft_launch::verify(d_e, d_r, d_s, d_slot, c->winv[k].as<uint32_t>(), tb->d_tabG,
                                tb->g_wbits, tb->d_keys.as<mbft::KeyDesc>(),
                                (uint32_t)tb->slots.size(), (long)n, d_status,
                                c->slowq[k].as<uint32_t>(), st, host_status, /*queue_zeroed=*/true));
  HIPCHK(c, hipEventRecord(c->ev_done[k], st));
  if (c->prof) {
    HIPCHK(c, hipEventRecord(ev.d, st));
    c->evs.push_back(ev);
  }
  return MBFT_OK;
}

// Host buffers in, host status out, on ONE engine.
int verify_host_engine(mbft_ctx* c, const uint8_t* e, const uint8_t* r, const uint8_t* s,
                       const uint32_t* slots, size_t n, uint8_t* status) {
  if (n == 0) return MBFT_OK;
  if (c->slots.empty()) {
    memset(status, MBFT_BAD_KEY, n);
    return MBFT_OK;
  }
  HIPCHK(c, c->e.ensure(32 * n));
  HIPCHK(c, c->r.ensure(32 * n));
  HIPCHK(c, c->s.ensure(32 * n));
  HIPCHK(c, c->slot.ensure(4 * n));
  HIPCHK(c, c->status.ensure(n));
  HIPCHK(c, hipMemcpyAsync(c->e.p, e, 32 * n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->r.p, r, 32 * n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->s.p, s, 32 * n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->slot.p, slots, 4 * n, hipMemcpyHostToDevice, c->stream));
  int rc = verify_device(c, c->e.as<uint8_t>(), c->r.as<uint8_t>(), c->s.as<uint8_t>(),
                         c->slot.as<uint32_t>(), n, c->status.as<uint8_t>(), c->stream);
  if (rc) return rc;
  HIPCHK(c, hipMemcpyAsync(status, c->status.p, n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return MBFT_OK;
}

// Register on the primary engine, then replay the same points on every peer
// engine (identical dedup order => identical slot numbers and windows).
int register_points(mbft_ctx* c, const uint8_t* xy64, size_t n, uint32_t* out_slots,
                    uint8_t* valid_out) {
  int rc = register_points_engine(c, xy64, n, out_slots, valid_out);
  if (rc) return rc;
  for (mbft_ctx* p : c->peers) {
    std::lock_guard<std::mutex> g(p->mu);
    if (hipSetDevice(p->device) != hipSuccess) return fail(c, MBFT_ERR_HIP, "hipSetDevice(peer)");
    p->q_wbits = c->q_wbits;
    rc = register_points_engine(p, xy64, n, nullptr, nullptr);
    if (rc) return fail(c, rc, std::string("peer engine: ") + p->err);
    if (p->slots.size() != c->slots.size()) return fail(c, MBFT_ERR_STATE, "peer slot mismatch");
  }
  if (hipSetDevice(c->device) != hipSuccess) return fail(c, MBFT_ERR_HIP, "hipSetDevice");
  return MBFT_OK;
}

// Host buffers in, host status out: split into contiguous shards over the
// primary and peer engines (one host thread each, each on its own device
// and stream), statuses written in place, so the result is in index order.
int verify_host(mbft_ctx* c, const uint8_t* e, const uint8_t* r, const uint8_t* s,
                const uint32_t* slots, size_t n, uint8_t* status) {
  const size_t engines = 1 + c->peers.size();
  size_t k = c->shard_min ? n / c->shard_min : engines;
  if (k > engines) k = engines;
  if (k <= 1) return verify_host_engine(c, e, r, s, slots, n, status);
  std::vector<int> rcs(k, MBFT_OK);
  // shards 1 .. k-1 on their engines' persistent threads, shard 0 here
  auto shard = [=, &rcs](size_t j) {
    const size_t lo = n * j / k, hi = n * (j + 1) / k;
    mbft_ctx* eng = j == 0 ? c : c->peers[j - 1];
    std::unique_lock<std::mutex> g(eng->mu, std::defer_lock);
    if (eng != c) g.lock();  // the primary's lock is held by the caller
    if (hipSetDevice(eng->device) != hipSuccess) {
      rcs[j] = MBFT_ERR_HIP;
      return;
    }
    rcs[j] = verify_host_engine(eng, e + 32 * lo, r + 32 * lo, s + 32 * lo, slots + lo, hi - lo, status + lo);
  };
  std::vector<uint64_t> tickets(k, 0);
  for (size_t j = 1; j < k; j++) tickets[j] = engine_worker(c->peers[j - 1]).submit([&shard, j] { shard(j); });
  shard(0);
  for (size_t j = 1; j < k; j++) engine_worker(c->peers[j - 1]).wait(tickets[j]);
  (void)hipSetDevice(c->device);
  for (size_t j = 0; j < k; j++)
    if (rcs[j]) {
      mbft_ctx* eng = j == 0 ? c : c->peers[j - 1];
      return eng == c ? rcs[j] : fail(c, rcs[j], std::string("peer engine: ") + eng->err);
    }
  return MBFT_OK;
}

size_t gpu_usig_min_calls() {
  const char* v = getenv("MBFT_GPU_USIG_MIN_CALLS");
  return v ? (size_t)strtoull(v, nullptr, 10) : 4096;
}


}  // namespace mbft_host

// ============================================================== C-ABI
extern "C" {

int mbft_version(void) { return kVersion; }

int mbft_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

void mbft_sha256(const uint8_t* data, size_t len, uint8_t out[32]) {
  mbft_host::sha256(data, len, out);
}

uint64_t mbft_debug_threads_started(void) { return mbft_host::g_threads_started.load(); }

}  // extern "C"

namespace mbft_host {

// A context (tables = true: builds the default generator table) or a lane
// (tables = false: streams, events and scratch only).
int create_engine(int device, bool tables, mbft_ctx** out) {
  if (!out) return MBFT_ERR_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return MBFT_ERR_NODEV;
  if (device < 0 || device >= ndev) return MBFT_ERR_ARG;
  mbft_ctx* c = new (std::nothrow) mbft_ctx();
  if (!c) return MBFT_ERR_NOMEM;
  c->device = device;
  auto bail = [&](int rc) {
    mbft_ctx_destroy(c);
    return rc;
  };
  if (hipSetDevice(device) != hipSuccess) return bail(MBFT_ERR_HIP);
  // The s^-1 pipeline stream gets the highest priority: a distinct hardware
  // queue, so the next batch's (latency-bound) inverse runs beside the
  // current verify kernel instead of queueing behind it.
  int prio_lo = 0, prio_hi = 0;
  hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithPriority(&c->istream, hipStreamNonBlocking, prio_hi) != hipSuccess ||
      hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->cstream2, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->vstream[0], hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->vstream[1], hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->kstream, hipStreamNonBlocking) != hipSuccess)
    return bail(MBFT_ERR_HIP);
  for (hipEvent_t* ev : {&c->ev_in, &c->ev_h2d, &c->ev_h2d2})
    if (hipEventCreateWithFlags(ev, hipEventDisableTiming) != hipSuccess) return bail(MBFT_ERR_HIP);
  for (int j = 0; j < mbft_ctx::kMsgChunks; j++)
    if (hipEventCreateWithFlags(&c->ev_msg[j], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_cnt[j], hipEventDisableTiming) != hipSuccess)
      return bail(MBFT_ERR_HIP);
  for (int k = 0; k < mbft_ctx::kPipe; k++)
    if (hipEventCreateWithFlags(&c->ev_inv[k], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_done[k], hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(c->ev_done[k], c->stream) != hipSuccess)
      return bail(MBFT_ERR_HIP);
  if (tables && mbft_host::build_generator(c, c->g_wbits) != MBFT_OK) return bail(MBFT_ERR_HIP);
  if (hipStreamSynchronize(c->stream) != hipSuccess) return bail(MBFT_ERR_HIP);
  *out = c;
  return MBFT_OK;
}

void destroy_lanes(mbft_ctx* c) {
  for (mbft_ctx* l : c->lanes) mbft_ctx_destroy(l);
  c->lanes.clear();
  c->lane_free.clear();
  c->lane_busy.clear();
  c->concurrency = 1;
}

// `count` lanes on the device of table engine `owner` (the context or a peer
// engine): engines with their own scratch, streams and pool that read the
// owner's tables (caller holds the context's KeyWriteGuard).
int add_lanes(mbft_ctx* c, mbft_ctx* owner, int count) {
  const int total = count * (1 + (int)c->peers.size());
  const int workers = host_pool_threads() / total > 2 ? host_pool_threads() / total : 2;
  for (int i = 0; i < count; i++) {
    mbft_ctx* l = nullptr;
    const int rc = create_engine(owner->device, /*tables=*/false, &l);
    if (rc) return fail(c, rc, "lane: create on device " + std::to_string(owner->device));
    l->owner = owner;
    l->pool_threads = workers;
    l->dev_prepare = c->dev_prepare;
    c->lanes.push_back(l);
    c->lane_free.push_back(l);
  }
  return MBFT_OK;
}

}  // namespace mbft_host

extern "C" {

int mbft_ctx_create(int device, mbft_ctx** out) { return create_engine(device, true, out); }

void mbft_ctx_destroy(mbft_ctx* c) {
  if (!c) return;
  resident_destroy(c);
  destroy_lanes(c);
  for (mbft_ctx* p : c->peers) mbft_ctx_destroy(p);
  c->peers.clear();
  hipSetDevice(c->device);
  c->pool.reset();
  for (hipStream_t st : {c->stream, c->istream, c->cstream, c->cstream2, c->vstream[0], c->vstream[1], c->kstream})
    if (st) hipStreamSynchronize(st);
  for (auto& ev : c->evs) {
    hipEventSynchronize(ev.d);
    hipEventDestroy(ev.a);
    hipEventDestroy(ev.b);
    hipEventDestroy(ev.c);
    hipEventDestroy(ev.d);
  }
  for (int k = 0; k < mbft_ctx::kPipe; k++)
    for (DevBuf* b : {&c->winv[k], &c->ws[k], &c->slowq[k]}) b->release();
  for (DevBuf* b : {&c->e, &c->r, &c->s, &c->slot, &c->status, &c->xy, &c->ok, &c->bpts, &c->priv_d, &c->sha_data,
                    &c->sha_off, &c->sha_out, &c->sha_ep, &c->sha_ctr, &c->b_e, &c->b_r, &c->b_s,
                    &c->b_slot, &c->b_status, &c->b_udata, &c->b_uoff, &c->b_uidx, &c->b_uep,
                    &c->b_uctr, &c->b_desc, &c->d_kmap_keys, &c->d_kmap_slots, &c->b_roles,
                    &c->b_ids, &c->b_moff, &c->b_toff, &c->b_msgs, &c->b_tags, &c->b_small,
                    &c->m_recs, &c->m_bytes, &c->m_chk, &c->m_flag, &c->m_cand, &c->m_chash,
                    &c->m_cslot, &c->m_uniq, &c->m_ref, &c->m_idx, &c->m_callof, &c->m_candof, &c->m_bounds,
                    &c->m_tkeys, &c->m_treps, &c->m_scan, &c->m_fpg, &c->m_info, &c->m_epset,
                    &c->m_epval, &c->m_cap, &c->m_out, &c->b_bad, &c->m_pack})
    b->release();
  for (PinnedBuf* b : {&c->h_e, &c->h_r, &c->h_s, &c->h_slot, &c->h_status, &c->h_udata, &c->h_uoff,
                       &c->h_uidx, &c->h_uep, &c->h_uctr, &c->h_desc, &c->h_small, &c->hm_small,
                       &c->hm_chk, &c->hm_callof, &c->hm_info, &c->hm_cap, &c->hm_out, &c->hm_recs,
                       &c->hm_bytes, &c->hm_bad, &c->hm_pack})
    b->release();
  if (c->zc_host) hipHostFree(c->zc_host);
  for (hipEvent_t ev : {c->ev_in, c->ev_h2d, c->ev_h2d2})
    if (ev) hipEventDestroy(ev);
  for (int j = 0; j < mbft_ctx::kMsgChunks; j++)
    for (hipEvent_t ev : {c->ev_msg[j], c->ev_cnt[j]})
      if (ev) hipEventDestroy(ev);
  for (int k = 0; k < mbft_ctx::kPipe; k++)
    for (hipEvent_t ev : {c->ev_inv[k], c->ev_done[k]})
      if (ev) hipEventDestroy(ev);
  for (hipStream_t st : {c->istream, c->cstream, c->cstream2, c->vstream[0], c->vstream[1], c->kstream})
    if (st) hipStreamDestroy(st);
  if (c->d_tabG) hipFree(c->d_tabG);
  for (void* b : c->tab_blocks) hipFree(b);
  for (auto& b : c->free_blocks) hipFree(b.first);
  c->d_keys.release();
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
}

const char* mbft_last_error(const mbft_ctx* c) { return c ? c->err.c_str() : "null ctx"; }

int mbft_profile_enable(mbft_ctx* c, int enable) {
  if (!c) return MBFT_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  c->prof = enable != 0;
  return MBFT_OK;
}

int mbft_profile_read(mbft_ctx* c, double out[4]) {
  if (!c || !out) return MBFT_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return MBFT_ERR_HIP;
  for (auto& ev : c->evs) {
    HIPCHK(c, hipEventSynchronize(ev.c));
    HIPCHK(c, hipEventSynchronize(ev.d));
    float inv = 0, ver = 0;
    HIPCHK(c, hipEventElapsedTime(&inv, ev.a, ev.b));
    HIPCHK(c, hipEventElapsedTime(&ver, ev.c, ev.d));
    c->prof_inv_ms += inv;
    c->prof_verify_ms += ver;
    c->prof_batches += 1;
    c->prof_items += (double)ev.n;
    hipEventDestroy(ev.a);
    hipEventDestroy(ev.b);
    hipEventDestroy(ev.c);
    hipEventDestroy(ev.d);
  }
  c->evs.clear();
  out[0] = c->prof_verify_ms;
  out[1] = c->prof_inv_ms;
  out[2] = c->prof_batches;
  out[3] = c->prof_items;
  c->prof_verify_ms = c->prof_inv_ms = c->prof_batches = c->prof_items = 0;
  return MBFT_OK;
}

int mbft_add_role(mbft_ctx* c, uint32_t role) {
  if (!c) return MBFT_ERR_ARG;
  KeyWriteGuard g(c);
  c->roles[role];
  c->key_gen++;
  return MBFT_OK;
}

int mbft_set_key_window(mbft_ctx* c, int wbits) {
  if (!c || wbits < mbft_launch::kMinWindow || wbits > mbft_launch::kMaxWindow)
    return MBFT_ERR_ARG;
  KeyWriteGuard g(c);
  c->q_wbits = wbits;
  return MBFT_OK;
}

int mbft_set_generator_window(mbft_ctx* c, int wbits) {
  if (!c || wbits < mbft_launch::kMinWindow || wbits > mbft_launch::kMaxWindow)
    return MBFT_ERR_ARG;
  KeyWriteGuard g(c);
  if (wbits == c->g_wbits && c->d_tabG) return MBFT_OK;
  if (hipSetDevice(c->device) != hipSuccess) return fail(c, MBFT_ERR_HIP, "hipSetDevice");
  // no verify/sign may be in flight on the old table
  if (c->stream) HIPCHK(c, hipStreamSynchronize(c->stream));
  resident_park(c);
  HIPCHK(c, hipDeviceSynchronize());
  int rc = build_generator(c, wbits);
  if (rc) return rc;
  for (mbft_ctx* p : c->peers) {
    rc = mbft_set_generator_window(p, wbits);
    if (rc) return fail(c, rc, std::string("peer engine: ") + p->err);
  }
  (void)hipSetDevice(c->device);
  return MBFT_OK;
}

int mbft_ctx_add_device(mbft_ctx* c, int device) {
  if (!c) return MBFT_ERR_ARG;
  mbft_ctx* p = nullptr;
  int rc = mbft_ctx_create(device, &p);
  if (rc) return fail(c, rc, "peer engine: create on device " + std::to_string(device));
  KeyWriteGuard g(c);
  auto bail = [&](int code, const std::string& what) {
    mbft_ctx_destroy(p);
    (void)hipSetDevice(c->device);
    return fail(c, code, what);
  };
  rc = mbft_set_generator_window(p, c->g_wbits);
  if (rc) return bail(rc, "peer engine: " + p->err);
  // replay every slot in order, in runs of equal key window
  const size_t ns = c->slots.size();
  size_t a = 0;
  (void)hipSetDevice(device);
  while (a < ns) {
    size_t b = a + 1;
    while (b < ns && c->keydesc[b].wbits == c->keydesc[a].wbits) b++;
    std::vector<uint8_t> xy(64 * (b - a));
    for (size_t j = a; j < b; j++) memcpy(&xy[64 * (j - a)], c->slots[j].xy.data(), 64);
    p->q_wbits = (int)c->keydesc[a].wbits;
    rc = register_points_engine(p, xy.data(), b - a, nullptr, nullptr);
    if (rc) return bail(rc, "peer engine: " + p->err);
    a = b;
  }
  if (p->slots.size() != ns) return bail(MBFT_ERR_STATE, "peer slot mismatch");
  p->q_wbits = c->q_wbits;
  p->prof = false;
  p->split_max = c->split_max;
  p->small_inv = c->small_inv;
  p->dev_prepare = c->dev_prepare;
  c->peers.push_back(p);
  if (c->concurrency > 1) {  // the new device gets its lanes too
    rc = add_lanes(c, p, c->concurrency);
    if (rc) {
      c->peers.pop_back();
      std::vector<mbft_ctx*> keep;
      for (mbft_ctx* l : c->lanes)
        if (l->owner == p) {
          mbft_ctx_destroy(l);
        } else {
          keep.push_back(l);
        }
      c->lanes = keep;
      c->lane_free = keep;  // (KeyWriteGuard: no lane is leased now)
      mbft_ctx_destroy(p);
      (void)hipSetDevice(c->device);
      return rc;
    }
  }
  (void)hipSetDevice(c->device);
  return MBFT_OK;
}

int mbft_ctx_devices(const mbft_ctx* c, int* devices, int cap) {
  if (!c) return MBFT_ERR_ARG;
  const int n = 1 + (int)c->peers.size();
  for (int i = 0; i < n && i < cap && devices; i++)
    devices[i] = i == 0 ? c->device : c->peers[i - 1]->device;
  return n;
}

int mbft_set_shard_min(mbft_ctx* c, size_t items) {
  if (!c) return MBFT_ERR_ARG;
  KeyWriteGuard g(c);
  c->shard_min = items;
  return MBFT_OK;
}

int mbft_get_windows(const mbft_ctx* c, int* g_wbits, int* q_wbits) {
  if (!c) return MBFT_ERR_ARG;
  if (g_wbits) *g_wbits = c->g_wbits;
  if (q_wbits) *q_wbits = c->q_wbits;
  return MBFT_OK;
}

int mbft_enable_usig(mbft_ctx* c, int enabled) {
  if (!c) return MBFT_ERR_ARG;
  KeyWriteGuard g(c);
  c->usig_enabled = enabled != 0;
  c->key_gen++;
  return MBFT_OK;
}

int mbft_register_points(mbft_ctx* c, const uint8_t* xy64, size_t n, uint32_t* out_slots,
                         uint8_t* valid_out) {
  if (!c || (n && !xy64)) return MBFT_ERR_ARG;
  KeyWriteGuard g(c);
  if (hipSetDevice(c->device) != hipSuccess) return MBFT_ERR_HIP;
  return register_points(c, xy64, n, out_slots, valid_out);
}

int mbft_set_public_key_xy(mbft_ctx* c, uint32_t role, uint32_t id, const uint8_t xy[64]) {
  if (!c || !xy) return MBFT_ERR_ARG;
  KeyWriteGuard g(c);
  if (hipSetDevice(c->device) != hipSuccess) return MBFT_ERR_HIP;
  uint32_t slot = 0;
  uint8_t valid = 0;
  int rc = register_points(c, xy, 1, &slot, &valid);
  if (rc) return rc;
  if (!valid) return fail(c, MBFT_ERR_KEY, "x509: invalid elliptic curve public key");
  c->roles[role][id] = KeyEntry{slot};
  c->key_gen++;
  return MBFT_OK;
}

int mbft_set_public_key_pkix(mbft_ctx* c, uint32_t role, uint32_t id, const uint8_t* pkix,
                             size_t len) {
  if (!c || !pkix) return MBFT_ERR_ARG;
  if (len != 91 || memcmp(pkix, kPkixPrefix, 26) != 0 || pkix[26] != 0x04)
    return fail(c, MBFT_ERR_KEY, "unsupported PKIX public key (expect uncompressed P-256)");
  return mbft_set_public_key_xy(c, role, id, pkix + 27);
}

int mbft_clear_keys(mbft_ctx* c) {
  if (!c) return MBFT_ERR_ARG;
  KeyWriteGuard g(c);
  for (mbft_ctx* p : c->peers) {
    const int rc = mbft_clear_keys(p);
    if (rc) return fail(c, rc, std::string("peer engine: ") + p->err);
  }
  if (hipSetDevice(c->device) != hipSuccess) return fail(c, MBFT_ERR_HIP, "hipSetDevice");
  // no verify may be in flight on the tables being freed
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipStreamSynchronize(c->istream));
  resident_park(c);
  HIPCHK(c, hipDeviceSynchronize());
  for (size_t i = 0; i < c->tab_blocks.size(); i++)
    c->free_blocks.emplace_back(c->tab_blocks[i], c->tab_sizes[i]);
  c->tab_blocks.clear();
  c->tab_sizes.clear();
  c->slots.clear();
  c->slot_of_xy.clear();
  c->keydesc.clear();
  for (auto& r : c->roles) r.second.clear();
  c->key_gen++;
  c->fp_group_of.clear();
  c->epoch_val.clear();
  c->epoch_set.clear();
  return MBFT_OK;
}

int mbft_key_slot(const mbft_ctx* c, uint32_t role, uint32_t id) {
  if (!c) return MBFT_ERR_ARG;
  auto rs = c->roles.find(role);
  if (rs == c->roles.end()) return MBFT_ERR_KEY;
  auto it = rs->second.find(id);
  if (it == rs->second.end()) return MBFT_ERR_KEY;
  return (int)it->second.slot;
}

int mbft_set_private_key(mbft_ctx* c, uint32_t role, const uint8_t d[32]) {
  if (!c || !d) return MBFT_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  std::array<uint8_t, 32> k;
  memcpy(k.data(), d, 32);
  c->priv[role] = k;
  return MBFT_OK;
}

int mbft_verify_batch(mbft_ctx* c, const mbft_item* items, size_t n, uint8_t* status_out) {
  if (!c || (n && (!items || !status_out))) return MBFT_ERR_ARG;
  Lease ls(c);
  if (hipSetDevice(c->device) != hipSuccess) return MBFT_ERR_HIP;
  return verify_batch_impl(c, items, n, status_out, ls.g);
}

int mbft_verify_message_authen_tag(mbft_ctx* c, uint32_t role, uint32_t id, const uint8_t* msg,
                                   size_t msg_len, const uint8_t* tag, size_t tag_len) {
  if (!c) return MBFT_ERR_ARG;
  mbft_item it{role, id, msg, msg_len, tag, tag_len};
  uint8_t st = 0;
  if (c->res_on.load(std::memory_order_relaxed)) {
    const int rc = resident_call(c, it, &st);
    if (rc != kNoResident) return rc ? rc : (int)st;
  }
  const int rc = c->co.enabled ? coalesced_call(c, it, &st) : mbft_verify_batch(c, &it, 1, &st);
  return rc ? rc : (int)st;
}

int mbft_verify_prehashed(mbft_ctx* c, const uint8_t* e, const uint8_t* r, const uint8_t* s,
                          const uint32_t* slots, size_t n, uint8_t* status) {
  if (!c || (n && (!e || !r || !s || !slots || !status))) return MBFT_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return MBFT_ERR_HIP;
  return verify_host(c, e, r, s, slots, n, status);
}

int mbft_verify_prehashed_device(mbft_ctx* c, const uint8_t* d_e, const uint8_t* d_r,
                                 const uint8_t* d_s, const uint32_t* d_slots, size_t n,
                                 uint8_t* d_status, void* hip_stream) {
  if (!c || (n && (!d_e || !d_r || !d_s || !d_slots || !d_status))) return MBFT_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return MBFT_ERR_HIP;
  if (c->slots.empty()) return fail(c, MBFT_ERR_STATE, "no keys registered");
  hipStream_t st = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
  return verify_device(c, d_e, d_r, d_s, d_slots, n, d_status, st);
}

int mbft_sign_prehashed(mbft_ctx* c, const uint8_t* priv32, size_t nkeys,
                        const uint32_t* key_idx, const uint8_t* e, size_t n, uint8_t* r_out,
                        uint8_t* s_out) {
  if (!c || !priv32 || nkeys == 0 || (n && (!e || !r_out || !s_out))) return MBFT_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return MBFT_ERR_HIP;
  if (n == 0) return MBFT_OK;
  HIPCHK(c, c->priv_d.ensure(32 * nkeys));
  HIPCHK(c, c->e.ensure(32 * n));
  HIPCHK(c, c->r.ensure(32 * n));
  HIPCHK(c, c->s.ensure(32 * n));
  HIPCHK(c, c->slot.ensure(4 * n));
  HIPCHK(c, hipMemcpyAsync(c->priv_d.p, priv32, 32 * nkeys, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->e.p, e, 32 * n, hipMemcpyHostToDevice, c->stream));
  if (key_idx)
    HIPCHK(c, hipMemcpyAsync(c->slot.p, key_idx, 4 * n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, mbft_launch::sign(c->priv_d.as<uint8_t>(), key_idx ? c->slot.as<uint32_t>() : nullptr,
                              c->e.as<uint8_t>(), nullptr, (long)n, c->d_tabG, c->g_wbits,
                              c->r.as<uint8_t>(), c->s.as<uint8_t>(), c->stream));
  HIPCHK(c, hipMemcpyAsync(r_out, c->r.p, 32 * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(s_out, c->s.p, 32 * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return MBFT_OK;
}

int mbft_sign_prehashed_device(mbft_ctx* c, const uint8_t* d_priv32, const uint32_t* d_key_idx,
                               const uint8_t* d_e, size_t n, uint8_t* d_r, uint8_t* d_s,
                               void* hip_stream) {
  if (!c || !d_priv32 || (n && (!d_e || !d_r || !d_s))) return MBFT_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return MBFT_ERR_HIP;
  hipStream_t st = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
  HIPCHK(c, mbft_launch::sign(d_priv32, d_key_idx, d_e, nullptr, (long)n, c->d_tabG, c->g_wbits, d_r,
                              d_s, st));
  return MBFT_OK;
}

int mbft_sign_nonce_device(mbft_ctx* c, const uint8_t* d_priv32, const uint32_t* d_key_idx,
                           const uint8_t* d_e, const uint8_t* d_k, size_t n, uint8_t* d_r,
                           uint8_t* d_s, void* hip_stream) {
  if (!c || !d_priv32 || (n && (!d_e || !d_k || !d_r || !d_s))) return MBFT_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return MBFT_ERR_HIP;
  hipStream_t st = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
  HIPCHK(c, mbft_launch::sign(d_priv32, d_key_idx, d_e, d_k, (long)n, c->d_tabG, c->g_wbits, d_r,
                              d_s, st));
  return MBFT_OK;
}

int mbft_request_digests_device(mbft_ctx* c, const uint64_t* d_seq, const uint8_t* d_ops,
                                uint32_t op_len, size_t n, uint8_t* d_e, void* hip_stream) {
  if (!c || (n && (!d_seq || !d_e || (op_len && !d_ops)))) return MBFT_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return MBFT_ERR_HIP;
  hipStream_t st = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
  HIPCHK(c, mbft_launch::request_e(d_seq, d_ops, op_len, (long)n, d_e, st));
  return MBFT_OK;
}

int mbft_sha256_device(mbft_ctx* c, const uint8_t* d_data, const uint64_t* d_off, size_t n,
                       uint8_t* d_out, void* hip_stream) {
  if (!c || (n && (!d_off || !d_out))) return MBFT_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return MBFT_ERR_HIP;
  hipStream_t st = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
  HIPCHK(c, mbft_launch::sha256_var(d_data, d_off, (long)n, d_out, st));
  return MBFT_OK;
}

int mbft_usig_digests_device(mbft_ctx* c, const uint8_t* d_data, const uint64_t* d_off,
                             const uint64_t* d_epoch, const uint64_t* d_counter, size_t n,
                             uint8_t* d_e, void* hip_stream) {
  if (!c || (n && (!d_off || !d_epoch || !d_counter || !d_e))) return MBFT_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return MBFT_ERR_HIP;
  hipStream_t st = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
  HIPCHK(c, mbft_launch::usig_e(d_data, d_off, d_epoch, d_counter, nullptr, (long)n, d_e, st));
  return MBFT_OK;
}

int mbft_generate_message_authen_tag(mbft_ctx* c, uint32_t role, const uint8_t* msg,
                                     size_t msg_len, uint8_t* tag_out, size_t tag_cap,
                                     size_t* tag_len) {
  if (!c || (msg_len && !msg) || !tag_out || !tag_len) return MBFT_ERR_ARG;
  std::array<uint8_t, 32> d;
  {
    std::lock_guard<std::mutex> g(c->mu);
    auto it = c->priv.find(role);
    if (it == c->priv.end() || role == MBFT_ROLE_USIG)
      return fail(c, MBFT_ERR_STATE, "no ECDSA private key for role");
    d = it->second;
  }
  uint8_t e32[32], r[32], s[32];
  for (size_t k = 0; k < 32; k++) e32[k] = k < msg_len ? msg[k] : kEmptyHash[k - msg_len];
  int rc = mbft_sign_prehashed(c, d.data(), 1, nullptr, e32, 1, r, s);
  if (rc) return rc;
  // asn1.Marshal(ecdsaSignature{r, s}) (crypto.go:69)
  uint8_t body[2 * 35];
  size_t bl = 0;
  for (const uint8_t* v : {r, s}) {
    size_t i = 0;
    while (i < 31 && v[i] == 0) i++;
    const bool pad = (v[i] & 0x80) != 0;
    body[bl++] = 0x02;
    body[bl++] = (uint8_t)(32 - i + (pad ? 1 : 0));
    if (pad) body[bl++] = 0x00;
    memcpy(body + bl, v + i, 32 - i);
    bl += 32 - i;
  }
  const size_t total = 2 + bl;
  *tag_len = total;
  if (tag_cap < total) return MBFT_ERR_ARG;
  tag_out[0] = 0x30;
  tag_out[1] = (uint8_t)bl;
  memcpy(tag_out + 2, body, bl);
  return MBFT_OK;
}

int mbft_set_concurrency(mbft_ctx* c, int lanes) {
  if (!c || c->owner || lanes < 1 || lanes > 64) return MBFT_ERR_ARG;
  KeyWriteGuard g(c);  // no batch is on a lane now
  if (lanes == c->concurrency) return MBFT_OK;
  destroy_lanes(c);
  if (lanes == 1) return MBFT_OK;
  // `lanes` lanes on every device: the context's, then each peer engine's
  for (size_t e = 0; e <= c->peers.size(); e++) {
    const int rc = add_lanes(c, e == 0 ? c : c->peers[e - 1], lanes);
    if (rc) {
      destroy_lanes(c);
      (void)hipSetDevice(c->device);
      return rc;
    }
  }
  c->concurrency = lanes;
  (void)hipSetDevice(c->device);
  return MBFT_OK;
}

int mbft_get_concurrency(const mbft_ctx* c) { return c ? c->concurrency : MBFT_ERR_ARG; }

// Comb windows from the HBM budget and the key counts: every class starts
// at 8 bits; then, greedily, the upgrade with the most additions saved per
// verify per byte of tables is taken while it fits.  A verify adds
// ceil(256 / W) entries of the generator table and as many of its key's
// table; the key class's share of verifies weights its saving: on a
// replica, per request, one client signature and ~n USIG UIs (SURVEY
// Appendix B), replica-role signatures rarely (REPLYs are verified by
// clients).  The budget is the device's free memory less 6 GiB for batch
// scratch (1M-call batches need ~0.4 GiB per lane).
int mbft_plan_windows(int device, size_t n_replica, size_t n_usig, size_t n_client, int* g_w,
                      int* replica_w, int* usig_w, int* client_w) {
  size_t free_b = 0, total_b = 0;
  int cur = 0;
  (void)hipGetDevice(&cur);
  if (hipSetDevice(device) != hipSuccess || hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
    (void)hipGetLastError();
    free_b = (size_t)16 << 30;  // unknown device: a conservative budget
  }
  (void)hipSetDevice(cur);
  const size_t reserve = (size_t)6 << 30;
  double budget = free_b > reserve ? (double)(free_b - reserve) : 0.0;
  struct Cls {
    double count, share;
    int w;
  } cls[4] = {
      {1.0, 1.0, 8},                                                       // generator
      {(double)n_replica, n_usig ? 0.01 : (n_client ? 0.3 : 1.0), 8},      // replica keys
      {(double)n_usig, n_usig ? (double)n_usig / (double)(n_usig + 1) : 0.0, 8},  // USIG keys
      {(double)n_client, n_usig ? 1.0 / (double)(n_usig + 1) : 1.0, 8},    // client keys
  };
  auto adds = [](int w) { return (256 + w - 1) / w; };
  auto bytes = [](int w) { return (double)mbft_launch::table_words(w) * 4.0; };
  for (const Cls& k : cls) budget -= k.count * bytes(k.w);
  for (;;) {
    int best = -1, best_w = 0;
    double best_ratio = 0;
    for (int i = 0; i < 4; i++) {
      Cls& k = cls[i];
      if (k.count == 0 || k.share == 0) continue;
      int w = k.w + 1;  // the next window that saves an addition
      while (w <= mbft_launch::kMaxWindow && adds(w) == adds(k.w)) w++;
      if (w > mbft_launch::kMaxWindow) continue;
      const double cost = k.count * (bytes(w) - bytes(k.w));
      if (cost > budget) continue;
      const double ratio = k.share * (double)(adds(k.w) - adds(w)) / cost;
      if (ratio > best_ratio) {
        best_ratio = ratio;
        best = i;
        best_w = w;
      }
    }
    if (best < 0) break;
    budget -= cls[best].count * (bytes(best_w) - bytes(cls[best].w));
    cls[best].w = best_w;
  }
  if (g_w) *g_w = cls[0].w;
  if (replica_w) *replica_w = cls[1].w;
  if (usig_w) *usig_w = cls[2].w;
  if (client_w) *client_w = cls[3].w;
  return MBFT_OK;
}

}  // extern "C"

extern "C" int mbft_set_small_batch_form(mbft_ctx* c, long split_max) {
  if (!c || c->owner) return MBFT_ERR_ARG;
  KeyWriteGuard g(c);
  c->split_max = split_max < 0 ? -1 : split_max;
  for (mbft_ctx* p : c->peers) p->split_max = c->split_max;  // (their lanes read it there)
  return MBFT_OK;
}

extern "C" int mbft_set_small_batch_inverse(mbft_ctx* c, int mode) {
  if (!c || c->owner || mode < -1 || mode > 3) return MBFT_ERR_ARG;
  KeyWriteGuard g(c);
  c->small_inv = mode;
  for (mbft_ctx* p : c->peers) p->small_inv = mode;
  return MBFT_OK;
}

// mbft_validate_messages_flat and mbft_pack_messages (include/minbft_gpu.h).
//
// A flat batch -- fixed-size records plus one byte arena -- in library
// page-locked memory runs the message layer on the GPU (msg_kernels.hip):
// the records and bytes go up raw, the checks, candidate calls, content
// hashes, deduplication, AuthenBytes digests, DER / UI decode and key lookups
// are kernels, the verifier runs over the unique calls, and the host only
// replays the outcomes in message order (messages.cpp replay_messages: stream
// stop, panic stop, the USIG epoch state), exactly as mbft_validate_messages
// does for its host-built calls.  Any other flat batch is turned into
// mbft_message structs over the arena and validated by the host message
// layer; both give identical results.
//
// mbft_check_messages_flat / mbft_resolve_message split the same validation
// like mbft_check_batch / mbft_resolve_checked: the device part (every
// signature, digest, decode and key lookup; no state) runs once for the
// batch, and the in-order part (the USIG epoch step, crypto.go:219-236) runs
// per message when the caller resolves it -- the core's stream loop, right
// before processing that message, so a message after one whose processing
// failed is never validated and captures nothing (exactly the reference's
// sequence, core/message-handling.go:204-246).
#include <algorithm>
#include <chrono>

#include "host_internal.h"
#include "msg_dev.h"

using namespace mbft_host;

namespace {

static_assert(sizeof(mbft::DevCallInfo) == sizeof(CallInfo), "DevCallInfo mirrors CallInfo");
static_assert(offsetof(mbft::DevCallInfo, fpg) == offsetof(CallInfo, fpg) &&
                  offsetof(mbft::DevCallInfo, ui_epoch) == offsetof(CallInfo, ui_epoch) &&
                  offsetof(mbft::DevCallInfo, counter) == offsetof(CallInfo, counter) &&
                  offsetof(mbft::DevCallInfo, usig) == offsetof(CallInfo, usig) &&
                  offsetof(mbft::DevCallInfo, usig_tail) == offsetof(CallInfo, usig_tail),
              "DevCallInfo mirrors CallInfo");

double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

// HIP-event timing of one device message-layer call (when profiling is on):
// up0 before the first upload and up1 after the last, both on the copy
// stream (the H2D time of the records and arena), end after the last device
// work on the compute stream; done() adds them to the engine's totals.
struct MsgProf {
  mbft_ctx* g;
  bool on;
  hipEvent_t up0 = nullptr, up1 = nullptr, end = nullptr;
  explicit MsgProf(mbft_ctx* e) : g(e), on(e->prof) {
    if (on && (hipEventCreate(&up0) != hipSuccess || hipEventCreate(&up1) != hipSuccess ||
               hipEventCreate(&end) != hipSuccess))
      on = false;
  }
  void done(size_t bytes) {
    if (!on) return;
    float h2d = 0, dev = 0;
    if (hipEventElapsedTime(&h2d, up0, up1) == hipSuccess &&
        hipEventElapsedTime(&dev, up0, end) == hipSuccess) {
      g->prof_msg[0] += 1;
      g->prof_msg[1] += h2d;
      g->prof_msg[2] += dev;
      g->prof_msg[3] += (double)bytes;
    }
  }
  ~MsgProf() {
    for (hipEvent_t e : {up0, up1, end})
      if (e) (void)hipEventDestroy(e);
  }
};

// The roles of nc device call records (DevCallInfo, as copied down).
void dev_roles(const uint8_t* info, size_t nc, std::vector<uint8_t>& role) {
  role.resize(nc);
  for (size_t k = 0; k < nc; k++) role[k] = info[sizeof(mbft::DevCallInfo) * k + offsetof(mbft::DevCallInfo, role)];
}

// The checks of messages [f, n) from the packed device words (one 32-bit
// word per message: the count, then per check kind, stage and candidate
// slot; msg_kernels.hip k_msg_cands) and the candidates' call numbers.
void unpack_checks(mbft_ctx* g, size_t f, size_t n, const uint32_t* chk, const uint32_t* callof,
                   MsgChecks* checks) {
  const size_t m = n - f;
  const int Tm = m >= 4096 ? g->pool->size() : 1;
  g->pool->run(Tm, [&](int t) {
    for (size_t i = f + m * t / Tm; i < f + m * (t + 1) / Tm; i++) {
      const uint32_t w = chk[i];
      MsgChecks& ck = checks[i];
      ck.n = (uint8_t)(w & 0xFFu);
      for (int q = 0; q < ck.n; q++) {
        const uint32_t b = (w >> (8 + 8 * q)) & 0xFFu;
        ck.c[q].kind = (uint8_t)(b & 3u);
        ck.c[q].stage = (uint8_t)((b >> 2) & 15u);
        ck.c[q].call = ck.c[q].kind == 0 ? callof[3 * i + ((b >> 6) & 3u)] : 0xFFFFFFFFu;
      }
    }
  });
}

// Everything a device check copies down, in ONE device block (and one
// page-locked host block of the same layout), so it comes down in one copy
// instead of six (each a blit kernel plus a gap: ~45 us of a 1,024-message
// pass, profiles/round6_midsize_timeline_1024.json): the unique-call count
// and chunk bounds, the argument flags, the packed checks, the candidates'
// call numbers, the call statuses, and last the call records (so a prefix of
// nc records ends the copy).
struct PackLayout {
  size_t bounds = 0, flags = 64, chk = 256, callof, status, info, end;
  explicit PackLayout(size_t n) {
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    callof = al(chk + 4 * n);
    status = al(callof + 12 * n);
    info = al(status + 3 * n + 1);
    end = info + sizeof(mbft::DevCallInfo) * 3 * n + 32;
  }
  size_t through(size_t nc) const { return info + sizeof(mbft::DevCallInfo) * nc; }
};

}  // namespace

// The checks, per-call outcomes and statuses of a device-checked batch
// (mbft_check_messages_flat), resolved message by message.
// The unique calls of one device pass: host outcome and GPU status per call
// (shared by every batch a coalesced pass served).
struct MsgCalls {
  std::vector<CallInfo> info;
  std::vector<uint8_t> gst;
  std::vector<uint8_t> role;  // each call's role (the in-order replay's panic rule)
};
struct mbft_msg_batch {
  mbft_ctx* c = nullptr;
  size_t n = 0;
  std::vector<MsgChecks> checks;
  std::shared_ptr<const MsgCalls> calls;
};

namespace {

// The device path (recs and bytes are library-owned page-locked memory,
// n > 0).  c: the key store and USIG epoch state; g: the engine whose
// buffers, streams and pool run the batch (c itself, or a lane leased by the
// caller).  Validate mode (chk == null, g == c, caller holds c->mu): the
// results of every message, replayed on the GPU and finished on the host.
// Check mode: no state read or written; the checks, call outcomes and
// statuses go to *chk.  Error returns may leave work queued on any of the
// three streams: validate_flat_device drains them.
// The rest of a one-wait check (validate_flat_device_impl): k_call_list /
// k_msg_calls and the verifier over the 3n upper bound, stopping at the
// device count bounds[1]; then the checks, call outcomes, statuses, count and
// argument flags in one synchronize.
int check_one_wait(mbft_ctx* c, mbft_ctx* g, const mbft::MsgDevArgs& a, size_t n, uint32_t* bounds,
                   uint8_t* dstatus, const PackLayout& L, MsgProf& prof, size_t nbytes,
                   mbft_msg_batch* chk, bool listed) {  // nbytes: uploaded; listed: msg_number_one ran
  (void)c;
  const size_t nc3 = 3 * n;
  // one stream for the whole pass: a single chunk has nothing to overlap
  // the calls and the verifier with, and each cross-stream event left a
  // 13-23 us gap (profiles/round6_midsize_timeline_1024*.json)
  hipStream_t st = g->stream, vb = st;
  HIPCHK(g, mbft_launch::msg_calls(a, 0, (long)n, 0, (long)nc3, vb, bounds + 1, listed));
  int rc = verify_device(g, a.e, a.r, a.s, a.slot, nc3, dstatus, vb, /*host_status=*/true,
                         /*latency=*/false, /*d_winv=*/nullptr, /*d_count=*/bounds + 1);
  if (rc) return rc;
  HIPCHK(g, g->hm_pack.ensure(L.end));
  HIPCHK(g, hipMemcpyAsync(g->hm_pack.p, g->m_pack.p, L.end, hipMemcpyDeviceToHost, st));
  if (prof.on) HIPCHK(g, hipEventRecord(prof.end, st));
  HIPCHK(g, hipStreamSynchronize(st));
  const uint8_t* hp = g->hm_pack.as<uint8_t>();
  const uint32_t bad = reinterpret_cast<const uint32_t*>(hp + L.flags)[0];
  if (bad & 3u) {  // an argument error: nothing written to the batch (the caller drains)
    if (bad & 1u) return fail(g, MBFT_ERR_ARG, "mbft_check_messages_flat: unknown message type");
    return fail(g, MBFT_ERR_ARG, "mbft_check_messages_flat: field outside the byte arena");
  }
  prof.done(sizeof(mbft_msg_rec) * n + nbytes);
  const size_t nc = reinterpret_cast<const uint32_t*>(hp + L.bounds)[1];
  chk->n = n;
  chk->checks.resize(n);
  auto calls = std::make_shared<MsgCalls>();
  const CallInfo* info = reinterpret_cast<const CallInfo*>(hp + L.info);
  calls->info.assign(info, info + nc);
  calls->gst.assign(hp + L.status, hp + L.status + nc);
  dev_roles(hp + L.info, nc, calls->role);
  chk->calls = std::move(calls);
  unpack_checks(g, 0, n, reinterpret_cast<const uint32_t*>(hp + L.chk),
                reinterpret_cast<const uint32_t*>(hp + L.callof), chk->checks.data());
  return MBFT_OK;
}

// abase: the records' fields all lie in [abase, nbytes) of `bytes` (8-aligned;
// a record shard of a larger pass), only that slice goes up, and the kernels
// read it at the same absolute offsets.
int validate_flat_device_impl(mbft_ctx* c, mbft_ctx* g, const mbft_msg_rec* recs, size_t n,
                              const uint8_t* bytes, size_t nbytes, uint32_t n_replicas, uint32_t flags,
                              int32_t* out, mbft_msg_batch* chk, size_t abase) {
  const size_t up = nbytes - abase;  // arena bytes uploaded
  const auto t0 = std::chrono::steady_clock::now();
  if (!g->pool) g->pool.reset(new Pool(pool_workers(g)));
  int rc = sync_keymap(c, g);
  if (rc) return rc;
  const size_t nc3 = 3 * n;
  size_t cap = 1024;
  while (cap < 2 * nc3) cap <<= 1;
  HIPCHK(g, g->m_recs.ensure(sizeof(mbft_msg_rec) * n));
  HIPCHK(g, g->m_bytes.ensure(((up + 3) & ~(size_t)3) + 32));
  const PackLayout L(n);
  HIPCHK(g, g->m_pack.ensure(L.end));
  uint8_t* pk = g->m_pack.as<uint8_t>();
  HIPCHK(g, g->m_cand.ensure(sizeof(mbft::MsgCand) * nc3));
  HIPCHK(g, g->m_chash.ensure(8 * nc3));
  HIPCHK(g, g->m_cslot.ensure(4 * nc3));
  HIPCHK(g, g->m_uniq.ensure(4 * nc3));
  HIPCHK(g, g->m_ref.ensure(4 * nc3));
  HIPCHK(g, g->m_idx.ensure(4 * nc3));
  HIPCHK(g, g->m_candof.ensure(4 * nc3));
  HIPCHK(g, g->m_tkeys.ensure(8 * cap));
  HIPCHK(g, g->m_treps.ensure(4 * cap));
  const mbft_ctx* tb = tabs(g);
  // the slots' USIG fingerprint groups -- the key store's numbering, which
  // the epoch state is indexed by (an engine on another device holds the same
  // slots) -- uploaded when the key store changed
  const bool fpg_new = g->fpg_gen != c->key_gen || g->fpg_n != c->slots.size();
  std::vector<uint32_t> fpg;
  if (fpg_new) {
    fpg.assign(c->slots.size() + 1, 0);
    for (size_t k = 0; k < c->slots.size(); k++) fpg[k] = c->slots[k].fp_group;
    HIPCHK(g, g->m_fpg.ensure(4 * fpg.size()));
  }
  HIPCHK(g, g->hm_small.ensure(64));

  mbft::MsgDevArgs a{};
  a.recs = g->m_recs.as<mbft_msg_rec>();
  a.bytes = g->m_bytes.as<uint8_t>() - abase;  // (read only at offsets >= abase)
  a.nbytes = nbytes;
  a.n = (long)n;
  a.n_replicas = n_replicas;
  a.chk = reinterpret_cast<uint32_t*>(pk + L.chk);
  a.bad = reinterpret_cast<uint32_t*>(pk + L.flags);
  a.cand = g->m_cand.as<mbft::MsgCand>();
  a.chash = g->m_chash.as<uint64_t>();
  a.cslot = g->m_cslot.as<uint32_t>();
  a.uniq = g->m_uniq.as<uint32_t>();
  a.ref = g->m_ref.as<uint32_t>();
  a.idx = g->m_idx.as<uint32_t>();
  a.call_of = reinterpret_cast<uint32_t*>(pk + L.callof);
  a.cand_of = g->m_candof.as<uint32_t>();
  a.tkeys = g->m_tkeys.as<unsigned long long>();
  a.treps = g->m_treps.as<uint32_t>();
  a.tmask = (uint32_t)(cap - 1);
  a.map = mbft::KeyMap{g->d_kmap_keys.as<uint64_t>(), g->d_kmap_slots.as<uint32_t>(), g->kmap_mask,
                       g->kmap_role_ok};
  a.keys = tb->d_keys.as<mbft::KeyDesc>();
  a.nslots = (uint32_t)tb->slots.size();
  a.fpg = g->m_fpg.as<uint32_t>();

  // per unique call (at most one per candidate)
  HIPCHK(g, g->b_e.ensure(32 * nc3 + 32));
  HIPCHK(g, g->b_r.ensure(32 * nc3 + 32));
  HIPCHK(g, g->b_s.ensure(32 * nc3 + 32));
  HIPCHK(g, g->b_slot.ensure(4 * nc3 + 4));

  a.e = g->b_e.as<uint8_t>();
  a.r = g->b_r.as<uint8_t>();
  a.s = g->b_s.as<uint8_t>();
  a.slot = g->b_slot.as<uint32_t>();
  a.info = reinterpret_cast<mbft::DevCallInfo*>(pk + L.info);
  uint32_t* bounds = reinterpret_cast<uint32_t*>(pk + L.bounds);  // kMsgChunks + 1 <= 16 words
  uint8_t* dstatus = pk + L.status;

  hipStream_t st = g->stream, cs = g->cstream, vb = g->vstream[0];
  const int K = n >= 65536 ? mbft_ctx::kMsgChunks : 1;
  // one chunk: its copies on the compute stream itself -- nothing to overlap
  // them with, and no cross-stream event between the last copy and the first
  // kernel (~35 us of a 1,024-message pass, round6_midsize_timeline_1024.json)
  if (K == 1) cs = vb = st;
  // The dedup table cleared on the compute stream; on the copy stream the
  // arena first (its tail padded with zeros: the kernels read whole words),
  // then the records in chunks.  Each chunk's kernels start as soon as its
  // records are in (a record may point anywhere in the arena, so the arena
  // goes whole): candidates, table inserts, and -- exact already, since a
  // slot keeps its smallest candidate and later chunks only add larger ones --
  // the full-compare resolve and the chunk's call numbering (a local scan plus
  // the running base in bounds[]), whose running end comes back to the host.
  // The verify runs in two stages on a second stream: the calls of the first
  // chunks (0..S, S = 3 of 8) as soon as their count is back, under the later
  // copies, then the rest (its s^-1 in one launch: nothing after it to hide a
  // chain behind).  Measured +0.9-1.5 % over one stage (within a few percent of
  // noise, profiles/round3_c3_split_sp*.jsonl); eight per-chunk verifies were
  // slower (a 70K-call verify is latency-bound).  The previous call ended with a synchronize, so nothing
  // still reads these buffers.
  HIPCHK(g, g->hm_small.ensure(4 * (mbft_ctx::kMsgChunks + 8)));
  uint32_t* hs = g->hm_small.as<uint32_t>();  // [0, K) running chunk ends, [K] the argument-check flags
  uint32_t* tail6 = reinterpret_cast<uint32_t*>(g->m_bytes.as<uint8_t>() + (up & ~(size_t)3));
  // A one-chunk pass of up to MBFT_MSG_KCOPY_MAX bytes (default 4 MiB; 0:
  // never) uploads its records and arena with k_msg_init's own threads
  // (reads of page-locked memory over PCIe) instead of two copy-engine
  // copies: each hand-off between the copy engine and the compute queue
  // cost ~8-11 us (init -> copy -> copy -> k_msg_cands: ~29 us of a
  // 1,024-message pass, profiles/round6_midsize_timeline_*.json).
  static const size_t kcopy_max = [] {
    const char* v = getenv("MBFT_MSG_KCOPY_MAX");
    return v ? (size_t)strtoull(v, nullptr, 10) : (size_t)4 << 20;
  }();
  const size_t rec_bytes = sizeof(mbft_msg_rec) * n;
  const bool kcopy = K == 1 && rec_bytes + up <= kcopy_max && (((uintptr_t)recs | (uintptr_t)(bytes + abase)) & 15u) == 0;
  MsgProf prof(g);
  if (kcopy) {
    // profiling: the upload events bracket the init kernel that does it
    if (prof.on) HIPCHK(g, hipEventRecord(prof.up0, st));
    const mbft::MsgUpload u_rec{reinterpret_cast<uint8_t*>(g->m_recs.p), reinterpret_cast<const uint8_t*>(recs),
                                rec_bytes, rec_bytes};
    const mbft::MsgUpload u_arena{g->m_bytes.as<uint8_t>(), bytes + abase, up, (up & ~(size_t)3) + 24};
    HIPCHK(g, mbft_launch::msg_init(a, a.bad, bounds, st, nullptr, &u_rec, &u_arena));
    if (prof.on) HIPCHK(g, hipEventRecord(prof.up1, st));
  } else {
    HIPCHK(g, mbft_launch::msg_init(a, a.bad, bounds, st, cs == st ? tail6 : nullptr));
  }
  // profiling (mbft_profile_msg_layer): HIP events on the copy stream around
  // every upload, and at the end of the device work on st
  if (prof.on && !kcopy) HIPCHK(g, hipEventRecord(prof.up0, cs));
  if (fpg_new) {
    HIPCHK(g, hipMemcpyAsync(g->m_fpg.p, fpg.data(), 4 * fpg.size(), hipMemcpyHostToDevice, cs));
    g->fpg_gen = c->key_gen;
    g->fpg_n = c->slots.size();
  }
  if (cs != st) HIPCHK(g, hipMemsetAsync(tail6, 0, 24, cs));
  if (up && !kcopy) HIPCHK(g, hipMemcpyAsync(g->m_bytes.p, bytes + abase, up, hipMemcpyHostToDevice, cs));
  static const int split_at = [] {  // env MBFT_MSG_VERIFY_SPLIT: the first stage's last chunk (-1: one stage)
    const char* v = getenv("MBFT_MSG_VERIFY_SPLIT");
    return v ? atoi(v) : 3;
  }();
  const int S = K > 1 && split_at >= 0 && split_at < K - 1 ? split_at : -1;
  // A small check (one chunk, <= kOneWaitMsgs messages) waits on the host
  // once: the unique-call count stays on the device, k_msg_calls and the
  // small-batch verifier (pairs / split: no s^-1 chain sized on the host) run
  // over the 3n upper bound and stop at the device count, and the count and
  // argument flags come down with the results.  Only where the two-wait form
  // would run the small-batch verifier too (3n <= 4,096 calls): for a
  // 4,096-message stream batch (12,288 calls) the per-lane s^-1 costs more
  // than the wait saves (0.56 vs 0.49 ms p50 alone, and half the rate with 4
  // lanes at once; profiles/round4_msg_pass_ab.txt).  Env MBFT_MSG_ONE_WAIT=0:
  // the two-wait form always.
  static const bool one_wait_env = [] {
    const char* v = getenv("MBFT_MSG_ONE_WAIT");
    return !(v && atoi(v) == 0);
  }();
  static const size_t kOneWaitMsgs = [] {  // env MBFT_MSG_ONE_WAIT_MAX (messages)
    const char* v = getenv("MBFT_MSG_ONE_WAIT_MAX");
    return v ? (size_t)strtoull(v, nullptr, 10) : (size_t)(4096 / 3);
  }();
  const bool one_wait = one_wait_env && chk && K == 1 && n <= kOneWaitMsgs;
  // A one-chunk pass of up to 1,365 messages numbers its calls in one
  // single-workgroup launch (msg_number_one) instead of the hipcub scan,
  // k_chunk_base and k_call_list; env MBFT_MSG_NUMBER_ONE=0: never.
  static const bool number_one_env = [] {
    const char* v = getenv("MBFT_MSG_NUMBER_ONE");
    return !(v && atoi(v) == 0);
  }();
  const bool listed = number_one_env && K == 1 && 3 * (long)n <= mbft_launch::kNumberOneMax;
  size_t tmp_bytes = 0;
  HIPCHK(g, mbft_launch::msg_scan(a, 0, 0, (long)((n + K - 1) / K + 1), nullptr, &tmp_bytes, st));
  HIPCHK(g, g->m_scan.ensure(tmp_bytes + 16));
  auto chunk_lo = [&](int j) { return (long)(n * (size_t)j / (size_t)K); };
  for (int j = 0; j < K; j++) {
    const long lo = chunk_lo(j), hi = chunk_lo(j + 1);
    if (!kcopy) {
      HIPCHK(g, hipMemcpyAsync(g->m_recs.as<mbft_msg_rec>() + lo, recs + lo, sizeof(mbft_msg_rec) * (hi - lo),
                               hipMemcpyHostToDevice, cs));
      if (prof.on && j == K - 1) HIPCHK(g, hipEventRecord(prof.up1, cs));
    }
    if (cs != st) {
      HIPCHK(g, hipEventRecord(g->ev_msg[j], cs));
      HIPCHK(g, hipStreamWaitEvent(st, g->ev_msg[j], 0));
    }
    HIPCHK(g, mbft_launch::msg_cands(a, lo, hi, st));  // (the table inserts too)
    HIPCHK(g, mbft_launch::msg_dedup_resolve(a, lo, hi, st));
    if (listed) {
      HIPCHK(g, mbft_launch::msg_number_one(a, lo, hi, bounds, j, st));
    } else {
      HIPCHK(g, mbft_launch::msg_scan(a, lo, hi, 0, g->m_scan.p, &tmp_bytes, st));
      HIPCHK(g, mbft_launch::msg_number(a, lo, hi, bounds, j, st));
    }
    if (one_wait) continue;  // (the count stays on the device)
    if (j == S || j == K - 1) {
      HIPCHK(g, hipMemcpyAsync(hs + j, bounds + j + 1, 4, hipMemcpyDeviceToHost, st));
      if (j == K - 1) HIPCHK(g, hipMemcpyAsync(hs + K, a.bad, 4, hipMemcpyDeviceToHost, st));
      HIPCHK(g, hipEventRecord(g->ev_cnt[j], st));
    }
  }
  if (one_wait) return check_one_wait(c, g, a, n, bounds, dstatus, L, prof, up, chk, listed);
  // stage 1: chunks [0, S]; stage 2: chunks (S, K)
  uint32_t base = 0;
  for (int stage = 0; stage < 2; stage++) {
    const int j0 = stage == 0 ? 0 : S + 1, j1 = stage == 0 ? S : K - 1;
    if (j1 < j0) continue;
    HIPCHK(g, hipEventSynchronize(g->ev_cnt[j1]));
    if (j1 == K - 1 && (hs[K] & 3u)) {  // an argument error: write nothing (the caller drains)
      if (hs[K] & 1u) return fail(g, MBFT_ERR_ARG, "mbft_validate_messages_flat: unknown message type");
      return fail(g, MBFT_ERR_ARG, "mbft_validate_messages_flat: field outside the byte arena");
    }
    const uint32_t end = hs[j1], cnt = end - base;
    if (vb != st) HIPCHK(g, hipStreamWaitEvent(vb, g->ev_cnt[j1], 0));
    HIPCHK(g, mbft_launch::msg_calls(a, chunk_lo(j0), chunk_lo(j1 + 1), (long)base, (long)cnt, vb, nullptr,
                                     listed));
    if (cnt) {
      rc = verify_device(g, a.e + 32 * (size_t)base, a.r + 32 * (size_t)base, a.s + 32 * (size_t)base,
                         a.slot + base, cnt, dstatus + base, vb, /*host_status=*/true,
                         /*latency=*/j1 == K - 1 && S >= 0);
      if (rc) return rc;
    }
    base = end;
  }
  const size_t nc = base;
  const auto t1 = std::chrono::steady_clock::now();
  if (chk) {
    // check mode: the checks, call outcomes and statuses come down; nothing
    // replayed, no epoch state read
    HIPCHK(g, g->hm_pack.ensure(L.end));
    if (vb != st) {  // st joins the verifies
      HIPCHK(g, hipEventRecord(g->ev_cnt[0], vb));
      HIPCHK(g, hipStreamWaitEvent(st, g->ev_cnt[0], 0));
    }
    // one copy: checks, call numbers, statuses and the first nc call records
    HIPCHK(g, hipMemcpyAsync(g->hm_pack.as<uint8_t>() + L.chk, pk + L.chk, L.through(nc) - L.chk,
                             hipMemcpyDeviceToHost, st));
    if (prof.on) HIPCHK(g, hipEventRecord(prof.end, st));
    HIPCHK(g, hipStreamSynchronize(st));
    prof.done(sizeof(mbft_msg_rec) * n + up);
    const uint8_t* hp = g->hm_pack.as<uint8_t>();
    chk->n = n;
    chk->checks.resize(n);
    auto calls = std::make_shared<MsgCalls>();
    const CallInfo* info = reinterpret_cast<const CallInfo*>(hp + L.info);
    calls->info.assign(info, info + nc);
    calls->gst.assign(hp + L.status, hp + L.status + nc);
    dev_roles(hp + L.info, nc, calls->role);
    chk->calls = std::move(calls);
    unpack_checks(g, 0, n, reinterpret_cast<const uint32_t*>(hp + L.chk),
                  reinterpret_cast<const uint32_t*>(hp + L.callof), chk->checks.data());
    return MBFT_OK;
  }
  if (vb != st) {  // st joins the verifies
    HIPCHK(g, hipEventRecord(g->ev_cnt[0], vb));
    HIPCHK(g, hipStreamWaitEvent(st, g->ev_cnt[0], 0));
  }
  // the optimistic in-order replay on the GPU (k_replay_*, messages.cpp
  // replay_parallel's rules): every message's result, the first message
  // whose result is not 0, and each key group's first capture
  const size_t G = c->epoch_val.size();
  HIPCHK(g, g->m_epset.ensure(G + 1));
  HIPCHK(g, g->m_epval.ensure(8 * G + 8));
  HIPCHK(g, g->m_cap.ensure(16 * G + 16));
  HIPCHK(g, g->m_out.ensure(4 * n));
  HIPCHK(g, g->hm_cap.ensure(16 * G + 16));
  HIPCHK(g, g->hm_out.ensure(4 * n));
  if (G) {
    HIPCHK(g, hipMemcpyAsync(g->m_epset.p, c->epoch_set.data(), G, hipMemcpyHostToDevice, st));
    HIPCHK(g, hipMemcpyAsync(g->m_epval.p, c->epoch_val.data(), 8 * G, hipMemcpyHostToDevice, st));
  }
  uint64_t* hcap = g->hm_cap.as<uint64_t>();  // [0, G) cap_pos, [G, 2G) cap_epoch, [2G] first_bad
  hcap[2 * G] = n;
  HIPCHK(g, hipMemsetAsync(g->m_cap.p, 0xFF, 8 * G, st));
  HIPCHK(g, hipMemcpyAsync(g->m_cap.as<uint64_t>() + 2 * G, hcap + 2 * G, 8, hipMemcpyHostToDevice, st));
  a.status = dstatus;
  a.epoch_set = g->m_epset.as<uint8_t>();
  a.epoch_val = g->m_epval.as<uint64_t>();
  a.ngroups = (uint32_t)G;
  a.cap_pos = g->m_cap.as<unsigned long long>();
  a.cap_epoch = g->m_cap.as<uint64_t>() + G;
  a.out = g->m_out.as<int32_t>();
  a.first_bad = g->m_cap.as<unsigned long long>() + 2 * G;
  HIPCHK(g, mbft_launch::msg_replay(a, st));
  HIPCHK(g, hipMemcpyAsync(g->hm_out.p, a.out, 4 * n, hipMemcpyDeviceToHost, st));
  HIPCHK(g, hipMemcpyAsync(hcap, g->m_cap.p, 16 * G + 8, hipMemcpyDeviceToHost, st));
  if (prof.on) HIPCHK(g, hipEventRecord(prof.end, st));
  HIPCHK(g, hipStreamSynchronize(st));
  prof.done(sizeof(mbft_msg_rec) * n + up);
  const auto t2 = std::chrono::steady_clock::now();
  const int T = n >= 4096 ? g->pool->size() : 1;
  const int32_t* hout = g->hm_out.as<int32_t>();
  g->pool->run(T, [&](int t) {
    const size_t lo = n * t / T, hi = n * (t + 1) / T;
    memcpy(out + lo, hout + lo, 4 * (hi - lo));
  });
  // commit the captures made before message f (exact: every check before f
  // ran); the sequential replay from f (adversarial batches only) sees the
  // state as it was there
  const size_t f = (size_t)hcap[2 * G];
  for (size_t g = 0; g < G; g++)
    if (hcap[g] < 3 * (uint64_t)f) {
      c->epoch_val[g] = hcap[G + g];
      c->epoch_set[g] = 1;
    }
  if (f < n) {
    HIPCHK(g, g->hm_pack.ensure(L.end));
    HIPCHK(g, hipMemcpyAsync(g->hm_pack.as<uint8_t>() + L.chk, pk + L.chk, L.through(nc) - L.chk,
                             hipMemcpyDeviceToHost, st));
    HIPCHK(g, hipStreamSynchronize(st));
    const uint8_t* hp = g->hm_pack.as<uint8_t>();
    // checks of messages f.. from the packed words
    static thread_local std::vector<MsgChecks> tl_checks;
    std::vector<MsgChecks>& checks = tl_checks;
    checks.resize(n);
    unpack_checks(g, f, n, reinterpret_cast<const uint32_t*>(hp + L.chk),
                  reinterpret_cast<const uint32_t*>(hp + L.callof), checks.data());
    const CallInfo* info = reinterpret_cast<const CallInfo*>(hp + L.info);
    const uint8_t* role_bytes = hp + L.info + offsetof(mbft::DevCallInfo, role);
    replay_tail(
        c, f, n, checks.data(), info, hp + L.status, flags, out,
        [&](size_t i) { return recs[i].stream; },
        [&](uint32_t k) { return (uint32_t)role_bytes[sizeof(CallInfo) * k]; });
  }
  static const bool trace = getenv("MBFT_STAGE_TRACE") != nullptr;
  if (trace)
    fprintf(stderr,
            "[mbft validate flat dev] n=%zu calls=%zu bytes=%zu up+cands+dedup=%.3f "
            "calls+verify+replay+down=%.3f host tail=%.3f ms (first non-zero result %zu)\n",
            n, nc, nbytes, std::chrono::duration<double, std::milli>(t1 - t0).count(),
            std::chrono::duration<double, std::milli>(t2 - t1).count(), ms_since(t2), f);
  return MBFT_OK;
}

// Every return after the first enqueue -- a failed launch or copy, a stage-1
// verify failure, an argument error found by the kernels -- may leave kernels
// and copies running on st, cs or vb over m_recs, m_bytes and the dedup
// table, which the next call overwrites from its copy stream without waiting
// on st: drain all three streams before returning an error.
int validate_flat_device(mbft_ctx* c, mbft_ctx* g, const mbft_msg_rec* recs, size_t n,
                         const uint8_t* bytes, size_t nbytes, uint32_t n_replicas, uint32_t flags,
                         int32_t* out, mbft_msg_batch* chk, size_t base = 0) {
  const int rc = validate_flat_device_impl(c, g, recs, n, bytes, nbytes, n_replicas, flags, out, chk, base);
  if (rc != MBFT_OK) {
    (void)hipStreamSynchronize(g->cstream);
    (void)hipStreamSynchronize(g->stream);
    (void)hipStreamSynchronize(g->vstream[0]);
    if (g != c && !g->err.empty()) c->err = g->err;
  }
  return rc;
}

bool field_ok(uint64_t off, uint32_t len, size_t nbytes) {
  return len == 0 || (off <= nbytes && (uint64_t)len <= nbytes - off);
}

// Records -> mbft_message structs over the arena, with k_msg_cands' argument
// checks: 1 = a type out of range (Go: panic("Unknown message type")), 2 = a
// field outside the arena (either way MBFT_ERR_ARG, as on the device);
// 0 = ok.
int recs_to_messages(const mbft_msg_rec* recs, size_t n, const uint8_t* bytes, size_t nbytes,
                     mbft_message* msgs) {
  int bad = 0;
  for (size_t i = 0; i < n; i++) {
    const mbft_msg_rec& r = recs[i];
    if (r.type < MBFT_MSG_REQUEST || r.type > MBFT_MSG_REQ_VIEW_CHANGE) bad |= 1;
    if (!field_ok(r.op_off, r.op_len, nbytes) || !field_ok(r.sig_off, r.sig_len, nbytes) ||
        !field_ok(r.ui_cert_off, r.ui_cert_len, nbytes) ||
        !field_ok(r.prep_ui_cert_off, r.prep_ui_cert_len, nbytes))
      bad |= 2;
    if (bad) continue;
    mbft_message& m = msgs[i];
    m.type = r.type;
    m.stream = r.stream;
    m.replica_id = r.replica_id;
    m.prep_replica_id = r.prep_replica_id;
    m.view = r.view;
    m.client_id = r.client_id;
    m.reserved = 0;
    m.seq = r.seq;
    m.op = bytes + r.op_off;
    m.op_len = r.op_len;
    m.sig = bytes + r.sig_off;
    m.sig_len = r.sig_len;
    m.ui_counter = r.ui_counter;
    m.ui_cert = bytes + r.ui_cert_off;
    m.ui_cert_len = r.ui_cert_len;
    m.prep_ui_counter = r.prep_ui_counter;
    m.prep_ui_cert = bytes + r.prep_ui_cert_off;
    m.prep_ui_cert_len = r.prep_ui_cert_len;
  }
  return bad & 1 ? 1 : bad;
}

int small_arg_error(mbft_ctx* c, int why) {
  return fail(c, MBFT_ERR_ARG, why == 1 ? "mbft_check_messages_flat: unknown message type"
                                        : "mbft_check_messages_flat: field outside the byte arena");
}

// The small route (mbft_set_small_check): messages over any host memory,
// checked on engine g by check_messages_small (messages.cpp) -- no device
// message layer, one verify launch.
int check_small(mbft_ctx* c, mbft_ctx* g, const mbft_message* msgs, size_t n, uint32_t n_replicas,
                mbft_msg_batch* chk);

}  // namespace

namespace {

int check_small(mbft_ctx* c, mbft_ctx* g, const mbft_message* msgs, size_t n, uint32_t n_replicas,
                mbft_msg_batch* chk) {
  const auto t0 = std::chrono::steady_clock::now();
  auto calls = std::make_shared<MsgCalls>();
  chk->n = n;
  chk->checks.resize(n);
  const int rc = check_messages_small(c, g, msgs, n, n_replicas, chk->checks.data(), calls->info, calls->gst,
                                      calls->role);
  if (rc) return rc;
  chk->calls = std::move(calls);
  static const bool trace = getenv("MBFT_STAGE_TRACE") != nullptr;
  if (trace)
    fprintf(stderr, "[mbft check small] n=%zu calls=%zu %.3f ms\n", n, chk->calls->gst.size(), ms_since(t0));
  return MBFT_OK;
}


// [lo, hi) of the arena bytes the fields of records r[0 .. m) reference (lo
// 8-aligned), with k_msg_cands' argument checks: returns 1 for a type out of
// range, 2 for a field outside [0, nbytes), else 0.
int shard_range(const mbft_msg_rec* r, size_t m, size_t nbytes, size_t* lo, size_t* hi) {
  size_t a = nbytes, b = 0;
  int bad = 0;
  auto f = [&](uint64_t off, uint32_t len) {
    if (len == 0) return;
    if (!field_ok(off, len, nbytes)) {
      bad |= 2;
      return;
    }
    a = std::min<size_t>(a, (size_t)off);
    b = std::max<size_t>(b, (size_t)(off + len));
  };
  for (size_t i = 0; i < m; i++) {
    if (r[i].type < MBFT_MSG_REQUEST || r[i].type > MBFT_MSG_REQ_VIEW_CHANGE) bad |= 1;
    f(r[i].op_off, r[i].op_len);
    f(r[i].sig_off, r[i].sig_len);
    f(r[i].ui_cert_off, r[i].ui_cert_len);
    f(r[i].prep_ui_cert_off, r[i].prep_ui_cert_len);
  }
  if (b < a) a = b = 0;  // no field bytes at all
  *lo = a & ~(size_t)7;
  *hi = b;
  return bad & 1 ? 1 : bad;
}

// The engines a device pass is split over (mbft_ctx_add_device): g0 -- the
// leased lane, or the context -- then one per other table engine: the peer
// engines, with the context itself instead of the peer whose lane g0 is.
std::vector<mbft_ctx*> shard_engines(mbft_ctx* c, mbft_ctx* g0) {
  std::vector<mbft_ctx*> e{g0};
  const mbft_ctx* own = tabs(g0);
  for (mbft_ctx* p : c->peers) e.push_back(p == own ? c : p);
  return e;
}

// A device pass of n messages (library page-locked records and arena) over
// k > 1 engines: contiguous record shards, each with only the arena bytes its
// records reference, checked on the engines' devices at once (one host
// thread each: engine 0 on this one, the others under their own mutex --
// the context's is not taken again when the caller holds it, c_held); the
// shards' checks and call outcomes concatenated in message order (call
// numbers offset).  Identical calls in different shards are verified once
// per shard.  No state read or written: the check form; validate_sharded
// replays it.
int check_sharded(mbft_ctx* c, const std::vector<mbft_ctx*>& eng, size_t k, const mbft_msg_rec* recs, size_t n,
                  const uint8_t* bytes, size_t nbytes, uint32_t n_replicas, mbft_msg_batch* out, bool c_held) {
  std::vector<size_t> lo(k), hi(k), blo(k), bhi(k);
  std::vector<int> why(k, 0), rcs(k, MBFT_OK);
  for (size_t j = 0; j < k; j++) {
    lo[j] = n * j / k;
    hi[j] = n * (j + 1) / k;
  }
  // shards 1 .. k-1 on their engines' persistent threads, shard 0 here (no
  // thread start per pass)
  std::vector<uint64_t> tickets(k, 0);
  for (size_t j = 1; j < k; j++)
    tickets[j] = engine_worker(eng[j]).submit(
        [&, j] { why[j] = shard_range(recs + lo[j], hi[j] - lo[j], nbytes, &blo[j], &bhi[j]); });
  why[0] = shard_range(recs, hi[0], nbytes, &blo[0], &bhi[0]);
  for (size_t j = 1; j < k; j++) engine_worker(eng[j]).wait(tickets[j]);
  int w = 0;
  for (int x : why) w |= x;
  if (w) return fail(c, MBFT_ERR_ARG, w & 1 ? "mbft_check_messages_flat: unknown message type"
                                            : "mbft_check_messages_flat: field outside the byte arena");
  std::vector<mbft_msg_batch> part(k);
  auto run = [&](size_t j) {
    mbft_ctx* g = eng[j];
    std::unique_lock<std::mutex> lk(g->mu, std::defer_lock);
    if (j != 0 && !(g == c && c_held)) lk.lock();  // shard 0: the caller holds its engine
    if (hipSetDevice(g->device) != hipSuccess) {
      rcs[j] = MBFT_ERR_HIP;
      return;
    }
    part[j].c = c;
    rcs[j] = validate_flat_device(c, g, recs + lo[j], hi[j] - lo[j], bytes, bhi[j], n_replicas, 0, nullptr,
                                  &part[j], blo[j]);
  };
  for (size_t j = 1; j < k; j++) tickets[j] = engine_worker(eng[j]).submit([&run, j] { run(j); });
  run(0);
  for (size_t j = 1; j < k; j++) engine_worker(eng[j]).wait(tickets[j]);
  (void)hipSetDevice(eng[0]->device);
  for (size_t j = 0; j < k; j++)
    if (rcs[j]) return eng[j] == c ? rcs[j] : fail(c, rcs[j], std::string("engine: ") + eng[j]->err);
  auto calls = std::make_shared<MsgCalls>();
  out->n = n;
  out->checks.resize(n);
  uint32_t off = 0;
  for (size_t j = 0; j < k; j++) {
    const MsgCalls& pc = *part[j].calls;
    calls->info.insert(calls->info.end(), pc.info.begin(), pc.info.end());
    calls->gst.insert(calls->gst.end(), pc.gst.begin(), pc.gst.end());
    calls->role.insert(calls->role.end(), pc.role.begin(), pc.role.end());
    for (size_t i = 0; i < part[j].n; i++) {
      MsgChecks ck = part[j].checks[i];
      for (int q = 0; q < ck.n; q++)
        if (ck.c[q].kind == 0) ck.c[q].call += off;
      out->checks[lo[j] + i] = ck;
    }
    off += (uint32_t)pc.gst.size();
  }
  out->calls = std::move(calls);
  return MBFT_OK;
}

// How many engines a device pass of n messages is split over: one per table
// engine, each shard at least shard_min messages (mbft_set_shard_min, the
// call-level batches' rule).
size_t shard_count(const mbft_ctx* c, size_t n) {
  const size_t engines = 1 + c->peers.size();
  if (engines == 1) return 1;
  const size_t k = c->shard_min ? n / c->shard_min : engines;
  return k < engines ? (k < 1 ? 1 : k) : engines;
}
}  // namespace

extern "C" int mbft_set_small_check(mbft_ctx* c, size_t max_messages) {
  if (!c) return MBFT_ERR_ARG;
  c->msg_small_max.store(max_messages);
  return MBFT_OK;
}

extern "C" int mbft_pack_messages(const mbft_message* msgs, size_t n, mbft_msg_rec* recs,
                                  uint8_t* bytes, size_t cap, size_t* used) {
  if (!used || (n && !msgs)) return MBFT_ERR_ARG;
  size_t need = 0;
  for (size_t i = 0; i < n; i++) {
    const mbft_message& m = msgs[i];
    if (m.op_len > 0xFFFFFFFFull || m.sig_len > 0xFFFFFFFFull || m.ui_cert_len > 0xFFFFFFFFull ||
        m.prep_ui_cert_len > 0xFFFFFFFFull)
      return MBFT_ERR_ARG;
    need += m.op_len + m.sig_len + m.ui_cert_len + m.prep_ui_cert_len;
  }
  *used = need;
  if (!recs) return MBFT_OK;  // size query
  if (need > cap || (need && !bytes)) return MBFT_ERR_ARG;
  size_t pos = 0;
  auto put = [&](const uint8_t* p, size_t len, uint64_t& off, uint32_t& l) {
    off = pos;
    l = (uint32_t)len;
    if (len) memcpy(bytes + pos, p, len);
    pos += len;
  };
  for (size_t i = 0; i < n; i++) {
    const mbft_message& m = msgs[i];
    mbft_msg_rec& r = recs[i];
    r.type = m.type;
    r.stream = m.stream;
    r.replica_id = m.replica_id;
    r.prep_replica_id = m.prep_replica_id;
    r.client_id = m.client_id;
    r.reserved = 0;
    r.view = m.view;
    r.seq = m.seq;
    r.ui_counter = m.ui_counter;
    r.prep_ui_counter = m.prep_ui_counter;
    put(m.op, m.op_len, r.op_off, r.op_len);
    put(m.sig, m.sig_len, r.sig_off, r.sig_len);
    put(m.ui_cert, m.ui_cert_len, r.ui_cert_off, r.ui_cert_len);
    put(m.prep_ui_cert, m.prep_ui_cert_len, r.prep_ui_cert_off, r.prep_ui_cert_len);
  }
  return MBFT_OK;
}

extern "C" int mbft_validate_replies_flat(mbft_ctx* c, const mbft_msg_rec* recs, size_t n, const uint8_t* bytes,
                                          size_t nbytes, uint32_t client_id, uint32_t flags, int32_t* out) {
  if (!c || (n && (!recs || !out)) || (nbytes && !bytes)) return MBFT_ERR_ARG;
  std::vector<mbft_message> msgs(n);
  if (recs_to_messages(recs, n, bytes, nbytes, msgs.data()))
    return fail(c, MBFT_ERR_ARG, "mbft_validate_replies_flat: unknown message type or field outside the arena");
  return mbft_validate_replies(c, msgs.data(), n, client_id, flags, out);
}

extern "C" int mbft_validate_messages_flat(mbft_ctx* c, const mbft_msg_rec* recs, size_t n,
                                           const uint8_t* bytes, size_t nbytes, uint32_t n_replicas,
                                           uint32_t flags, int32_t* out) {
  if (!c || (n && (!recs || !out)) || n_replicas == 0 || (nbytes && !bytes)) return MBFT_ERR_ARG;
  if (n == 0) return MBFT_OK;
  // the device path numbers candidates (3 per message) in 32-bit words and
  // scans them with int counts: batches past 2^28 messages take the host layer
  constexpr size_t kMaxDevMessages = (size_t)1 << 28;
  const bool dev = c->dev_prepare != 0 && !c->slots.empty() && n <= kMaxDevMessages &&
                   host_owned(recs, sizeof(mbft_msg_rec) * n) && host_owned(bytes, nbytes);
  if (dev) {
    // the engine: a lane on the least busy device when there are lanes
    // (mbft_ctx_add_device gives every device its own), else the context;
    // the epoch state held for the whole call (the in-order replay writes it)
    std::unique_ptr<Lease> ls;
    if (c->concurrency > 1) ls.reset(new Lease(c, /*any_device=*/true));
    std::lock_guard<std::mutex> lk(c->mu);
    mbft_ctx* g = ls ? ls->g : c;
    if (hipSetDevice(g->device) != hipSuccess) return MBFT_ERR_HIP;
    sync_host_keymap(c);
    const size_t k = shard_count(c, n);
    if (k <= 1) return validate_flat_device(c, g, recs, n, bytes, nbytes, n_replicas, flags, out, nullptr);
    // record shards over every table engine (check form), then the in-order
    // replay of the whole batch on the host
    mbft_msg_batch b;
    b.c = c;
    const int rc = check_sharded(c, shard_engines(c, g), k, recs, n, bytes, nbytes, n_replicas, &b, /*c_held=*/true);
    if (rc) return rc;
    const MsgCalls& mc = *b.calls;
    return replay_messages(c, n, b.checks.data(), mc.info.data(), mc.gst.data(), flags, out,
                           [&](size_t i) { return recs[i].stream; }, [&](uint32_t q) { return (uint32_t)mc.role[q]; });
  }
  // host message layer over structs that point into the arena
  std::vector<mbft_message> msgs(n);
  for (size_t i = 0; i < n; i++) {
    const mbft_msg_rec& r = recs[i];
    if (!field_ok(r.op_off, r.op_len, nbytes) || !field_ok(r.sig_off, r.sig_len, nbytes) ||
        !field_ok(r.ui_cert_off, r.ui_cert_len, nbytes) ||
        !field_ok(r.prep_ui_cert_off, r.prep_ui_cert_len, nbytes))
      return MBFT_ERR_ARG;
    mbft_message& m = msgs[i];
    m.type = r.type;
    m.stream = r.stream;
    m.replica_id = r.replica_id;
    m.prep_replica_id = r.prep_replica_id;
    m.view = r.view;
    m.client_id = r.client_id;
    m.reserved = 0;
    m.seq = r.seq;
    m.op = bytes + r.op_off;
    m.op_len = r.op_len;
    m.sig = bytes + r.sig_off;
    m.sig_len = r.sig_len;
    m.ui_counter = r.ui_counter;
    m.ui_cert = bytes + r.ui_cert_off;
    m.ui_cert_len = r.ui_cert_len;
    m.prep_ui_counter = r.prep_ui_counter;
    m.prep_ui_cert = bytes + r.prep_ui_cert_off;
    m.prep_ui_cert_len = r.prep_ui_cert_len;
  }
  return mbft_validate_messages(c, msgs.data(), n, n_replicas, flags, out);
}

// One caller's batch in the check coalescer (mbft_set_check_coalescing).
struct mbft_check_req {
  const mbft_msg_rec* recs;
  size_t n;
  const uint8_t* bytes;
  size_t nbytes;
  uint32_t n_replicas;
  mbft_msg_batch* out = nullptr;
  int rc = MBFT_OK;
  bool done = false, lead = false;
};

namespace {

// What k_msg_cands rejects with MBFT_ERR_ARG (an unknown message type, a
// field outside the arena), checked per caller before its batch joins a
// coalesced pass, so one caller's bad batch fails that caller alone.
bool records_ok(const mbft_check_req& r) {
  auto in = [&](uint64_t off, uint32_t len) { return len == 0 || (off <= r.nbytes && len <= r.nbytes - off); };
  for (size_t i = 0; i < r.n; i++) {
    const mbft_msg_rec& m = r.recs[i];
    if (m.type < MBFT_MSG_REQUEST || m.type > MBFT_MSG_REQ_VIEW_CHANGE) return false;
    if (!in(m.op_off, m.op_len) || !in(m.sig_off, m.sig_len) || !in(m.ui_cert_off, m.ui_cert_len) ||
        !in(m.prep_ui_cert_off, m.prep_ui_cert_len))
      return false;
  }
  return true;
}

// One device pass over the requests rs (same n_replicas) on lane g: their
// records and arenas concatenated into g's page-locked staging (the offsets
// rebased to the merged arena), checked together, and the merged batch's
// checks handed out per request, every request sharing the pass's calls.
// A request whose records fail records_ok gets MBFT_ERR_ARG and is left out.
void check_merged(mbft_ctx* c, mbft_ctx* g, const std::vector<mbft_check_req*>& rs, Pool* pool) {
  const auto t0 = std::chrono::steady_clock::now();
  if (!g->pool) g->pool.reset(new Pool(pool_workers(g)));
  const size_t R = rs.size();
  std::vector<char> ok(R, 1);
  size_t total = 0;
  for (const mbft_check_req* r : rs) total += r->n;
  // a small pass checks its few records on this thread (no pool wake-ups)
  const int Tr = total <= c->msg_small_max.load() ? 1 : (int)std::min<size_t>(R, (size_t)g->pool->size());
  g->pool->run(Tr, [&](int t) {
    for (size_t j = (size_t)t; j < R; j += (size_t)Tr) ok[j] = records_ok(*rs[j]) ? 1 : 0;
  });
  std::vector<size_t> mbase(R + 1, 0), bbase(R + 1, 0);
  for (size_t j = 0; j < R; j++) {
    if (!ok[j]) {
      rs[j]->rc = fail(c, MBFT_ERR_ARG, "mbft_check_messages_flat: unknown message type or field outside the arena");
      mbase[j + 1] = mbase[j];
      bbase[j + 1] = bbase[j];
      continue;
    }
    mbase[j + 1] = mbase[j] + rs[j]->n;
    bbase[j + 1] = (bbase[j] + rs[j]->nbytes + 7) & ~(size_t)7;
  }
  const size_t N = mbase[R], NB = bbase[R];
  auto fail_all = [&](int rc) {
    for (size_t j = 0; j < R; j++)
      if (ok[j]) rs[j]->rc = rc;
  };
  if (N == 0) {
    for (size_t j = 0; j < R; j++)
      if (ok[j]) {
        rs[j]->out = new mbft_msg_batch;
        rs[j]->out->c = c;
      }
    return;
  }
  if (N <= c->msg_small_max.load()) {
    // a small pass: the callers' records as messages over their own arenas
    // (no staging copy), checked together on the calling thread
    std::vector<mbft_message> msgs(N);
    for (size_t j = 0; j < R; j++)
      if (ok[j]) (void)recs_to_messages(rs[j]->recs, rs[j]->n, rs[j]->bytes, rs[j]->nbytes, msgs.data() + mbase[j]);
    mbft_msg_batch merged;
    merged.c = c;
    const int rc = check_small(c, g, msgs.data(), N, rs[0]->n_replicas, &merged);
    if (rc) {
      fail_all(rc);
      return;
    }
    for (size_t j = 0; j < R; j++) {
      if (!ok[j]) continue;
      mbft_msg_batch* b = new mbft_msg_batch;
      b->c = c;
      b->n = rs[j]->n;
      b->checks.assign(merged.checks.begin() + mbase[j], merged.checks.begin() + mbase[j + 1]);
      b->calls = merged.calls;
      rs[j]->out = b;
    }
    auto& co = c->cco;
    std::lock_guard<std::mutex> lk(co.m);
    co.passes += 1;
    co.requests += (double)R;
    co.messages += (double)N;
    return;
  }
  if (g->hm_recs.ensure(sizeof(mbft_msg_rec) * N) != hipSuccess || g->hm_bytes.ensure(NB + 8) != hipSuccess) {
    fail_all(hip_fail(c, hipErrorOutOfMemory, "mbft_check_messages_flat: coalesced staging"));
    return;
  }
  mbft_msg_rec* recs = g->hm_recs.as<mbft_msg_rec>();
  uint8_t* bytes = g->hm_bytes.as<uint8_t>();
  const int T = pool->size();
  pool->run(T, [&](int t) {
    for (size_t j = 0; j < R; j++) {
      if (!ok[j]) continue;
      const mbft_check_req& r = *rs[j];
      const size_t m0 = r.n * (size_t)t / (size_t)T, m1 = r.n * (size_t)(t + 1) / (size_t)T;
      const uint64_t b = bbase[j];
      for (size_t i = m0; i < m1; i++) {
        mbft_msg_rec m = r.recs[i];
        m.op_off += b;
        m.sig_off += b;
        m.ui_cert_off += b;
        m.prep_ui_cert_off += b;
        recs[mbase[j] + i] = m;
      }
      const size_t b0 = r.nbytes * (size_t)t / (size_t)T, b1 = r.nbytes * (size_t)(t + 1) / (size_t)T;
      if (b1 > b0) memcpy(bytes + bbase[j] + b0, r.bytes + b0, b1 - b0);
    }
  });
  mbft_msg_batch merged;
  merged.c = c;
  const double t_stage = ms_since(t0);
  const size_t k = shard_count(c, N);
  const int rc = k > 1 ? check_sharded(c, shard_engines(c, g), k, recs, N, bytes, NB, rs[0]->n_replicas, &merged,
                                       /*c_held=*/g == c)
                       : validate_flat_device(c, g, recs, N, bytes, NB, rs[0]->n_replicas, 0, nullptr, &merged);
  const double t_dev = ms_since(t0) - t_stage;
  if (rc) {
    fail_all(rc);
    return;
  }
  for (size_t j = 0; j < R; j++) {
    if (!ok[j]) continue;
    mbft_msg_batch* b = new mbft_msg_batch;
    b->c = c;
    b->n = rs[j]->n;
    b->checks.assign(merged.checks.begin() + mbase[j], merged.checks.begin() + mbase[j + 1]);
    b->calls = merged.calls;
    rs[j]->out = b;
  }
  static const bool trace = getenv("MBFT_STAGE_TRACE") != nullptr;
  if (trace)
    fprintf(stderr, "[mbft check pass] batches=%zu messages=%zu bytes=%zu stage=%.3f device=%.3f split=%.3f ms\n",
            R, N, NB, t_stage, t_dev, ms_since(t0) - t_stage - t_dev);
  auto& co = c->cco;
  std::lock_guard<std::mutex> lk(co.m);
  co.passes += 1;
  co.requests += (double)R;
  co.messages += (double)N;
}

// The coalesced form of mbft_check_messages_flat: queue; lead if no other
// caller is collecting (wait up to max_wait_us for company, then for a
// lane), take every queued request with the leader's n_replicas (up to
// max_messages), run them as one pass, wake them.  Requests left behind
// (another n_replicas, or past the cap) get a new leader at once.
int check_coalesced(mbft_ctx* c, mbft_check_req& me) {
  auto& co = c->cco;
  std::unique_lock<std::mutex> lk(co.m);
  co.q.push_back(&me);
  if (co.collecting) {
    // a leader is collecting: it takes this request, or hands this caller
    // the lead (collecting stays set for it) for what it left behind
    co.cv.wait(lk, [&] { return me.done || me.lead; });
    if (me.done) return me.rc;
  } else {
    co.collecting = true;  // this caller leads the next pass
  }
  me.lead = false;
  if (co.max_wait_us) {
    const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(co.max_wait_us);
    co.cv.wait_until(lk, until, [&] { return false; });
  }
  // At most max_passes coalesced passes at once (env MBFT_CHECK_PASSES,
  // default 2), whatever the lane count: more concurrent passes make each
  // merge smaller and their streams share the hardware queues (C3 Go wiring:
  // 24.4 M messages/s on 2 lanes against 20.2 M on 4,
  // profiles/round4_msg_pass_ab.txt).  The queue fills meanwhile.
  static const int max_passes = [] {
    const char* v = getenv("MBFT_CHECK_PASSES");
    return v && atoi(v) > 0 ? atoi(v) : 2;
  }();
  co.cv.wait(lk, [&] { return co.running < max_passes; });
  co.running++;
  if (co.pools.empty()) {
    const int share = host_pool_threads() / max_passes > 2 ? host_pool_threads() / max_passes : 2;
    for (int k = 0; k < max_passes; k++) co.pools.emplace_back(new Pool(share - 1));
    co.pool_busy.assign((size_t)max_passes, 0);
  }
  size_t slot = 0;
  while (co.pool_busy[slot]) slot++;  // running < max_passes: one is free
  co.pool_busy[slot] = 1;
  Pool* pool = co.pools[slot].get();
  lk.unlock();
  Lease ls(c, /*any_device=*/true);  // waits while every lane runs a pass: the queue fills meanwhile
  lk.lock();
  std::vector<mbft_check_req*> take, rest;
  size_t msgs = 0;
  for (mbft_check_req* r : co.q) {
    const bool fits = r == &me || (r->n_replicas == me.n_replicas && msgs + r->n <= co.max_messages);
    if (fits) {
      take.push_back(r);
      msgs += r->n;
    } else {
      rest.push_back(r);
    }
  }
  co.q.swap(rest);
  co.collecting = false;
  if (!co.q.empty()) {  // a new leader for the rest (it waits for its own lane)
    co.q.front()->lead = true;
    co.collecting = true;
    co.cv.notify_all();
  }
  lk.unlock();
  mbft_ctx* g = ls.g;
  if (hipSetDevice(g->device) != hipSuccess) {
    for (mbft_check_req* r : take) r->rc = MBFT_ERR_HIP;
  } else {
    if (g == c) sync_host_keymap(c);
    check_merged(c, g, take, pool);
  }
  lk.lock();
  for (mbft_check_req* r : take) r->done = true;
  co.running--;
  co.pool_busy[slot] = 0;
  co.cv.notify_all();
  co.cv.wait(lk, [&] { return me.done; });  // (always in `take`: the sole collector)
  return me.rc;
}

}  // namespace

extern "C" int mbft_set_check_coalescing(mbft_ctx* c, int enabled, uint32_t max_wait_us, size_t max_messages) {
  if (!c) return MBFT_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->cco.m);
  c->cco.max_wait_us = max_wait_us;
  c->cco.max_messages = max_messages ? max_messages : ((size_t)1 << 20);
  c->cco.enabled = enabled != 0;
  return MBFT_OK;
}

extern "C" int mbft_check_coalescing_stats(mbft_ctx* c, double out[3]) {
  if (!c || !out) return MBFT_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->cco.m);
  out[0] = c->cco.passes;
  out[1] = c->cco.requests;
  out[2] = c->cco.messages;
  c->cco.passes = c->cco.requests = c->cco.messages = 0;
  return MBFT_OK;
}

extern "C" int mbft_check_messages_flat(mbft_ctx* c, const mbft_msg_rec* recs, size_t n,
                                        const uint8_t* bytes, size_t nbytes, uint32_t n_replicas,
                                        mbft_msg_batch** out) {
  if (!c || !out || (n && !recs) || n_replicas == 0 || (nbytes && !bytes)) return MBFT_ERR_ARG;
  *out = nullptr;
  constexpr size_t kMaxDevMessages = (size_t)1 << 28;
  if (n > kMaxDevMessages) return fail(c, MBFT_ERR_ARG, "mbft_check_messages_flat: more than 2^28 messages");
  if (n && c->cco.enabled.load()) {
    {
      std::shared_lock<std::shared_mutex> tl(c->tab_mu);
      if (c->slots.empty()) return fail(c, MBFT_ERR_STATE, "mbft_check_messages_flat: no keys registered");
    }
    mbft_check_req me{recs, n, bytes, nbytes, n_replicas};
    const int rc = check_coalesced(c, me);
    if (rc) {
      delete me.out;
      return rc;
    }
    *out = me.out;
    return MBFT_OK;
  }
  std::unique_ptr<mbft_msg_batch> b(new mbft_msg_batch);
  b->c = c;
  if (n == 0) {
    *out = b.release();
    return MBFT_OK;
  }
  Lease ls(c, /*any_device=*/true);
  if (hipSetDevice(ls.g->device) != hipSuccess) return MBFT_ERR_HIP;
  if (c->slots.empty()) {
    // no key yet: every check is decided without a signature (a role or key
    // lookup fails first); the host message layer's check part gives them
    return fail(c, MBFT_ERR_STATE, "mbft_check_messages_flat: no keys registered");
  }
  mbft_ctx* g = ls.g;
  if (g == c) sync_host_keymap(c);
  if (n <= c->msg_small_max.load()) {
    std::vector<mbft_message> msgs(n);
    const int why = recs_to_messages(recs, n, bytes, nbytes, msgs.data());
    if (why) return small_arg_error(c, why);
    const int rc = check_small(c, g, msgs.data(), n, n_replicas, b.get());
    if (rc) return rc;
    *out = b.release();
    return MBFT_OK;
  }
  // records and arena outside library page-locked memory are staged into the
  // engine's own (the DMA engines read only page-locked memory)
  if (!host_owned(recs, sizeof(mbft_msg_rec) * n)) {
    HIPCHK(c, g->hm_recs.ensure(sizeof(mbft_msg_rec) * n));
    memcpy(g->hm_recs.p, recs, sizeof(mbft_msg_rec) * n);
    recs = g->hm_recs.as<mbft_msg_rec>();
  }
  if (nbytes && !host_owned(bytes, nbytes)) {
    HIPCHK(c, g->hm_bytes.ensure(nbytes));
    memcpy(g->hm_bytes.p, bytes, nbytes);
    bytes = g->hm_bytes.as<uint8_t>();
  }
  const size_t k = shard_count(c, n);
  const int rc = k > 1 ? check_sharded(c, shard_engines(c, g), k, recs, n, bytes, nbytes, n_replicas, b.get(),
                                       /*c_held=*/g == c)
                       : validate_flat_device(c, g, recs, n, bytes, nbytes, n_replicas, 0, nullptr, b.get());
  if (rc) return rc;
  *out = b.release();
  return MBFT_OK;
}

namespace {

// Message i's result with the USIG epoch step applied now (caller holds
// c->mu): the validator's checks in order, the first failing one decides.
int32_t resolve_one(mbft_ctx* c, const mbft_msg_batch* b, size_t i) {
  const MsgChecks& ck = b->checks[i];
  for (int q = 0; q < ck.n; q++) {
    const Check& k = ck.c[q];
    if (k.kind == 1 || k.kind == 3) return k.stage << 8;
    if (k.kind == 2) return (k.stage << 8) | MBFT_ZERO_COUNTER;
    const uint8_t st = resolve_call(c, b->calls->info[k.call], b->calls->gst[k.call]);
    if (st != MBFT_ACCEPT) return (k.stage << 8) | st;
  }
  return 0;
}

}  // namespace

extern "C" int mbft_resolve_message(mbft_ctx* c, mbft_msg_batch* b, size_t i) {
  if (!c || !b || b->c != c || i >= b->n) return MBFT_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);  // the USIG epoch state
  return resolve_one(c, b, i);
}

extern "C" int mbft_resolve_messages(mbft_ctx* c, mbft_msg_batch* b, size_t i0, size_t count,
                                     int32_t* out) {
  if (!c || !b || b->c != c || i0 > b->n || count > b->n - i0 || (count && !out)) return MBFT_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  for (size_t k = 0; k < count; k++) out[k] = resolve_one(c, b, i0 + k);
  return MBFT_OK;
}

extern "C" void mbft_msg_batch_free(mbft_msg_batch* b) { delete b; }

extern "C" int mbft_profile_msg_layer(mbft_ctx* c, double out[4]) {
  if (!c || !out) return MBFT_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  for (int k = 0; k < 4; k++) out[k] = c->prof_msg[k];
  for (const std::vector<mbft_ctx*>* v : {&c->lanes, &c->peers})
    for (mbft_ctx* l : *v)
      for (int k = 0; k < 4; k++) {
        out[k] += l->prof_msg[k];
        l->prof_msg[k] = 0;
      }
  for (int k = 0; k < 4; k++) c->prof_msg[k] = 0;
  return MBFT_OK;
}

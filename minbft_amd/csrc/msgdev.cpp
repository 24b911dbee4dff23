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

// The device path (caller holds c->mu; recs and bytes are library-owned
// page-locked memory, n > 0).  Error returns may leave work queued on any of
// the three streams: validate_flat_device drains them.
int validate_flat_device_impl(mbft_ctx* c, const mbft_msg_rec* recs, size_t n, const uint8_t* bytes,
                         size_t nbytes, uint32_t n_replicas, uint32_t flags, int32_t* out) {
  const auto t0 = std::chrono::steady_clock::now();
  if (!c->pool) c->pool.reset(new Pool(host_pool_threads() - 1));
  sync_host_keymap(c);
  int rc = sync_keymap(c, c);
  if (rc) return rc;
  const size_t nc3 = 3 * n;
  size_t cap = 1024;
  while (cap < 2 * nc3) cap <<= 1;
  HIPCHK(c, c->m_recs.ensure(sizeof(mbft_msg_rec) * n));
  HIPCHK(c, c->m_bytes.ensure(((nbytes + 3) & ~(size_t)3) + 32));
  HIPCHK(c, c->m_chk.ensure(4 * n));
  HIPCHK(c, c->m_flag.ensure(64));
  HIPCHK(c, c->m_cand.ensure(sizeof(mbft::MsgCand) * nc3));
  HIPCHK(c, c->m_chash.ensure(8 * nc3));
  HIPCHK(c, c->m_cslot.ensure(4 * nc3));
  HIPCHK(c, c->m_uniq.ensure(4 * nc3));
  HIPCHK(c, c->m_ref.ensure(4 * nc3));
  HIPCHK(c, c->m_idx.ensure(4 * nc3));
  HIPCHK(c, c->m_callof.ensure(4 * nc3));
  HIPCHK(c, c->m_candof.ensure(4 * nc3));
  HIPCHK(c, c->m_tkeys.ensure(8 * cap));
  HIPCHK(c, c->m_treps.ensure(4 * cap));
  const mbft_ctx* tb = tabs(c);
  std::vector<uint32_t> fpg(tb->slots.size() + 1, 0);
  for (size_t k = 0; k < tb->slots.size(); k++) fpg[k] = tb->slots[k].fp_group;
  HIPCHK(c, c->m_fpg.ensure(4 * fpg.size()));
  HIPCHK(c, c->hm_small.ensure(64));

  mbft::MsgDevArgs a{};
  a.recs = c->m_recs.as<mbft_msg_rec>();
  a.bytes = c->m_bytes.as<uint8_t>();
  a.nbytes = nbytes;
  a.n = (long)n;
  a.n_replicas = n_replicas;
  a.chk = c->m_chk.as<uint32_t>();
  a.bad = c->m_flag.as<uint32_t>();
  a.cand = c->m_cand.as<mbft::MsgCand>();
  a.chash = c->m_chash.as<uint64_t>();
  a.cslot = c->m_cslot.as<uint32_t>();
  a.uniq = c->m_uniq.as<uint32_t>();
  a.ref = c->m_ref.as<uint32_t>();
  a.idx = c->m_idx.as<uint32_t>();
  a.call_of = c->m_callof.as<uint32_t>();
  a.cand_of = c->m_candof.as<uint32_t>();
  a.tkeys = c->m_tkeys.as<unsigned long long>();
  a.treps = c->m_treps.as<uint32_t>();
  a.tmask = (uint32_t)(cap - 1);
  a.map = mbft::KeyMap{c->d_kmap_keys.as<uint64_t>(), c->d_kmap_slots.as<uint32_t>(), c->kmap_mask,
                       c->kmap_role_ok};
  a.keys = tb->d_keys.as<mbft::KeyDesc>();
  a.nslots = (uint32_t)tb->slots.size();
  a.fpg = c->m_fpg.as<uint32_t>();

  // per unique call (at most one per candidate)
  HIPCHK(c, c->b_e.ensure(32 * nc3 + 32));
  HIPCHK(c, c->b_r.ensure(32 * nc3 + 32));
  HIPCHK(c, c->b_s.ensure(32 * nc3 + 32));
  HIPCHK(c, c->b_slot.ensure(4 * nc3 + 4));
  HIPCHK(c, c->m_info.ensure(sizeof(mbft::DevCallInfo) * nc3 + 32));
  HIPCHK(c, c->m_bounds.ensure(4 * (mbft_ctx::kMsgChunks + 1)));
  a.e = c->b_e.as<uint8_t>();
  a.r = c->b_r.as<uint8_t>();
  a.s = c->b_s.as<uint8_t>();
  a.slot = c->b_slot.as<uint32_t>();
  a.info = c->m_info.as<mbft::DevCallInfo>();
  uint32_t* bounds = c->m_bounds.as<uint32_t>();

  hipStream_t st = c->stream, cs = c->cstream, vb = c->vstream[0];
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
  HIPCHK(c, c->hm_small.ensure(4 * (mbft_ctx::kMsgChunks + 8)));
  uint32_t* hs = c->hm_small.as<uint32_t>();  // [0, K) running chunk ends, [K] the argument-check flags
  HIPCHK(c, hipMemsetAsync(c->m_flag.p, 0, 64, st));
  HIPCHK(c, hipMemsetAsync(bounds, 0, 4, st));
  HIPCHK(c, hipMemsetAsync(c->m_tkeys.p, 0, 8 * cap, st));
  HIPCHK(c, hipMemsetAsync(c->m_treps.p, 0xFF, 4 * cap, st));
  HIPCHK(c, hipMemcpyAsync(c->m_fpg.p, fpg.data(), 4 * fpg.size(), hipMemcpyHostToDevice, cs));
  HIPCHK(c, hipMemsetAsync(c->m_bytes.as<uint8_t>() + (nbytes & ~(size_t)3), 0, 24, cs));
  if (nbytes) HIPCHK(c, hipMemcpyAsync(c->m_bytes.p, bytes, nbytes, hipMemcpyHostToDevice, cs));
  const int K = n >= 65536 ? mbft_ctx::kMsgChunks : 1;
  static const int split_at = [] {  // env MBFT_MSG_VERIFY_SPLIT: the first stage's last chunk (-1: one stage)
    const char* v = getenv("MBFT_MSG_VERIFY_SPLIT");
    return v ? atoi(v) : 3;
  }();
  const int S = K > 1 && split_at >= 0 && split_at < K - 1 ? split_at : -1;
  size_t tmp_bytes = 0;
  HIPCHK(c, mbft_launch::msg_scan(a, 0, 0, (long)((n + K - 1) / K + 1), nullptr, &tmp_bytes, st));
  HIPCHK(c, c->m_scan.ensure(tmp_bytes + 16));
  HIPCHK(c, c->b_status.ensure(nc3 + 1));
  auto chunk_lo = [&](int j) { return (long)(n * (size_t)j / (size_t)K); };
  for (int j = 0; j < K; j++) {
    const long lo = chunk_lo(j), hi = chunk_lo(j + 1);
    HIPCHK(c, hipMemcpyAsync(c->m_recs.as<mbft_msg_rec>() + lo, recs + lo, sizeof(mbft_msg_rec) * (hi - lo),
                             hipMemcpyHostToDevice, cs));
    HIPCHK(c, hipEventRecord(c->ev_msg[j], cs));
    HIPCHK(c, hipStreamWaitEvent(st, c->ev_msg[j], 0));
    HIPCHK(c, mbft_launch::msg_cands(a, lo, hi, st));
    HIPCHK(c, mbft_launch::msg_dedup_insert(a, lo, hi, st));
    HIPCHK(c, mbft_launch::msg_dedup_resolve(a, lo, hi, st));
    HIPCHK(c, mbft_launch::msg_scan(a, lo, hi, 0, c->m_scan.p, &tmp_bytes, st));
    HIPCHK(c, mbft_launch::msg_number(a, lo, hi, bounds, j, st));
    if (j == S || j == K - 1) {
      HIPCHK(c, hipMemcpyAsync(hs + j, bounds + j + 1, 4, hipMemcpyDeviceToHost, st));
      if (j == K - 1) HIPCHK(c, hipMemcpyAsync(hs + K, a.bad, 4, hipMemcpyDeviceToHost, st));
      HIPCHK(c, hipEventRecord(c->ev_cnt[j], st));
    }
  }
  // stage 1: chunks [0, S]; stage 2: chunks (S, K)
  uint32_t base = 0;
  for (int stage = 0; stage < 2; stage++) {
    const int j0 = stage == 0 ? 0 : S + 1, j1 = stage == 0 ? S : K - 1;
    if (j1 < j0) continue;
    HIPCHK(c, hipEventSynchronize(c->ev_cnt[j1]));
    if (j1 == K - 1 && (hs[K] & 3u)) {  // an argument error: write nothing (the caller drains)
      if (hs[K] & 1u) return fail(c, MBFT_ERR_ARG, "mbft_validate_messages_flat: unknown message type");
      return fail(c, MBFT_ERR_ARG, "mbft_validate_messages_flat: field outside the byte arena");
    }
    const uint32_t end = hs[j1], cnt = end - base;
    HIPCHK(c, hipStreamWaitEvent(vb, c->ev_cnt[j1], 0));
    HIPCHK(c, mbft_launch::msg_calls(a, chunk_lo(j0), chunk_lo(j1 + 1), (long)base, (long)cnt, vb));
    if (cnt) {
      rc = verify_device(c, a.e + 32 * (size_t)base, a.r + 32 * (size_t)base, a.s + 32 * (size_t)base,
                         a.slot + base, cnt, c->b_status.as<uint8_t>() + base, vb, /*host_status=*/true,
                         /*latency=*/j1 == K - 1 && S >= 0);
      if (rc) return rc;
    }
    base = end;
  }
  const size_t nc = base;
  const auto t1 = std::chrono::steady_clock::now();
  HIPCHK(c, hipEventRecord(c->ev_cnt[0], vb));  // st joins the verifies
  HIPCHK(c, hipStreamWaitEvent(st, c->ev_cnt[0], 0));
  // the optimistic in-order replay on the GPU (k_replay_*, messages.cpp
  // replay_parallel's rules): every message's result, the first message
  // whose result is not 0, and each key group's first capture
  const size_t G = c->epoch_val.size();
  HIPCHK(c, c->m_epset.ensure(G + 1));
  HIPCHK(c, c->m_epval.ensure(8 * G + 8));
  HIPCHK(c, c->m_cap.ensure(16 * G + 16));
  HIPCHK(c, c->m_out.ensure(4 * n));
  HIPCHK(c, c->hm_cap.ensure(16 * G + 16));
  HIPCHK(c, c->hm_out.ensure(4 * n));
  if (G) {
    HIPCHK(c, hipMemcpyAsync(c->m_epset.p, c->epoch_set.data(), G, hipMemcpyHostToDevice, st));
    HIPCHK(c, hipMemcpyAsync(c->m_epval.p, c->epoch_val.data(), 8 * G, hipMemcpyHostToDevice, st));
  }
  uint64_t* hcap = c->hm_cap.as<uint64_t>();  // [0, G) cap_pos, [G, 2G) cap_epoch, [2G] first_bad
  hcap[2 * G] = n;
  HIPCHK(c, hipMemsetAsync(c->m_cap.p, 0xFF, 8 * G, st));
  HIPCHK(c, hipMemcpyAsync(c->m_cap.as<uint64_t>() + 2 * G, hcap + 2 * G, 8, hipMemcpyHostToDevice, st));
  a.status = c->b_status.as<uint8_t>();
  a.epoch_set = c->m_epset.as<uint8_t>();
  a.epoch_val = c->m_epval.as<uint64_t>();
  a.ngroups = (uint32_t)G;
  a.cap_pos = c->m_cap.as<unsigned long long>();
  a.cap_epoch = c->m_cap.as<uint64_t>() + G;
  a.out = c->m_out.as<int32_t>();
  a.first_bad = c->m_cap.as<unsigned long long>() + 2 * G;
  HIPCHK(c, mbft_launch::msg_replay(a, st));
  HIPCHK(c, hipMemcpyAsync(c->hm_out.p, a.out, 4 * n, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipMemcpyAsync(hcap, c->m_cap.p, 16 * G + 8, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  const auto t2 = std::chrono::steady_clock::now();
  const int T = n >= 4096 ? c->pool->size() : 1;
  const int32_t* hout = c->hm_out.as<int32_t>();
  c->pool->run(T, [&](int t) {
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
    HIPCHK(c, c->hm_chk.ensure(4 * n));
    HIPCHK(c, c->hm_callof.ensure(4 * nc3));
    HIPCHK(c, c->hm_info.ensure(sizeof(CallInfo) * nc + 32));
    HIPCHK(c, c->h_status.ensure(nc + 1));
    HIPCHK(c, hipMemcpyAsync(c->hm_chk.p, a.chk, 4 * n, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpyAsync(c->hm_callof.p, a.call_of, 4 * nc3, hipMemcpyDeviceToHost, st));
    if (nc) {
      HIPCHK(c, hipMemcpyAsync(c->hm_info.p, a.info, sizeof(CallInfo) * nc, hipMemcpyDeviceToHost, st));
      HIPCHK(c, hipMemcpyAsync(c->h_status.p, c->b_status.p, nc, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(c, hipStreamSynchronize(st));
    // checks of messages f.. from the packed words
    static thread_local std::vector<MsgChecks> tl_checks;
    std::vector<MsgChecks>& checks = tl_checks;
    checks.resize(n);
    const uint32_t* chk = c->hm_chk.as<uint32_t>();
    const uint32_t* callof = c->hm_callof.as<uint32_t>();
    const size_t m = n - f;
    const int Tm = m >= 4096 ? c->pool->size() : 1;
    c->pool->run(Tm, [&](int t) {
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
    const CallInfo* info = c->hm_info.as<CallInfo>();
    const uint8_t* role_bytes = c->hm_info.as<uint8_t>() + offsetof(mbft::DevCallInfo, role);
    replay_tail(
        c, f, n, checks.data(), info, c->h_status.as<uint8_t>(), flags, out,
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
int validate_flat_device(mbft_ctx* c, const mbft_msg_rec* recs, size_t n, const uint8_t* bytes,
                         size_t nbytes, uint32_t n_replicas, uint32_t flags, int32_t* out) {
  const int rc = validate_flat_device_impl(c, recs, n, bytes, nbytes, n_replicas, flags, out);
  if (rc != MBFT_OK) {
    (void)hipStreamSynchronize(c->cstream);
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->vstream[0]);
  }
  return rc;
}

bool field_ok(uint64_t off, uint32_t len, size_t nbytes) {
  return len == 0 || (off <= nbytes && (uint64_t)len <= nbytes - off);
}

}  // namespace

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
    std::lock_guard<std::mutex> g(c->mu);
    if (hipSetDevice(c->device) != hipSuccess) return MBFT_ERR_HIP;
    return validate_flat_device(c, recs, n, bytes, nbytes, n_replicas, flags, out);
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

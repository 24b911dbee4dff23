// MinBFT message layer over the batch authenticator: AuthenBytes and the
// core validators, batched.
//
//  * mbft_authen_bytes            messages/authen.go:27-82
//  * mbft_validate_messages       core/message-handling.go:409-424
//                                 (makeMessageValidator) with
//      REQUEST  core/request.go:146-150 -> core/utils.go:57-76
//      PREPARE  core/prepare.go:46-65  (isPrimary, Request, UI)
//      COMMIT   core/commit.go:74-92   (not from primary, Prepare, UI)
//      UI       core/usig-ui.go:62-77  (zero counter, USIG authenticator)
//    plus the stream semantics of core/message-handling.go:204-246: a
//    rejected message ends its stream, and a Go panic (malformed DER in an
//    ECDSA role, crypto.go:82-84; a REPLY reaching the replica's validator,
//    core/message-handling.go:420-421) ends the process.
//  * mbft_validate_replies        client side, client/message-handling.go:
//                                 93-110 (per-replica loop: a rejected REPLY
//                                 is logged, the loop goes on) and 140-170
//                                 (ClientID check, then ReplicaAuthen).
//
// Batching: every authenticator call of every message is collected,
// identical calls are verified once (a COMMIT repeats
// its PREPARE's and REQUEST's checks), and the whole batch makes ONE GPU
// round trip (§8(f) row 3): the operations go up once, k_sha256_var hashes
// them, k_authen_e builds every call's AuthenBytes from the raw fields in
// registers and its digest input e (the ECDSA-role quirk prefix, or the USIG
// chain SHA256(SHA256(AuthenBytes) || epoch_le || counter_le)), and the
// verify kernels check every signature; the host only parses DER and UIs.
// Then the validators replay in message order with short-circuit
// evaluation so that the USIG epoch state evolves exactly as the sequential
// reference would make it.
#include <algorithm>
#include <string>
#include <unordered_map>

#include <chrono>

#include "host_internal.h"
#include "kernels.h"

using namespace mbft_host;

namespace {

constexpr uint32_t kNone = 0xFFFFFFFFu;

// writeAuthenBytes for the embedded request fields: seq_be64 || H(op)
void put_request_fields(std::string& b, uint64_t seq, const uint8_t h[32]) {
  uint8_t q[8];
  put_be64(q, seq);
  b.append((const char*)q, 8);
  b.append((const char*)h, 32);
}

void put_prepare_fields(std::string& b, uint64_t view, uint32_t client, uint64_t seq,
                        const uint8_t h[32]) {
  uint8_t q[12];
  put_be64(q, view);
  put_be32(q + 8, client);
  b.append((const char*)q, 12);
  put_request_fields(b, seq, h);
}

// AuthenBytes given H(op) (or H(result) for REPLY)
std::string authen_bytes(const mbft_message& m, const uint8_t h[32], uint32_t which) {
  std::string b;
  uint8_t q[8];
  switch (which) {
    case MBFT_MSG_REQUEST:
      b = "REQUEST";
      put_request_fields(b, m.seq, h);
      break;
    case MBFT_MSG_REPLY:
      b = "REPLY";
      put_be32(q, m.client_id);
      b.append((const char*)q, 4);
      put_request_fields(b, m.seq, h);
      break;
    case MBFT_MSG_PREPARE: {
      // the PREPARE itself, or a COMMIT's embedded PREPARE
      b = "PREPARE";
      put_prepare_fields(b, m.view, m.client_id, m.seq, h);
      break;
    }
    case MBFT_MSG_COMMIT:
      b = "COMMIT";
      put_be32(q, m.prep_replica_id);
      b.append((const char*)q, 4);
      put_prepare_fields(b, m.view, m.client_id, m.seq, h);
      put_be64(q, m.prep_ui_counter);
      b.append((const char*)q, 8);
      break;
    case MBFT_MSG_REQ_VIEW_CHANGE:
      b = "REQ-VIEW-CHANGE";
      put_be64(q, m.view);
      b.append((const char*)q, 8);
      break;
  }
  return b;
}

// The same bytes into out (>= 70 B); returns their length.
size_t authen_bytes_into(const mbft_message& m, const uint8_t h[32], uint32_t which, uint8_t* out) {
  size_t o = 0;
  auto put = [&](const void* p, size_t k) {
    memcpy(out + o, p, k);
    o += k;
  };
  auto req = [&] {  // seq_be64 || H(op)
    put_be64(out + o, m.seq);
    o += 8;
    put(h, 32);
  };
  auto prep = [&] {  // view_be64 || client_be32 || seq_be64 || H(op)
    put_be64(out + o, m.view);
    put_be32(out + o + 8, m.client_id);
    o += 12;
    req();
  };
  switch (which) {
    case MBFT_MSG_REQUEST:
      put("REQUEST", 7);
      req();
      break;
    case MBFT_MSG_REPLY:
      put("REPLY", 5);
      put_be32(out + o, m.client_id);
      o += 4;
      req();
      break;
    case MBFT_MSG_PREPARE:
      put("PREPARE", 7);
      prep();
      break;
    case MBFT_MSG_COMMIT:
      put("COMMIT", 6);
      put_be32(out + o, m.prep_replica_id);
      o += 4;
      prep();
      put_be64(out + o, m.prep_ui_counter);
      o += 8;
      break;
    case MBFT_MSG_REQ_VIEW_CHANGE:
      put("REQ-VIEW-CHANGE", 15);
      put_be64(out + o, m.view);
      o += 8;
      break;
  }
  return o;
}

// One unique authenticator call of a message batch: who, which AuthenBytes
// layout over which message's fields, and the tag -- a signature, or for
// USIG the UI counter_be64 || cert (usig.MustMarshalUI) given as counter +
// cert bytes.
struct MCall {
  uint32_t role, id, kind, msg;  // kind: mbft::AuthenKind; msg: message index (fields)
  uint32_t primary;              // COMMIT: the embedded PREPARE's replica
  uint64_t prep_ctr;             // COMMIT: the embedded PREPARE's UI counter
  uint64_t counter;              // USIG kinds: the UI counter
  const uint8_t* tag;            // signature (ECDSA kinds) or UI cert (USIG kinds)
  size_t tag_len;
  bool usig() const { return kind == mbft::kAuthenPrepare || kind == mbft::kAuthenCommit; }
};

// Multiply-xorshift over 8-byte words in 4 independent lanes (no long
// multiply chain), then the tail: a bucket index only -- every hit is
// compared in full.
inline uint64_t mix(uint64_t h) {
  h ^= h >> 32;
  h *= 0xD6E8FEB86659FD93ull;
  return h ^ (h >> 32);
}

uint64_t fnv(uint64_t h, const void* p, size_t n) {
  const uint8_t* b = static_cast<const uint8_t*>(p);
  uint64_t l0 = h, l1 = h ^ 0x9E3779B97F4A7C15ull, l2 = h + 0x632BE59BD9B4E019ull,
           l3 = h ^ 0x85EBCA77C2B2AE63ull;
  size_t i = 0;
  for (; i + 32 <= n; i += 32) {
    uint64_t w[4];
    memcpy(w, b + i, 32);
    l0 = (l0 ^ w[0]) * 0x9FB21C651E98DF25ull;
    l1 = (l1 ^ w[1]) * 0xC2B2AE3D27D4EB4Full;
    l2 = (l2 ^ w[2]) * 0x165667B19E3779F9ull;
    l3 = (l3 ^ w[3]) * 0xD6E8FEB86659FD93ull;
  }
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    memcpy(&w, b + i, 8);
    l0 = mix(l0 ^ w);
  }
  uint64_t t = n;
  for (; i < n; i++) t = (t << 8) | b[i];
  return mix(l0 ^ mix(l1 ^ mix(l2 ^ mix(l3 ^ t))));
}

// The AuthenBytes-relevant fields of message m for a call of this kind
// (messages/authen.go:52-76): equal fields, op and tag <=> identical call.
struct CallKey {
  uint32_t role, id, kind, client, primary, pad;
  uint64_t view, seq, prep_ctr, counter;
};

CallKey call_key(const MCall& c, const mbft_message& m) {
  CallKey k{c.role, c.id, c.kind, 0, 0, 0, 0, m.seq, 0, c.counter};
  if (c.kind == mbft::kAuthenReply) k.client = m.client_id;
  if (c.usig()) {
    k.view = m.view;
    k.client = m.client_id;
  }
  if (c.kind == mbft::kAuthenCommit) {
    k.primary = c.primary;
    k.prep_ctr = c.prep_ctr;
  }
  return k;
}

bool same_key(const CallKey& a, const CallKey& b) { return memcmp(&a, &b, sizeof(CallKey)) == 0; }

bool same_bytes(const uint8_t* a, size_t na, const uint8_t* b, size_t nb) {
  return na == nb && (na == 0 || a == b || memcmp(a, b, na) == 0);
}

// Hash of a call's identity: its key, operation bytes and tag bytes (a
// bucket index only -- every hash hit is compared in full, so crafted
// collisions cannot merge two calls).
// op_hash: fnv(seed, m.op, m.op_len), computed once per message (all of a
// message's candidate calls include its operation).
uint64_t call_hash(const MCall& c, uint64_t op_hash, const CallKey& k) {
  const uint64_t h = fnv(op_hash, &k, sizeof(k));
  return fnv(h ^ 0x9E37u, c.tag, c.tag_len);
}

bool same_call(const MCall& a, const CallKey& ka, const mbft_message& ma, const MCall& b,
               const CallKey& kb, const mbft_message& mb) {
  return same_key(ka, kb) && same_bytes(ma.op, ma.op_len, mb.op, mb.op_len) &&
         same_bytes(a.tag, a.tag_len, b.tag, b.tag_len);
}

// The validator's steps for message m (index mi) in order, each
// authenticator call proposed through add(MCall) -> the index the check
// records (makeMessageValidator, core/message-handling.go:409-424: REQUEST
// core/request.go:146-150; PREPARE core/prepare.go:46-65 (isPrimary,
// core/utils.go:80-82); COMMIT core/commit.go:74-92; UI core/usig-ui.go:62-77).
template <class Add>
void message_checks(const mbft_message& m, uint32_t mi, uint32_t n_replicas, MsgChecks& ck, Add&& add) {
  ck.n = 0;
  auto request_checks = [&]() {
    ck.push(Check{MBFT_ST_REQUEST_SIG, 0,
                  add(MCall{MBFT_ROLE_CLIENT, m.client_id, mbft::kAuthenRequest, mi, 0, 0, 0, m.sig,
                            m.sig_len})});
  };
  auto prepare_checks = [&](uint32_t primary, uint64_t ctr, const uint8_t* cert, size_t clen) {
    if ((uint64_t)primary != m.view % (uint64_t)n_replicas) {  // isPrimary, core/utils.go:80-82
      ck.push(Check{MBFT_ST_NOT_PRIMARY, 1, kNone});
      return;
    }
    request_checks();
    if (ctr == 0) {
      ck.push(Check{MBFT_ST_PREPARE_UI, 2, kNone});
      return;
    }
    ck.push(Check{MBFT_ST_PREPARE_UI, 0,
                  add(MCall{MBFT_ROLE_USIG, primary, mbft::kAuthenPrepare, mi, 0, 0, ctr, cert, clen})});
  };
  switch (m.type) {
    case MBFT_MSG_REQUEST:
      request_checks();
      break;
    case MBFT_MSG_REPLY:
      // not a replica-side message: makeMessageValidator panics
      // ("Unknown message type", core/message-handling.go:420-421)
      ck.push(Check{MBFT_ST_UNKNOWN_TYPE, 3, kNone});
      break;
    case MBFT_MSG_PREPARE:
      prepare_checks(m.replica_id, m.ui_counter, m.ui_cert, m.ui_cert_len);
      break;
    case MBFT_MSG_COMMIT:
      if (m.replica_id == m.prep_replica_id) {
        ck.push(Check{MBFT_ST_COMMIT_FROM_PRIMARY, 1, kNone});
        break;
      }
      prepare_checks(m.prep_replica_id, m.prep_ui_counter, m.prep_ui_cert, m.prep_ui_cert_len);
      if (ck.c[ck.n - 1].kind != 0) break;  // the embedded PREPARE's checks ended early
      if (m.ui_counter == 0) {
        ck.push(Check{MBFT_ST_COMMIT_UI, 2, kNone});
        break;
      }
      ck.push(Check{MBFT_ST_COMMIT_UI, 0,
                    add(MCall{MBFT_ROLE_USIG, m.replica_id, mbft::kAuthenCommit, mi, m.prep_replica_id,
                              m.prep_ui_counter, m.ui_counter, m.ui_cert, m.ui_cert_len})});
      break;
    case MBFT_MSG_REQ_VIEW_CHANGE:
      ck.push(Check{MBFT_ST_NOT_IMPLEMENTED, 1, kNone});
      break;
  }
}

// The authenticator calls of a message batch, deduplicated in parallel.
// Every message proposes up to 3 candidate calls (slot 3 i + q) while its
// checks are built (pool, over messages); each candidate is hashed there
// too.  Then P partitions of the hash space are deduplicated at once, each
// by one worker with its own open-addressing table, and the unique calls are
// numbered partition by partition: the numbering is internal (statuses are
// read back through the checks), the first occurrence in message order
// represents each call.
struct CallDedup {
  std::vector<MCall> cand;
  std::vector<CallKey> ckey;
  std::vector<uint64_t> chash;
  std::vector<uint8_t> cpart;       // candidate -> hash partition (kNoPart: unused slot,
                                    // kRecent: a repeat of the builder's recent call rep[i])
  std::vector<uint32_t> rep;        // kRecent candidates: the earlier equal candidate
  std::vector<uint32_t> cglob;      // candidate -> unique call index
  std::vector<uint32_t> local;      // candidate -> index within its partition
  std::vector<MCall> calls;         // unique calls
  std::vector<std::vector<uint32_t>> part_first;  // per partition: first-occurrence candidates
  std::vector<std::vector<uint64_t>> part_tab;    // per partition: (hash tag << 32 | cand + 1)
  // lists[t * P + p]: the candidates builder t put in partition p, ascending
  // (builders own ascending message ranges, so partition p's candidates in
  // call order are lists[0 * P + p], lists[1 * P + p], ...)
  std::vector<std::vector<uint32_t>> lists;
  std::vector<std::vector<uint32_t>> prank;  // per partition: call number of each first occurrence
};

inline int part_of(uint64_t h, int P) { return (int)(((h >> 32) * (uint64_t)P) >> 32); }
constexpr uint8_t kNoPart = 0xFF;
constexpr uint8_t kRecent = 0xFE;
// Builder-local cache of recent calls (direct-mapped by hash): a COMMIT
// repeats the REQUEST signature and the PREPARE UI of the messages just
// before it, so most repeats are caught here, on data still in cache, and
// never reach the partitioned tables.
constexpr int kRecentSlots = 1024;

void dedup_candidates(CallDedup& D, const mbft_message* msgs, size_t ncand, Pool* pool, int T) {
  const int P = T;  // <= 64 (host_pool_threads), so a partition fits in cpart
  D.part_first.resize(P);
  D.part_tab.resize(P);
  D.cglob.resize(ncand);
  D.local.resize(ncand);
  std::vector<uint32_t>& local = D.local;
  pool->run(P, [&](int p) {
    std::vector<uint32_t>& first = D.part_first[p];
    first.clear();
    size_t cnt = 0;
    for (int t = 0; t < T; t++) cnt += D.lists[(size_t)t * P + p].size();
    size_t cap = 16;
    while (cap < 2 * cnt) cap <<= 1;
    std::vector<uint64_t>& tab = D.part_tab[p];
    tab.assign(cap, 0);
    for (int t = 0; t < T; t++)
    for (const uint32_t i : D.lists[(size_t)t * P + p]) {
      const uint64_t h = D.chash[i];
      const uint32_t tagv = (uint32_t)h | 1u;
      for (size_t sl = (size_t)(h ^ (h >> 29)) & (cap - 1);; sl = (sl + 1) & (cap - 1)) {
        const uint64_t e = tab[sl];
        if (e == 0) {
          tab[sl] = ((uint64_t)tagv << 32) | (uint32_t)(first.size());
          local[i] = (uint32_t)first.size();
          first.push_back((uint32_t)i);
          break;
        }
        if ((uint32_t)(e >> 32) != tagv) continue;
        const uint32_t j = first[(uint32_t)e];
        if (same_call(D.cand[j], D.ckey[j], msgs[D.cand[j].msg], D.cand[i], D.ckey[i],
                      msgs[D.cand[i].msg])) {
          local[i] = (uint32_t)e;
          break;
        }
      }
    }
  });
  // Number the unique calls in first-occurrence (= message) order, so that
  // the host part of the calls and the in-order replay walk them
  // sequentially: a parallel count of first occurrences per candidate range,
  // their prefix, then every candidate takes its first occurrence's number.
  auto is_first = [&](size_t i) {
    return D.cpart[i] < P && D.part_first[D.cpart[i]][local[i]] == (uint32_t)i;
  };
  D.prank.resize(P);
  for (int p = 0; p < P; p++) D.prank[p].resize(D.part_first[p].size());
  std::vector<uint32_t> cnt(T + 1, 0);
  pool->run(T, [&](int t) {
    uint32_t k = 0;
    for (size_t i = ncand * t / T; i < ncand * (t + 1) / T; i++) k += is_first(i) ? 1u : 0u;
    cnt[t + 1] = k;
  });
  for (int t = 0; t < T; t++) cnt[t + 1] += cnt[t];
  D.calls.resize(cnt[T]);
  pool->run(T, [&](int t) {
    uint32_t k = cnt[t];
    for (size_t i = ncand * t / T; i < ncand * (t + 1) / T; i++)
      if (is_first(i)) {
        D.prank[D.cpart[i]][local[i]] = k;
        D.calls[k++] = D.cand[i];
      }
  });
  pool->run(T, [&](int t) {
    for (size_t i = ncand * t / T; i < ncand * (t + 1) / T; i++) {
      const uint8_t pt = D.cpart[i];
      if (pt < P) {
        D.cglob[i] = D.prank[pt][local[i]];
      } else if (pt == kRecent) {  // its representative is never kRecent itself
        const uint32_t r = D.rep[i];
        D.cglob[i] = D.prank[D.cpart[r]][local[r]];
      }
    }
  });
}

// Distinct operations of a batch (same pointer and length = same bytes;
// equal bytes behind different pointers are simply hashed twice): op_of[i]
// = operation index of message i, first[j] = a message holding operation j.
// On the pool: messages are partitioned by a hash of (pointer, length), each
// partition deduplicated by one worker with its own table, and operations
// numbered partition by partition (any numbering works: op_of and first are
// consistent, and the packed operation bytes follow it).
size_t dedup_ops(const mbft_message* msgs, size_t n, std::vector<uint32_t>& op_of,
                 std::vector<uint32_t>& first, Pool* pool, int T) {
  op_of.resize(n);
  first.clear();
  if (n == 0) return 0;
  const int P = T;
  // per-thread scratch of the CALLING thread, reused across calls; the
  // workers reach it through these references (a thread_local named inside
  // the lambdas would be each worker's own)
  static thread_local std::vector<std::vector<uint32_t>> tl_lists, tl_pfirst;
  static thread_local std::vector<uint32_t> tl_local;
  std::vector<std::vector<uint32_t>>& lists = tl_lists;
  std::vector<std::vector<uint32_t>>& pfirst = tl_pfirst;
  std::vector<uint32_t>& local = tl_local;
  lists.resize((size_t)T * P);
  pfirst.resize(P);
  local.resize(n);
  auto hash = [&](size_t i) {
    return ((uint64_t)(uintptr_t)msgs[i].op * 0x9E3779B97F4A7C15ull) ^ msgs[i].op_len;
  };
  pool->run(T, [&](int t) {
    std::vector<uint32_t>* L = &lists[(size_t)t * P];
    for (int p = 0; p < P; p++) L[p].clear();
    for (size_t i = n * t / T; i < n * (t + 1) / T; i++) {
      const uint64_t h = hash(i);
      L[(int)(((h >> 32) * (uint64_t)P) >> 32)].push_back((uint32_t)i);
    }
  });
  pool->run(P, [&](int p) {
    std::vector<uint32_t>& f = pfirst[p];
    f.clear();
    size_t cnt = 0;
    for (int t = 0; t < T; t++) cnt += lists[(size_t)t * P + p].size();
    size_t cap = 16;
    while (cap < 2 * cnt) cap <<= 1;
    std::vector<uint32_t> tab(cap, 0);
    for (int t = 0; t < T; t++)
      for (const uint32_t i : lists[(size_t)t * P + p]) {
        const uint64_t h = hash(i);
        for (size_t sl = (size_t)(h ^ (h >> 31)) & (cap - 1);; sl = (sl + 1) & (cap - 1)) {
          const uint32_t j = tab[sl];
          if (j == 0) {
            tab[sl] = (uint32_t)f.size() + 1;
            local[i] = (uint32_t)f.size();
            f.push_back(i);
            break;
          }
          const mbft_message& o = msgs[f[j - 1]];
          if (o.op == msgs[i].op && o.op_len == msgs[i].op_len) {
            local[i] = j - 1;
            break;
          }
        }
      }
  });
  std::vector<uint32_t> off(P + 1, 0);
  for (int p = 0; p < P; p++) off[p + 1] = off[p] + (uint32_t)pfirst[p].size();
  first.resize(off[P]);
  pool->run(P, [&](int p) {
    std::copy(pfirst[p].begin(), pfirst[p].end(), first.begin() + off[p]);
    for (int t = 0; t < T; t++)
      for (const uint32_t i : lists[(size_t)t * P + p]) op_of[i] = off[p] + local[i];
  });
  return first.size();
}

// One GPU round trip for the calls of a message batch: H(op) of every
// distinct operation (k_sha256_var), e of every call from its fields
// (k_authen_e), then s^-1 + verify.  The host part of the calls (DER, UI,
// key lookups) runs on the worker pool.  info[k] / gst[k]: host outcome and
// status of call k.
int run_message_calls(mbft_ctx* c, const mbft_message* msgs, size_t n,
                      const std::vector<MCall>& calls, std::vector<CallInfo>& info,
                      std::vector<uint8_t>& gst) {
  const size_t nc = calls.size();
  info.resize(nc);  // every entry written by prepare_item
  gst.resize(nc);
  if (nc == 0) return MBFT_OK;
  if (!c->pool) c->pool.reset(new Pool(host_pool_threads() - 1));
  sync_host_keymap(c);
  const int T = nc >= 4096 ? c->pool->size() : 1;
  // distinct operations, packed
  std::vector<uint32_t> op_of, first;
  const auto tc0 = std::chrono::steady_clock::now();
  const size_t nop = dedup_ops(msgs, n, op_of, first, c->pool.get(), n >= 4096 ? c->pool->size() : 1);
  const auto tc1 = std::chrono::steady_clock::now();
  size_t obytes = 0;
  for (uint32_t i : first) obytes += msgs[i].op_len;
  HIPCHK(c, c->h_udata.ensure(obytes + 1));
  HIPCHK(c, c->h_uoff.ensure(8 * (nop + 1)));
  HIPCHK(c, c->b_udata.ensure(obytes + 1));
  HIPCHK(c, c->b_uoff.ensure(8 * (nop + 1)));
  HIPCHK(c, c->sha_out.ensure(32 * nop));
  uint8_t* ob = c->h_udata.as<uint8_t>();
  uint64_t* oo = c->h_uoff.as<uint64_t>();
  size_t pos = 0;
  for (size_t j = 0; j < nop; j++) {
    oo[j] = pos;
    pos += msgs[first[j]].op_len;
  }
  oo[nop] = pos;
  HIPCHK(c, c->h_e.ensure(32 * nc));
  HIPCHK(c, c->h_r.ensure(32 * nc));
  HIPCHK(c, c->h_s.ensure(32 * nc));
  HIPCHK(c, c->h_slot.ensure(4 * nc));
  HIPCHK(c, c->h_status.ensure(nc));
  HIPCHK(c, c->b_e.ensure(32 * nc));
  HIPCHK(c, c->b_r.ensure(32 * nc));
  HIPCHK(c, c->b_s.ensure(32 * nc));
  HIPCHK(c, c->b_slot.ensure(4 * nc));
  HIPCHK(c, c->b_status.ensure(nc));
  HIPCHK(c, c->h_desc.ensure(sizeof(mbft::AuthenDesc) * nc));
  HIPCHK(c, c->b_desc.ensure(sizeof(mbft::AuthenDesc) * nc));
  mbft::AuthenDesc* desc = c->h_desc.as<mbft::AuthenDesc>();
  uint32_t* hslot = c->h_slot.as<uint32_t>();
  c->pool->run(T, [&](int t) {
    // operations
    for (size_t j = nop * t / T; j < nop * (t + 1) / T; j++) {
      const mbft_message& m = msgs[first[j]];
      if (m.op_len) memcpy(ob + oo[j], m.op, m.op_len);
    }
    // the host part of every call; e comes from the GPU (every call gets a
    // descriptor; a host-decided call's e is computed and ignored)
    Lookup lk;
    std::vector<uint8_t> ui;  // a USIG call's UI, counter_be64 || cert (usig.MustMarshalUI)
    for (size_t k = nc * t / T; k < nc * (t + 1) / T; k++) {
      const MCall& cl = calls[k];
      const mbft_message& m = msgs[cl.msg];
      const uint8_t* tag = cl.tag;
      size_t tag_len = cl.tag_len;
      if (cl.usig()) {
        if (ui.size() < 8 + cl.tag_len) ui.resize(8 + cl.tag_len);
        put_be64(ui.data(), cl.counter);
        if (cl.tag_len) memcpy(ui.data() + 8, cl.tag, cl.tag_len);
        tag = ui.data();
        tag_len = 8 + cl.tag_len;
      }
      const mbft_item it{cl.role, cl.id, nullptr, 0, tag, tag_len};
      prepare_item(c, it, info[k], c->h_e.as<uint8_t>() + 32 * k, c->h_r.as<uint8_t>() + 32 * k,
                   c->h_s.as<uint8_t>() + 32 * k, hslot + k, true, lk);
      desc[k] = mbft::AuthenDesc{cl.kind, op_of[cl.msg], (uint32_t)k, m.client_id, cl.primary, 0,
                                 m.view, m.seq, cl.prep_ctr, info[k].ui_epoch, info[k].counter};
    }
  });
  const auto tg0 = std::chrono::steady_clock::now();
  hipStream_t st = c->stream;
  HIPCHK(c, hipMemcpyAsync(c->b_udata.p, ob, obytes + 1, hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpyAsync(c->b_uoff.p, oo, 8 * (nop + 1), hipMemcpyHostToDevice, st));
  HIPCHK(c, mbft_launch::sha256_var(c->b_udata.as<uint8_t>(), c->b_uoff.as<uint64_t>(), (long)nop,
                                    c->sha_out.as<uint8_t>(), st));
  HIPCHK(c, hipMemcpyAsync(c->b_r.p, c->h_r.p, 32 * nc, hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpyAsync(c->b_s.p, c->h_s.p, 32 * nc, hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpyAsync(c->b_slot.p, hslot, 4 * nc, hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpyAsync(c->b_desc.p, desc, sizeof(mbft::AuthenDesc) * nc, hipMemcpyHostToDevice,
                           st));
  HIPCHK(c, mbft_launch::authen_e(c->sha_out.as<uint8_t>(), c->b_desc.as<mbft::AuthenDesc>(),
                                  (long)nc, c->b_e.as<uint8_t>(), st));
  int rc = verify_device(c, c->b_e.as<uint8_t>(), c->b_r.as<uint8_t>(), c->b_s.as<uint8_t>(),
                         c->b_slot.as<uint32_t>(), nc, c->b_status.as<uint8_t>(), st);
  if (rc) return rc;
  HIPCHK(c, hipMemcpyAsync(c->h_status.p, c->b_status.p, nc, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  const auto tg1 = std::chrono::steady_clock::now();
  const uint8_t* hs = c->h_status.as<uint8_t>();
  c->pool->run(T, [&](int t) {
    for (size_t k = nc * t / T; k < nc * (t + 1) / T; k++)
      gst[k] = info[k].pre != 0xFF ? info[k].pre : hs[k];
  });
  static const bool trace = getenv("MBFT_STAGE_TRACE") != nullptr;
  if (trace)
    fprintf(stderr, "[mbft calls] nc=%zu nop=%zu T=%d dedup_ops=%.3f host_prep=%.3f gpu_round_trip=%.3f "
            "statuses=%.3f ms\n", nc, nop, T,
            std::chrono::duration<double, std::milli>(tc1 - tc0).count(),
            std::chrono::duration<double, std::milli>(tg0 - tc1).count(),
            std::chrono::duration<double, std::milli>(tg1 - tg0).count(),
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tg1).count());
  return MBFT_OK;
}

// The USIG epoch step of resolve_call (batch.cpp) against an explicit
// state (set, value) instead of the context's map.  *captures: the call
// would set the state (it accepts while the state is unset).
uint8_t resolve_with(const CallInfo& p, uint8_t g, bool set, uint64_t val, bool* captures) {
  *captures = false;
  if (p.pre != 0xFF) return p.pre;
  if (!p.usig) return g;
  const uint64_t epoch = set ? val : (p.counter == 1 ? p.ui_epoch : 0);
  if (p.ui_epoch != epoch) return MBFT_EPOCH_MISMATCH;  // sgx-usig.go:92-94
  if (p.usig_tail != 0xFF) return p.usig_tail;
  if (g == MBFT_ACCEPT && !set) *captures = true;
  return g;
}

// Message i's result given the state of every key group (epoch_set /
// epoch_val of the context, or the first capture cap_pos[g] < pos with
// cap_epoch[g]); pos = 3 i + q is a check's place in message order.
int32_t eval_message(const mbft_ctx* c, const MsgChecks& ck, size_t i, const CallInfo* info,
                     const uint8_t* gst, const std::vector<uint64_t>& cap_pos,
                     const std::vector<uint64_t>& cap_epoch) {
  for (int q = 0; q < ck.n; q++) {
    const Check& k = ck.c[q];
    if (k.kind == 1) return k.stage << 8;
    if (k.kind == 2) return (k.stage << 8) | MBFT_ZERO_COUNTER;
    if (k.kind == 3) return k.stage << 8;
    const CallInfo& p = info[k.call];
    bool set = false;
    uint64_t val = 0;
    if (p.usig) {
      const uint64_t pos = 3 * (uint64_t)i + (uint64_t)q;
      if (c->epoch_set[p.fpg]) {
        set = true;
        val = c->epoch_val[p.fpg];
      } else if (cap_pos[p.fpg] < pos) {
        set = true;
        val = cap_epoch[p.fpg];
      }
    }
    bool cap;
    const uint8_t st = resolve_with(p, gst[k.call], set, val, &cap);
    if (st != MBFT_ACCEPT) return (k.stage << 8) | st;
  }
  return 0;
}

// Replay step (a) of mbft_validate_messages: writes out[i] for every message
// before the first non-zero result, commits the epoch captures made before
// it to the context, and returns its index (n if there is none).
size_t replay_parallel(mbft_ctx* c, size_t n, const MsgChecks* checks, const CallInfo* info,
                       const uint8_t* gst, int32_t* out, Pool* pool, int T) {
  const size_t G = c->epoch_val.size();
  constexpr uint64_t kInf = ~0ull;
  // the first check of each key group that would capture (every check run,
  // the state unset until then): per-thread minima, then merged
  std::vector<std::vector<uint64_t>> tmin(T, std::vector<uint64_t>(G, kInf));
  pool->run(T, [&](int t) {
    std::vector<uint64_t>& mn = tmin[t];
    for (size_t i = n * t / T; i < n * (t + 1) / T; i++) {
      const MsgChecks& ck = checks[i];
      for (int q = 0; q < ck.n; q++) {
        const Check& k = ck.c[q];
        if (k.kind != 0) break;
        const CallInfo& p = info[k.call];
        if (!p.usig || c->epoch_set[p.fpg]) continue;
        bool cap;
        resolve_with(p, gst[k.call], false, 0, &cap);
        const uint64_t pos = 3 * (uint64_t)i + (uint64_t)q;
        if (cap && pos < mn[p.fpg]) mn[p.fpg] = pos;
      }
    }
  });
  std::vector<uint64_t> cap_pos(G, kInf), cap_epoch(G, 0);
  for (int t = 0; t < T; t++)
    for (size_t g = 0; g < G; g++) cap_pos[g] = std::min(cap_pos[g], tmin[t][g]);
  for (size_t g = 0; g < G; g++)
    if (cap_pos[g] != kInf) {
      const size_t i = cap_pos[g] / 3;
      const Check& k = checks[i].c[cap_pos[g] % 3];
      const CallInfo& p = info[k.call];
      cap_epoch[g] = p.counter == 1 ? p.ui_epoch : 0;
    }
  // every message's result on that state; the first non-zero one
  std::vector<size_t> first_bad(T, n);
  pool->run(T, [&](int t) {
    for (size_t i = n * t / T; i < n * (t + 1) / T; i++) {
      out[i] = eval_message(c, checks[i], i, info, gst, cap_pos, cap_epoch);
      if (out[i] != 0) {
        first_bad[t] = i;
        break;
      }
    }
  });
  size_t f = n;
  for (int t = 0; t < T; t++) f = std::min(f, first_bad[t]);
  // commit the captures made before message f (exact: every check before f
  // ran); the sequential replay from f sees the state as it was there
  for (size_t g = 0; g < G; g++)
    if (cap_pos[g] < 3 * (uint64_t)f) {
      c->epoch_val[g] = cap_epoch[g];
      c->epoch_set[g] = 1;
    }
  return f;
}

}  // namespace

namespace mbft_host {

// In-order replay (host_internal.h): short-circuit per message, stop per
// stream, stop all after a panic, the USIG epoch state evolving call by call.
//  (a) Optimistic pass, in parallel over messages: every message as if no
//      stream had stopped and nothing had panicked, the epoch state of each
//      key group read from the first CAPTURING check in message order (a
//      per-group minimum: the state changes only there).  It is exact for
//      every message before the first one whose result is not 0: nothing
//      before it stopped or panicked, so every check before it ran.
//  (b) From that message on (adversarial batches only), the sequential
//      replay continues from the exact state.
int replay_messages(mbft_ctx* c, size_t n, const MsgChecks* checks, const CallInfo* info,
                    const uint8_t* gst, uint32_t flags, int32_t* out,
                    const std::function<uint32_t(size_t)>& stream_of,
                    const std::function<uint32_t(uint32_t)>& role_of) {
  if (n == 0) return MBFT_OK;
  if (!c->pool) c->pool.reset(new Pool(host_pool_threads() - 1));
  const int T = n >= 4096 ? c->pool->size() : 1;
  const size_t f = replay_parallel(c, n, checks, info, gst, out, c->pool.get(), T);
  replay_tail(c, f, n, checks, info, gst, flags, out, stream_of, role_of);
  return MBFT_OK;
}

// (b): the sequential replay from message f, whose state is exact (every
// capture before f committed).  checks / info / gst indexed as above.
void replay_tail(mbft_ctx* c, size_t f, size_t n, const MsgChecks* checks, const CallInfo* info,
                 const uint8_t* gst, uint32_t flags, int32_t* out,
                 const std::function<uint32_t(size_t)>& stream_of,
                 const std::function<uint32_t(uint32_t)>& role_of) {
  std::unordered_map<uint32_t, bool> stopped;
  bool panicked = false;
  for (size_t i = f; i < n; i++) {
    if (panicked) {
      out[i] = MBFT_ST_AFTER_PANIC << 8;
      continue;
    }
    const uint32_t sid = stream_of(i);
    if (!(flags & MBFT_VF_NO_STREAM_STOP) && stopped.count(sid)) {
      out[i] = MBFT_ST_STREAM_STOPPED << 8;
      continue;
    }
    int32_t res = 0;
    for (int q = 0; q < checks[i].n; q++) {
      const Check& ck = checks[i].c[q];
      if (ck.kind == 1) {
        res = ck.stage << 8;
        break;
      }
      if (ck.kind == 2) {
        res = (ck.stage << 8) | MBFT_ZERO_COUNTER;
        break;
      }
      if (ck.kind == 3) {
        res = ck.stage << 8;
        if (!(flags & MBFT_VF_NO_PANIC_STOP)) panicked = true;
        break;
      }
      const uint8_t st = resolve_call(c, info[ck.call], gst[ck.call]);
      if (st != MBFT_ACCEPT) {
        res = (ck.stage << 8) | st;
        if (st == MBFT_MALFORMED_DER && role_of(ck.call) != MBFT_ROLE_USIG &&
            !(flags & MBFT_VF_NO_PANIC_STOP))
          panicked = true;
        break;
      }
    }
    out[i] = res;
    if (res != 0) stopped[sid] = true;
  }
}

// The unique calls of a small check (calls over messages msgs[0 .. n), oph[i]
// = fnv of message i's operation bytes) verified on engine g with no device
// message layer: SHA256(op) once per distinct operation content, each call's
// AuthenBytes built and hashed on the host, then the batch pipeline's
// small-batch launch (zero-copy staging, host s^-1; check_calls_on).
int run_calls_small(mbft_ctx* c, mbft_ctx* g, const mbft_message* msgs, size_t n,
                    const std::vector<MCall>& calls, const std::vector<uint64_t>& oph,
                    std::vector<CallInfo>& info, std::vector<uint8_t>& gst) {
  const size_t nc = calls.size();
  info.assign(nc, CallInfo());
  gst.assign(nc, 0);
  if (nc == 0) return MBFT_OK;
  static const bool trace = getenv("MBFT_STAGE_TRACE") != nullptr;
  const auto ta = std::chrono::steady_clock::now();
  size_t cap = 16;
  while (cap < 2 * n) cap <<= 1;
  // SHA256(op) once per distinct operation CONTENT (a request's REQUEST,
  // PREPARE and COMMITs carry the same op, each in its own arena bytes): a
  // table over the operations' fnv hashes, equal bytes confirmed; the
  // distinct operations hashed together (sha256_many); then each call's
  // AuthenBytes (messages/authen.go:52-76) and tag -- the signature, or for
  // USIG the UI counter_be64 || cert (usig.MustMarshalUI) -- into two flat
  // buffers (no allocation per call)
  std::vector<uint32_t> opsrc(n);     // message -> message whose digest it uses
  std::vector<uint32_t> otab(cap, 0);  // message index + 1
  std::vector<uint32_t> ops;           // distinct operations (source messages)
  std::vector<uint8_t> need(n, 0);
  for (size_t k = 0; k < nc; k++) need[calls[k].msg] = 1;
  for (uint32_t i = 0; i < (uint32_t)n; i++) {
    if (!need[i]) continue;
    const mbft_message& m = msgs[i];
    for (size_t sl = (size_t)(oph[i] ^ (oph[i] >> 31)) & (cap - 1);; sl = (sl + 1) & (cap - 1)) {
      const uint32_t j = otab[sl];
      if (j == 0) {
        otab[sl] = i + 1;
        opsrc[i] = i;
        ops.push_back(i);
        break;
      }
      const mbft_message& o = msgs[j - 1];
      if (oph[j - 1] == oph[i] && same_bytes(o.op, o.op_len, m.op, m.op_len)) {
        opsrc[i] = opsrc[j - 1];
        break;
      }
    }
  }
  std::vector<uint8_t> opdig(32 * n);  // digest, at the source message
  {
    std::vector<const uint8_t*> pp(ops.size());
    std::vector<size_t> ln(ops.size());
    std::vector<uint8_t*> oo(ops.size());
    for (size_t j = 0; j < ops.size(); j++) {
      pp[j] = msgs[ops[j]].op;
      ln[j] = msgs[ops[j]].op_len;
      oo[j] = opdig.data() + 32 * ops[j];
    }
    sha256_many(ops.size(), pp.data(), ln.data(), oo.data());
  }
  constexpr size_t kAb = 72;  // the longest AuthenBytes (COMMIT) is 70 B
  size_t uib = 0;
  for (size_t k = 0; k < nc; k++)
    if (calls[k].usig()) uib += 8 + calls[k].tag_len;
  std::vector<uint8_t> ab(kAb * nc), ui(uib + 1);
  std::vector<mbft_item> items(nc);
  size_t up = 0;
  for (size_t k = 0; k < nc; k++) {
    const MCall& cl = calls[k];
    const mbft_message& m = msgs[cl.msg];
    static constexpr uint32_t kType[4] = {MBFT_MSG_REQUEST, MBFT_MSG_REPLY, MBFT_MSG_PREPARE, MBFT_MSG_COMMIT};
    uint8_t* a = ab.data() + kAb * k;
    const size_t alen = authen_bytes_into(m, opdig.data() + 32 * opsrc[cl.msg], kType[cl.kind], a);
    const uint8_t* tag = cl.tag;
    size_t tag_len = cl.tag_len;
    if (cl.usig()) {
      uint8_t* u = ui.data() + up;
      put_be64(u, cl.counter);
      if (cl.tag_len) memcpy(u + 8, cl.tag, cl.tag_len);
      tag = u;
      tag_len = 8 + cl.tag_len;
      up += tag_len;
    }
    items[k] = mbft_item{cl.role, cl.id, a, alen, tag, tag_len};
  }
  const auto tb = std::chrono::steady_clock::now();
  std::vector<UsigCall> usig;
  const int rc = check_calls_on(c, g, items.data(), nc, gst.data(), &usig);
  if (rc) return rc;
  for (const UsigCall& u : usig) info[u.i] = u.p;
  if (trace)
    fprintf(stderr, "[mbft small calls] n=%zu calls=%zu ops=%zu digests+authen=%.3f verify=%.3f ms\n", n, nc,
            ops.size(), std::chrono::duration<double, std::milli>(tb - ta).count(),
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb).count());
  return MBFT_OK;
}

// A small check (msgdev.cpp, mbft_set_small_check): the checks of n
// messages and their unique calls' outcomes with no device message layer.
// The checks and candidate calls are built as above, deduplicated through a
// table over the content hash (every hit compared in full), each unique call's AuthenBytes
// built and hashed on the host (SHA256(op) once per operation), and the
// calls verified by the batch pipeline on engine g in one launch (the
// small-batch kernel from zero-copy staging, s^-1 on the host: the lone-call
// path).  info[k] / gst[k]: unique call k's host outcome and status, as the
// device layer hands them to resolve_call.
int check_messages_small(mbft_ctx* c, mbft_ctx* g, const mbft_message* msgs, size_t n,
                         uint32_t n_replicas, MsgChecks* checks, std::vector<CallInfo>& info,
                         std::vector<uint8_t>& gst, std::vector<uint8_t>& role) {
  std::vector<MCall> calls;
  std::vector<CallKey> keys;
  std::vector<uint64_t> hs;
  calls.reserve(3 * n);
  keys.reserve(3 * n);
  hs.reserve(3 * n);
  // the unique calls: an open-addressing table over the content hash, every
  // hit compared in full (crafted collisions only cost a verify)
  size_t cap = 16;
  while (cap < 6 * n) cap <<= 1;
  std::vector<uint32_t> tab(cap, 0);  // call index + 1
  std::vector<uint64_t> oph(n);       // fnv of each message's operation bytes
  for (size_t i = 0; i < n; i++) {
    const mbft_message& m = msgs[i];
    oph[i] = fnv(1469598103934665603ull, m.op, m.op_len);
    message_checks(m, (uint32_t)i, n_replicas, checks[i], [&](const MCall& cl) {
      const CallKey k = call_key(cl, m);
      const uint64_t h = call_hash(cl, oph[i], k);
      size_t sl = (size_t)(h ^ (h >> 29)) & (cap - 1);
      for (;; sl = (sl + 1) & (cap - 1)) {
        const uint32_t j = tab[sl];
        if (j == 0) break;
        if (hs[j - 1] == h && same_call(calls[j - 1], keys[j - 1], msgs[calls[j - 1].msg], cl, k, m))
          return j - 1;
      }
      calls.push_back(cl);
      keys.push_back(k);
      hs.push_back(h);
      tab[sl] = (uint32_t)calls.size();
      return (uint32_t)(calls.size() - 1);
    });
  }
  role.resize(calls.size());
  for (size_t k = 0; k < calls.size(); k++) role[k] = (uint8_t)calls[k].role;
  return run_calls_small(c, g, msgs, n, calls, oph, info, gst);
}

}  // namespace mbft_host

namespace {
}  // namespace

extern "C" int mbft_authen_bytes(const mbft_message* m, uint8_t* out, size_t cap, size_t* len) {
  if (!m || !len) return MBFT_ERR_ARG;
  if (m->type < MBFT_MSG_REQUEST || m->type > MBFT_MSG_REQ_VIEW_CHANGE) return MBFT_ERR_ARG;
  uint8_t h[32];
  sha256(m->op, m->op_len, h);
  const std::string b = authen_bytes(*m, h, m->type);
  *len = b.size();
  if (cap < b.size() || !out) return MBFT_ERR_ARG;
  memcpy(out, b.data(), b.size());
  return MBFT_OK;
}

extern "C" int mbft_validate_messages(mbft_ctx* c, const mbft_message* msgs, size_t n,
                                      uint32_t n_replicas, uint32_t flags, int32_t* out) {
  if (!c || (n && (!msgs || !out)) || n_replicas == 0) return MBFT_ERR_ARG;
  for (size_t i = 0; i < n; i++)
    if (msgs[i].type < MBFT_MSG_REQUEST || msgs[i].type > MBFT_MSG_REQ_VIEW_CHANGE)
      return MBFT_ERR_ARG;  // Go: panic("Unknown message type")
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return MBFT_ERR_HIP;
  const auto t0 = std::chrono::steady_clock::now();

  // 1. checks per message (pool, over messages); each authenticator call a
  //    candidate in slot 3 i + q, hashed; then the calls deduplicated
  if (!c->pool) c->pool.reset(new Pool(host_pool_threads() - 1));
  const int T = n >= 4096 ? c->pool->size() : 1;
  // per-thread scratch, reused across calls; the workers below reach it
  // through these references (a thread_local named inside the lambdas would
  // be each worker's own)
  static thread_local CallDedup tl_dedup;
  static thread_local std::vector<MsgChecks> tl_checks;
  CallDedup& D = tl_dedup;
  std::vector<MsgChecks>& checks = tl_checks;
  D.cand.resize(3 * n);
  D.ckey.resize(3 * n);
  D.chash.resize(3 * n);
  D.cpart.resize(3 * n);
  D.rep.resize(3 * n);
  D.lists.resize((size_t)T * T);
  checks.resize(n);
  c->pool->run(T, [&](int t) {
    std::vector<uint32_t>* lists = &D.lists[(size_t)t * T];
    for (int p = 0; p < T; p++) lists[p].clear();
    uint32_t recent[kRecentSlots];  // candidate id + 1 of a representative, 0 = empty
    memset(recent, 0, sizeof recent);
    for (size_t i = n * t / T; i < n * (t + 1) / T; i++) {
      const mbft_message& m = msgs[i];
      MsgChecks& ck = checks[i];
      const uint32_t mi = (uint32_t)i;
      int q = 0;
      uint64_t oph = 0;
      bool have_oph = false;
      auto add = [&](const MCall& cl) {
        const size_t id = 3 * i + (size_t)q++;
        if (!have_oph) {
          oph = fnv(1469598103934665603ull, m.op, m.op_len);
          have_oph = true;
        }
        D.cand[id] = cl;
        D.ckey[id] = call_key(cl, m);
        const uint64_t h = call_hash(cl, oph, D.ckey[id]);
        D.chash[id] = h;
        uint32_t& slot = recent[(h ^ (h >> 41)) & (kRecentSlots - 1)];
        if (slot) {
          const uint32_t r = slot - 1;
          if (D.chash[r] == h && same_call(D.cand[r], D.ckey[r], msgs[D.cand[r].msg], cl,
                                           D.ckey[id], m)) {
            D.cpart[id] = kRecent;
            D.rep[id] = r;
            return (uint32_t)id;
          }
        }
        slot = (uint32_t)id + 1;
        const int part = part_of(h, T);
        D.cpart[id] = (uint8_t)part;
        lists[part].push_back((uint32_t)id);
        return (uint32_t)id;
      };
      message_checks(m, mi, n_replicas, ck, add);
      for (; q < 3; q++) D.cpart[3 * i + (size_t)q] = kNoPart;
    }
  });
  const auto t0b = std::chrono::steady_clock::now();
  dedup_candidates(D, msgs, 3 * n, c->pool.get(), T);
  const auto t0c = std::chrono::steady_clock::now();
  c->pool->run(T, [&](int t) {
    for (size_t i = n * t / T; i < n * (t + 1) / T; i++)
      for (int q = 0; q < checks[i].n; q++)
        if (checks[i].c[q].kind == 0) checks[i].c[q].call = D.cglob[checks[i].c[q].call];
  });

  // 2. every unique call in one GPU round trip
  const auto t1 = std::chrono::steady_clock::now();
  static thread_local std::vector<CallInfo> tl_info;
  static thread_local std::vector<uint8_t> tl_gst;
  std::vector<CallInfo>& info = tl_info;
  std::vector<uint8_t>& gst = tl_gst;
  int rc = run_message_calls(c, msgs, n, D.calls, info, gst);
  if (rc) return rc;
  const std::vector<MCall>& calls = D.calls;
  const auto t2 = std::chrono::steady_clock::now();

  // 4. in-order replay
  rc = replay_messages(c, n, checks.data(), info.data(), gst.data(), flags, out,
                       [&](size_t i) { return msgs[i].stream; },
                       [&](uint32_t k) { return calls[k].role; });
  if (rc) return rc;
  static const bool trace = getenv("MBFT_STAGE_TRACE") != nullptr;
  if (trace) {
    const auto t3 = std::chrono::steady_clock::now();
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    fprintf(stderr,
            "[mbft validate] n=%zu calls=%zu checks=%.3f (build+hash %.3f, dedup %.3f, remap %.3f) "
            "calls_gpu=%.3f replay=%.3f ms\n",
            n, calls.size(), ms(t0, t1), ms(t0, t0b), ms(t0b, t0c), ms(t0c, t1), ms(t1, t2), ms(t2, t3));
  }
  return MBFT_OK;
}

extern "C" int mbft_authen_digests(mbft_ctx* c, const mbft_message* msgs, size_t n, uint32_t kind,
                                   const uint64_t* epochs, const uint64_t* counters, uint8_t* e_out) {
  if (!c || (n && (!msgs || !e_out))) return MBFT_ERR_ARG;
  if (kind > mbft::kAuthenCommit) return MBFT_ERR_ARG;
  const bool usig = kind == mbft::kAuthenPrepare || kind == mbft::kAuthenCommit;
  if (usig && n && (!epochs || !counters)) return MBFT_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return MBFT_ERR_HIP;
  if (n == 0) return MBFT_OK;
  size_t obytes = 0;
  for (size_t i = 0; i < n; i++) obytes += msgs[i].op_len;
  HIPCHK(c, c->h_udata.ensure(obytes + 1));
  HIPCHK(c, c->h_uoff.ensure(8 * (n + 1)));
  HIPCHK(c, c->b_udata.ensure(obytes + 1));
  HIPCHK(c, c->b_uoff.ensure(8 * (n + 1)));
  HIPCHK(c, c->sha_out.ensure(32 * n));
  HIPCHK(c, c->h_desc.ensure(sizeof(mbft::AuthenDesc) * n));
  HIPCHK(c, c->b_desc.ensure(sizeof(mbft::AuthenDesc) * n));
  HIPCHK(c, c->b_e.ensure(32 * n));
  uint8_t* ob = c->h_udata.as<uint8_t>();
  uint64_t* oo = c->h_uoff.as<uint64_t>();
  mbft::AuthenDesc* desc = c->h_desc.as<mbft::AuthenDesc>();
  size_t pos = 0;
  for (size_t i = 0; i < n; i++) {
    const mbft_message& m = msgs[i];
    oo[i] = pos;
    if (m.op_len) memcpy(ob + pos, m.op, m.op_len);
    pos += m.op_len;
    desc[i] = mbft::AuthenDesc{kind, (uint32_t)i, (uint32_t)i, m.client_id, m.prep_replica_id, 0,
                               m.view, m.seq, m.prep_ui_counter, usig ? epochs[i] : 0,
                               usig ? counters[i] : 0};
  }
  oo[n] = pos;
  hipStream_t st = c->stream;
  HIPCHK(c, hipMemcpyAsync(c->b_udata.p, ob, obytes + 1, hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpyAsync(c->b_uoff.p, oo, 8 * (n + 1), hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpyAsync(c->b_desc.p, desc, sizeof(mbft::AuthenDesc) * n, hipMemcpyHostToDevice,
                           st));
  HIPCHK(c, mbft_launch::sha256_var(c->b_udata.as<uint8_t>(), c->b_uoff.as<uint64_t>(), (long)n,
                                    c->sha_out.as<uint8_t>(), st));
  HIPCHK(c, mbft_launch::authen_e(c->sha_out.as<uint8_t>(), c->b_desc.as<mbft::AuthenDesc>(),
                                  (long)n, c->b_e.as<uint8_t>(), st));
  HIPCHK(c, hipMemcpyAsync(e_out, c->b_e.p, 32 * n, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  return MBFT_OK;
}

extern "C" int mbft_validate_replies(mbft_ctx* c, const mbft_message* msgs, size_t n,
                                     uint32_t client_id, uint32_t flags, int32_t* out) {
  if (!c || (n && (!msgs || !out))) return MBFT_ERR_ARG;
  for (size_t i = 0; i < n; i++)
    if (msgs[i].type != MBFT_MSG_REPLY) return MBFT_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return MBFT_ERR_HIP;

  // one ReplicaAuthen call per REPLY whose ClientID matches
  // (client/message-handling.go:163-168), all in one GPU round trip
  std::vector<uint8_t> checked(n, 0);
  std::vector<MCall> calls;
  std::vector<size_t> call_of(n, 0);
  for (size_t i = 0; i < n; i++) {
    const mbft_message& m = msgs[i];
    if (m.client_id != client_id) continue;
    call_of[i] = calls.size();
    calls.push_back(MCall{MBFT_ROLE_REPLICA, m.replica_id, mbft::kAuthenReply, (uint32_t)i, 0, 0, 0,
                          m.sig, m.sig_len});
    checked[i] = 1;
  }
  std::vector<CallInfo> info;
  std::vector<uint8_t> gst;
  int rc;
  if (n <= c->msg_small_max.load() && !c->slots.empty()) {
    // few replies (a client waits for f + 1 of each request's): the small
    // route, AuthenBytes hashed on the host, one zero-copy verify launch
    std::vector<uint64_t> oph(n);
    for (size_t i = 0; i < n; i++) oph[i] = fnv(1469598103934665603ull, msgs[i].op, msgs[i].op_len);
    sync_host_keymap(c);
    rc = run_calls_small(c, c, msgs, n, calls, oph, info, gst);
  } else {
    rc = run_message_calls(c, msgs, n, calls, info, gst);
  }
  if (rc) return rc;

  // in order: no stream stop (a rejected REPLY is only logged), but a
  // malformed DER signature panics the client process (crypto.go:82-84)
  bool panicked = false;
  for (size_t i = 0; i < n; i++) {
    if (panicked) {
      out[i] = MBFT_ST_AFTER_PANIC << 8;
      continue;
    }
    if (!checked[i]) {
      out[i] = MBFT_ST_REPLY_CLIENT_ID << 8;
      continue;
    }
    const uint8_t st = resolve_call(c, info[call_of[i]], gst[call_of[i]]);
    out[i] = st == MBFT_ACCEPT ? 0 : ((MBFT_ST_REPLY_SIG << 8) | st);
    if (st == MBFT_MALFORMED_DER && !(flags & MBFT_VF_NO_PANIC_STOP)) panicked = true;
  }
  return MBFT_OK;
}

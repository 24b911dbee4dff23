// The message layer on the GPU (mbft_validate_messages_flat over library
// page-locked memory; driver in msgdev.cpp).  The same steps as the host
// message layer in messages.cpp, which cites the reference validators
// (core/message-handling.go:409-424; REQUEST core/request.go:146-150,
// PREPARE core/prepare.go:46-65, COMMIT core/commit.go:74-92, UI
// core/usig-ui.go:62-77), one lane per message or per candidate call:
//   k_msg_cands      a message's checks in validator order and its candidate
//                    authenticator calls (<= 3: a COMMIT repeats its PREPARE's
//                    REQUEST signature and PREPARE UI), each with a 64-bit
//                    content hash (call key fields, operation bytes, tag bytes),
//                    and every candidate into an open-addressing table keyed by
//                    the hash; the slot keeps the smallest candidate index
//                    (first occurrence in message order) -- atomicCAS/atomicMin
//                    (round 6: inserted here, no k_dedup_insert launch)
//   k_dedup_resolve  every candidate compared IN FULL with its slot's
//                    representative: equal -> a repeat of that call; a hash
//                    collision with different content -> a call of its own
//                    (dedup is an optimization: a crafted collision only costs
//                    one more verify)
//   (hipcub exclusive scan: unique calls numbered in first-occurrence order)
//   k_call_list      call_of per candidate, the unique calls' list
//   k_msg_calls      each unique call decoded as batch.cpp prepare_item /
//                    k_prepare do (key lookup, Go-exact DER, USIG UI / cert
//                    split, the reference's check order), its digest input e
//                    from the AuthenBytes layout and SHA256(op) (authen_dev.h),
//                    and the outcome the host's in-order replay needs
// The verifier then runs over the unique calls (verify_device).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include "arena_dev.h"
#include "authen_dev.h"
#include "der_dev.h"
#include "msg_dev.h"
#include "sha256_dev.h"

using namespace mbft;

namespace {

constexpr uint32_t kStMalformedDer = MBFT_MALFORMED_DER, kStDerTrailing = MBFT_DER_TRAILING,
                   kStUnknownKey = MBFT_UNKNOWN_KEY, kStBadKey = MBFT_BAD_KEY,
                   kStBadCert = MBFT_BAD_CERT, kStUnknownRole = MBFT_UNKNOWN_ROLE;
constexpr uint32_t kDeadSlotDev = kHostSlot | MBFT_BAD_KEY;

__device__ __forceinline__ bool field_in(uint64_t off, uint32_t len, uint64_t nbytes) {
  return len == 0 || (off <= nbytes && (uint64_t)len <= nbytes - off);
}


// Two independent 32-bit murmur3-style lanes -> a 64-bit bucket key.  Not a
// security boundary: every hit is compared in full.
struct H2 {
  uint32_t a, b;
};
__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ void hmix(H2& h, uint32_t w) {
  uint32_t k = rotl(w * 0xcc9e2d51u, 15) * 0x1b873593u;
  h.a = rotl(h.a ^ k, 13) * 5u + 0xe6546b64u;
  uint32_t j = rotl(w * 0x85ebca6bu, 13) * 0xc2b2ae35u;
  h.b = rotl(h.b ^ j, 17) * 9u + 0x7fb5d329u;
}
__device__ __forceinline__ void hmix64(H2& h, uint64_t v) {
  hmix(h, (uint32_t)v);
  hmix(h, (uint32_t)(v >> 32));
}
__device__ __forceinline__ void hbytes(H2& h, const uint8_t* b, uint64_t off, uint32_t len) {
  hmix(h, len);
  if (len == 0) return;
  const ArenaField f = arena_field(b, off, len);
  const uint32_t nw = (len + 3u) / 4u;
  // the next block's words in flight while this block is mixed
  uint32_t cur[9], nxt[9];
  arena_load(f, 0u, cur);
  for (uint32_t k0 = 0; k0 < nw; k0 += 8) {
    if (k0 + 8 < nw) arena_load(f, k0 + 8u, nxt);
    uint32_t o[8];
    arena_shift(f, cur, o);
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint32_t k = k0 + (uint32_t)j;
      if (k < nw) hmix(h, 4u * k + 4u <= len ? o[j] : o[j] & tail_mask(len - 4u * k));
    }
#pragma unroll
    for (int j = 0; j < 9; j++) cur[j] = nxt[j];
  }
}
__device__ __forceinline__ uint32_t fmix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  return x ^ (x >> 16);
}
__device__ __forceinline__ uint64_t hfinal(const H2& h) {
  return (((uint64_t)fmix(h.a ^ h.b) << 32) | fmix(h.b + 0x9e3779b9u * h.a)) | 1ull;  // never 0
}

__device__ __forceinline__ bool same_arena(const uint8_t* b, uint64_t o1, uint64_t o2, uint32_t len) {
  if (o1 == o2 || len == 0) return true;
  const ArenaField f1 = arena_field(b, o1, len), f2 = arena_field(b, o2, len);
  const uint32_t nw = (len + 3u) / 4u;
  uint32_t diff = 0;
  for (uint32_t k0 = 0; k0 < nw && diff == 0; k0 += 8) {
    uint32_t x[8], y[8];
    arena_block(f1, k0, x);
    arena_block(f2, k0, y);
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint32_t k = k0 + (uint32_t)j;
      if (k < nw) diff |= (x[j] ^ y[j]) & (4u * k + 4u <= len ? ~0u : tail_mask(len - 4u * k));
    }
  }
  return diff == 0;
}

// The fields of message m a call of this kind reads (messages.cpp call_key:
// equal key fields, operation and tag <=> identical call).
struct CKey {
  uint32_t client, primary;
  uint64_t view, prep_ctr;
};
__device__ __forceinline__ CKey call_key(const MsgCand& c, const mbft_msg_rec& m) {
  CKey k{0, 0, 0, 0};
  const bool usig = c.kind == kAuthenPrepare || c.kind == kAuthenCommit;
  if (c.kind == kAuthenReply || usig) k.client = m.client_id;
  if (usig) k.view = m.view;
  if (c.kind == kAuthenCommit) {
    k.primary = c.primary;
    k.prep_ctr = c.prep_ctr;
  }
  return k;
}

__device__ __forceinline__ uint64_t be64_at(const uint8_t* b) {
  uint64_t v = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) v = (v << 8) | b[k];
  return v;
}


__device__ __forceinline__ void store_words8_g(uint8_t* p, const uint32_t w[8]) {
  uint4* q = reinterpret_cast<uint4*>(p);
  q[0] = make_uint4(w[0], w[1], w[2], w[3]);
  q[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

}  // namespace

// Candidate slot c (content hash h != 0) into the dedup table (capacity >=
// 2 x 3n, so the probe always ends); the slot keeps the smallest candidate
// index (first occurrence in message order: atomicMin, so the order of the
// inserts does not matter).
__device__ __forceinline__ void dedup_insert(const MsgDevArgs& A, long c, uint64_t h) {
  uint32_t s = (uint32_t)(h ^ (h >> 29)) & A.tmask;
  for (uint32_t probe = 0; probe <= A.tmask; probe++, s = (s + 1) & A.tmask) {
    const unsigned long long old = atomicCAS(&A.tkeys[s], 0ull, (unsigned long long)h);
    if (old == 0ull || old == (unsigned long long)h) {
      atomicMin(&A.treps[s], (uint32_t)c);
      A.cslot[c] = s;
      return;
    }
  }
}

// One lane per message: its checks and candidate calls (messages.cpp
// mbft_validate_messages step 1, same order and stages).
__global__ void __launch_bounds__(256) k_msg_cands(MsgDevArgs A, long lo, long hi) {
  const long i = lo + (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= hi) return;
  const mbft_msg_rec m = A.recs[i];
  const bool type_ok = m.type >= MBFT_MSG_REQUEST && m.type <= MBFT_MSG_REQ_VIEW_CHANGE;
  const bool fields_ok = field_in(m.op_off, m.op_len, A.nbytes) &&
                         field_in(m.sig_off, m.sig_len, A.nbytes) &&
                         field_in(m.ui_cert_off, m.ui_cert_len, A.nbytes) &&
                         field_in(m.prep_ui_cert_off, m.prep_ui_cert_len, A.nbytes);
  if (!type_ok || !fields_ok) {
    // Go: panic("Unknown message type"); a field past the arena is a caller
    // error -- either way the C-ABI returns MBFT_ERR_ARG, and no byte of
    // this message is read
    atomicOr(A.bad, (type_ok ? 0u : 1u) | (fields_ok ? 0u : 2u));
    A.chk[i] = 0;
    for (int q = 0; q < 3; q++) A.chash[3 * i + q] = 0;
    return;
  }
  {
    // every field this lane will hash, one round trip for all of them (the
    // hashing below walks each field 8 words per memory wait)
    uint32_t t0[8], t1[2], t2[2], t3[2];
    touch_lines(A.bytes, m.op_off, m.op_len, t0);
    touch_lines(A.bytes, m.sig_off, m.sig_len, t1);
    touch_lines(A.bytes, m.ui_cert_off, m.ui_cert_len, t2);
    touch_lines(A.bytes, m.prep_ui_cert_off, m.prep_ui_cert_len, t3);
    uint32_t x = t1[0] ^ t1[1] ^ t2[0] ^ t2[1] ^ t3[0] ^ t3[1];
#pragma unroll
    for (int j = 0; j < 8; j++) x ^= t0[j];
    asm volatile("" ::"v"(x));
  }
  uint32_t packed = 0, nchk = 0;
  auto check = [&](uint32_t kind, uint32_t stage, uint32_t cq) __attribute__((always_inline)) {
    packed |= (kind | (stage << 2) | (cq << 6)) << (8 + 8 * nchk);
    nchk++;
  };
  // The candidates by slot: a message's calls are a prefix of (REQUEST
  // signature, PREPARE UI, COMMIT UI), so each site's slot is fixed.  The
  // validator walk below only records them; the hashing runs after it, in
  // one convergent loop -- hashed at their sites, a wave mixing REQUESTs,
  // PREPAREs and COMMITs walked the operation three times and six tags one
  // after another (~46 us for a 4,096-message pass).
  MsgCand c0{}, c1{}, c2{};
  int nq = 0;
  auto request_checks = [&]() __attribute__((always_inline)) {
    c0 = MsgCand{MBFT_ROLE_CLIENT, m.client_id, kAuthenRequest, (uint32_t)i, 0, m.sig_len, m.sig_off, 0, 0};
    nq = 1;
    check(kChkCall, MBFT_ST_REQUEST_SIG, 0);
  };
  // core/prepare.go:46-65 (also the embedded PREPARE of a COMMIT)
  auto prepare_checks = [&](uint32_t primary, uint64_t ctr, uint64_t cert_off, uint32_t cert_len) __attribute__((always_inline)) {
    if ((uint64_t)primary != m.view % (uint64_t)A.n_replicas) {  // isPrimary, core/utils.go:80-82
      check(kChkFail, MBFT_ST_NOT_PRIMARY, 0);
      return false;
    }
    request_checks();
    if (ctr == 0) {
      check(kChkZeroCtr, MBFT_ST_PREPARE_UI, 0);
      return false;
    }
    c1 = MsgCand{MBFT_ROLE_USIG, primary, kAuthenPrepare, (uint32_t)i, 0, cert_len, cert_off, 0, ctr};
    nq = 2;
    check(kChkCall, MBFT_ST_PREPARE_UI, 1);
    return true;
  };
  switch (m.type) {
    case MBFT_MSG_REQUEST:
      request_checks();
      break;
    case MBFT_MSG_REPLY:
      // not a replica-side message: makeMessageValidator panics
      // ("Unknown message type", core/message-handling.go:420-421)
      check(kChkPanic, MBFT_ST_UNKNOWN_TYPE, 0);
      break;
    case MBFT_MSG_PREPARE:
      prepare_checks(m.replica_id, m.ui_counter, m.ui_cert_off, m.ui_cert_len);
      break;
    case MBFT_MSG_COMMIT:
      if (m.replica_id == m.prep_replica_id) {  // core/commit.go:78-80
        check(kChkFail, MBFT_ST_COMMIT_FROM_PRIMARY, 0);
        break;
      }
      if (!prepare_checks(m.prep_replica_id, m.prep_ui_counter, m.prep_ui_cert_off,
                          m.prep_ui_cert_len))
        break;  // the embedded PREPARE's checks ended early
      if (m.ui_counter == 0) {
        check(kChkZeroCtr, MBFT_ST_COMMIT_UI, 0);
        break;
      }
      c2 = MsgCand{MBFT_ROLE_USIG, m.replica_id, kAuthenCommit, (uint32_t)i, m.prep_replica_id,
                   m.ui_cert_len, m.ui_cert_off, m.prep_ui_counter, m.ui_counter};
      nq = 3;
      check(kChkCall, MBFT_ST_COMMIT_UI, 2);
      break;
    default:  // MBFT_MSG_REQ_VIEW_CHANGE: core/message-handling.go:418-419
      check(kChkFail, MBFT_ST_NOT_IMPLEMENTED, 0);
      break;
  }
  // each candidate: key fields, then the operation's hash state, then its tag
  H2 oh{0x243f6a88u, 0x85a308d3u};
  if (nq > 0) hbytes(oh, A.bytes, m.op_off, m.op_len);
#pragma unroll 1
  for (int q = 0; q < 3; q++) {
    const long c = 3 * i + q;
    if (q >= nq) {
      A.chash[c] = 0;
      continue;
    }
    const MsgCand cd = q == 0 ? c0 : (q == 1 ? c1 : c2);
    A.cand[c] = cd;
    const CKey k = call_key(cd, m);
    H2 h = oh;
    hmix(h, cd.role);
    hmix(h, cd.id);
    hmix(h, cd.kind);
    hmix(h, k.client);
    hmix(h, k.primary);
    hmix64(h, k.view);
    hmix64(h, m.seq);
    hmix64(h, k.prep_ctr);
    hmix64(h, cd.counter);
    hbytes(h, A.bytes, cd.tag_off, cd.tag_len);
    const uint64_t hv = hfinal(h);
    A.chash[c] = hv;
    dedup_insert(A, c, hv);  // (the table was cleared by k_msg_init; k_dedup_resolve follows)
  }
  A.chk[i] = packed | nchk;
}

__global__ void __launch_bounds__(256) k_dedup_resolve(MsgDevArgs A, long lo, long hi) {
  const long c = 3 * lo + (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= 3 * hi) return;
  const uint64_t h = A.chash[c];
  if (h == 0) {
    A.uniq[c] = 0;
    A.ref[c] = (uint32_t)c;
    return;
  }
  const uint32_t r = A.treps[A.cslot[c]];
  bool same = r == (uint32_t)c;
  if (!same) {
    const MsgCand a = A.cand[c], b = A.cand[r];
    const mbft_msg_rec& ma = A.recs[a.msg];
    const mbft_msg_rec& mb = A.recs[b.msg];
    const CKey ka = call_key(a, ma), kb = call_key(b, mb);
    same = a.role == b.role && a.id == b.id && a.kind == b.kind && a.counter == b.counter &&
           ka.client == kb.client && ka.primary == kb.primary && ka.view == kb.view &&
           ka.prep_ctr == kb.prep_ctr && ma.seq == mb.seq && ma.op_len == mb.op_len &&
           a.tag_len == b.tag_len && same_arena(A.bytes, ma.op_off, mb.op_off, ma.op_len) &&
           same_arena(A.bytes, a.tag_off, b.tag_off, a.tag_len);
  }
  // a representative always represents itself; a collision with different
  // content makes this candidate a call of its own
  A.uniq[c] = (r == (uint32_t)c || !same) ? 1u : 0u;
  A.ref[c] = same ? r : (uint32_t)c;
}

// call_of of every candidate, and the list of unique calls (call k -> its
// candidate), so that k_msg_calls runs one dense lane per call: in a C3 batch
// two of a COMMIT's three candidates are repeats, and a lane per candidate
// left two thirds of every wave idle through the SHA rounds.
// Chunk j's call numbers made global: idx += bounds[j]; its last slot also
// sets bounds[j + 1] (from its chunk-local idx, read before the add).
__global__ void __launch_bounds__(256) k_chunk_base(MsgDevArgs A, long lo, long hi, uint32_t* bounds,
                                                    int j) {
  const long c = 3 * lo + (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= 3 * hi) return;
  const uint32_t base = bounds[j], v = A.idx[c];
  if (c == 3 * hi - 1) bounds[j + 1] = base + v + A.uniq[c];
  A.idx[c] = base + v;
}

// call_of of every candidate (its representative's number) and the list of
// unique calls (call k -> its candidate), so that k_msg_calls runs one dense
// lane per call: in a C3 batch two of a COMMIT's three candidates are repeats,
// and a lane per candidate left two thirds of every wave idle through the SHA
// rounds.
__global__ void __launch_bounds__(256) k_call_list(MsgDevArgs A, long lo, long hi) {
  const long c = 3 * lo + (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= 3 * hi) return;
  if (A.chash[c] == 0) return;
  A.call_of[c] = A.idx[A.ref[c]];
  if (A.uniq[c]) A.cand_of[A.idx[c]] = (uint32_t)c;
}

// A small chunk's numbering in ONE workgroup (kNumberOneMax candidate slots
// or fewer): the exclusive scan of uniq (each thread a contiguous run, a wave
// scan of the run totals, then the 16 wave totals), the chunk's base from
// bounds[j] and its end to bounds[j + 1] (k_chunk_base), then -- after a
// barrier, every idx written -- call_of and the unique-call list
// (k_call_list).  Replaces the hipcub scan's launches, k_chunk_base and
// k_call_list, each ~5 us of dispatch in a mid-size pass.
__global__ void __launch_bounds__(1024) k_number_one(MsgDevArgs A, long lo, long hi, uint32_t* bounds, int j) {
  __shared__ uint32_t wsum[16];
  const long c0 = 3 * lo, m = 3 * (hi - lo);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const long per = (m + 1023) / 1024;
  const long b = c0 + (long)t * per, e = b + per < c0 + m ? b + per : c0 + m;
  uint32_t s = 0;
  for (long c = b; c < e; c++) s += A.uniq[c];
  uint32_t x = s;  // inclusive scan over the wave
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  if (t < 64) {
    uint32_t w = t < 16 ? wsum[t] : 0u;
#pragma unroll
    for (int d = 1; d < 16; d <<= 1) {
      const uint32_t y = __shfl_up(w, d);
      if (lane >= d) w += y;
    }
    if (t < 16) wsum[t] = w;
  }
  __syncthreads();
  const uint32_t base = bounds[j];
  uint32_t run = base + (x - s) + (wv ? wsum[wv - 1] : 0u);
  for (long c = b; c < e; c++) {
    const uint32_t u = A.uniq[c];
    A.idx[c] = run;
    run += u;
  }
  if (t == 1023) bounds[j + 1] = base + wsum[15];
  __syncthreads();  // every idx of the chunk written (a representative may be anywhere in it)
  for (long c = b; c < e; c++) {
    if (A.chash[c] == 0) continue;
    A.call_of[c] = A.idx[A.ref[c]];
    if (A.uniq[c]) A.cand_of[A.idx[c]] = (uint32_t)c;
  }
}

// Each unique call's decode (batch.cpp prepare_item's rules and order, as
// k_prepare), digest input and outcome.
__global__ void __launch_bounds__(256) k_msg_calls(MsgDevArgs A, long base, long cnt,
                                                   const uint32_t* __restrict__ cnt_dev) {
  const long k = base + (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= base + cnt) return;
  if (cnt_dev && k >= base + (long)*cnt_dev) return;  // grid sized for an upper bound
  const MsgCand cd = A.cand[A.cand_of[k]];
  const mbft_msg_rec& m = A.recs[cd.msg];
  DevCallInfo inf{0xFF, 0xFF, 0, (uint8_t)cd.role, 0, 0, 0};
  uint32_t sl = 0, slot = kDeadSlotDev;
  uint32_t ew[8], rw[8], sw[8];
#pragma unroll
  for (int j = 0; j < 8; j++) ew[j] = rw[j] = sw[j] = 0;
  const uint32_t role = cd.role;
  bool digest = false;
  uint64_t epoch = 0;
  // this lane's copy of the tag in LDS (one batch of word loads), when its
  // covering words fit the slot
  __shared__ uint32_t tagbuf[256 * kTagWords];
  uint32_t* tw = tagbuf + threadIdx.x * kTagWords;
  const bool staged = stage_field(tw, A.bytes, cd.tag_off, cd.tag_len);
  if (role > 3u || ((A.map.role_ok >> role) & 1u) == 0) {
    inf.pre = kStUnknownRole;  // keymanager.go:100, authenticator.go:126-129
  } else {
    const uint64_t key = ((uint64_t)role << 32) | cd.id;
    bool known = false;
    for (uint32_t h = keymap_hash(key) & A.map.mask, probe = 0; probe <= A.map.mask;
         probe++, h = (h + 1) & A.map.mask) {
      const uint64_t kk = A.map.keys[h];
      if (kk == key) {
        known = true;
        sl = A.map.slots[h];
        break;
      }
      if (kk == ~0ull) break;
    }
    const bool valid = known && sl < A.nslots && A.keys[sl].valid != 0;
    // the tag's checks read it from the lane's LDS copy when it fits (byte
    // parsing at LDS latency), from the arena otherwise (a flat pointer
    // either way: one copy of the DER parser, run once by a wave whatever
    // its mix of ECDSA and USIG calls)
    const uint8_t* t = staged ? reinterpret_cast<const uint8_t*>(tw) + (cd.tag_off & 3u) : A.bytes + cd.tag_off;
    const bool usig_role = role == MBFT_ROLE_USIG;
    // crypto.go:79-89: an ECDSA tag's DER first (Go panics on a decode
    // error), then the key; a USIG UI is counter || cert, never shorter than
    // 8 (usig.go:75-80), its cert's DER read after the key checks
    // (ParseCert, sgx-usig.go:159-168; usig-enclave.go:217-221)
    const bool want_der = !usig_role || (known && valid && cd.tag_len >= 8);
    const uint32_t dl = usig_role ? cd.tag_len - 8 : cd.tag_len;
    bool der_ok = false;
    uint32_t used = 0;
    if (want_der) der_ok = der_sig(usig_role ? t + 8 : t, dl, rw, sw, used);
    if (!usig_role) {
      if (!der_ok) {
        inf.pre = kStMalformedDer;
      } else if (!known) {
        inf.pre = kStUnknownKey;
      } else if (!valid) {
        inf.pre = kStBadKey;
      } else {
        slot = sl;
        digest = true;
      }
    } else if (!known) {
      inf.pre = kStUnknownKey;
    } else if (!valid) {
      inf.pre = kStBadKey;
    } else if (cd.tag_len < 8) {
      inf.pre = kStBadCert;
    } else {
      inf.usig = 1;
      inf.fpg = A.fpg[sl];
      inf.counter = cd.counter;
      epoch = be64_at(t);
      inf.ui_epoch = epoch;
      if (!der_ok) {
        inf.usig_tail = kStMalformedDer;
      } else if (used != dl) {  // usig-enclave.go:220-221
        inf.usig_tail = kStDerTrailing;
      } else {
        slot = sl;
        digest = true;
      }
    }
  }
  if (digest) {
    uint32_t hw[8], out[8];
    sha256_arena(hw, A.bytes, m.op_off, m.op_len);  // H(op), messages/authen.go:78-82
    authen_digest(out, cd.kind, hw, m.seq, m.client_id, m.view, cd.primary, cd.prep_ctr, epoch,
                  cd.counter);
#pragma unroll
    for (int j = 0; j < 8; j++) ew[j] = __builtin_bswap32(out[j]);
  } else {
#pragma unroll
    for (int j = 0; j < 8; j++) rw[j] = sw[j] = 0;
  }
  store_words8_g(A.e + 32 * (size_t)k, ew);
  store_words8_g(A.r + 32 * (size_t)k, rw);
  store_words8_g(A.s + 32 * (size_t)k, sw);
  A.slot[k] = slot;
  A.info[k] = inf;
}


// The optimistic replay on the GPU (messages.cpp replay_parallel, same
// rules): resolve_with is the USIG epoch step of batch.cpp resolve_call
// against an explicit state (crypto.go:219-236, sgx-usig.go:92-94).
__device__ __forceinline__ uint32_t resolve_dev(const DevCallInfo& p, uint32_t g, bool set,
                                                uint64_t val, bool* captures) {
  *captures = false;
  if (p.pre != 0xFF) return p.pre;
  if (!p.usig) return g;
  const uint64_t epoch = set ? val : (p.counter == 1 ? p.ui_epoch : 0);
  if (p.ui_epoch != epoch) return MBFT_EPOCH_MISMATCH;
  if (p.usig_tail != 0xFF) return p.usig_tail;
  if (g == MBFT_ACCEPT && !set) *captures = true;
  return g;
}

// per message: its capturing checks (every call check up to the first
// non-call check, the state unset) -> the group's minimum position
__global__ void __launch_bounds__(256) k_replay_caps(MsgDevArgs A) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= A.n) return;
  const uint32_t w = A.chk[i], nq = w & 0xFFu;
  for (uint32_t q = 0; q < nq; q++) {
    const uint32_t b = (w >> (8 + 8 * q)) & 0xFFu;
    if ((b & 3u) != kChkCall) break;
    const uint32_t k = A.call_of[3 * i + ((b >> 6) & 3u)];
    const DevCallInfo p = A.info[k];
    if (!p.usig || A.epoch_set[p.fpg]) continue;
    bool cap;
    resolve_dev(p, A.status[k], false, 0, &cap);
    if (cap) atomicMin(&A.cap_pos[p.fpg], (unsigned long long)(3 * i + q));
  }
}

// per group: the epoch its first capturing check captures
__global__ void k_replay_cap_epoch(MsgDevArgs A) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= A.ngroups) return;
  const unsigned long long pos = A.cap_pos[g];
  uint64_t e = 0;
  if (pos != ~0ull) {
    const long i = (long)(pos / 3);
    const uint32_t q = (uint32_t)(pos % 3);
    const uint32_t b = (A.chk[i] >> (8 + 8 * q)) & 0xFFu;
    const DevCallInfo p = A.info[A.call_of[3 * i + ((b >> 6) & 3u)]];
    e = p.counter == 1 ? p.ui_epoch : 0;
  }
  A.cap_epoch[g] = e;
}

// per message: its result on that state (messages.cpp eval_message)
__global__ void __launch_bounds__(256) k_replay_eval(MsgDevArgs A) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= A.n) return;
  const uint32_t w = A.chk[i], nq = w & 0xFFu;
  int32_t res = 0;
  for (uint32_t q = 0; q < nq && res == 0; q++) {
    const uint32_t b = (w >> (8 + 8 * q)) & 0xFFu;
    const uint32_t kind = b & 3u, stage = (b >> 2) & 15u;
    if (kind == kChkFail || kind == kChkPanic) {
      res = (int32_t)(stage << 8);
    } else if (kind == kChkZeroCtr) {
      res = (int32_t)((stage << 8) | MBFT_ZERO_COUNTER);
    } else {
      const uint32_t k = A.call_of[3 * i + ((b >> 6) & 3u)];
      const DevCallInfo p = A.info[k];
      bool set = false, cap;
      uint64_t val = 0;
      if (p.usig) {
        if (A.epoch_set[p.fpg]) {
          set = true;
          val = A.epoch_val[p.fpg];
        } else if (A.cap_pos[p.fpg] < (unsigned long long)(3 * i + q)) {
          set = true;
          val = A.cap_epoch[p.fpg];
        }
      }
      const uint32_t st = resolve_dev(p, A.status[k], set, val, &cap);
      if (st != MBFT_ACCEPT) res = (int32_t)((stage << 8) | st);
    }
  }
  A.out[i] = res;
  if (res != 0) atomicMin(A.first_bad, (unsigned long long)i);
}

// A pass's zeroed state in one launch (instead of four memsets): the
// argument-check flags (16 words), the first chunk bound, the dedup table's
// keys (0 = empty) and representatives (~0 = none yet).
// (16-byte stores: cap is a power of two >= 1024, both arrays 16-B aligned)
// Upload u: bytes [0, u.bytes) of page-locked host memory (16-B aligned)
// to device memory (16-B aligned), then zero words up to u.fill: the body in
// 16-B chunks, two per thread and iteration (both loads in flight before
// either store), the last partial chunk and the padding by the first threads
// of the grid, word by word (bytes past u.bytes read as zero).  The host
// reuses these buffers pass after pass, so every read is system scope (sc0
// sc1: never served from a GPU cache line of an earlier pass).
__device__ __forceinline__ void host_load2(const uint4* p, const uint4* q, uint4& a, uint4& b) {
  asm volatile(
      "global_load_dwordx4 %0, %2, off sc0 sc1\n\t"
      "global_load_dwordx4 %1, %3, off sc0 sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(a), "=&v"(b)
      : "v"(p), "v"(q)
      : "memory");
}
__device__ __forceinline__ void upload_body(const MsgUpload& u, long t, long stride) {
  const uint64_t n16 = u.bytes / 16u;
  const uint4* s4 = reinterpret_cast<const uint4*>(u.src);
  uint4* d4 = reinterpret_cast<uint4*>(u.dst);
  for (uint64_t i = (uint64_t)t; i < n16; i += 2u * (uint64_t)stride) {
    const uint64_t j = i + (uint64_t)stride;
    uint4 a, b;
    host_load2(s4 + i, s4 + (j < n16 ? j : i), a, b);
    d4[i] = a;
    if (j < n16) d4[j] = b;
  }
  const uint64_t w = 16u * n16 / 4u + (uint64_t)t;  // this thread's tail word
  if (t < 16 && 4u * w < u.fill) {
    uint32_t v = 0;
    if (4u * w < u.bytes) {  // (the aligned word lies in the same 16-B chunk as the field's last bytes)
      v = __hip_atomic_load(reinterpret_cast<const uint32_t*>(u.src) + w, __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_SYSTEM);
      const uint64_t nb = u.bytes - 4u * w;
      if (nb < 4u) v &= (1u << (8u * (uint32_t)nb)) - 1u;
    }
    reinterpret_cast<uint32_t*>(u.dst)[w] = v;
  }
}

__global__ void __launch_bounds__(256) k_msg_init(uint32_t* flags, uint32_t* bounds,
                                                  unsigned long long* tkeys, uint32_t* treps, long cap,
                                                  uint32_t* tail6, MsgUpload up0, MsgUpload up1,
                                                  int ublocks) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long stride = (long)gridDim.x * blockDim.x;
  if (t < 16) flags[t] = 0;
  if (t == 0) bounds[0] = 0;
  if (tail6 && t < 6) tail6[t] = 0;  // the arena's zero padding (before its upload, same stream)
  // the uploads by the first `ublocks` workgroups only (block-uniform)
  if ((int)blockIdx.x < ublocks) {
    const long ustride = (long)ublocks * blockDim.x;
    if (up0.dst) upload_body(up0, t, ustride);
    if (up1.dst) upload_body(up1, t, ustride);
  }
  uint4* k4 = reinterpret_cast<uint4*>(tkeys);
  uint4* r4 = reinterpret_cast<uint4*>(treps);
  for (long i = t; i < cap / 2; i += stride) k4[i] = make_uint4(0u, 0u, 0u, 0u);
  for (long i = t; i < cap / 4; i += stride) r4[i] = make_uint4(~0u, ~0u, ~0u, ~0u);
}

namespace mbft_launch {

hipError_t msg_init(const MsgDevArgs& a, uint32_t* flags, uint32_t* bounds, hipStream_t st, uint32_t* tail6,
                    const MsgUpload* up0, const MsgUpload* up1) {
  const long cap = (long)a.tmask + 1;
  long blocks = (cap / 2 + 255) / 256;
  // an upload: at least a block per 64 KB (env MBFT_MSG_KCOPY_BLOCK).  Fewer
  // workgroups streaming host memory beat many: 1,024 / 4,096 messages 19.0 /
  // 66.8 us at 8 KB a block, 27 / 104 at 2 KB, 14.5 / 47.3 at 64 KB -- the
  // table-clearing grid (16 / 64 blocks) then sets the spread
  // (profiles/round6_kcopy_block_ab.json).
  const uint64_t ub = (up0 ? up0->bytes : 0) + (up1 ? up1->bytes : 0);
  static const uint64_t per_block = [] {
    const char* v = getenv("MBFT_MSG_KCOPY_BLOCK");
    const uint64_t x = v ? strtoull(v, nullptr, 10) : 65536u;
    return x >= 256u ? x : (uint64_t)65536u;
  }();
  long ublocks = (long)((ub + per_block - 1) / per_block);
  if (ublocks > blocks) blocks = ublocks;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  static const long umax = [] {  // env MBFT_MSG_KCOPY_UBLOCKS: at most this many workgroups upload (A/B)
    const char* v = getenv("MBFT_MSG_KCOPY_UBLOCKS");
    return v ? atol(v) : 2048L;
  }();
  ublocks = blocks < umax ? blocks : (umax > 0 ? umax : 1);
  const MsgUpload none{nullptr, nullptr, 0, 0};
  hipLaunchKernelGGL(k_msg_init, dim3((unsigned)blocks), dim3(256), 0, st, flags, bounds, a.tkeys, a.treps,
                     cap, tail6, up0 ? *up0 : none, up1 ? *up1 : none, (int)ublocks);
  return hipGetLastError();
}

hipError_t msg_cands(const MsgDevArgs& a, long lo, long hi, hipStream_t st) {
  if (hi <= lo) return hipSuccess;
  hipLaunchKernelGGL(k_msg_cands, dim3((unsigned)((hi - lo + 255) / 256)), dim3(256), 0, st, a, lo,
                     hi);
  return hipGetLastError();
}

hipError_t msg_dedup_resolve(const MsgDevArgs& a, long lo, long hi, hipStream_t st) {
  if (hi <= lo) return hipSuccess;
  hipLaunchKernelGGL(k_dedup_resolve, dim3((unsigned)((3 * (hi - lo) + 255) / 256)), dim3(256), 0, st,
                     a, lo, hi);
  return hipGetLastError();
}

hipError_t msg_scan(const MsgDevArgs& a, long lo, long hi, long maxn, void* tmp, size_t* tmp_bytes,
                    hipStream_t st) {
  if (!tmp) return hipcub::DeviceScan::ExclusiveSum(tmp, *tmp_bytes, a.uniq, a.idx, (int)(3 * maxn), st);
  if (hi <= lo) return hipSuccess;
  return hipcub::DeviceScan::ExclusiveSum(tmp, *tmp_bytes, a.uniq + 3 * lo, a.idx + 3 * lo,
                                          (int)(3 * (hi - lo)), st);
}

hipError_t msg_number(const MsgDevArgs& a, long lo, long hi, uint32_t* bounds, int j, hipStream_t st) {
  if (hi <= lo) return hipSuccess;
  hipLaunchKernelGGL(k_chunk_base, dim3((unsigned)((3 * (hi - lo) + 255) / 256)), dim3(256), 0, st, a, lo,
                     hi, bounds, j);
  return hipGetLastError();
}

hipError_t msg_number_one(const MsgDevArgs& a, long lo, long hi, uint32_t* bounds, int j, hipStream_t st) {
  if (hi <= lo) return hipSuccess;
  if (3 * (hi - lo) > kNumberOneMax) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_number_one, dim3(1), dim3(1024), 0, st, a, lo, hi, bounds, j);
  return hipGetLastError();
}

hipError_t msg_calls(const MsgDevArgs& a, long lo, long hi, long base, long cnt, hipStream_t st,
                     const uint32_t* cnt_dev, bool listed) {
  if (hi <= lo) return hipSuccess;
  if (!listed)
    hipLaunchKernelGGL(k_call_list, dim3((unsigned)((3 * (hi - lo) + 255) / 256)), dim3(256), 0, st, a, lo,
                       hi);
  if (cnt > 0)
    hipLaunchKernelGGL(k_msg_calls, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, st, a, base, cnt,
                       cnt_dev);
  return hipGetLastError();
}

hipError_t msg_replay(const MsgDevArgs& a, hipStream_t st) {
  if (a.n <= 0) return hipSuccess;
  const dim3 grid((unsigned)((a.n + 255) / 256)), block(256);
  hipLaunchKernelGGL(k_replay_caps, grid, block, 0, st, a);
  if (a.ngroups)
    hipLaunchKernelGGL(k_replay_cap_epoch, dim3((a.ngroups + 63) / 64), dim3(64), 0, st, a);
  hipLaunchKernelGGL(k_replay_eval, grid, block, 0, st, a);
  return hipGetLastError();
}

}  // namespace mbft_launch

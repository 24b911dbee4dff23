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
// its PREPARE's and REQUEST's checks), all signatures go to the GPU in one
// batch, then the validators replay in message order with short-circuit
// evaluation so that the USIG epoch state evolves exactly as the sequential
// reference would make it.
#include <string>
#include <unordered_map>

#include "host_internal.h"

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

std::string ui_tag(uint64_t counter, const uint8_t* cert, size_t cert_len) {
  std::string t(8, '\0');
  put_be64((uint8_t*)&t[0], counter);  // usig.MustMarshalUI (usig/usig.go:54-70)
  if (cert_len) t.append((const char*)cert, cert_len);
  return t;
}

// One step of a message's validation.
struct Check {
  uint8_t stage;  // mbft_stage
  uint8_t kind;   // 0 = authenticator call, 1 = fail (no call), 2 = zero-counter UI,
                  // 3 = Go panic (no call)
  uint32_t call;  // unique call index (kind 0)
};

struct Call {
  uint32_t role, id;
  std::string msg, tag;
};

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

  // 1. H(op) for every message (GPU SHA stage when the batch is large)
  std::vector<uint8_t> ops;
  std::vector<uint64_t> off{0};
  ops.reserve(n * 64);
  for (size_t i = 0; i < n; i++) {
    if (msgs[i].op_len) ops.insert(ops.end(), msgs[i].op, msgs[i].op + msgs[i].op_len);
    off.push_back(ops.size());
  }
  std::vector<uint8_t> hops;
  int rc = sha256_many(c, ops, off, hops);
  if (rc) return rc;

  // 2. checks per message, with deduplicated authenticator calls
  std::vector<Call> calls;
  std::unordered_map<std::string, uint32_t> call_ix;
  std::vector<std::vector<Check>> checks(n);
  auto add_call = [&](uint32_t role, uint32_t id, std::string msg, std::string tag) {
    std::string key;
    key.reserve(16 + msg.size() + tag.size());
    key.append((const char*)&role, 4).append((const char*)&id, 4);
    const uint64_t ml = msg.size();
    key.append((const char*)&ml, 8).append(msg).append(tag);
    auto it = call_ix.find(key);
    if (it != call_ix.end()) return it->second;
    const uint32_t ix = (uint32_t)calls.size();
    calls.push_back(Call{role, id, std::move(msg), std::move(tag)});
    call_ix.emplace(std::move(key), ix);
    return ix;
  };
  auto sig = [&](const mbft_message& m) {
    return std::string((const char*)m.sig, m.sig_len);
  };
  for (size_t i = 0; i < n; i++) {
    const mbft_message& m = msgs[i];
    const uint8_t* h = &hops[32 * i];
    auto& ck = checks[i];
    auto request_checks = [&]() {
      ck.push_back(Check{MBFT_ST_REQUEST_SIG, 0,
                         add_call(MBFT_ROLE_CLIENT, m.client_id,
                                  authen_bytes(m, h, MBFT_MSG_REQUEST), sig(m))});
    };
    auto prepare_checks = [&](uint32_t primary, uint64_t ctr, const uint8_t* cert, size_t clen) {
      if ((uint64_t)primary != m.view % (uint64_t)n_replicas) {  // isPrimary, core/utils.go:80-82
        ck.push_back(Check{MBFT_ST_NOT_PRIMARY, 1, kNone});
        return;
      }
      request_checks();
      if (ctr == 0) {
        ck.push_back(Check{MBFT_ST_PREPARE_UI, 2, kNone});
        return;
      }
      ck.push_back(Check{MBFT_ST_PREPARE_UI, 0,
                         add_call(MBFT_ROLE_USIG, primary, authen_bytes(m, h, MBFT_MSG_PREPARE),
                                  ui_tag(ctr, cert, clen))});
    };
    switch (m.type) {
      case MBFT_MSG_REQUEST:
        request_checks();
        break;
      case MBFT_MSG_REPLY:
        // not a replica-side message: makeMessageValidator panics
        // ("Unknown message type", core/message-handling.go:420-421)
        ck.push_back(Check{MBFT_ST_UNKNOWN_TYPE, 3, kNone});
        break;
      case MBFT_MSG_PREPARE:
        prepare_checks(m.replica_id, m.ui_counter, m.ui_cert, m.ui_cert_len);
        break;
      case MBFT_MSG_COMMIT:
        if (m.replica_id == m.prep_replica_id) {
          ck.push_back(Check{MBFT_ST_COMMIT_FROM_PRIMARY, 1, kNone});
          break;
        }
        prepare_checks(m.prep_replica_id, m.prep_ui_counter, m.prep_ui_cert, m.prep_ui_cert_len);
        if (m.ui_counter == 0) {
          ck.push_back(Check{MBFT_ST_COMMIT_UI, 2, kNone});
          break;
        }
        ck.push_back(Check{MBFT_ST_COMMIT_UI, 0,
                           add_call(MBFT_ROLE_USIG, m.replica_id,
                                    authen_bytes(m, h, MBFT_MSG_COMMIT),
                                    ui_tag(m.ui_counter, m.ui_cert, m.ui_cert_len))});
        break;
      case MBFT_MSG_REQ_VIEW_CHANGE:
        ck.push_back(Check{MBFT_ST_NOT_IMPLEMENTED, 1, kNone});
        break;
    }
  }

  // 3. pure part of every unique call + one GPU batch (batch.cpp)
  std::vector<mbft_item> items(calls.size());
  for (size_t k = 0; k < calls.size(); k++) {
    const Call& cl = calls[k];
    items[k] = mbft_item{cl.role, cl.id, (const uint8_t*)cl.msg.data(), cl.msg.size(),
                         (const uint8_t*)cl.tag.data(), cl.tag.size()};
  }
  std::vector<CallInfo> info(calls.size());
  std::vector<uint8_t> gst(calls.size());
  rc = check_calls(c, items.data(), items.size(), info.data(), gst.data());
  if (rc) return rc;

  // 4. in-order replay: short-circuit per message, stop per stream, stop all
  //    after a panic
  std::unordered_map<uint32_t, bool> stopped;
  bool panicked = false;
  for (size_t i = 0; i < n; i++) {
    if (panicked) {
      out[i] = MBFT_ST_AFTER_PANIC << 8;
      continue;
    }
    const uint32_t sid = msgs[i].stream;
    if (!(flags & MBFT_VF_NO_STREAM_STOP) && stopped.count(sid)) {
      out[i] = MBFT_ST_STREAM_STOPPED << 8;
      continue;
    }
    int32_t res = 0;
    for (const Check& ck : checks[i]) {
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
        if (st == MBFT_MALFORMED_DER && calls[ck.call].role != MBFT_ROLE_USIG &&
            !(flags & MBFT_VF_NO_PANIC_STOP))
          panicked = true;
        break;
      }
    }
    out[i] = res;
    if (res != 0) stopped[sid] = true;
  }
  return MBFT_OK;
}

extern "C" int mbft_validate_replies(mbft_ctx* c, const mbft_message* msgs, size_t n,
                                     uint32_t client_id, uint32_t flags, int32_t* out) {
  if (!c || (n && (!msgs || !out))) return MBFT_ERR_ARG;
  for (size_t i = 0; i < n; i++)
    if (msgs[i].type != MBFT_MSG_REPLY) return MBFT_ERR_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) return MBFT_ERR_HIP;

  // H(result) for every REPLY (GPU SHA stage when the batch is large)
  std::vector<uint8_t> ops;
  std::vector<uint64_t> off{0};
  for (size_t i = 0; i < n; i++) {
    if (msgs[i].op_len) ops.insert(ops.end(), msgs[i].op, msgs[i].op + msgs[i].op_len);
    off.push_back(ops.size());
  }
  std::vector<uint8_t> hops;
  int rc = sha256_many(c, ops, off, hops);
  if (rc) return rc;

  // one ReplicaAuthen call per REPLY whose ClientID matches
  // (client/message-handling.go:163-168), all verified in one GPU batch
  std::vector<uint8_t> checked(n, 0);
  std::vector<std::string> abytes(n);
  std::vector<mbft_item> items;
  std::vector<size_t> call_of(n, 0);
  for (size_t i = 0; i < n; i++) {
    const mbft_message& m = msgs[i];
    if (m.client_id != client_id) continue;
    abytes[i] = authen_bytes(m, &hops[32 * i], MBFT_MSG_REPLY);
    call_of[i] = items.size();
    items.push_back(mbft_item{MBFT_ROLE_REPLICA, m.replica_id, (const uint8_t*)abytes[i].data(),
                              abytes[i].size(), m.sig, m.sig_len});
    checked[i] = 1;
  }
  std::vector<CallInfo> info(items.size());
  std::vector<uint8_t> gst(items.size());
  rc = check_calls(c, items.data(), items.size(), info.data(), gst.data());
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

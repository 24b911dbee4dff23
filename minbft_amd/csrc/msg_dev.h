// The device-side message layer (mbft_validate_messages_flat over library
// page-locked memory): structures shared by msg_kernels.hip and the host
// driver in msgdev.cpp.  What the kernels restate is messages.cpp's host
// message layer, which follows the core validators
// (core/message-handling.go:409-424, core/request.go:146-150,
// core/prepare.go:46-65, core/commit.go:74-92, core/usig-ui.go:62-77).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "kernels.h"
#include "minbft_gpu.h"

namespace mbft {

// One candidate authenticator call of a message (slot 3 i + q of message i):
// who, which AuthenBytes layout over which message's fields, and the tag --
// the ECDSA signature, or for the USIG kinds the UI cert (the UI is
// counter_be64 || cert, usig.MustMarshalUI).
struct MsgCand {
  uint32_t role, id, kind, msg;  // kind: AuthenKind; msg: the message whose fields it reads
  uint32_t primary, tag_len;     // COMMIT: the embedded PREPARE's replica
  uint64_t tag_off;              // into the byte arena
  uint64_t prep_ctr, counter;    // COMMIT: the embedded PREPARE's UI counter; USIG: UI counter
};

// A unique call's host-side outcome for the in-order replay: the layout of
// mbft_host::CallInfo (pre, usig_tail, usig, fpg, ui_epoch, counter), plus
// the call's role in the padding byte (a malformed DER signature panics only
// in an ECDSA role).
struct DevCallInfo {
  uint8_t pre, usig_tail, usig, role;
  uint32_t fpg;
  uint64_t ui_epoch, counter;
};

// Per message, the checks in validator order, packed: bits 0..7 the count
// (<= 3), then 8 bits per check: kind (2: 0 call, 1 fail, 2 zero-counter UI,
// 3 Go panic), stage (4, mbft_stage), candidate q (2: the call is candidate
// slot 3 i + q).
constexpr uint32_t kChkCall = 0, kChkFail = 1, kChkZeroCtr = 2, kChkPanic = 3;

struct MsgDevArgs {
  const mbft_msg_rec* recs;  // device copy of the records (all n)
  const uint8_t* bytes;      // device copy of the byte arena (+16 B of padding)
  uint64_t nbytes;           // arena length (every field must lie inside it)
  long n;
  uint32_t n_replicas;
  uint32_t* chk;             // n: packed checks
  uint32_t* bad;             // 1 word: bit 0 a type out of range, bit 1 a field outside the arena
  MsgCand* cand;             // 3n
  uint64_t* chash;           // 3n: content hash (0: no candidate in this slot)
  uint32_t* cslot;           // 3n: the candidate's dedup-table slot
  uint32_t* uniq;            // 3n: 1 = first occurrence of its content (a unique call)
  uint32_t* ref;             // 3n: the candidate whose call this one is
  uint32_t* idx;             // 3n: exclusive prefix sum of uniq = unique-call number
  uint32_t* call_of;         // 3n: the unique-call number of each candidate
  uint32_t* cand_of;         // unique call k -> its representative candidate
  unsigned long long* tkeys; // dedup table: content hash per slot (0 = empty)
  uint32_t* treps;           // dedup table: smallest candidate slot with that hash
  uint32_t tmask;            // table capacity - 1 (power of two, >= 2 x 3n)
  KeyMap map;                // (role, id) -> key slot
  const KeyDesc* keys;
  uint32_t nslots;
  const uint32_t* fpg;       // per key slot: its USIG fingerprint group
  uint8_t* e;                // per unique call: verifier inputs
  uint8_t* r;
  uint8_t* s;
  uint32_t* slot;
  DevCallInfo* info;
  // the optimistic replay (k_replay_*): messages.cpp replay_parallel on the GPU
  const uint8_t* status;          // per unique call: the verifier's status
  const uint8_t* epoch_set;       // per fingerprint group: the context's USIG epoch state
  const uint64_t* epoch_val;
  uint32_t ngroups;
  unsigned long long* cap_pos;    // per group: first capturing check (3 i + q), ~0 = none
  uint64_t* cap_epoch;            // per group: the epoch that check captures
  int32_t* out;                   // per message: the result
  unsigned long long* first_bad;  // the first message whose result is not 0 (n = none)
};

}  // namespace mbft

namespace mbft {
// A host -> device upload done by k_msg_init's threads (page-locked host
// memory read over PCIe; src and dst 16-B aligned): bytes [0, bytes) copied,
// then words up to `fill` (>= bytes) zeroed past them.
struct MsgUpload {
  uint8_t* dst;
  const uint8_t* src;
  uint64_t bytes, fill;
};
}  // namespace mbft

namespace mbft_launch {
// a pass's zeroed state: flags[0..16), bounds[0], the dedup table (a.tkeys /
// a.treps, a.tmask + 1 slots)
// tail6 (optional): 6 words zeroed too -- the arena's padding, when its upload
// follows on the same stream
// up0 / up1 (optional): uploads done by the same kernel (no copy-engine
// hand-offs for a small pass; then tail6 is null: the upload writes the padding)
hipError_t msg_init(const mbft::MsgDevArgs& a, uint32_t* flags, uint32_t* bounds, hipStream_t st,
                    uint32_t* tail6 = nullptr, const mbft::MsgUpload* up0 = nullptr,
                    const mbft::MsgUpload* up1 = nullptr);
// messages [lo, hi): checks, candidates, content hashes, each candidate into
// the dedup table
hipError_t msg_cands(const mbft::MsgDevArgs& a, long lo, long hi, hipStream_t st);
// every candidate of messages [lo, hi) against its table representative
// (full comparison).  Exact as soon as the table holds the candidates of
// messages [0, hi): a slot keeps its smallest candidate, and the candidates of
// later messages (larger indices) never lower it.
hipError_t msg_dedup_resolve(const mbft::MsgDevArgs& a, long lo, long hi, hipStream_t st);
// idx = exclusive prefix sum of uniq over the 3 (hi - lo) slots of messages
// [lo, hi), numbered from 0; tmp == nullptr: *tmp_bytes receives the scratch
// size for up to `maxn` messages
hipError_t msg_scan(const mbft::MsgDevArgs& a, long lo, long hi, long maxn, void* tmp,
                    size_t* tmp_bytes, hipStream_t st);
// chunk j = messages [lo, hi), after msg_scan: its calls numbered from
// bounds[j] (device; bounds[j + 1] = bounds[j] + its unique calls)
hipError_t msg_number(const mbft::MsgDevArgs& a, long lo, long hi, uint32_t* bounds, int j,
                      hipStream_t st);
// msg_scan + msg_number + the call list of msg_calls in ONE single-workgroup
// launch, for a chunk of at most kNumberOneMax candidate slots (3 per
// message: 1,365 messages).  Each thread walks a run of up to 4 slots; longer
// runs made the one workgroup slower than the three launches it replaces
// (4,096 messages: 434-447 against 406-418 us, profiles/round6_number_one_ab.json).
constexpr long kNumberOneMax = 4096;
hipError_t msg_number_one(const mbft::MsgDevArgs& a, long lo, long hi, uint32_t* bounds, int j,
                          hipStream_t st);
// messages [lo, hi), numbered (msg_number): their candidates' call_of, their
// unique calls' list (skipped when `listed`: msg_number_one did it), and those
// calls [base, base + cnt) decoded (one dense lane each)
// (cnt_dev: the unique-call count on the device, cnt only an upper bound)
hipError_t msg_calls(const mbft::MsgDevArgs& a, long lo, long hi, long base, long cnt, hipStream_t st,
                     const uint32_t* cnt_dev = nullptr, bool listed = false);
// the optimistic in-order replay: every message's result as if no stream had
// stopped and nothing had panicked, the epoch state of each key group taken
// from its first capturing check; exact up to first_bad (cap_pos / first_bad
// initialized to ~0 / n by the caller)
hipError_t msg_replay(const mbft::MsgDevArgs& a, hipStream_t st);
}  // namespace mbft_launch

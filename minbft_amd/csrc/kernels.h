// Host-side launch wrappers for the kernels in kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace mbft {
// Per key slot, read by k_verify (16 B): the key's comb table, its window and
// whether the key passed validation.
struct KeyDesc {
  const uint32_t* tab;
  uint32_t wbits;
  uint32_t valid;
};
// Key slots >= kHostSlot carry a status the host decided for the item
// (batch pipeline): k_verify writes the slot's low byte as the status.
constexpr uint32_t kHostSlot = 0xFFFFFF00u;
}  // namespace mbft

namespace mbft {
// One ECDSA input e built on the GPU from a message's raw fields and the
// SHA-256 of its operation (mbft_validate_messages / _replies; k_authen_e).
enum AuthenKind : uint32_t {
  kAuthenRequest = 0,  // e = ("REQUEST" || seq || H(op) || SHA256(""))[0:32]
  kAuthenReply = 1,    // e = ("REPLY" || client || seq || H(result) || ...)[0:32]
  kAuthenPrepare = 2,  // e = SHA256(SHA256("PREPARE" || view || client || seq || H(op))
                       //            || epoch_le || counter_le)
  kAuthenCommit = 3    // same over "COMMIT" || primary || view || client || seq || H(op) || prep_ctr
};
struct AuthenDesc {
  uint32_t kind, msg;        // kind, index of the message's H(op)
  uint32_t item, client;     // destination item of e; client id
  uint32_t primary, pad;
  uint64_t view, seq, prep_ctr, epoch, counter;
};
}  // namespace mbft

namespace mbft {
// (role, id) -> key slot on the device, for k_prepare: open addressing over
// keys[] = (role << 32) | id (empty: ~0), cap = mask + 1 a power of two at
// load <= 1/2, linear probing.  role_ok bit r: role r has a verification
// scheme in this context (Replica / Client registered; USIG registered and
// enabled), exactly the host's keymanager.go:100 / authenticator.go:126-129
// dispatch.
struct KeyMap {
  const uint64_t* keys;
  const uint32_t* slots;
  uint32_t mask;
  uint32_t role_ok;
};
__host__ __device__ inline uint32_t keymap_hash(uint64_t k) {
  return (uint32_t)((k * 0x9E3779B97F4A7C15ull) >> 32);
}
// Raw VerifyMessageAuthenTag calls i in [0, n) of one chunk, decoded on the
// GPU (mbft_verify_batch_flat over library-owned page-locked buffers): call
// i = (roles[i], ids[i], msgs + moff[i] - mbase .. moff[i + 1] - mbase, tags
// likewise).  Outputs the verifier's items: e, r, s (32 B big-endian each)
// and the key slot, or kHostSlot | status where the call is decided before
// the signature check (kHostSlot | MBFT_BAD_KEY where the host's USIG epoch
// step decides it).
struct PrepArgs {
  const uint32_t* roles;    // wide form (or null: roles8)
  const uint32_t* ids;
  const uint64_t* moff;     // wide form (or null: moff32 / toff32)
  const uint64_t* toff;
  const uint8_t* roles8;    // compact form (mbft_verify_batch_flat32)
  const uint32_t* moff32;
  const uint32_t* toff32;
  const uint8_t* msgs;
  const uint8_t* tags;
  uint64_t mbase, tbase;    // absolute offset of msgs[0] / tags[0]
  uint64_t mlo, mhi, tlo, thi;  // this chunk's byte ranges (absolute): a call outside sets *bad
  uint32_t* bad;
  long n;
  KeyMap map;
  const KeyDesc* keys;
  uint32_t nslots;
  uint8_t* e;
  uint8_t* r;
  uint8_t* s;
  uint32_t* slot;
};
}  // namespace mbft

namespace mbft {
// The resident single-call verifier (k_verify_server, resident.cpp): a kernel
// that stays on the GPU while single calls keep arriving, two 256-thread
// workgroups per mailbox slot in host-mapped memory.  The host fills a slot's
// fields, then its seq (24 bits, never 0); the workgroups see the new seq,
// run the item's comb sums, and write (seq << 8) | status to the slot's done
// words.  No launch and no stream synchronize per call.
constexpr int kSrvMaxSlots = 64;
constexpr int kSrvMaxParts = 16;  // partial sums per item (two workgroups, 8 each)
struct alignas(256) SrvSlot {
  uint32_t seq;           // written last by the host
  uint32_t key0;          // 0: the item's index into kd
  uint32_t wg;            // generator window
  uint32_t ugiven;        // 1: u[] holds u1, u2 (computed by the host)
  const uint32_t* tabG;   // generator comb table (per item: it may be rebuilt)
  uint32_t gjoin;         // 1: the joins and the x test on the GPU, a final status (no partials)
  uint32_t pad1;
  KeyDesc kd;             // the signer's table (offset 32)
  uint8_t e[32], r[32], s[32];  // offsets 48, 80, 112 (16-B aligned)
  uint32_t winv[12];      // s^-1 R mod N, 9 limbs (planes of one item)
  uint32_t u[16];         // u1 = e s^-1, u2 = r s^-1 mod N, 8 LE words each (ugiven)
};
static_assert(sizeof(SrvSlot) == 256 && __builtin_offsetof(SrvSlot, kd) == 32 &&
                  __builtin_offsetof(SrvSlot, e) == 48 && __builtin_offsetof(SrvSlot, winv) == 144 &&
                  __builtin_offsetof(SrvSlot, u) == 192,
              "mailbox slot layout");
// A post's tag from its seq: 1..255, the next post's tag always the
// successor t % 255 + 1 of this one's (seq steps by one per post, skipping
// 0); the servers open a job only for the successor of its claim.
inline uint32_t srv_tag(uint32_t seq) { return seq % 255u + 1u; }
struct SrvCtl {
  // the doorbell line: slot b's post tag in byte b (srv_tag of its seq; 0:
  // never posted), written by the host after the slot and its seq
  uint32_t tag32[kSrvMaxSlots / 4];
  uint32_t exited_gen;    // kernel: the generation that decided to exit
  uint32_t stop_gen;      // host: the generation told to stop (set_resident(0), destroy)
  uint32_t pad1[14];
  // (seq << 8) | status, one cache line per slot: word 0, and word 8 for the
  // second workgroup of the two-workgroup form
  uint32_t done[kSrvMaxSlots][16];
  // status kSrvPartials: the item's partial comb sums, one per wave (G's
  // window ranges, then Q's), 40 words each -- X, Y, ZZ, ZZZ (9 device limbs
  // each, Montgomery form), a flags word (1: infinity) -- for the host to
  // join and x-check (join_host.cpp); 4 sums, or 16 in the two-workgroup form
  // (unused ones flagged infinity)
  uint32_t part[kSrvMaxSlots][kSrvMaxParts * 40];
};
constexpr uint8_t kSrvPartials = 0xFE;
struct ServerArgs {
  SrvCtl* ctl;        // device views of the host-mapped control block
  SrvSlot* slots;     // ... and mailbox
  uint8_t* st;        // device scratch: each slot's status byte
  uint32_t* dexit;    // device: [0] generation told to exit, [2..3] last activity (u64)
  uint32_t* claim;    // device: [half * kSrvMaxSlots + b] the tag of slot b's last claimed job
  uint32_t gen;       // this launch's generation (never 0)
  uint32_t nslots;    // mailbox slots (1..kSrvMaxSlots)
  uint64_t idle_ticks;   // exit after this long without a post (100 MHz ticks)
  uint64_t life_ticks;   // ... or this long after the start
  uint32_t poll_sleep;   // s_sleep(8) steps between two empty doorbell polls (>= 1)
  uint32_t pad;
};
}  // namespace mbft

namespace mbft_launch {

using mbft::AuthenDesc;
using mbft::KeyDesc;
using mbft::PrepArgs;

hipError_t prepare_calls(const PrepArgs& a, hipStream_t st);

// Comb windows: W bits per SIGNED digit, S = ceil(256/W) windows, 2^(W-1)
// affine entries per window (|d|; the last window holds the 2^(256-(S-1)W)
// its digits reach), 64 B per entry.  W = 8 -> 32 mixed additions per
// scalar, 0.25 MiB; 16 -> 16 additions, 34 MiB; 20 -> 13, 388 MiB;
// 22 -> 12, 1.4 GiB; 24 -> 11, 5.0 GiB; 26 -> 10, 18.3 GiB; 29 -> 9, 129 GiB.
constexpr int kMinWindow = 4, kMaxWindow = 29;
size_t table_entries(int wbits);
size_t table_words(int wbits);
int table_steps(int wbits);

hipError_t sha256_var(const uint8_t* data, const uint64_t* off, long n, uint8_t* out,
                      hipStream_t st);
hipError_t usig_e(const uint8_t* data, const uint64_t* off, const uint64_t* epoch,
                  const uint64_t* counter, const uint32_t* idx, long n, uint8_t* e,
                  hipStream_t st);
hipError_t request_e(const uint64_t* seq, const uint8_t* ops, uint32_t op_len, long n, uint8_t* e,
                     hipStream_t st);
hipError_t authen_e(const uint8_t* H, const AuthenDesc* d, long n, uint8_t* e, hipStream_t st);
hipError_t check_points(const uint32_t* xy, int n, uint32_t* ok, hipStream_t st);
hipError_t build_tables(const uint32_t* xy, int npts, int wbits, uint32_t* bpts, uint32_t* tab,
                        hipStream_t st);
hipError_t generator_xy(uint32_t* xy16, hipStream_t st);
size_t ninv_workspace_words(long n);
// One launch, one root inversion per 2,048 items (k_ninv_block, per workgroup;
// MBFT_NINV_FORM=wave: per wave, k_ninv_local): for a batch issued while
// the GPU is idle (latency), not for the steady-state pipeline (VALU work).
// zero_word (optional): zeroed by the kernel (the exact-path queue counter
// of the verify that follows on the same stream).
hipError_t batch_inverse_s_local(const uint8_t* s, long n, uint32_t* winv, uint32_t* zero_word,
                                 hipStream_t st);
// The pipelined form (earlier batches in flight): per-wave chains of 16.
hipError_t batch_inverse_s_pipelined(const uint8_t* s, long n, uint32_t* winv, uint32_t* zero_word,
                                     hipStream_t st);
// The level chain for the pipeline (k_ninv_up / k_ninv_top / k_ninv_down);
// zero_word as above (zeroed by the last kernel of the chain).
hipError_t batch_inverse_s(const uint8_t* s, long n, uint32_t* ws, uint32_t* winv,
                           uint32_t* zero_word, hipStream_t st);
hipError_t sign(const uint8_t* priv, const uint32_t* key_idx, const uint8_t* e, const uint8_t* k_in,
                long n, const uint32_t* tabG, int wg, uint8_t* r_out, uint8_t* s_out,
                hipStream_t st);
// words of the `slowq` buffer verify() needs for n items (exact-path queue,
// its length, the rare comb steps' scratch; `pairs`: the small-batch kernels,
// up to four threads per item)
size_t verify_words(long n, bool pairs = false);
size_t verify_scratch_offset(long n);
hipError_t verify(const uint8_t* e, const uint8_t* r, const uint8_t* s, const uint32_t* slot,
                  const uint32_t* winv, const uint32_t* tabG, int wg, const KeyDesc* keys,
                  uint32_t nslots, long n, uint8_t* status, uint32_t* slowq, hipStream_t st,
                  bool host_status = false, bool queue_zeroed = false, long split_max = -1,
                  bool split_winv = false, const uint32_t* ndev = nullptr,
                  uint32_t* planes_ws = nullptr, int small_form = -1);
// (planes_ws: 9 n words the small-batch forms may use for the batched s^-1
// planes; small_form: their form, mbft_set_small_batch_inverse's modes)
// The resident verifier: one 256-thread workgroup per mailbox slot, or two
// (`two`: one per scalar, each on its own CU).
hipError_t verify_server(const mbft::ServerArgs& a, int servers, bool two, hipStream_t st);

}  // namespace mbft_launch

// Internal declarations shared by the host translation units of
// libminbft_amd.so (host.cpp: context, key store, batch verifier, C-ABI;
// messages.cpp: AuthenBytes and the MinBFT validators).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <array>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/minbft_gpu.h"
#include "kernels.h"
#include "sha256.h"

namespace mbft_host {

constexpr int kVersion = 1;

extern const uint8_t kPkixPrefix[26];
extern const uint8_t kEmptyHash[32];  // SHA256("")

inline void sha256(const uint8_t* p, size_t n, uint8_t out[32]) {
  mbft::Sha256 h;
  h.init();
  h.update(p, n);
  h.final(out);
}

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

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = bytes < 4096 ? 4096 : bytes;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
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
};

}  // namespace mbft_host

struct mbft_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  std::mutex mu;

  // Comb tables.  The generator table is built at create time
  // (and rebuilt by mbft_set_generator_window); each registration call that
  // brings new valid keys allocates one block holding their tables.  d_keys
  // mirrors `slots` on the device as KeyDesc {table, window, valid}.
  uint32_t* d_tabG = nullptr;
  int g_wbits = 16;  // generator comb window (16: 64 MiB, 26: 36 GiB)
  int q_wbits = 16;  // key comb window for keys registered from now on
  std::vector<void*> tab_blocks;
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

  std::map<uint32_t, std::map<uint32_t, mbft_host::KeyEntry>> roles;  // role -> id -> key
  bool usig_enabled = false;
  std::map<uint64_t, uint64_t> usig_epoch;  // fingerprint -> captured epoch
  std::map<uint32_t, std::array<uint8_t, 32>> priv;

  // scratch
  mbft_host::DevBuf e, r, s, slot, status, xy, ok, bpts, priv_d;
  mbft_host::DevBuf sha_data, sha_off, sha_out, sha_ep, sha_ctr;

  // Batched-inverse pipeline: s^-1 of batch i+1 runs on `istream` while the
  // verify kernel of batch i runs on the caller's stream; the s^-1 planes and
  // workspace are double-buffered and guarded by events.
  hipStream_t istream = nullptr;
  mbft_host::DevBuf winv[2], ws[2];
  hipEvent_t ev_in = nullptr, ev_inv[2] = {nullptr, nullptr}, ev_done[2] = {nullptr, nullptr};
  int pipe = 0;

  // profiling (HIP events around the kernels of each batch)
  bool prof = false;
  struct Ev {
    hipEvent_t a, b, c, d;
    size_t n;
  };
  std::vector<Ev> evs;
  double prof_verify_ms = 0, prof_inv_ms = 0, prof_batches = 0, prof_items = 0;
};

namespace mbft_host {

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
                  const uint32_t* d_slot, size_t n, uint8_t* d_status, hipStream_t st);
int verify_host(mbft_ctx* c, const uint8_t* e, const uint8_t* r, const uint8_t* s,
                const uint32_t* slots, size_t n, uint8_t* status);

// One VerifyMessageAuthenTag call split into a pure part (everything that
// depends only on the call's own bytes, including the GPU signature check)
// and the stateful USIG epoch step, applied later in call order.
struct CallInfo {
  uint8_t pre = 0xFF;        // final status decided on the host, or 0xFF
  bool usig = false;
  uint64_t fp = 0, ui_epoch = 0, counter = 0;
  uint8_t usig_tail = 0xFF;  // DER outcome if the epoch matches (USIG)
  int64_t gpu = -1;          // GPU item index, or -1
};

// GPU work collected from many calls; USIG digests may be deferred to the
// GPU SHA stage (k_usig_e) when there are many.
struct GpuWork {
  std::vector<uint8_t> e, r, s;
  std::vector<uint32_t> slot;
  // deferred USIG digests: GPU item index + message bytes + epoch/counter
  std::vector<int64_t> u_item;
  std::vector<uint8_t> u_data;
  std::vector<uint64_t> u_off{0}, u_epoch, u_ctr;
};

void prepare_call(mbft_ctx* c, const mbft_item& it, CallInfo& ci, GpuWork& w, bool defer_usig);
int run_gpu_work(mbft_ctx* c, GpuWork& w, std::vector<uint8_t>& gst);
uint8_t resolve_call(mbft_ctx* c, const CallInfo& ci, const std::vector<uint8_t>& gst);
// Thresholds for the GPU SHA stage (env MBFT_GPU_SHA_MIN_BYTES,
// MBFT_GPU_USIG_MIN_CALLS; defaults 1 MiB of message bytes, 4096 USIG calls).
size_t gpu_sha_min_bytes();
size_t gpu_usig_min_calls();
// SHA-256 of many byte strings (GPU when the batch is large): out n x 32 B
int sha256_many(mbft_ctx* c, const std::vector<uint8_t>& data, const std::vector<uint64_t>& off,
                std::vector<uint8_t>& out);

}  // namespace mbft_host

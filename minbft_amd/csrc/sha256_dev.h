// Device-side SHA-256 message feeders (one message per lane, state in VGPRs).
//
// sha256_msg: hashes `len` bytes at a global pointer with the standard
// padding, 32-bit loads where a word lies inside the message and the pointer
// is 4-byte aligned (the common case), byte loads otherwise.  Digest words
// are returned big-endian-numeric (h[0] = first 4 digest bytes).
#pragma once
#include "sha256.h"

namespace mbft {

// word j (0..15) of 64-byte block b of the padded message
__device__ __forceinline__ uint32_t sha_pad_word(const uint8_t* p, uint32_t len, bool aligned,
                                                 uint64_t base, bool last, int j,
                                                 uint64_t bits) {
  if (last && j == 14) return (uint32_t)(bits >> 32);
  if (last && j == 15) return (uint32_t)bits;
  if (aligned && base + 4 <= len)
    return __builtin_bswap32(*reinterpret_cast<const uint32_t*>(p + base));
  uint32_t w = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint64_t idx = base + k;
    const uint32_t byte = idx < len ? p[idx] : (idx == len ? 0x80u : 0u);
    w = (w << 8) | byte;
  }
  return w;
}

__device__ __forceinline__ void sha256_msg(uint32_t h[8], const uint8_t* p, uint32_t len) {
  sha256_init(h);
  // 64-bit counts: len + 72 and 64 b wrap in 32 bits for len near 2^32
  const uint64_t nblk = ((uint64_t)len + 9 + 63) / 64;
  const bool aligned = ((uintptr_t)p & 3u) == 0;
  const uint64_t bits = (uint64_t)len * 8u;
#pragma unroll 1
  for (uint64_t b = 0; b < nblk; b++) {
    uint32_t m[16];
    const bool last = b + 1 == nblk;
#pragma unroll
    for (int j = 0; j < 16; j++) m[j] = sha_pad_word(p, len, aligned, 64u * b + 4u * j, last, j, bits);
    sha256_block(h, m);
  }
}

// SHA256(d32 || epoch_le64 || counter_le64) for a 32-byte digest given as
// big-endian-numeric words (usig/sgx/usig-enclave.go:204-214).
__device__ __forceinline__ void sha256_usig_chain(uint32_t out[8], const uint32_t d[8],
                                                  uint64_t epoch, uint64_t counter) {
  uint32_t m[16];
#pragma unroll
  for (int j = 0; j < 8; j++) m[j] = d[j];
  m[8] = __builtin_bswap32((uint32_t)epoch);
  m[9] = __builtin_bswap32((uint32_t)(epoch >> 32));
  m[10] = __builtin_bswap32((uint32_t)counter);
  m[11] = __builtin_bswap32((uint32_t)(counter >> 32));
  m[12] = 0x80000000u;
  m[13] = 0;
  m[14] = 0;
  m[15] = 48u * 8u;
  sha256_init(out);
  sha256_block(out, m);
}

}  // namespace mbft

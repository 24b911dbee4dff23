// Blocked reads of byte fields at any offset in a device buffer whose
// allocation extends at least 3 bytes past every field (the message layer's
// arena, the batch pipeline's message and tag buffers: padded on upload).
// One lane per message has no other latency to hide behind (the whole grid
// is resident at once), so a field is read 8 words per memory wait, or
// staged once into the lane's LDS slot for byte-serial parsing (DER).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sha256.h"

namespace mbft {

__device__ __forceinline__ uint32_t tail_mask(uint32_t nb) {  // low nb bytes, nb in 1..3
  return (1u << (8u * nb)) - 1u;
}

// The nine aligned words covering a block of 8 output words are loaded
// together (indices clamped to the field's last covering word, so nothing
// past it is touched) and funnel-shifted into place.
struct ArenaField {
  const uint32_t* p;  // aligned word holding the first byte
  uint32_t sh;        // bit offset of the first byte in it
  uint32_t last;      // index of the last covering word
};
__device__ __forceinline__ ArenaField arena_field(const uint8_t* b, uint64_t off, uint32_t len) {
  return ArenaField{reinterpret_cast<const uint32_t*>(b + (off & ~3ull)), (uint32_t)(off & 3u) * 8u,
                    (uint32_t)(((off & 3u) + len + 3u) / 4u) - 1u};
}
// output words k0 .. k0 + 7 of the field (little-endian, bytes past its end
// unspecified)
__device__ __forceinline__ void arena_block(const ArenaField& f, uint32_t k0, uint32_t (&o)[8]) {
  uint32_t w[9];
#pragma unroll
  for (int j = 0; j < 9; j++) w[j] = f.p[min(k0 + (uint32_t)j, f.last)];
#pragma unroll
  for (int j = 0; j < 8; j++) o[j] = __builtin_amdgcn_alignbit(w[j + 1], w[j], f.sh);
}

// The same in two steps, so a loop can issue block k + 1's loads before it
// works on block k (one memory wait per field instead of one per block).
__device__ __forceinline__ void arena_load(const ArenaField& f, uint32_t k0, uint32_t (&w)[9]) {
#pragma unroll
  for (int j = 0; j < 9; j++) w[j] = f.p[min(k0 + (uint32_t)j, f.last)];
}
__device__ __forceinline__ void arena_shift(const ArenaField& f, const uint32_t (&w)[9], uint32_t (&o)[8]) {
#pragma unroll
  for (int j = 0; j < 8; j++) o[j] = __builtin_amdgcn_alignbit(w[j + 1], w[j], f.sh);
}

// One load per 64-byte line of the first L lines of [off, off + len), all
// issued before any is waited for, into t (0 past the field): a lane that
// then walks the field block by block (hashing it, 8 words per memory wait)
// finds its lines in the L2 instead of paying a miss -- and a TLB walk --
// per block.  (Addresses stay inside the field's covering lines.)
template <int L>
__device__ __forceinline__ void touch_lines(const uint8_t* b, uint64_t off, uint32_t len, uint32_t (&t)[L]) {
  const uint64_t first = off & ~63ull, end = off + len;
#pragma unroll
  for (int j = 0; j < L; j++) {
    const uint64_t a = first + 64ull * (uint64_t)j;
    t[j] = (len != 0 && a < end) ? *reinterpret_cast<const uint32_t*>(b + (a < off ? (off & ~3ull) : a)) : 0u;
  }
}

// Per-lane LDS slot for a tag's covering words (odd stride: lanes' slots
// start in different banks); 25 words = any field up to 97 bytes.
constexpr int kTagWords = 25;

// The covering words of [off, off + len) into the lane's slot, in one batch
// of loads; false (nothing staged) if the field is empty or does not fit.
// The staged copy of the field starts at byte (off & 3) of the slot.
__device__ __forceinline__ bool stage_field(uint32_t* slot, const uint8_t* b, uint64_t off,
                                            uint32_t len) {
  if (len == 0 || ((off & 3u) + len + 3u) / 4u > (uint64_t)kTagWords) return false;
  const ArenaField f = arena_field(b, off, len);
  uint32_t w[kTagWords];
#pragma unroll
  for (int j = 0; j < kTagWords; j++) w[j] = f.p[min((uint32_t)j, f.last)];
#pragma unroll
  for (int j = 0; j < kTagWords; j++) slot[j] = w[j];
  return true;
}

// SHA-256 of an arena field (standard padding), each 64-byte block's words
// loaded together through arena_block (sha256_msg reads an unaligned field
// byte by byte).
__device__ __forceinline__ void sha256_arena(uint32_t h[8], const uint8_t* b, uint64_t off,
                                             uint32_t len) {
  sha256_init(h);
  // 64-bit block and byte counts: a field may be up to 2^32 - 1 bytes (an
  // arena >= 4 GiB), where len + 72 and 64 blk wrap in 32 bits
  const uint64_t nblk = ((uint64_t)len + 9u + 63u) / 64u;
  // (an empty field may carry any offset: read the arena's first word instead)
  const ArenaField f = len ? arena_field(b, off, len) : arena_field(b, 0, 1u);
  const uint64_t bits = (uint64_t)len * 8u;
  // block blk + 1's words are loaded while block blk is compressed
  uint32_t cur[2][9], nxt[2][9];
  arena_load(f, 0u, cur[0]);
  arena_load(f, 8u, cur[1]);
#pragma unroll 1
  for (uint64_t blk = 0; blk < nblk; blk++) {
    if (blk + 1 < nblk) {
      arena_load(f, (uint32_t)(16u * (blk + 1)), nxt[0]);
      arena_load(f, (uint32_t)(16u * (blk + 1)) + 8u, nxt[1]);
    }
    uint32_t m[16];
#pragma unroll
    for (int half = 0; half < 2; half++) {
      uint32_t o[8];
      arena_shift(f, cur[half], o);
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const uint64_t base = 64u * blk + 32u * (uint32_t)half + 4u * (uint32_t)j;
        uint32_t v = o[j];
        if (base + 4u > len) {
          const uint32_t nb = base >= len ? 0u : (uint32_t)(len - base);  // 0..3 bytes of the field
          v = nb ? v & tail_mask(nb) : 0u;
          if (base + nb == len) v |= 0x80u << (8u * nb);
        }
        m[8 * half + j] = __builtin_bswap32(v);
      }
    }
    if (blk + 1 == nblk) {
      m[14] = (uint32_t)(bits >> 32);
      m[15] = (uint32_t)bits;
    }
    sha256_block(h, m);
#pragma unroll
    for (int half = 0; half < 2; half++)
#pragma unroll
      for (int j = 0; j < 9; j++) cur[half][j] = nxt[half][j];
  }
}

}  // namespace mbft

// Host SHA-256 (FIPS 180-4) for the host parts of the path: the USIG digest
// chain of host-decoded calls (usig/sgx/sgx-usig.go:99-101,
// usig/sgx/usig-enclave.go:204-214), AuthenBytes' SHA256(op) of the small
// message checks (messages/authen.go:78-82), key fingerprints
// (crypto.go:134-144).  Whole 64-byte blocks go through the x86 SHA
// extensions when the CPU has them (CPUID leaf 7, EBX bit 29: sha256rnds2 /
// sha256msg1 / sha256msg2, ~2 cycles a byte), else through sha256.h's
// portable compression; only the final one or two padded blocks are built in
// a stack buffer.  The byte-at-a-time mbft::Sha256 stays the device form.
#include <cpuid.h>
#include <immintrin.h>

#include "host_internal.h"

namespace mbft_host {

bool cpu_has_shani() {
  unsigned a = 0, b = 0, c = 0, d = 0;
  if (!__get_cpuid(1, &a, &b, &c, &d)) return false;
  const bool ssse3 = (c >> 9) & 1u, sse41 = (c >> 19) & 1u;
  if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return false;
  return ssse3 && sse41 && ((b >> 29) & 1u);
}

namespace {

// Env MBFT_HOST_SHA=portable forces the portable compression (A/B only).
int default_form() {
  static const int f = [] {
    const char* v = getenv("MBFT_HOST_SHA");
    if (v && strcmp(v, "portable") == 0) return 0;
    return cpu_has_shani() ? 1 : 0;
  }();
  return f;
}

void blocks_portable(uint32_t st[8], const uint8_t* p, size_t nb) {
  for (size_t k = 0; k < nb; k++, p += 64) {
    uint32_t w[16];
    for (int i = 0; i < 16; i++)
      w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) | ((uint32_t)p[4 * i + 2] << 8) |
             p[4 * i + 3];
    mbft::sha256_block(st, w);
  }
}

alignas(16) const uint32_t kK[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

// The state lives as (A B E F) and (C D G H) across the blocks, the layout
// sha256rnds2 works on.  Each group of 4 rounds: W + K, two sha256rnds2 (two
// rounds each); message words 16.. from the previous four groups:
// W[i] = msg2(msg1(W[i-4], W[i-3]) + (W[i-2] : W[i-1] shifted by one word), W[i-1]).
__attribute__((target("sha,sse4.1,ssse3"))) void blocks_shani(uint32_t st[8], const uint8_t* p, size_t nb) {
  const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bll, 0x0405060700010203ll);
  __m128i t = _mm_loadu_si128(reinterpret_cast<const __m128i*>(st));       // D C B A
  __m128i s1 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(st + 4));  // H G F E
  t = _mm_shuffle_epi32(t, 0xB1);                                          // C D A B
  s1 = _mm_shuffle_epi32(s1, 0x1B);                                        // E F G H
  __m128i s0 = _mm_alignr_epi8(t, s1, 8);                                  // A B E F
  s1 = _mm_blend_epi16(s1, t, 0xF0);                                       // C D G H
  for (size_t k = 0; k < nb; k++, p += 64) {
    const __m128i abef = s0, cdgh = s1;
    __m128i w[4];
    for (int g = 0; g < 16; g++) {
      __m128i x;
      if (g < 4) {
        x = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(p + 16 * g)), bswap);
      } else {
        const __m128i a4 = w[g & 3], a3 = w[(g + 1) & 3], a2 = w[(g + 2) & 3], a1 = w[(g + 3) & 3];
        x = _mm_sha256msg1_epu32(a4, a3);
        x = _mm_add_epi32(x, _mm_alignr_epi8(a1, a2, 4));
        x = _mm_sha256msg2_epu32(x, a1);
      }
      w[g & 3] = x;
      __m128i m = _mm_add_epi32(x, _mm_load_si128(reinterpret_cast<const __m128i*>(kK + 4 * g)));
      s1 = _mm_sha256rnds2_epu32(s1, s0, m);
      m = _mm_shuffle_epi32(m, 0x0E);
      s0 = _mm_sha256rnds2_epu32(s0, s1, m);
    }
    s0 = _mm_add_epi32(s0, abef);
    s1 = _mm_add_epi32(s1, cdgh);
  }
  t = _mm_shuffle_epi32(s0, 0x1B);      // F E B A
  s1 = _mm_shuffle_epi32(s1, 0xB1);     // D C H G
  s0 = _mm_blend_epi16(t, s1, 0xF0);    // D C B A
  s1 = _mm_alignr_epi8(s1, t, 8);       // H G F E
  _mm_storeu_si128(reinterpret_cast<__m128i*>(st), s0);
  _mm_storeu_si128(reinterpret_cast<__m128i*>(st + 4), s1);
}

#ifndef SHA_LANES
#define SHA_LANES 4
#endif
// L independent messages at once, one block of each per step: a lane's
// rounds are one long dependent chain (each sha256rnds2 waits for the
// previous), so four chains in flight fill the unit's pipeline -- ~3x the
// one-stream rate for the small-route digests on the GPU box's EPYC (4
// lanes: 57 -> 32 ns a 48-byte digest, 189 -> 114 ns a 256-byte one;
// tools/sha_x4_bench.cpp, profiles/round6_sha_lanes.txt).
// blk(i, k): lane i's k-th block; every lane has nb blocks.
template <int L, class Blk>
__attribute__((target("sha,sse4.1,ssse3"))) inline void blocks_shani_xl(uint32_t* const* st, size_t nb,
                                                                         Blk&& blk) {
  const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bll, 0x0405060700010203ll);
  __m128i s0[L], s1[L];
  for (int i = 0; i < L; i++) {
    __m128i t = _mm_loadu_si128(reinterpret_cast<const __m128i*>(st[i]));
    __m128i u = _mm_loadu_si128(reinterpret_cast<const __m128i*>(st[i] + 4));
    t = _mm_shuffle_epi32(t, 0xB1);
    u = _mm_shuffle_epi32(u, 0x1B);
    s0[i] = _mm_alignr_epi8(t, u, 8);
    s1[i] = _mm_blend_epi16(u, t, 0xF0);
  }
  for (size_t k = 0; k < nb; k++) {
    const uint8_t* p[L];
    for (int i = 0; i < L; i++) p[i] = blk(i, k);
    __m128i abef[L], cdgh[L], w[L][4];
    for (int i = 0; i < L; i++) {
      abef[i] = s0[i];
      cdgh[i] = s1[i];
    }
    for (int g = 0; g < 16; g++) {
      const __m128i kk = _mm_load_si128(reinterpret_cast<const __m128i*>(kK + 4 * g));
      for (int i = 0; i < L; i++) {
        __m128i x;
        if (g < 4) {
          x = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(p[i] + 16 * g)), bswap);
        } else {
          const __m128i a4 = w[i][g & 3], a3 = w[i][(g + 1) & 3], a2 = w[i][(g + 2) & 3], a1 = w[i][(g + 3) & 3];
          x = _mm_sha256msg1_epu32(a4, a3);
          x = _mm_add_epi32(x, _mm_alignr_epi8(a1, a2, 4));
          x = _mm_sha256msg2_epu32(x, a1);
        }
        w[i][g & 3] = x;
        __m128i m = _mm_add_epi32(x, kk);
        s1[i] = _mm_sha256rnds2_epu32(s1[i], s0[i], m);
        m = _mm_shuffle_epi32(m, 0x0E);
        s0[i] = _mm_sha256rnds2_epu32(s0[i], s1[i], m);
      }
    }
    for (int i = 0; i < L; i++) {
      s0[i] = _mm_add_epi32(s0[i], abef[i]);
      s1[i] = _mm_add_epi32(s1[i], cdgh[i]);
    }
  }
  for (int i = 0; i < L; i++) {
    const __m128i t = _mm_shuffle_epi32(s0[i], 0x1B);
    const __m128i u = _mm_shuffle_epi32(s1[i], 0xB1);
    _mm_storeu_si128(reinterpret_cast<__m128i*>(st[i]), _mm_blend_epi16(t, u, 0xF0));
    _mm_storeu_si128(reinterpret_cast<__m128i*>(st[i] + 4), _mm_alignr_epi8(u, t, 8));
  }
}

// A message's padded tail: its last n % 64 bytes, 0x80, zeros, the bit
// length; returns the tail's block count (1 or 2).
size_t pad_tail(const uint8_t* p, size_t n, uint8_t tail[128]) {
  const size_t full = n / 64, rem = n - 64 * full;
  if (rem) memcpy(tail, p + 64 * full, rem);
  tail[rem] = 0x80;
  const size_t tb = rem + 9 <= 64 ? 1 : 2;
  memset(tail + rem + 1, 0, 64 * tb - rem - 1 - 8);
  put_be64(tail + 64 * tb - 8, (uint64_t)n * 8);
  return tb;
}

}  // namespace

void sha256_many(size_t m, const uint8_t* const* p, const size_t* n, uint8_t* const* out) {
  constexpr int L = SHA_LANES;
  const bool xl = default_form() == 1;
  size_t i = 0;
  if (xl) {
    // L at a time while the next L have the same padded block count
    for (; i + L <= m; i += L) {
      size_t nb[L], full[L];
      alignas(16) uint8_t tail[L][128];
      uint32_t stv[L][8];
      uint32_t* st[L];
      bool same = true;
      for (int j = 0; j < L; j++) {
        full[j] = n[i + j] / 64;
        nb[j] = full[j] + pad_tail(p[i + j], n[i + j], tail[j]);
        same = same && nb[j] == nb[0];
        mbft::sha256_init(stv[j]);
        st[j] = stv[j];
      }
      if (!same) {
        for (int j = 0; j < L; j++) sha256(p[i + j], n[i + j], out[i + j]);
        continue;
      }
      blocks_shani_xl<L>(st, nb[0], [&](int j, size_t k) -> const uint8_t* {
        return k < full[j] ? p[i + j] + 64 * k : tail[j] + 64 * (k - full[j]);
      });
      for (int j = 0; j < L; j++)
        for (int w = 0; w < 8; w++) put_be32(out[i + j] + 4 * w, stv[j][w]);
    }
  }
  for (; i < m; i++) sha256(p[i], n[i], out[i]);
}

void sha256_form(int form, const uint8_t* p, size_t n, uint8_t out[32]) {
  void (*blocks)(uint32_t*, const uint8_t*, size_t) = form == 1 ? blocks_shani : blocks_portable;
  uint32_t st[8];
  mbft::sha256_init(st);
  const size_t full = n / 64;
  if (full) blocks(st, p, full);
  uint8_t tail[128];
  const size_t rem = n - 64 * full;
  if (rem) memcpy(tail, p + 64 * full, rem);
  tail[rem] = 0x80;
  const size_t tb = rem + 9 <= 64 ? 1 : 2;
  memset(tail + rem + 1, 0, 64 * tb - rem - 1 - 8);
  put_be64(tail + 64 * tb - 8, (uint64_t)n * 8);
  blocks(st, tail, tb);
  for (int i = 0; i < 8; i++) put_be32(out + 4 * i, st[i]);
}

void sha256(const uint8_t* p, size_t n, uint8_t out[32]) { sha256_form(default_form(), p, n, out); }

}  // namespace mbft_host

// Test hook (include/minbft_gpu.h): SHA-256 of [data, data + len) through
// the portable compression (form 0) or the SHA extensions (form 1;
// MBFT_ERR_STATE when the CPU lacks them).
extern "C" int mbft_debug_sha256(int form, const uint8_t* data, size_t len, uint8_t out[32]) {
  if ((len && !data) || !out || (form != 0 && form != 1)) return MBFT_ERR_ARG;
  static const bool shani = mbft_host::cpu_has_shani();  // (CPUID may trap to a hypervisor: once)
  if (form == 1 && !shani) return MBFT_ERR_STATE;
  mbft_host::sha256_form(form, data, len, out);
  return MBFT_OK;
}

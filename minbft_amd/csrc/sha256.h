// SHA-256 (FIPS 180-4) usable from host and device code.
//
// On the GPU one message is hashed per lane with the state and the 16-word
// schedule window in registers; messages are fed as big-endian 32-bit words.
// Used for: AuthenBytes' SHA256(op) (messages/authen.go:78-82), the USIG
// digest chain SHA256(SHA256(m) || epoch_le || counter_le)
// (usig/sgx/sgx-usig.go:99-101, usig/sgx/usig-enclave.go:204-214), the USIG
// key fingerprint (sample/authentication/crypto.go:134-144) and the
// deterministic signing nonce.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace mbft {

#define MBFT_HD __host__ __device__ __forceinline__

struct Sha256Consts {
  static MBFT_HD uint32_t k(int i) {
    constexpr uint32_t K[64] = {
        0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u,
        0x923f82a4u, 0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u,
        0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u,
        0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
        0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u,
        0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u,
        0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
        0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
        0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au,
        0x5b9cca4fu, 0x682e6ff3u, 0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u,
        0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
    return K[i];
  }
};

MBFT_HD uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

MBFT_HD void sha256_init(uint32_t h[8]) {
  h[0] = 0x6a09e667u; h[1] = 0xbb67ae85u; h[2] = 0x3c6ef372u; h[3] = 0xa54ff53au;
  h[4] = 0x510e527fu; h[5] = 0x9b05688cu; h[6] = 0x1f83d9abu; h[7] = 0x5be0cd19u;
}

// One compression over 16 big-endian message words.
MBFT_HD void sha256_block(uint32_t h[8], const uint32_t m[16]) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = m[i];
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      const uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
      const uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      w[i & 15] = wi;
    }
    const uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = hh + S1 + ch + Sha256Consts::k(i) + wi;
    const uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    const uint32_t t2 = S0 + mj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d;
  h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// Streaming byte interface (host and device).
struct Sha256 {
  uint32_t h[8];
  uint32_t buf[16];
  uint32_t nbuf;   // bytes in buf
  uint64_t total;  // bytes hashed

  MBFT_HD void init() {
    sha256_init(h);
    nbuf = 0;
    total = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) buf[i] = 0;
  }
  MBFT_HD void put(uint8_t byte) {
    const int wi = nbuf >> 2, sh = 24 - 8 * (nbuf & 3);
    buf[wi] |= (uint32_t)byte << sh;
    nbuf++;
    total++;
    if (nbuf == 64) {
      sha256_block(h, buf);
      nbuf = 0;
#pragma unroll
      for (int i = 0; i < 16; i++) buf[i] = 0;
    }
  }
  MBFT_HD void update(const uint8_t* p, size_t n) {
    for (size_t i = 0; i < n; i++) put(p[i]);
  }
  MBFT_HD void final(uint8_t out[32]) {
    const uint64_t bits = total * 8;
    put(0x80);
    while (nbuf != 56) put(0);
    for (int i = 7; i >= 0; i--) put((uint8_t)(bits >> (8 * i)));
    for (int i = 0; i < 8; i++) {
      out[4 * i + 0] = (uint8_t)(h[i] >> 24);
      out[4 * i + 1] = (uint8_t)(h[i] >> 16);
      out[4 * i + 2] = (uint8_t)(h[i] >> 8);
      out[4 * i + 3] = (uint8_t)(h[i]);
    }
  }
};

}  // namespace mbft

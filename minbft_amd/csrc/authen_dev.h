// AuthenBytes (messages/authen.go:52-76) built in registers from a message's
// raw fields and H(op), then the digest input e of the authenticator call
// that checks it: the ECDSA-role quirk (sample/authentication/crypto.go:121,
// e = (AuthenBytes || SHA256(""))[0:32]) or the USIG chain
// (usig/sgx/sgx-usig.go:99-101, usig-enclave.go:204-214,
// e = SHA256(SHA256(AuthenBytes) || epoch_le || counter_le)).  One call per
// lane; the message bytes sit in big-endian words w[], placed at
// compile-time offsets.  Used by k_authen_e (kernels.hip) and the device
// message layer (msg_kernels.hip).
#pragma once
#include "kernels.h"
#include "sha256_dev.h"

namespace mbft {

template <int NW>
__device__ __forceinline__ void put_byte(uint32_t (&w)[NW], int off, uint32_t b) {
  w[off >> 2] |= (b & 0xFFu) << (24 - 8 * (off & 3));
}
template <int NW>
__device__ __forceinline__ void put_be(uint32_t (&w)[NW], int off, uint64_t v, int len) {
#pragma unroll
  for (int k = 0; k < len; k++) put_byte(w, off + k, (uint32_t)(v >> (8 * (len - 1 - k))));
}
template <int NW>
__device__ __forceinline__ void put_str(uint32_t (&w)[NW], int off, const char* s, int len) {
#pragma unroll
  for (int k = 0; k < len; k++) put_byte(w, off + k, (uint32_t)(uint8_t)s[k]);
}
template <int NW>
__device__ __forceinline__ void put_h(uint32_t (&w)[NW], int off, const uint32_t h[8], int len) {
#pragma unroll
  for (int k = 0; k < len; k++) put_byte(w, off + k, h[k >> 2] >> (24 - 8 * (k & 3)));
}

// SHA-256 of the first len bytes of w (2 blocks: len <= 119), padded here
__device__ __forceinline__ void sha256_w32(uint32_t out[8], uint32_t (&w)[32], int len) {
  put_byte(w, len, 0x80u);
  const int nblk = (len + 9 + 63) / 64;
  w[16 * nblk - 1] = (uint32_t)len * 8u;
  sha256_init(out);
  sha256_block(out, w);
  if (nblk > 1) sha256_block(out, w + 16);
}

// e (big-endian-numeric words: out[0] = bytes 0..3) of one authenticator
// call over the AuthenBytes of `kind` (AuthenKind), given H(op) as
// big-endian-numeric words hw.
__device__ __forceinline__ void authen_digest(uint32_t out[8], uint32_t kind, const uint32_t hw[8],
                                              uint64_t seq, uint32_t client, uint64_t view,
                                              uint32_t primary, uint64_t prep_ctr, uint64_t epoch,
                                              uint64_t counter) {
  uint32_t w[32];
#pragma unroll
  for (int k = 0; k < 32; k++) w[k] = 0;
  if (kind == kAuthenRequest) {
    // "REQUEST" || seq || H[0:17] (the first 32 of the 47 AuthenBytes)
    put_str(w, 0, "REQUEST", 7);
    put_be(w, 7, seq, 8);
    put_h(w, 15, hw, 17);
#pragma unroll
    for (int k = 0; k < 8; k++) out[k] = w[k];
  } else if (kind == kAuthenReply) {
    // "REPLY" || client || seq || H[0:15] (first 32 of 49)
    put_str(w, 0, "REPLY", 5);
    put_be(w, 5, client, 4);
    put_be(w, 9, seq, 8);
    put_h(w, 17, hw, 15);
#pragma unroll
    for (int k = 0; k < 8; k++) out[k] = w[k];
  } else {
    // both layouts are two padded blocks: laid out per kind, hashed once (a
    // wave holding PREPARE and COMMIT calls runs the compression once, not
    // once per kind)
    if (kind == kAuthenPrepare) {
      put_str(w, 0, "PREPARE", 7);  // 59 B
      put_be(w, 7, view, 8);
      put_be(w, 15, client, 4);
      put_be(w, 19, seq, 8);
      put_h(w, 27, hw, 32);
      put_byte(w, 59, 0x80u);
      w[31] = 59u * 8u;
    } else {
      put_str(w, 0, "COMMIT", 6);  // 70 B
      put_be(w, 6, primary, 4);
      put_be(w, 10, view, 8);
      put_be(w, 18, client, 4);
      put_be(w, 22, seq, 8);
      put_h(w, 30, hw, 32);
      put_be(w, 62, prep_ctr, 8);
      put_byte(w, 70, 0x80u);
      w[31] = 70u * 8u;
    }
    uint32_t dig[8];
    sha256_init(dig);
    sha256_block(dig, w);
    sha256_block(dig, w + 16);
    sha256_usig_chain(out, dig, epoch, counter);
  }
}

}  // namespace mbft

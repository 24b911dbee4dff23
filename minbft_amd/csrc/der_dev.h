// Go encoding/asn1 decode of `struct { R, S *big.Int }` for ONE lane, on the
// GPU (k_prepare, the device-side decode of raw VerifyMessageAuthenTag calls)
// and, compiled for the host, in the CPU test that checks it against the
// host parser (der.cpp, mbft_der_parse_sig) rule by rule.  The rules are
// der.cpp's (which cites encoding/asn1, Go 1.11/1.14; decode sites
// sample/authentication/crypto.go:81 and usig/sgx/usig-enclave.go:217):
//  * tag: high-tag-number form -> error; indefinite length -> error;
//    long-form length with a leading zero byte, >= 2^23 before a shift, or
//    < 128 -> error; truncation -> error;
//  * SEQUENCE (universal, constructed, 16) of two INTEGERs (universal,
//    primitive, 2); a field running past its container or a missing S ->
//    error; bytes after S inside the SEQUENCE are ignored;
//  * INTEGER: empty, or 00 followed by < 0x80, or FF followed by >= 0x80 ->
//    error; a negative value or one >= 2^256 decodes (Verify rejects it), as
//    32 zero bytes here, exactly like der.cpp.
// Output: r and s as 32 big-endian bytes each, packed in 8 words in memory
// order (word j = bytes 4j..4j+3 little-endian), ready for one 32-byte store.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mbft {

#define MBFT_DER_HD __host__ __device__ __forceinline__

// One tag + length at p[off]; false on any Go asn1 error.
MBFT_DER_HD bool der_tag_len(const uint8_t* p, uint32_t n, uint32_t& off, uint32_t& ident,
                             uint32_t& length) {
  if (off >= n) return false;
  ident = p[off++];
  if ((ident & 0x1fu) == 0x1fu) return false;  // high tag number
  if (off >= n) return false;
  uint32_t c = p[off++];
  if ((c & 0x80u) == 0) {
    length = c;
    return true;
  }
  const uint32_t nbytes = c & 0x7fu;
  if (nbytes == 0) return false;  // indefinite length
  uint32_t len = 0;
  for (uint32_t i = 0; i < nbytes; i++) {
    if (off >= n) return false;
    c = p[off++];
    if (len >= (1u << 23)) return false;  // length too large
    len = (len << 8) | c;
    if (len == 0) return false;  // superfluous leading zeros
  }
  if (len < 0x80u) return false;  // non-minimal length
  length = len;
  return true;
}

// INTEGER contents p[0 .. len) -> w (32 B big-endian, zeros for a negative
// value or one >= 2^256); false if Go rejects the encoding.
MBFT_DER_HD bool der_int(const uint8_t* p, uint32_t len, uint32_t (&w)[8]) {
#pragma unroll
  for (int j = 0; j < 8; j++) w[j] = 0;
  if (len == 0) return false;
  const uint32_t b0 = p[0];
  if (len > 1) {
    const uint32_t b1 = p[1];
    if ((b0 == 0 && (b1 & 0x80u) == 0) || (b0 == 0xffu && (b1 & 0x80u) != 0)) return false;
  }
  if (b0 & 0x80u) return true;  // negative: r, s <= 0 -> Verify rejects
  // minimal encoding: at most one leading zero byte
  const uint32_t lead = b0 == 0 ? 1u : 0u;
  const uint32_t mag = len - lead;
  if (mag > 32) return true;  // >= 2^256 > N -> Verify rejects
  const uint8_t* v = p + lead;
  const uint32_t pad = 32 - mag;  // output byte k = v[k - pad] for k >= pad
#pragma unroll
  for (int k = 0; k < 32; k++) {
    const uint32_t b = (uint32_t)k >= pad ? (uint32_t)v[k - pad] : 0u;
    w[k >> 2] |= b << (8 * (k & 3));
  }
  return true;
}

MBFT_DER_HD bool der_int_field(const uint8_t* q, uint32_t n, uint32_t& off, uint32_t (&w)[8]) {
  if (off == n) return false;  // sequence truncated
  uint32_t ident, length;
  if (!der_tag_len(q, n, off, ident, length)) return false;
  if (ident != 0x02u) return false;  // universal, primitive, INTEGER
  if (length > n - off) return false;  // data truncated
  const bool ok = der_int(q + off, length, w);
  off += length;
  return ok;
}

// The whole signature: true iff Go's asn1.Unmarshal succeeds; *consumed =
// the SEQUENCE's encoded size (bytes after it are Go's `rest`).  r, s are
// zero on failure.
MBFT_DER_HD bool der_sig(const uint8_t* p, uint32_t len, uint32_t (&r)[8], uint32_t (&s)[8],
                         uint32_t& consumed) {
#pragma unroll
  for (int j = 0; j < 8; j++) r[j] = s[j] = 0;
  consumed = 0;
  uint32_t off = 0, ident, length;
  if (len == 0) return false;
  if (!der_tag_len(p, len, off, ident, length)) return false;
  if (ident != 0x30u) return false;  // universal, constructed, SEQUENCE
  if (length > len - off) return false;
  const uint8_t* q = p + off;
  uint32_t io = 0;
  uint32_t rr[8], ss[8];
  if (!der_int_field(q, length, io, rr) || !der_int_field(q, length, io, ss)) return false;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    r[j] = rr[j];
    s[j] = ss[j];
  }
  consumed = off + length;
  return true;
}

}  // namespace mbft

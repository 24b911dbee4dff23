// Host-side restatement of Go encoding/asn1 for `struct { R, S *big.Int }`
// (the decode at sample/authentication/crypto.go:81 and
// usig/sgx/usig-enclave.go:217).  Product code: this is what the
// authenticator runs, not the test oracle.
//
// Go rules reproduced (encoding/asn1, Go 1.11/1.14):
//  * parseTagAndLength: high-tag-number form -> always an error here (a tag
//    >= 31 can never match SEQUENCE(16)/INTEGER(2)); indefinite length ->
//    error; long-form lengths with a leading zero byte ("superfluous leading
//    zeros"), >= 2^23 before a shift ("length too large"), or < 128
//    ("non-minimal length") -> error; truncation -> error.
//  * outer element must be universal, constructed, tag 16; each field
//    universal, primitive, tag 2; a field running past its container ->
//    "data truncated"; a missing S -> "sequence truncated".
//  * checkInteger: empty -> error; 00 followed by a byte < 0x80, or FF
//    followed by a byte >= 0x80 -> "not minimally-encoded".
//  * extra bytes inside the SEQUENCE after S are ignored; bytes after the
//    SEQUENCE are `rest` (ignored by the ECDSA roles, an error for USIG).
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "../../include/minbft_gpu.h"

namespace {

struct TL {
  int cls;
  bool compound;
  int tag;
  uint64_t length;
};

// returns false on any Go asn1 error
bool parse_tag_len(const uint8_t* b, size_t n, size_t& off, TL& t) {
  if (off >= n) return false;
  uint8_t c = b[off++];
  t.cls = c >> 6;
  t.compound = (c & 0x20) != 0;
  t.tag = c & 0x1f;
  if (t.tag == 0x1f) return false;  // high tag number: parse error or mismatch
  if (off >= n) return false;       // truncated tag or length
  c = b[off++];
  if ((c & 0x80) == 0) {
    t.length = c & 0x7f;
    return true;
  }
  const int nbytes = c & 0x7f;
  if (nbytes == 0) return false;  // indefinite length (not DER)
  uint64_t len = 0;
  for (int i = 0; i < nbytes; i++) {
    if (off >= n) return false;
    c = b[off++];
    if (len >= (1u << 23)) return false;  // length too large
    len = (len << 8) | c;
    if (len == 0) return false;  // superfluous leading zeros
  }
  if (len < 0x80) return false;  // non-minimal length
  t.length = len;
  return true;
}

// INTEGER contents -> 32-byte big-endian if 0 < v < 2^256, else zeros.
bool parse_int(const uint8_t* v, size_t len, uint8_t out[32]) {
  memset(out, 0, 32);
  if (len == 0) return false;  // empty integer
  if (len > 1 && ((v[0] == 0 && (v[1] & 0x80) == 0) || (v[0] == 0xff && (v[1] & 0x80) == 0x80)))
    return false;  // not minimally encoded
  if (v[0] & 0x80) return true;  // negative: Verify rejects (r <= 0)
  size_t i = 0;
  while (i < len && v[i] == 0) i++;
  const size_t mag = len - i;
  if (mag > 32) return true;  // >= 2^256 >= N: Verify rejects
  memcpy(out + 32 - mag, v + i, mag);
  return true;
}

bool parse_int_field(const uint8_t* inner, size_t n, size_t& off, uint8_t out[32]) {
  if (off == n) return false;  // sequence truncated
  TL t;
  if (!parse_tag_len(inner, n, off, t)) return false;
  if (t.cls != 0 || t.tag != 2 || t.compound) return false;  // tags don't match
  if (t.length > n - off) return false;                       // data truncated
  const bool ok = parse_int(inner + off, (size_t)t.length, out);
  off += (size_t)t.length;
  return ok;
}

}  // namespace

extern "C" int mbft_der_parse_sig(const uint8_t* sig, size_t len, uint8_t r32[32],
                                  uint8_t s32[32], size_t* consumed) {
  uint8_t r[32], s[32];
  memset(r32, 0, 32);
  memset(s32, 0, 32);
  if (len == 0 || sig == nullptr) return 0;  // sequence truncated
  size_t off = 0;
  TL t;
  if (!parse_tag_len(sig, len, off, t)) return 0;
  if (t.cls != 0 || t.tag != 16 || !t.compound) return 0;
  if (t.length > len - off) return 0;
  const uint8_t* inner = sig + off;
  const size_t n = (size_t)t.length;
  size_t ioff = 0;
  if (!parse_int_field(inner, n, ioff, r)) return 0;
  if (!parse_int_field(inner, n, ioff, s)) return 0;
  memcpy(r32, r, 32);
  memcpy(s32, s, 32);
  if (consumed) *consumed = off + n;
  return 1;
}

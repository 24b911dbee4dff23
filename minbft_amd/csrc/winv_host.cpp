// The lone calls' s^-1 on the host (declared in host_internal.h): s^-1 R
// mod N in the 29-bit-limb planes k_verify_split reads (A.winv), by
// modinv.h's divsteps with the Montgomery scale folded into the start value.
// A TU of its own so the CPU tests link it alone (tests/csrc/modinv_check.cpp).
// Go's verify inverts s on the CPU too (crypto/ecdsa.Verify, called at
// sample/authentication/crypto.go:86).
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "modinv.h"

namespace mbft_host {

// R mod N (R = 2^261, the 29-bit-limb Montgomery radix mod the group
// order), 8 LE words: the scale of modinv_n_var_scaled below.
static const uint32_t kRmodN[8] = {0x739B55E0u, 0x88C6A7A0u, 0x1D0C2F61u, 0x6320AA4Bu,
                                   0x00000008u, 0x00000000u, 0xFFFFFFE0u, 0x0000001Fu};
static const uint32_t kNwords[8] = {0xFC632551u, 0xF3B9CAC2u, 0xA7179E84u, 0xBCE6FAADu,
                                    0xFFFFFFFFu, 0xFFFFFFFFu, 0x00000000u, 0xFFFFFFFFu};

namespace {

// mod-N Montgomery arithmetic on 4 x 64-bit limbs (R = 2^256), for the
// batched form (Montgomery's trick: 3 products per item, one inversion)
using u128 = unsigned __int128;
const uint64_t kN64[4] = {0xF3B9CAC2FC632551ULL, 0xBCE6FAADA7179E84ULL, 0xFFFFFFFFFFFFFFFFULL,
                          0xFFFFFFFF00000000ULL};
const uint64_t kR1[4] = {0x0C46353D039CDAAFULL, 0x4319055258E8617BULL, 0x0000000000000000ULL,
                         0x00000000FFFFFFFFULL};  // 2^256 mod N
const uint64_t kR2[4] = {0x83244C95BE79EEA2ULL, 0x4699799C49BD6FA6ULL, 0x2845B2392B6BEC59ULL,
                         0x66E12D94F3D95620ULL};  // 2^512 mod N
const uint32_t kR2w[8] = {0xBE79EEA2u, 0x83244C95u, 0x49BD6FA6u, 0x4699799Cu,
                          0x2B6BEC59u, 0x2845B239u, 0xF3D95620u, 0x66E12D94u};
const uint64_t kN0inv = 0xCCD1C8AAEE00BC4FULL;  // -N^-1 mod 2^64

bool geq_n(const uint64_t a[4]) {
  for (int j = 3; j >= 0; j--)
    if (a[j] != kN64[j]) return a[j] > kN64[j];
  return true;
}
void sub_n(uint64_t a[4]) {
  u128 b = 0;
  for (int j = 0; j < 4; j++) {
    const u128 d = (u128)a[j] - kN64[j] - b;
    a[j] = (uint64_t)d;
    b = (d >> 64) & 1;
  }
}
// r = a b 2^-256 mod N (CIOS), inputs < N, output < N; r may alias a or b
void mont_n(uint64_t r[4], const uint64_t a[4], const uint64_t b[4]) {
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      c += (u128)a[j] * b[i] + t[j];
      t[j] = (uint64_t)c;
      c >>= 64;
    }
    c += t[4];
    t[4] = (uint64_t)c;
    t[5] = (uint64_t)(c >> 64);
    const uint64_t m = t[0] * kN0inv;
    c = ((u128)m * kN64[0] + t[0]) >> 64;
    for (int j = 1; j < 4; j++) {
      c += (u128)m * kN64[j] + t[j];
      t[j - 1] = (uint64_t)c;
      c >>= 64;
    }
    c += t[4];
    t[3] = (uint64_t)c;
    t[4] = t[5] + (uint64_t)(c >> 64);
  }
  if (t[4] || geq_n(t)) sub_n(t);
  for (int j = 0; j < 4; j++) r[j] = t[j];
}
// a 2^5 mod N (a < N): five doublings with a conditional subtraction
void times32_n(uint64_t a[4]) {
  for (int k = 0; k < 5; k++) {
    const uint64_t top = a[3] >> 63;
    for (int j = 3; j > 0; j--) a[j] = a[j] << 1 | a[j - 1] >> 63;
    a[0] <<= 1;
    if (top || geq_n(a)) sub_n(a);
  }
}

// big-endian 32 bytes -> 8 LE words; true if 0 < s < N
bool load_s(uint32_t w[8], const uint8_t* b) {
  for (int j = 0; j < 8; j++)
    w[j] = (uint32_t)b[31 - 4 * j] | (uint32_t)b[30 - 4 * j] << 8 | (uint32_t)b[29 - 4 * j] << 16 |
           (uint32_t)b[28 - 4 * j] << 24;
  bool lt = false, nz = false;
  for (int j = 0; j < 8; j++) nz = nz || w[j] != 0;
  for (int j = 7; j >= 0; j--) {
    if (w[j] != kNwords[j]) {
      lt = w[j] < kNwords[j];
      break;
    }
  }
  return nz && lt;
}

// 8 LE words (< 2^256) -> 9 29-bit limbs (fe29.h fe_from_words) at plane
// stride n
void store_planes(uint32_t* planes, size_t n, size_t i, const uint32_t iw[8]) {
  for (int k = 0; k < 9; k++) {
    const int bit = 29 * k, j = bit >> 5, sh = bit & 31;
    const uint64_t x = ((uint64_t)(j + 1 < 8 ? iw[j + 1] : 0u) << 32 | iw[j]) >> sh;
    planes[(size_t)k * n + i] = (uint32_t)x & 0x1FFFFFFFu;
  }
}

// a / 2 mod N (N odd): add N when a is odd, then shift the 257-bit sum
void half_n(uint64_t a[4]) {
  uint64_t c = 0;
  if (a[0] & 1) {
    u128 t = 0;
    for (int j = 0; j < 4; j++) {
      t += (u128)a[j] + kN64[j];
      a[j] = (uint64_t)t;
      t >>= 64;
    }
    c = (uint64_t)t;
  }
  for (int j = 0; j < 3; j++) a[j] = a[j] >> 1 | a[j + 1] << 63;
  a[3] = a[3] >> 1 | c << 63;
}

void load_be64(uint64_t v[4], const uint8_t* b) {
  for (int j = 0; j < 4; j++) {
    uint64_t x = 0;
    for (int k = 0; k < 8; k++) x = x << 8 | b[31 - 8 * j - 7 + k];
    v[j] = x;
  }
}

}  // namespace

// One resident call's scalars (resident.cpp post_slot): s^-1 R planes as
// host_winv(s, 1, ...), and u1 = e s^-1, u2 = r s^-1 mod N (canonical, 8 LE
// words each) for the kernel's comb digits -- crypto/ecdsa.Verify's
// u1 = e w, u2 = r w (Go: verifyGeneric, called at
// sample/authentication/crypto.go:86).  e < 2^256 as it is (CIOS takes
// a < 2^256 when b < N).  Invalid s: zero planes and zero u (the kernel
// rejects the range before reading either).
void host_scalars(const uint8_t* e, const uint8_t* r, const uint8_t* s, uint32_t* planes, uint32_t u[16]) {
  uint32_t w[8], iw[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (!load_s(w, s) || !mbft::modinv_n_var_scaled(iw, w, kRmodN))
    for (int j = 0; j < 8; j++) iw[j] = 0;
  store_planes(planes, 1, 0, iw);
  uint64_t wi[4], a[4], o[4];
  for (int j = 0; j < 4; j++) wi[j] = (uint64_t)iw[2 * j + 1] << 32 | iw[2 * j];
  for (int k = 0; k < 5; k++) half_n(wi);  // s^-1 2^261 -> s^-1 2^256
  for (int h = 0; h < 2; h++) {
    load_be64(a, h ? r : e);
    mont_n(o, a, wi);  // x s^-1 mod N
    for (int j = 0; j < 4; j++) {
      u[8 * h + 2 * j] = (uint32_t)o[j];
      u[8 * h + 2 * j + 1] = (uint32_t)(o[j] >> 32);
    }
  }
}

// One call: the scaled divsteps inversion alone (~2 us).  Several: Montgomery's
// trick in the R = 2^256 domain -- prefix products, ONE scaled inversion of the
// total (c = R^2: the result is already (prod s)^-1 R), the way back -- then
// x 2^5 to the kernel's R = 2^261 form.  Invalid s (0, >= N) count as one and
// get zero planes (the kernel rejects them before reading w).
void host_winv_u(const uint8_t* e, const uint8_t* r, const uint8_t* s, size_t n, uint32_t* planes);
void host_winv(const uint8_t* s, size_t n, uint32_t* planes) { host_winv_u(nullptr, nullptr, s, n, planes); }

// host_winv, and with e, r given also u1 = e s^-1, u2 = r s^-1 mod N after the
// planes (planes + 9 n: 16 LE words an item, zeros for an invalid s) -- the
// batched form has s_i^-1 R in the 2^256 domain on the way back, so each u is
// one more product.
void host_winv_u(const uint8_t* e, const uint8_t* r, const uint8_t* s, size_t n, uint32_t* planes) {
  uint32_t* u = e ? planes + 9 * n : nullptr;
  if (n == 1 && u) {
    host_scalars(e, r, s, planes, u);
    return;
  }
  if (n == 1) {
    uint32_t w[8], iw[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (!load_s(w, s) || !mbft::modinv_n_var_scaled(iw, w, kRmodN))
      for (int j = 0; j < 8; j++) iw[j] = 0;
    store_planes(planes, n, 0, iw);
    return;
  }
  std::vector<uint64_t> a(4 * n), pre(4 * n);
  std::vector<char> ok(n);
  uint64_t acc[4];
  for (int j = 0; j < 4; j++) acc[j] = kR1[j];  // the domain's one
  for (size_t i = 0; i < n; i++) {
    uint32_t w[8];
    ok[i] = load_s(w, s + 32 * i) ? 1 : 0;
    uint64_t* ai = &a[4 * i];
    if (ok[i]) {
      uint64_t v[4];
      for (int j = 0; j < 4; j++) v[j] = (uint64_t)w[2 * j + 1] << 32 | w[2 * j];
      mont_n(ai, v, kR2);  // s R
    } else {
      for (int j = 0; j < 4; j++) ai[j] = kR1[j];
    }
    for (int j = 0; j < 4; j++) pre[4 * i + j] = acc[j];
    mont_n(acc, acc, ai);
  }
  // (prod s)^-1 R = R^2 (prod s R)^-1
  uint32_t tw[8], iw[8];
  for (int j = 0; j < 4; j++) {
    tw[2 * j] = (uint32_t)acc[j];
    tw[2 * j + 1] = (uint32_t)(acc[j] >> 32);
  }
  uint64_t inv[4] = {0, 0, 0, 0};
  if (mbft::modinv_n_var_scaled(iw, tw, kR2w))
    for (int j = 0; j < 4; j++) inv[j] = (uint64_t)iw[2 * j + 1] << 32 | iw[2 * j];
  for (size_t i = n; i-- > 0;) {
    uint64_t wi[4];
    mont_n(wi, inv, &pre[4 * i]);  // s_i^-1 R
    mont_n(inv, inv, &a[4 * i]);
    uint32_t ow[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (u) {
      uint32_t* ui = u + 16 * i;
      for (int h = 0; h < 2; h++) {
        uint64_t a[4], o[4] = {0, 0, 0, 0};
        load_be64(a, (h ? r : e) + 32 * i);
        if (ok[i]) mont_n(o, a, wi);  // x s_i^-1 mod N
        for (int j = 0; j < 4; j++) {
          ui[8 * h + 2 * j] = (uint32_t)o[j];
          ui[8 * h + 2 * j + 1] = (uint32_t)(o[j] >> 32);
        }
      }
    }
    if (ok[i]) {
      times32_n(wi);  // s_i^-1 2^261
      for (int j = 0; j < 4; j++) {
        ow[2 * j] = (uint32_t)wi[j];
        ow[2 * j + 1] = (uint32_t)(wi[j] >> 32);
      }
    }
    store_planes(planes, n, i, ow);
  }
}

}  // namespace mbft_host

// Test hook (CPU): host_scalars of one (e, r, s), 32 B big-endian each.
extern "C" int mbft_debug_host_scalars(const uint8_t* e, const uint8_t* r, const uint8_t* s, uint32_t u[16]) {
  if (!e || !r || !s || !u) return -1;
  uint32_t planes[9];
  mbft_host::host_scalars(e, r, s, planes, u);
  return 0;
}

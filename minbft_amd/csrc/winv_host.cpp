// The lone calls' s^-1 on the host (declared in host_internal.h): s^-1 R
// mod N in the 29-bit-limb planes k_verify_split reads (A.winv), by
// modinv.h's divsteps with the Montgomery scale folded into the start value.
// A TU of its own so the CPU tests link it alone (tests/csrc/modinv_check.cpp).
// Go's verify inverts s on the CPU too (crypto/ecdsa.Verify, called at
// sample/authentication/crypto.go:86).
#include <stddef.h>
#include <stdint.h>

#include "modinv.h"

namespace mbft_host {

// R mod N (R = 2^261, the 29-bit-limb Montgomery radix mod the group
// order), 8 LE words: the scale of modinv_n_var_scaled below.
static const uint32_t kRmodN[8] = {0x739B55E0u, 0x88C6A7A0u, 0x1D0C2F61u, 0x6320AA4Bu,
                                   0x00000008u, 0x00000000u, 0xFFFFFFE0u, 0x0000001Fu};
static const uint32_t kNwords[8] = {0xFC632551u, 0xF3B9CAC2u, 0xA7179E84u, 0xBCE6FAADu,
                                    0xFFFFFFFFu, 0xFFFFFFFFu, 0x00000000u, 0xFFFFFFFFu};

void host_winv(const uint8_t* s, size_t n, uint32_t* planes) {
  for (size_t i = 0; i < n; i++) {
    uint32_t w[8], iw[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const uint8_t* b = s + 32 * i;
    for (int j = 0; j < 8; j++)
      w[j] = (uint32_t)b[31 - 4 * j] | (uint32_t)b[30 - 4 * j] << 8 | (uint32_t)b[29 - 4 * j] << 16 |
             (uint32_t)b[28 - 4 * j] << 24;
    bool lt = false, nz = false;  // 0 < s < N
    for (int j = 0; j < 8; j++) nz = nz || w[j] != 0;
    for (int j = 7; j >= 0; j--) {
      if (w[j] != kNwords[j]) {
        lt = w[j] < kNwords[j];
        break;
      }
    }
    if (!(nz && lt) || !mbft::modinv_n_var_scaled(iw, w, kRmodN))
      for (int j = 0; j < 8; j++) iw[j] = 0;
    // 29-bit limbs (fe29.h fe_from_words), plane k at k n
    for (int k = 0; k < 9; k++) {
      const int bit = 29 * k, j = bit >> 5, sh = bit & 31;
      const uint64_t x = ((uint64_t)(j + 1 < 8 ? iw[j + 1] : 0u) << 32 | iw[j]) >> sh;
      planes[(size_t)k * n + i] = (uint32_t)x & 0x1FFFFFFFu;
    }
  }
}

}  // namespace mbft_host

// The end of a resident-kernel verify on the host (declared in
// host_internal.h; resident.cpp).  k_verify_server leaves the four partial
// comb sums of an item -- u1's low and high windows times G, u2's times Q,
// Chudnovsky (X, Y, ZZ = Z^2, ZZZ = Z^3) in the device's 9 x 29-bit
// Montgomery limbs (R = 2^261) -- in host-mapped memory, and the caller's
// thread joins them and runs crypto/ecdsa.Verify's final test (the point at
// infinity rejects, else accept iff x mod N == r; Go: crypto/ecdsa
// verifyGeneric, called at sample/authentication/crypto.go:86) instead of
// one GPU wave running the three joins and the x-check one product level at
// a time (~10 us of a lone call).  Complete: equal partial sums double,
// opposite ones give infinity.  A TU of its own so the CPU tests link it
// alone (mbft_debug_host_join).
#include <stddef.h>
#include <stdint.h>
#include <string.h>

namespace mbft_host {

namespace join_plain {
namespace {
#include "join_core.inc"
}  // namespace
}  // namespace join_plain

#pragma clang attribute push(__attribute__((target("bmi2,adx"))), apply_to = function)
namespace join_bmi2 {
namespace {
#include "join_core.inc"
}  // namespace
}  // namespace join_bmi2
#pragma clang attribute pop

// part: nparts partial sums, 40 words each: X, Y, ZZ, ZZZ (9 device limbs each),
// then a flags word (1: infinity -- every digit of the range was zero);
// r_be: the signature's r (32 B big-endian, 0 < r < N already checked).
// Returns 0 (accept) or 1 (reject).  The BMI2 / ADX build of the products
// where the CPU has them (~25 % faster per product on the test host).
uint8_t host_join_check(const uint32_t* part, int nparts, const uint8_t* r_be) {
  static const bool fast = __builtin_cpu_supports("bmi2") && __builtin_cpu_supports("adx");
  return fast ? join_bmi2::join(part, nparts, r_be) : join_plain::join(part, nparts, r_be);
}

}  // namespace mbft_host


extern "C" int mbft_debug_host_join(const uint32_t* part, int nparts, const uint8_t* r_be) {
  if (!part || !r_be || nparts < 1 || nparts > 16) return -1;
  return mbft_host::host_join_check(part, nparts, r_be);
}

// Test-only: runs minbft_amd/csrc/modinv.h (the divsteps inversion mod N of
// the batched s^-1 root) on the HOST over caller-given inputs, so the CPU
// test suite can check it against Python big integers (tests/test_modinv.py).
// Built into tests/libmodinv_check.so by __graft_entry__.build().
#include "../../minbft_amd/csrc/modinv.h"
#include "../../minbft_amd/csrc/winv_host.cpp"

extern "C" int modinv_check_run(const uint32_t* x, uint32_t* out, uint8_t* ok, int n) {
  for (int i = 0; i < n; i++) ok[i] = mbft::modinv_n_var(out + 8 * i, x + 8 * i) ? 1 : 0;
  return 0;
}

// the product's host s^-1 R planes (winv_host.cpp, the lone calls' form)
extern "C" int winv_check_run(const uint8_t* s_be, size_t n, uint32_t* planes) {
  mbft_host::host_winv(s_be, n, planes);
  return 0;
}

// ... and with u1 = e s^-1, u2 = r s^-1 after the planes (host_winv_u: the
// split kernel's host-staged scalars)
extern "C" int winv_u_check_run(const uint8_t* e_be, const uint8_t* r_be, const uint8_t* s_be, size_t n,
                                uint32_t* planes) {
  mbft_host::host_winv_u(e_be, r_be, s_be, n, planes);
  return 0;
}

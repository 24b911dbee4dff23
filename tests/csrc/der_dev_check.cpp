// Test-only: runs minbft_amd/csrc/der_dev.h (the per-lane Go encoding/asn1
// decode k_prepare uses on the GPU) on the HOST over caller-given strings,
// so the CPU suite can check it rule by rule against the host parser
// (der.cpp, mbft_der_parse_sig) -- tests/test_der_dev.py.  Built into
// tests/libder_dev_check.so by __graft_entry__.build().
#include <string.h>

#include "../../minbft_amd/csrc/der_dev.h"

extern "C" int der_dev_run(const uint8_t* data, const uint64_t* off, int n, uint8_t* ok,
                           uint8_t* r, uint8_t* s, uint32_t* consumed) {
  for (int i = 0; i < n; i++) {
    uint32_t rw[8], sw[8], used = 0;
    ok[i] = mbft::der_sig(data + off[i], (uint32_t)(off[i + 1] - off[i]), rw, sw, used) ? 1 : 0;
    memcpy(r + 32 * i, rw, 32);  // words hold the bytes in memory order
    memcpy(s + 32 * i, sw, 32);
    consumed[i] = used;
  }
  return 0;
}

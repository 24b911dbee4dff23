// Host-side launch wrappers for the kernels in kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace mbft_launch {

// Comb table for window W bits: (256/W) windows x 2^W digits x (x, y) as 16
// LE words: W = 8 -> 512 KiB, W = 16 -> 64 MiB.
size_t table_words(int wbits);
int generator_window();

hipError_t sha256_var(const uint8_t* data, const uint64_t* off, long n, uint8_t* out,
                      hipStream_t st);
hipError_t usig_e(const uint8_t* data, const uint64_t* off, const uint64_t* epoch,
                  const uint64_t* counter, long n, uint8_t* e, hipStream_t st);
hipError_t request_e(const uint64_t* seq, const uint8_t* ops, uint32_t op_len, long n, uint8_t* e,
                     hipStream_t st);
hipError_t check_points(const uint32_t* xy, int n, uint32_t* ok, hipStream_t st);
hipError_t build_tables(const uint32_t* xy, int npts, int wbits, uint32_t* bpts, uint32_t* tab,
                        hipStream_t st);
hipError_t generator_xy(uint32_t* xy16, hipStream_t st);
size_t ninv_workspace_words(long n);
hipError_t batch_inverse_s(const uint8_t* s, long n, uint32_t* ws, uint32_t* winv,
                           hipStream_t st);
hipError_t sign(const uint8_t* priv, const uint32_t* key_idx, const uint8_t* e, long n,
                const uint32_t* tabG, uint8_t* r_out, uint8_t* s_out, hipStream_t st);
hipError_t verify(const uint8_t* e, const uint8_t* r, const uint8_t* s, const uint32_t* slot,
                  const uint32_t* winv, const uint32_t* tabG, const uint32_t* tabQ,
                  const uint8_t* slot_ok, uint32_t nslots, int q_wbits, long n,
                  uint8_t* status, hipStream_t st);

}  // namespace mbft_launch

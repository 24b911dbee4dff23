// Test-only harness (tests/test_gpu_field.py): runs the library's P-256
// field and group primitives (minbft_amd/csrc/fe29.h, ecc.h) on caller-given
// limb inputs, one case per lane, so that Python can check every result
// against big-integer arithmetic and every documented bound.  Built into
// tests/libfield_check.so by __graft_entry__.build(); never part of the
// product library.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../minbft_amd/csrc/ecc.h"

using namespace mbft;

enum Op : uint32_t {
  OP_MUL = 0, OP_SQR = 1, OP_SUB = 2, OP_NEG = 3, OP_ADD = 4, OP_MUL2 = 5,
  OP_CANON = 6, OP_MULSMALL8 = 7, OP_MADD = 8, OP_DBL = 9, OP_SUB2X = 10,
  OP_MULADD_P5B = 11, OP_MULADD_P2B = 12, OP_SUB5 = 13,
  OP_CHUD_P = 16, OP_CHUD_N = 17, OP_AFF_CHUD_P = 18, OP_AFF_CHUD_N = 19,
  OP_CHUD_LAZY_P = 20, OP_CHUD_LAZY_N = 21, OP_CHUD_LAST_P = 22, OP_CHUD_LAST_N = 23,
  OP_NORM_LAZY = 24
};

// in: per case 6 field elements (9 limbs each): a, b, c, d, e, f
// MADD: (X, Y, Z) = (a, b, c) Jacobian, (x2, y2) = (d, e) affine
// MULADD_P5B: fe_mul_add(a, b, kP5B - c)   (ec_madd_chud's H)
// MULADD_P2B: fe_mul_add(kP2B - a, b, c)   (ec_madd_chud's R' with a negative y2)
// CHUD_P / _N: ec_madd_chud((X, Y, ZZ, ZZZ) = (a, b, c, d), (e, f)), add_s2 = false / true
// AFF_CHUD_P / _N: ec_add_affine_chud((a, b), (e, f)), add_s2 = false / true
// CHUD_LAZY_P / _N: ec_madd_chud<LAZY> (ZZ in and out with lazy low limbs)
// CHUD_LAST_P / _N: ec_madd_chud<LAZY, LAST> (X and ZZ only; Y, ZZZ = inputs)
// NORM_LAZY: fe_norm_lazy(a)
// DBL:  (X, Y, Z) = (a, b, c)
// out: per case 4 field elements (9 limbs each)
__global__ void k_field(const uint32_t* op, const uint32_t* in, uint32_t* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fe v[6];
  for (int k = 0; k < 6; k++)
    for (int l = 0; l < NL; l++) v[k].v[l] = in[(size_t)i * 54 + 9 * k + l];
  fe r0, r1, r2, r3;
  fe_zero(r0); fe_zero(r1); fe_zero(r2); fe_zero(r3);
  switch (op[i]) {
    case OP_MUL: fe_mul(r0, v[0], v[1]); break;
    case OP_SQR: fe_sqr(r0, v[0]); break;
    case OP_SUB: fe_sub(r0, v[0], v[1]); break;
    case OP_NEG: fe_neg(r0, v[0]); break;
    case OP_ADD: fe_add(r0, v[0], v[1]); break;
    case OP_MUL2: fe_mul2(r0, v[0], v[1], v[2], v[3]); break;
    case OP_CANON: r0 = v[0]; fe_canon(r0); break;
    case OP_MULSMALL8: fe_mulsmall(r0, v[0], 8); break;
    case OP_SUB2X: fe_sub_2x(r0, v[0], v[1], v[2]); break;
    case OP_SUB5: fe_sub5(r0, v[0], v[1]); break;
    case OP_MULADD_P5B: {
      fe w;
      for (int l = 0; l < NL; l++) w.v[l] = kP5B[l] - v[2].v[l];
      fe_mul_add(r0, v[0], v[1], w);
      break;
    }
    case OP_MULADD_P2B: {
      fe a;
      for (int l = 0; l < NL; l++) a.v[l] = kP2B[l] - v[0].v[l];
      fe_mul_add(r0, a, v[1], v[2]);
      break;
    }
    case OP_MADD: {
      jac a{v[0], v[1], v[2]};
      ec_madd(a, a, v[3], v[4]);
      r0 = a.X; r1 = a.Y; r2 = a.Z;
      break;
    }
    case OP_CHUD_P:
    case OP_CHUD_N: {
      chud a{v[0], v[1], v[2], v[3]};
      ec_madd_chud(a, a, v[4], v[5], op[i] == OP_CHUD_N);
      r0 = a.X; r1 = a.Y; r2 = a.ZZ; r3 = a.ZZZ;
      break;
    }
    case OP_CHUD_LAZY_P:
    case OP_CHUD_LAZY_N: {
      chud a{v[0], v[1], v[2], v[3]};
      ec_madd_chud<true>(a, a, v[4], v[5], op[i] == OP_CHUD_LAZY_N);
      r0 = a.X; r1 = a.Y; r2 = a.ZZ; r3 = a.ZZZ;
      break;
    }
    case OP_CHUD_LAST_P:
    case OP_CHUD_LAST_N: {
      chud a{v[0], v[1], v[2], v[3]};
      ec_madd_chud<true, true>(a, a, v[4], v[5], op[i] == OP_CHUD_LAST_N);
      r0 = a.X; r1 = a.Y; r2 = a.ZZ; r3 = a.ZZZ;
      break;
    }
    case OP_NORM_LAZY: r0 = v[0]; fe_norm_lazy(r0); break;
    case OP_AFF_CHUD_P:
    case OP_AFF_CHUD_N: {
      chud a;
      ec_add_affine_chud(a, v[0], v[1], v[4], v[5], op[i] == OP_AFF_CHUD_N);
      r0 = a.X; r1 = a.Y; r2 = a.ZZ; r3 = a.ZZZ;
      break;
    }
    case OP_DBL: {
      jac a{v[0], v[1], v[2]};
      ec_dbl(a, a);
      r0 = a.X; r1 = a.Y; r2 = a.Z;
      break;
    }
  }
  for (int l = 0; l < NL; l++) {
    out[(size_t)i * 36 + l] = r0.v[l];
    out[(size_t)i * 36 + 9 + l] = r1.v[l];
    out[(size_t)i * 36 + 18 + l] = r2.v[l];
    out[(size_t)i * 36 + 27 + l] = r3.v[l];
  }
}

extern "C" int field_check_run(const uint32_t* h_op, const uint32_t* h_in, uint32_t* h_out,
                               int n) {
  uint32_t *d_op = nullptr, *d_in = nullptr, *d_out = nullptr;
  if (hipMalloc(&d_op, 4 * (size_t)n) != hipSuccess ||
      hipMalloc(&d_in, 54 * 4 * (size_t)n) != hipSuccess ||
      hipMalloc(&d_out, 36 * 4 * (size_t)n) != hipSuccess)
    return -1;
  int rc = 0;
  if (hipMemcpy(d_op, h_op, 4 * (size_t)n, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(d_in, h_in, 54 * 4 * (size_t)n, hipMemcpyHostToDevice) != hipSuccess)
    rc = -2;
  if (!rc) {
    hipLaunchKernelGGL(k_field, dim3((n + 63) / 64), dim3(64), 0, 0, d_op, d_in, d_out, n);
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(h_out, d_out, 36 * 4 * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess)
      rc = -3;
  }
  (void)hipFree(d_op);
  (void)hipFree(d_in);
  (void)hipFree(d_out);
  return rc;
}

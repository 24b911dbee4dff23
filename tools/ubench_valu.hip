// VALU integer / fp64 issue-rate microbenchmark for gfx950.
//
// Measures the sustained per-CU throughput of the instructions the P-256
// field arithmetic is built from, so that the roofline "peak" used by
// bench.py is a measured number rather than a datasheet guess.  Each thread
// runs NCHAIN independent dependency chains of one instruction inside
// inline asm (so the compiler can neither fold nor re-schedule them), and a
// grid of many waves per SIMD hides the dependent latency.
//
// Output: one JSON line per instruction with lane-ops/s and lane-ops per
// CU per clock (at the nominal 2.4 GHz).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_),       \
              __FILE__, __LINE__);                                            \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

constexpr int NCHAIN = 8;
constexpr int ITERS = 65536;

enum Op { MAD_U64_U32 = 0, MUL_LO_U32, MUL_HI_U32, MAD_U32_U24, FMA_F64,
          ADD_U32, LSHL_ADD_U64, ADD_CO_CHAIN, ADD3_U32, ALIGNBIT, LSHRREV_B64, AND_B32,
          AND_B32_E64, LSHRREV_B32, SUB_U32, CNDMASK_B32, MAD_I64_I32, LSHL_OR_B32, NOPS };
static const char* kNames[NOPS] = {
    "v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u32_u24",
    "v_fma_f64", "v_add_u32", "v_lshl_add_u64", "v_add_co+v_addc(e64,2 chains)",
    "v_add3_u32", "v_alignbit_b32", "v_lshrrev_b64", "v_and_b32 (e32)", "v_and_b32 (e64)",
    "v_lshrrev_b32 (e32)", "v_sub_u32 (e32)", "v_cndmask_b32 (e32, vcc)", "v_mad_i64_i32",
    "v_lshl_or_b32"};
// lane-ops counted per inner step per chain
static const int kOpsPerStep[NOPS] = {1, 1, 1, 1, 1, 1, 1, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1};

template <int OP>
__global__ void __launch_bounds__(256) k_bench(uint64_t* out, uint32_t seed) {
  uint32_t t = threadIdx.x + blockIdx.x * 256u + seed;
  uint64_t a64[NCHAIN];
  uint32_t a32[NCHAIN];
  double f[NCHAIN];
#pragma unroll
  for (int c = 0; c < NCHAIN; c++) {
    a64[c] = (uint64_t)(t * 2654435761u + c) << 7 | c;
    a32[c] = t * 40503u + c * 977u;
    f[c] = (double)(t + c) * 1e-3;
  }
  uint32_t m1 = t | 1u, m2 = t ^ 0x9e3779b9u;
  double g1 = 1.0000001, g2 = 1e-9;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int c = 0; c < NCHAIN; c++) {
      if constexpr (OP == MAD_U64_U32) {
        uint64_t sc;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0"
                     : "+v"(a64[c]), "=s"(sc) : "v"(m1), "v"(m2));
      } else if constexpr (OP == MUL_LO_U32) {
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a32[c]) : "v"(m1));
      } else if constexpr (OP == MUL_HI_U32) {
        asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a32[c]) : "v"(m1));
      } else if constexpr (OP == MAD_U32_U24) {
        asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a32[c]) : "v"(m1), "v"(m2));
      } else if constexpr (OP == FMA_F64) {
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(f[c]) : "v"(g1), "v"(g2));
      } else if constexpr (OP == ADD_U32) {
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a32[c]) : "v"(m1));
      } else if constexpr (OP == LSHL_ADD_U64) {
        uint64_t k = m1;
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a64[c]) : "v"(k));
      } else if constexpr (OP == ADD_CO_CHAIN) {
        // two interleaved 2-word carry chains on distinct SGPR pairs, padded
        // for the VALU-SGPR-write -> VALU-read hazard with independent work.
        uint32_t lo = (uint32_t)a64[c], hi = (uint32_t)(a64[c] >> 32);
        uint64_t c0, c1;
        asm volatile(
            "v_add_co_u32_e64 %0, %2, %0, %4\n\t"
            "v_add_co_u32_e64 %1, %3, %1, %4\n\t"
            "s_nop 1\n\t"
            "v_addc_co_u32_e64 %0, %2, %0, %5, %2\n\t"
            "v_addc_co_u32_e64 %1, %3, %1, %5, %3"
            : "+v"(lo), "+v"(hi), "=&s"(c0), "=&s"(c1) : "v"(m1), "v"(m2));
        a64[c] = ((uint64_t)hi << 32) | lo;
      } else if constexpr (OP == ADD3_U32) {
        asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a32[c]) : "v"(m1), "v"(m2));
      } else if constexpr (OP == ALIGNBIT) {
        asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a32[c]) : "v"(m1));
      } else if constexpr (OP == LSHRREV_B64) {
        asm volatile("v_lshrrev_b64 %0, 29, %0" : "+v"(a64[c]));
      } else if constexpr (OP == AND_B32) {
        asm volatile("v_and_b32_e32 %0, %1, %0" : "+v"(a32[c]) : "v"(m1));
      } else if constexpr (OP == AND_B32_E64) {
        asm volatile("v_and_b32_e64 %0, %0, %1" : "+v"(a32[c]) : "v"(m1));
      } else if constexpr (OP == LSHRREV_B32) {
        asm volatile("v_lshrrev_b32_e32 %0, 3, %0" : "+v"(a32[c]));
      } else if constexpr (OP == SUB_U32) {
        asm volatile("v_sub_u32_e32 %0, %1, %0" : "+v"(a32[c]) : "v"(m1));
      } else if constexpr (OP == CNDMASK_B32) {
        asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a32[c]) : "v"(m1));
      } else if constexpr (OP == MAD_I64_I32) {
        uint64_t sc;
        asm volatile("v_mad_i64_i32 %0, %1, %2, %3, %0"
                     : "+v"(a64[c]), "=s"(sc) : "v"(m1), "v"(m2));
      } else if constexpr (OP == LSHL_OR_B32) {
        asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(a32[c]) : "v"(m1));
      }
    }
  }
  uint64_t acc = 0;
#pragma unroll
  for (int c = 0; c < NCHAIN; c++) {
    acc ^= a64[c] ^ a32[c];
    uint64_t fb;
    memcpy(&fb, &f[c], 8);
    acc ^= fb;
  }
  out[threadIdx.x + blockIdx.x * 256u] = acc;
}

template <int OP>
double run(uint64_t* d_out, int blocks) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_bench<OP>, dim3(blocks), dim3(256), 0, 0, d_out, 1u);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 5; rep++) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_bench<OP>, dim3(blocks), dim3(256), 0, 0, d_out, (uint32_t)rep);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  double lane_ops = (double)blocks * 256.0 * ITERS * NCHAIN * kOpsPerStep[OP];
  double rate = lane_ops / (best * 1e-3);
  int cus = 0;
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  cus = p.multiProcessorCount;
  printf("{\"op\": \"%s\", \"lane_ops_per_s\": %.4e, \"per_cu_per_clk_at_2.4GHz\": %.2f, "
         "\"ms\": %.3f, \"cus\": %d}\n",
         kNames[OP], rate, rate / (cus * 2.4e9), best, cus);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return rate;
}

int main(int argc, char** argv) {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  int blocks = p.multiProcessorCount * 8;  // 8 blocks x 4 waves = 32 waves/CU
  if (argc > 1 && atoi(argv[1]) > 0) blocks = atoi(argv[1]);
  const bool mad_only = argc > 2 && strcmp(argv[2], "mad") == 0;
  uint64_t* d_out;
  CHECK(hipMalloc(&d_out, (size_t)blocks * 256 * sizeof(uint64_t)));
  run<MAD_U64_U32>(d_out, blocks);
  if (mad_only) {
    CHECK(hipFree(d_out));
    return 0;
  }
  run<MUL_LO_U32>(d_out, blocks);
  run<MUL_HI_U32>(d_out, blocks);
  run<MAD_U32_U24>(d_out, blocks);
  run<FMA_F64>(d_out, blocks);
  run<ADD_U32>(d_out, blocks);
  run<LSHL_ADD_U64>(d_out, blocks);
  run<ADD_CO_CHAIN>(d_out, blocks);
  run<ADD3_U32>(d_out, blocks);
  run<ALIGNBIT>(d_out, blocks);
  run<LSHRREV_B64>(d_out, blocks);
  run<AND_B32>(d_out, blocks);
  run<AND_B32_E64>(d_out, blocks);
  run<LSHRREV_B32>(d_out, blocks);
  run<SUB_U32>(d_out, blocks);
  run<CNDMASK_B32>(d_out, blocks);
  run<MAD_I64_I32>(d_out, blocks);
  run<LSHL_OR_B32>(d_out, blocks);
  CHECK(hipFree(d_out));
  return 0;
}

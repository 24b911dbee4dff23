// Calibration of rocprofv3 FETCH_SIZE for the verifier's access pattern
// (MI355X_MICROARCH.md §HBM: the 1/2 factor is calibrated only for wide
// coalesced streaming reads).  Three kernels over a 16 GiB table (far past
// the 256 MiB Infinity Cache), each reading a known byte count with 16-B
// loads:
//   stream   coalesced streaming read of 1 GiB
//   rand64   2^24 random 64-B entries (4 lanes x 16 B each, k_verify's
//            cooperative gather shape: 16 entries per wave instruction)
//   rand128  2^23 random 128-B aligned blocks (8 lanes x 16 B each)
// Run each under `rocprofv3 --pmc FETCH_SIZE` (tools/pmc_gather.sh): the
// FETCH_SIZE per requested byte of rand64 against rand128 tells whether a
// random 64-B entry costs a whole 128-B line from HBM.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t hash64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  return x ^ (x >> 33);
}

__global__ void k_stream(const u32x4* __restrict__ t, size_t n16, u32x4* out) {
  u32x4 acc = {0, 0, 0, 0};
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
       i += (size_t)gridDim.x * blockDim.x) {
    acc ^= __builtin_nontemporal_load(t + i);
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = acc;
}

// LANES lanes read one random aligned block of 16 * LANES bytes
template <int LANES>
__global__ void k_rand(const u32x4* __restrict__ t, size_t nblocks_table, size_t nreq, u32x4* out) {
  u32x4 acc = {0, 0, 0, 0};
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (size_t g = tid / LANES; g < nreq; g += (size_t)gridDim.x * blockDim.x / LANES) {
    const size_t blk = hash64(g * 0x9E3779B97F4A7C15ull + 17) % nblocks_table;
    acc ^= __builtin_nontemporal_load(t + blk * LANES + (tid % LANES));
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = acc;
}

// k_verify's own gather instruction: 16-B chunks of random 64-B entries
// straight into LDS (global_load_lds_dwordx4), with cache policy CPOL
// (SC0 = 1, NT = 2, SC1 = 16), to see which request size each policy makes.
template <int CPOL>
__global__ void __launch_bounds__(256) k_rand64_lds(const u32x4* __restrict__ t, size_t nblocks_table,
                                                    size_t nreq, u32x4* out) {
  __shared__ u32x4 buf[4][64];
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  u32x4 acc = {0, 0, 0, 0};
  for (size_t g = tid / 4; g < nreq; g += (size_t)gridDim.x * blockDim.x / 4) {
    const size_t blk = hash64(g * 0x9E3779B97F4A7C15ull + 17) % nblocks_table;
    __builtin_amdgcn_global_load_lds(t + blk * 4 + (tid % 4), &buf[threadIdx.x >> 6][0], 16, 0, CPOL);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    acc ^= buf[threadIdx.x >> 6][threadIdx.x & 63];
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
  const char* which = argc > 1 ? argv[1] : "all";
  const size_t table = (size_t)16 << 30;
  u32x4* t;
  u32x4* out;
  // argv[2]: table memory type -- default hipMalloc (coarse-grained), "uc"
  // uncached, "fg" fine-grained
  const char* mem = argc > 2 ? argv[2] : "";
  if (!strcmp(mem, "uc"))
    CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&t), table, hipDeviceMallocUncached));
  else if (!strcmp(mem, "fg"))
    CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&t), table, hipDeviceMallocFinegrained));
  else
    CHECK(hipMalloc(&t, table));
  CHECK(hipMalloc(&out, 64));
  CHECK(hipMemset(t, 1, table));
  const dim3 grid(256 * 16), block(256);
  const size_t req = (size_t)1 << 30;  // bytes requested by each kernel
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  auto run = [&](const char* name, auto launch) {
    if (strcmp(which, "all") && strcmp(which, name)) return;
    launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a, 0));
    launch();
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    printf("{\"kernel\": \"%s\", \"requested_bytes\": %zu, \"ms\": %.3f, \"GB_per_s\": %.1f}\n", name, req,
           ms, req / (ms * 1e-3) / 1e9);
  };
  run("stream", [&] { hipLaunchKernelGGL(k_stream, grid, block, 0, 0, t, req / 16, out); });
  run("rand64", [&] {
    hipLaunchKernelGGL(k_rand<4>, grid, block, 0, 0, t, table / 64, req / 64, out);
  });
  run("rand128", [&] {
    hipLaunchKernelGGL(k_rand<8>, grid, block, 0, 0, t, table / 128, req / 128, out);
  });
  const size_t nb = table / 64, nr = req / 64;
  run("lds_cpol0", [&] { hipLaunchKernelGGL(k_rand64_lds<0>, grid, block, 0, 0, t, nb, nr, out); });
  run("lds_cpol1", [&] { hipLaunchKernelGGL(k_rand64_lds<1>, grid, block, 0, 0, t, nb, nr, out); });
  run("lds_cpol2", [&] { hipLaunchKernelGGL(k_rand64_lds<2>, grid, block, 0, 0, t, nb, nr, out); });
  run("lds_cpol3", [&] { hipLaunchKernelGGL(k_rand64_lds<3>, grid, block, 0, 0, t, nb, nr, out); });
  run("lds_cpol16", [&] { hipLaunchKernelGGL(k_rand64_lds<16>, grid, block, 0, 0, t, nb, nr, out); });
  run("lds_cpol17", [&] { hipLaunchKernelGGL(k_rand64_lds<17>, grid, block, 0, 0, t, nb, nr, out); });
  run("lds_cpol18", [&] { hipLaunchKernelGGL(k_rand64_lds<18>, grid, block, 0, 0, t, nb, nr, out); });
  run("lds_cpol19", [&] { hipLaunchKernelGGL(k_rand64_lds<19>, grid, block, 0, 0, t, nb, nr, out); });
  CHECK(hipFree(t));
  CHECK(hipFree(out));
  return 0;
}

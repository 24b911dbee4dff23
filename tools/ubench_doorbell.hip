// Host <-> resident-kernel round trip (round 5, resident verifier design):
// the host writes a sequence number, one GPU wave polling for it writes an
// ack to host-mapped memory, the host spins on the ack.  Mailbox in
// host-mapped memory (mode H: the GPU polls over PCIe) or in fine-grained
// device memory written by the CPU through the BAR (mode D: the GPU polls
// its own memory, the host's write is posted).  Prints the p50 / p10 / p90
// round trip.  Diagnostic only.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_doorbell tools/ubench_doorbell.hip
//   ./tools/ubench_doorbell H ; ./tools/ubench_doorbell D
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

__global__ void pong(const uint32_t* box, uint32_t* ack, int n) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = wall_clock64();
  for (int k = 1; k <= n; k++) {
    for (;;) {
      const uint32_t v = __hip_atomic_load(box, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (v == (uint32_t)k) break;
      if (wall_clock64() - t0 > 300000000ull) return;  // 3 s: give up
      __builtin_amdgcn_s_sleep(1);
    }
    __hip_atomic_store(ack, (uint32_t)k, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

int main(int argc, char** argv) {
  const char mode = argc > 1 ? argv[1][0] : 'H';
  const int n = 20000;
  uint32_t* ack_h = nullptr;
  uint32_t* ack_d = nullptr;
  if (hipHostMalloc((void**)&ack_h, 4096, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return 1;
  if (hipHostGetDevicePointer((void**)&ack_d, ack_h, 0) != hipSuccess) return 1;
  volatile uint32_t* box_host = nullptr;  // what the CPU writes
  uint32_t* box_dev = nullptr;            // what the kernel polls
  if (mode == 'H') {
    uint32_t* h = nullptr;
    if (hipHostMalloc((void**)&h, 4096, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return 1;
    if (hipHostGetDevicePointer((void**)&box_dev, h, 0) != hipSuccess) return 1;
    box_host = h;
  } else {
    if (hipExtMallocWithFlags((void**)&box_dev, 4096, hipDeviceMallocFinegrained) != hipSuccess) {
      printf("D: fine-grained device allocation failed\n");
      return 2;
    }
    hipPointerAttribute_t at;
    memset(&at, 0, sizeof(at));
    const hipError_t e = hipPointerGetAttributes(&at, box_dev);
    printf("D: attributes rc %d hostPointer %p devicePointer %p type %d\n", (int)e, at.hostPointer,
           at.devicePointer, (int)at.type);
    if (!at.hostPointer) {
      printf("D: no host pointer for fine-grained device memory\n");
      return 3;
    }
    box_host = static_cast<volatile uint32_t*>(at.hostPointer);
    if (hipMemset(box_dev, 0, 4096) != hipSuccess) return 1;
  }
  *box_host = 0;
  ack_h[0] = 0;
  hipLaunchKernelGGL(pong, dim3(1), dim3(64), 0, 0, box_dev, ack_d, n);
  std::vector<double> rt;
  rt.reserve(n);
  volatile uint32_t* ack = ack_h;
  for (int k = 1; k <= n; k++) {
    const auto t0 = std::chrono::steady_clock::now();
    *box_host = (uint32_t)k;
    long spins = 0;
    while (*ack != (uint32_t)k) {
      __builtin_ia32_pause();
      if (++spins > 2000000000L) break;
    }
    rt.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  std::sort(rt.begin() + 100, rt.end());
  const size_t m = rt.size() - 100;
  printf("%c: round trip p10 %.2f us  p50 %.2f us  p90 %.2f us  (%d pings)\n", mode, rt[100 + m / 10],
         rt[100 + m / 2], rt[100 + 9 * m / 10], n);
  return 0;
}

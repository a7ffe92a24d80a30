// Per-lane SHA-256 throughput at one vs two waves per SIMD (the question behind k_sha's
// per-lane mode): every lane compresses `blocks` blocks of its own message (register data, no
// memory traffic), one workgroup per CU (LDS padding), 4 or 8 waves per workgroup. Prints the
// chip-wide blocks per microsecond and cycles per wave-block.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include "../../bs_amd/csrc/sha256_device.h"
using namespace bsg;

template <int WAVES>
__global__ __launch_bounds__(64 * WAVES, 1) void k_lanes(uint32_t* out, int blocks, uint32_t seed) {
  extern __shared__ uint32_t pad[];
  if (blocks < 0) pad[threadIdx.x] = 0;  // never: keeps the LDS request
  uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                    0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint32_t W[16];
  const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
  for (int b = 0; b < blocks; ++b) {
#pragma unroll
    for (int i = 0; i < 16; ++i) W[i] = (id * 2654435761u) ^ (seed + 31u * (uint32_t)(b * 16 + i));
    sha256_compress(st, W);
  }
  uint32_t x = 0;
  for (int i = 0; i < 8; ++i) x ^= st[i];
  out[id] = x;
}

template <int WAVES> void run(int cus, int blocks) {
  uint32_t* out;
  (void)hipMalloc(&out, (size_t)cus * 64 * WAVES * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_lanes<WAVES>, dim3(cus), dim3(64 * WAVES), 84 * 1024, 0, out, blocks, 7u);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
  }
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  const double total = (double)cus * 64 * WAVES * blocks;
  printf("%d waves/WG (%d per SIMD): %d blocks/lane, %.3f ms, %.1f blocks/us chip-wide, "
         "%.0f cycles per wave-block at 2.4 GHz\n", WAVES, WAVES / 4, blocks, ms,
         total / (ms * 1e3), ms * 1e-3 * 2.4e9 / blocks);
  (void)hipFree(out);
}

int main() {
  int dev = 0; hipDeviceProp_t p; (void)hipGetDeviceProperties(&p, dev);
  const int cus = p.multiProcessorCount;
  run<4>(cus, 400);
  run<8>(cus, 400);
  run<4>(cus, 400);
  run<8>(cus, 400);
  return 0;
}

// Microbenchmark: how waves sharing one SIMD split VALU issue (every wave timed), with and
// without s_setprio on one of them.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../../bs_amd/csrc/sha256_device.h"
using namespace bsg;

template <int PRIO>
__global__ void kb(uint64_t* out, uint32_t* io, int blocks) {
  const int wave = threadIdx.x / 64;
  if (PRIO && wave == 0) __builtin_amdgcn_s_setprio(3);
  uint32_t st[8], W[16];
  for (int i = 0; i < 8; ++i) st[i] = io[i] + threadIdx.x;
  for (int i = 0; i < 16; ++i) W[i] = io[8 + i] ^ threadIdx.x;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int b = 0; b < blocks; ++b) {
    uint32_t w[16];
    for (int i = 0; i < 16; ++i) w[i] = W[i] ^ st[i & 7];
    sha256_compress_v<true>(st, w);
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t x = 0;
  for (int i = 0; i < 8; ++i) x ^= st[i];
  io[100 + threadIdx.x] = x;
  if ((threadIdx.x & 63) == 0) out[wave] = t1 - t0;
}

template <int PRIO> void run(int waves_per_simd) {
  uint64_t* d; uint32_t* io; hipMalloc(&d, 64 * 8); hipMalloc(&io, 8192 * 4);
  hipMemset(io, 1, 8192 * 4);
  int blocks = 100, threads = 256 * waves_per_simd;  // waves are dealt over the 4 SIMDs
  for (int k = 0; k < 2; ++k) {
    hipLaunchKernelGGL(kb<PRIO>, dim3(1), dim3(threads), 0, 0, d, io, blocks);
    hipDeviceSynchronize();
  }
  uint64_t h[64]; hipMemcpy(h, d, 8 * threads / 64, hipMemcpyDeviceToHost);
  printf("waves/SIMD=%d prio=%d cycles/block per wave:", waves_per_simd, PRIO);
  for (int w = 0; w < threads / 64; ++w) printf(" %.0f", (double)h[w] / blocks);
  printf("\n");
  hipFree(d); hipFree(io);
}
int main() {
  run<0>(1); run<0>(2); run<0>(3); run<0>(4);
  run<1>(2); run<1>(3);
  return 0;
}

// Microbenchmark: cycles per SHA-256 compression for a lone wave (register data, no memory).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../../bs_amd/csrc/sha256_device.h"
using namespace bsg;

#define STAMP(t) asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory")

template <int V>
__global__ void kb(uint64_t* out, uint32_t* io, int blocks) {
  uint32_t st[8], st2[8], W[16], KW[64];
  for (int i = 0; i < 8; ++i) { st[i] = io[i] + threadIdx.x; st2[i] = st[i] * 3; }
  for (int i = 0; i < 16; ++i) W[i] = io[8 + i] ^ threadIdx.x;
  for (int i = 0; i < 64; ++i) KW[i] = io[24 + i] + threadIdx.x;
  uint64_t t0, t1;
  STAMP(t0);
  for (int b = 0; b < blocks; ++b) {
    if (V == 0 || V == 1) {
      uint32_t w[16];
      for (int i = 0; i < 16; ++i) w[i] = W[i] ^ st[i & 7];  // not loop-invariant
      if (V == 0) sha256_compress_v<true>(st, w); else sha256_compress_v<false>(st, w);
    } else if (V == 2 || V == 3) {
      uint32_t kw[64];
      for (int i = 0; i < 64; ++i) kw[i] = KW[i] ^ st[i & 7];
      if (V == 2) sha256_rounds_kw<true>(st, kw); else sha256_rounds_kw<false>(st, kw);
    } else if (V == 4) {  // two independent chains per lane
      uint32_t w[16], w2[16];
      for (int i = 0; i < 16; ++i) { w[i] = W[i] ^ st[i & 7]; w2[i] = W[i] ^ st2[i & 7]; }
      sha256_compress_v<false>(st, w);
      sha256_compress_v<false>(st2, w2);
    }
  }
  STAMP(t1);
  uint32_t x = 0;
  for (int i = 0; i < 8; ++i) x ^= st[i] ^ st2[i];
  io[100 + threadIdx.x] = x;
  if (threadIdx.x == 0) out[0] = t1 - t0;
}

template <int V> void run(const char* name, int wg_threads) {
  uint64_t* d; uint32_t* io; hipMalloc(&d, 16); hipMalloc(&io, 8192 * 4);
  hipMemset(io, 1, 8192 * 4);
  int blocks = 200;
  hipLaunchKernelGGL(kb<V>, dim3(1), dim3(wg_threads), 0, 0, d, io, blocks);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(kb<V>, dim3(1), dim3(wg_threads), 0, 0, d, io, blocks);
  hipDeviceSynchronize();
  uint64_t h; hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  printf("%-48s threads=%4d  %8.0f cycles/block\n", name, wg_threads, (double)h / blocks);
  hipFree(d); hipFree(io);
}

int main() {
  run<0>("compress, asm bitop3/xor3", 64);
  run<1>("compress, plain C", 64);
  run<2>("rounds only (KW given), asm", 64);
  run<3>("rounds only (KW given), plain C", 64);
  run<4>("compress x2 chains/lane (per 2 blocks), C", 64);
  run<1>("compress, plain C, 8 waves (2/SIMD)", 512);
  run<1>("compress, plain C, 16 waves (4/SIMD)", 1024);
  return 0;
}

// Per-lane SHA-256 (k_sha's per-lane compression) on the whole chip, one wave per SIMD (or two:
// argv[1] = 2), message words from registers: hipcc's sha256_compress against the generated asm
// statements (tools/gen_lane_asm.py: V1 aligned, V2 + no st copies, V3 + K through an SGPR; the
// product's sha256_compress_aligned is V3). Prints cycles per block per wave (s_memtime) and
// whether all give the same digests.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include "../../bs_amd/csrc/sha256_device.h"

using namespace bsg;
#include "lane_variants.inc"

#define LANE_FN(NAME, MACRO)                                                                  \
  __device__ __forceinline__ void NAME(uint32_t (&st)[8], uint32_t (&W)[16]) {                \
    uint32_t x0, x1, x2, x3, x4, x5, x6, x7, t0, t1, t2, t3, t4, t5, k;                      \
    asm volatile(MACRO                                                                         \
                 : [st0] "+v"(st[0]), [st1] "+v"(st[1]), [st2] "+v"(st[2]), [st3] "+v"(st[3]), \
                   [st4] "+v"(st[4]), [st5] "+v"(st[5]), [st6] "+v"(st[6]), [st7] "+v"(st[7]), \
                   [w0] "+v"(W[0]), [w1] "+v"(W[1]), [w2] "+v"(W[2]), [w3] "+v"(W[3]),         \
                   [w4] "+v"(W[4]), [w5] "+v"(W[5]), [w6] "+v"(W[6]), [w7] "+v"(W[7]),         \
                   [w8] "+v"(W[8]), [w9] "+v"(W[9]), [w10] "+v"(W[10]), [w11] "+v"(W[11]),     \
                   [w12] "+v"(W[12]), [w13] "+v"(W[13]), [w14] "+v"(W[14]), [w15] "+v"(W[15]), \
                   [x0] "=&v"(x0), [x1] "=&v"(x1), [x2] "=&v"(x2), [x3] "=&v"(x3),             \
                   [x4] "=&v"(x4), [x5] "=&v"(x5), [x6] "=&v"(x6), [x7] "=&v"(x7),             \
                   [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3),             \
                   [t4] "=&v"(t4), [t5] "=&v"(t5), [k] "=&s"(k));                               \
  }
LANE_FN(lane_v1, LANE_V1)
LANE_FN(lane_v2, LANE_V2)
LANE_FN(lane_v3, LANE_V3)

template <int V>
__global__ __launch_bounds__(512) void k_lanes(uint32_t* out, int blocks, uint64_t* stamps) {
  extern __shared__ uint32_t pad[];
  if (blocks < 0) pad[threadIdx.x] = 0;  // never: keeps the LDS request (one workgroup per CU)
  uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                    0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int b = 0; b < blocks; ++b) {
    uint32_t W[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) W[i] = (id * 2654435761u) ^ (0x9E3779B9u * (uint32_t)(b * 16 + i + 1));
    if (V == 1) lane_v1(st, W);
    else if (V == 2) lane_v2(st, W);
    else if (V == 3) lane_v3(st, W);
    else sha256_compress(st, W);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 8; ++i) out[8 * id + i] = st[i];
  if ((threadIdx.x & 63) == 0) stamps[id >> 6] = t1 - t0;
}

int main(int argc, char** argv) {
  const int wps = argc > 1 ? atoi(argv[1]) : 1;  // waves per SIMD
  const int cus = 256, blocks = 1000, tpb = 256 * wps, n = cus * tpb, nw = n / 64;
  uint32_t* o[4]; uint64_t* st;
  for (int v = 0; v < 4; ++v) (void)hipMalloc(&o[v], n * 32);
  (void)hipMalloc(&st, nw * 8);
  uint64_t* hs = new uint64_t[nw];
  const char* names[4] = {"hipcc sha256_compress", "V1 aligned", "V2 +no copies", "V3 +K in SGPR"};
  printf("%d wave(s) per SIMD\n", wps);
  for (int r = 0; r < 3; ++r) {
    for (int v = 0; v < 4; ++v) {
      hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
      (void)hipEventRecord(e0);
      const size_t lds = 100 * 1024;
      if (v == 0) hipLaunchKernelGGL(k_lanes<0>, dim3(cus), dim3(tpb), lds, 0, o[0], blocks, st);
      if (v == 1) hipLaunchKernelGGL(k_lanes<1>, dim3(cus), dim3(tpb), lds, 0, o[1], blocks, st);
      if (v == 2) hipLaunchKernelGGL(k_lanes<2>, dim3(cus), dim3(tpb), lds, 0, o[2], blocks, st);
      if (v == 3) hipLaunchKernelGGL(k_lanes<3>, dim3(cus), dim3(tpb), lds, 0, o[3], blocks, st);
      (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
      float ms; (void)hipEventElapsedTime(&ms, e0, e1);
      (void)hipMemcpy(hs, st, nw * 8, hipMemcpyDeviceToHost);
      double avg = 0; for (int i = 0; i < nw; ++i) avg += hs[i]; avg /= nw;
      printf("%-22s %8.1f cycles/block/wave  %.3f ms  %.1f k blocks/us\n", names[v], avg / blocks,
             ms, (double)n * blocks / (ms * 1e3) / 1e3);
    }
  }
  int bad = 0;
  uint32_t* h0 = new uint32_t[n * 8]; uint32_t* h1 = new uint32_t[n * 8];
  (void)hipMemcpy(h0, o[0], n * 32, hipMemcpyDeviceToHost);
  for (int v = 1; v < 4; ++v) {
    (void)hipMemcpy(h1, o[v], n * 32, hipMemcpyDeviceToHost);
    int b = 0; for (int i = 0; i < n * 8; ++i) b += h0[i] != h1[i];
    printf("%s digests %s (%d words differ)\n", names[v], b ? "DIFFER" : "MATCH", b);
    bad += b;
  }
  return bad ? 1 : 0;
}

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
__device__ constexpr uint32_t kK256h[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

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

// V4: K from 64 VGPRs the caller keeps resident (kv, set once by opaque moves)
__device__ __forceinline__ void lane_v4(uint32_t (&st)[8], uint32_t (&W)[16], const uint32_t (&kv)[64]) {
  uint32_t x0, x1, x2, x3, x4, x5, x6, x7, t0, t1, t2, t3, t4, t5;
  asm volatile(LANE_V4
               : [st0] "+v"(st[0]), [st1] "+v"(st[1]), [st2] "+v"(st[2]), [st3] "+v"(st[3]),
                 [st4] "+v"(st[4]), [st5] "+v"(st[5]), [st6] "+v"(st[6]), [st7] "+v"(st[7]),
                 [w0] "+v"(W[0]), [w1] "+v"(W[1]), [w2] "+v"(W[2]), [w3] "+v"(W[3]),
                 [w4] "+v"(W[4]), [w5] "+v"(W[5]), [w6] "+v"(W[6]), [w7] "+v"(W[7]),
                 [w8] "+v"(W[8]), [w9] "+v"(W[9]), [w10] "+v"(W[10]), [w11] "+v"(W[11]),
                 [w12] "+v"(W[12]), [w13] "+v"(W[13]), [w14] "+v"(W[14]), [w15] "+v"(W[15]),
                 [x0] "=&v"(x0), [x1] "=&v"(x1), [x2] "=&v"(x2), [x3] "=&v"(x3),
                 [x4] "=&v"(x4), [x5] "=&v"(x5), [x6] "=&v"(x6), [x7] "=&v"(x7),
                 [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3),
                 [t4] "=&v"(t4), [t5] "=&v"(t5)
               : [k0] "v"(kv[0]), [k1] "v"(kv[1]), [k2] "v"(kv[2]), [k3] "v"(kv[3]), [k4] "v"(kv[4]), [k5] "v"(kv[5]), [k6] "v"(kv[6]), [k7] "v"(kv[7]), [k8] "v"(kv[8]), [k9] "v"(kv[9]), [k10] "v"(kv[10]), [k11] "v"(kv[11]), [k12] "v"(kv[12]), [k13] "v"(kv[13]), [k14] "v"(kv[14]), [k15] "v"(kv[15]), [k16] "v"(kv[16]), [k17] "v"(kv[17]), [k18] "v"(kv[18]), [k19] "v"(kv[19]), [k20] "v"(kv[20]), [k21] "v"(kv[21]), [k22] "v"(kv[22]), [k23] "v"(kv[23]), [k24] "v"(kv[24]), [k25] "v"(kv[25]), [k26] "v"(kv[26]), [k27] "v"(kv[27]), [k28] "v"(kv[28]), [k29] "v"(kv[29]), [k30] "v"(kv[30]), [k31] "v"(kv[31]), [k32] "v"(kv[32]), [k33] "v"(kv[33]), [k34] "v"(kv[34]), [k35] "v"(kv[35]), [k36] "v"(kv[36]), [k37] "v"(kv[37]), [k38] "v"(kv[38]), [k39] "v"(kv[39]), [k40] "v"(kv[40]), [k41] "v"(kv[41]), [k42] "v"(kv[42]), [k43] "v"(kv[43]), [k44] "v"(kv[44]), [k45] "v"(kv[45]), [k46] "v"(kv[46]), [k47] "v"(kv[47]), [k48] "v"(kv[48]), [k49] "v"(kv[49]), [k50] "v"(kv[50]), [k51] "v"(kv[51]), [k52] "v"(kv[52]), [k53] "v"(kv[53]), [k54] "v"(kv[54]), [k55] "v"(kv[55]), [k56] "v"(kv[56]), [k57] "v"(kv[57]), [k58] "v"(kv[58]), [k59] "v"(kv[59]), [k60] "v"(kv[60]), [k61] "v"(kv[61]), [k62] "v"(kv[62]), [k63] "v"(kv[63]));
}

template <int V>
__global__ __launch_bounds__(512) void k_lanes(uint32_t* out, int blocks, uint64_t* stamps,
                                               int prio = 0) {
  if (prio && (threadIdx.x >> 6) < 4) __builtin_amdgcn_s_setprio(3);  // waves 0-3: one per SIMD
  extern __shared__ uint32_t pad[];
  if (blocks < 0) pad[threadIdx.x] = 0;  // never: keeps the LDS request (one workgroup per CU)
  uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                    0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t kv[64];
  if (V == 4) {
#pragma unroll
    for (int i = 0; i < 64; ++i) asm volatile("v_mov_b32 %0, %1" : "=v"(kv[i]) : "i"(kK256h[i]));
  }
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int b = 0; b < blocks; ++b) {
    uint32_t W[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) W[i] = (id * 2654435761u) ^ (0x9E3779B9u * (uint32_t)(b * 16 + i + 1));
    if (V == 1) lane_v1(st, W);
    else if (V == 2) lane_v2(st, W);
    else if (V == 3) lane_v3(st, W);
    else if (V == 4) lane_v4(st, W, kv);
    else sha256_compress(st, W);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 8; ++i) out[8 * id + i] = st[i];
  if ((threadIdx.x & 63) == 0) stamps[id >> 6] = t1 - t0;
}

int main(int argc, char** argv) {
  const int wps = argc > 1 ? atoi(argv[1]) : 1;  // waves per SIMD
  const int prio = argc > 2 ? atoi(argv[2]) : 0;  // 1: waves 0-3 of each workgroup at s_setprio 3
  const int cus = 256, blocks = 1000, tpb = 256 * wps, n = cus * tpb, nw = n / 64;
  uint32_t* o[5]; uint64_t* st;
  for (int v = 0; v < 5; ++v) (void)hipMalloc(&o[v], n * 32);
  (void)hipMalloc(&st, nw * 8);
  uint64_t* hs = new uint64_t[nw];
  const char* names[5] = {"hipcc sha256_compress", "V1 aligned", "V2 +no copies", "V3 +K in SGPR",
                          "V4 +K in VGPRs"};
  printf("%d wave(s) per SIMD%s\n", wps, prio ? ", waves 0-3 at s_setprio 3" : "");
  for (int r = 0; r < 3; ++r) {
    for (int v = 0; v < 5; ++v) {
      hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
      (void)hipEventRecord(e0);
      const size_t lds = 100 * 1024;
      if (v == 0) hipLaunchKernelGGL(k_lanes<0>, dim3(cus), dim3(tpb), lds, 0, o[0], blocks, st, prio);
      if (v == 1) hipLaunchKernelGGL(k_lanes<1>, dim3(cus), dim3(tpb), lds, 0, o[1], blocks, st, prio);
      if (v == 2) hipLaunchKernelGGL(k_lanes<2>, dim3(cus), dim3(tpb), lds, 0, o[2], blocks, st, prio);
      if (v == 3) hipLaunchKernelGGL(k_lanes<3>, dim3(cus), dim3(tpb), lds, 0, o[3], blocks, st, prio);
      if (v == 4) hipLaunchKernelGGL(k_lanes<4>, dim3(cus), dim3(tpb), lds, 0, o[4], blocks, st, prio);
      (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
      float ms; (void)hipEventElapsedTime(&ms, e0, e1);
      (void)hipMemcpy(hs, st, nw * 8, hipMemcpyDeviceToHost);
      double avg = 0; for (int i = 0; i < nw; ++i) avg += hs[i]; avg /= nw;
      double hi = 0, lo = 0; int nh = 0, nl = 0;  // waves 0-3 / 4-7 of each workgroup
      for (int i = 0; i < nw; ++i) {
        if ((i % (tpb / 64)) < 4) { hi += hs[i]; ++nh; } else { lo += hs[i]; ++nl; }
      }
      printf("%-22s %8.1f cycles/block/wave  %.3f ms  %.1f k blocks/us", names[v], avg / blocks,
             ms, (double)n * blocks / (ms * 1e3) / 1e3);
      if (nl) printf("   waves 0-3 %.1f, 4-7 %.1f", hi / nh / blocks, lo / nl / blocks);
      printf("\n");
    }
  }
  int bad = 0;
  uint32_t* h0 = new uint32_t[n * 8]; uint32_t* h1 = new uint32_t[n * 8];
  (void)hipMemcpy(h0, o[0], n * 32, hipMemcpyDeviceToHost);
  for (int v = 1; v < 5; ++v) {
    (void)hipMemcpy(h1, o[v], n * 32, hipMemcpyDeviceToHost);
    int b = 0; for (int i = 0; i < n * 8; ++i) b += h0[i] != h1[i];
    printf("%s digests %s (%d words differ)\n", names[v], b ? "DIFFER" : "MATCH", b);
    bad += b;
  }
  return bad ? 1 : 0;
}

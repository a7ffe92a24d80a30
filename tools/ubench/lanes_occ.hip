// Per-lane SHA-256 throughput against occupancy: the k_sha per-lane pattern (one message per
// lane, sha256_compress, the message realigned with v_perm_b32 and prefetched a block ahead)
// with 1, 2 or 3 waves per SIMD (workgroups of 256 threads; LDS padding admits 1, 2 or 3 per
// CU), register messages and HBM messages. Question: can a second wave per SIMD
// raise per-lane SHA-256 throughput enough to change configs[2]'s work bound?
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench/lanes_occ tools/ubench/lanes_occ.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include "../../bs_amd/csrc/sha256_device.h"
using namespace bsg;

typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const uint32_t g32;
typedef __attribute__((address_space(1))) const u32x4v g32x4;
struct Raw { uint32_t r[17]; };

__device__ __forceinline__ void load_raw(const uint8_t* p, Raw& rb) {
  g32* al = reinterpret_cast<g32*>(reinterpret_cast<uintptr_t>(p) & ~(uintptr_t)3);
  g32x4* q = reinterpret_cast<g32x4*>(al);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const u32x4v x = q[i];
    rb.r[4 * i] = x.x; rb.r[4 * i + 1] = x.y; rb.r[4 * i + 2] = x.z; rb.r[4 * i + 3] = x.w;
  }
  rb.r[16] = al[16];
}

template <bool MEM>
__global__ __launch_bounds__(256, 1) void k_lanes(const uint8_t* d, uint64_t region, uint32_t* out,
                                                  int blocks, uint64_t* stamps) {
  extern __shared__ uint32_t pad[];
  if (blocks < 0) pad[threadIdx.x] = 0;  // never: keeps the LDS request
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                    0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
  const uint8_t* base = d + (uint64_t)id * region + 5;
  const uint32_t sel = (1u << 24) | (2u << 16) | (3u << 8) | 4u;
  Raw rb;
  if (MEM) load_raw(base, rb);
  for (int b = 0; b < blocks; ++b) {
    uint32_t W[16];
    if (MEM) {
#pragma unroll
      for (int i = 0; i < 16; ++i) W[i] = __builtin_amdgcn_perm(rb.r[i + 1], rb.r[i], sel);
      load_raw(base + 64ull * (b + 1), rb);
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) W[i] = (id * 2654435761u) ^ (sel + 31u * (uint32_t)(b * 16 + i));
    }
    sha256_compress(st, W);
  }
  uint32_t x = 0;
  for (int i = 0; i < 8; ++i) x ^= st[i];
  out[id] = x;
  if ((threadIdx.x & 63) == 0) stamps[id >> 6] = __builtin_amdgcn_s_memtime() - t0;
}

template <bool MEM>
void run(const uint8_t* d, int cus, int per_cu, int blocks) {
  const int wgs = cus * per_cu;
  const uint64_t region = 64ull * (blocks + 2);
  uint32_t* out;
  uint64_t* stamps;
  (void)hipMalloc(&out, (size_t)wgs * 256 * 4);
  (void)hipMalloc(&stamps, (size_t)wgs * 4 * 8);
  // LDS padding: 160 KiB per CU admits per_cu workgroups
  const size_t lds = per_cu == 1 ? 100 * 1024 : per_cu == 2 ? 72 * 1024 : 48 * 1024;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_lanes<MEM>, dim3(wgs), dim3(256), lds, 0, d, region, out, blocks, stamps);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  static uint64_t h[8 * 1024 * 4];
  (void)hipMemcpy(h, stamps, (size_t)wgs * 4 * 8, hipMemcpyDeviceToHost);
  double cyc = 0;
  for (int i = 0; i < wgs * 4; ++i) cyc += (double)h[i];
  cyc /= wgs * 4;
  const double total = (double)wgs * 256 * blocks;
  printf("%s, %d wave(s) per SIMD: %.3f ms, %.1f blocks/us chip-wide (%.0f GB/s), %.0f cycles "
         "per wave-block (s_memtime, per wave)\n", MEM ? "HBM message " : "register msg", per_cu,
         best, total / (best * 1e3), total * 64 / (best * 1e6), cyc / blocks);
  (void)hipFree(out);
  (void)hipFree(stamps);
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const int blocks = 300;
  const uint64_t bytes = (uint64_t)cus * 3 * 256 * 64ull * (blocks + 2) + 4096;
  uint8_t* d;
  if (hipMalloc(&d, bytes) != hipSuccess) return 1;
  (void)hipMemset(d, 0x5a, bytes);
  for (int rep = 0; rep < 2; ++rep)
    for (int per_cu = 1; per_cu <= 3; ++per_cu) {
      run<false>(d, cus, per_cu, blocks);
      run<true>(d, cus, per_cu, blocks);
    }
  (void)hipFree(d);
  return 0;
}

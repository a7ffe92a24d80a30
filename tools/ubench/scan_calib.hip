// scan_calib.hip — calibrates rocprofv3's FETCH_SIZE for k_scan's load pattern on gfx950.
//
// MI355X_MICROARCH.md (HBM section): FETCH_SIZE reports half the bytes of a wide coalesced
// streaming read; other access patterns are uncalibrated and must be calibrated on a known byte
// count. This program reads exactly 1 GiB (plus the 64-byte warm-up block before each strip,
// as k_scan does) in two patterns and writes one word per lane:
//   k_strips    k_scan's pattern: each lane owns a 2 KiB strip, 512-thread workgroups, reads
//               the 64 bytes before its strip, then the strip as 64-byte blocks of 4 x 16 B
//   k_coalesced the guide's calibrated case: lane i of a wave reads 16 B at base + 16 i
// Run each under `rocprofv3 --pmc FETCH_SIZE`; FETCH_SIZE x 1024 / algorithmic bytes gives the
// factor to apply to k_scan's counter (tools/pmc_summary.py).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4* g_u32x4p;

constexpr int kStrip = 2048;

__global__ __launch_bounds__(512) void k_strips(const uint8_t* d, uint64_t nstrips, uint32_t* out) {
  const uint64_t strip = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (strip >= nstrips) return;
  const uint8_t* base = d + strip * kStrip;
  uint32_t acc = 0;
  if (strip) {  // warm-up block: the 64 bytes before the strip
    g_u32x4p q = (g_u32x4p)(base - 64);
    for (int i = 0; i < 4; ++i) { u32x4 v = q[i]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
  }
  for (int b = 0; b < kStrip / 64; ++b) {
    g_u32x4p q = (g_u32x4p)(base + 64 * b);
#pragma unroll
    for (int i = 0; i < 4; ++i) { u32x4 v = q[i]; acc = (acc ^ v.x ^ v.y ^ v.z ^ v.w) * 0x9E3779B1u; }
  }
  out[strip] = acc;
}

__global__ __launch_bounds__(256) void k_coalesced(const uint8_t* d, uint64_t n16, uint32_t* out) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    u32x4 v = ((g_u32x4p)d)[i];
    acc = (acc ^ v.x ^ v.y ^ v.z ^ v.w) * 0x9E3779B1u;
  }
  out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  const uint64_t n = 1ull << 30;
  uint8_t* d;
  uint32_t* out;
  if (hipMalloc(&d, n + 256) != hipSuccess || hipMalloc(&out, (n / kStrip) * 4) != hipSuccess) return 1;
  hipMemset(d, 0x5a, n);
  const uint64_t nstrips = n / kStrip;
  hipLaunchKernelGGL(k_strips, dim3((uint32_t)((nstrips + 511) / 512)), dim3(512), 0, 0, d, nstrips, out);
  hipLaunchKernelGGL(k_coalesced, dim3(2048), dim3(256), 0, 0, d, n / 16, out);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::printf("k_strips: %llu strips, algorithmic bytes %llu (strips) + %llu (warm-up)\n",
              (unsigned long long)nstrips, (unsigned long long)n,
              (unsigned long long)((nstrips - 1) * 64));
  std::printf("k_coalesced: algorithmic bytes %llu\n", (unsigned long long)n);
  hipFree(d);
  hipFree(out);
  return 0;
}

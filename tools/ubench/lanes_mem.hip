// Per-lane SHA-256 with its message read from HBM, as k_sha's per-lane mode reads it (one
// chunk per lane, 4 x dwordx4 + 1 dword per block, realigned by v_perm_b32, issued one block
// ahead), against the same loop on register data (lanes.hip). One workgroup per CU (LDS
// padding), 4 waves (one per SIMD). Question: does the HBM read cost k_sha's per-lane mode the
// ~30 % it runs below lanes.hip under full load?
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

// MEM: message from HBM (else from registers). SCATTER: lane i's region is region slot
// perm(i) of a large buffer (k_sha's per-lane jobs sit anywhere in 16 GiB; adjacent lanes'
// regions are otherwise adjacent). AHEAD: blocks prefetched ahead (1: k_sha today; 2: two
// register sets, loop unrolled by two).
template <bool MEM, int SCATTER, int AHEAD>
__global__ __launch_bounds__(256, 1) void k_lanes_mem(const uint8_t* d, uint64_t region,
                                                     uint64_t nslots, uint32_t* out, int blocks,
                                                     uint32_t mis, uint64_t rbytes) {
  extern __shared__ uint32_t pad[];
  if (blocks < 0) pad[threadIdx.x] = 0;  // never: keeps the LDS request
  uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                    0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
  // SCATTER 2: scattered, but inside a 64 MiB range per CU (a stream per CU, as in
  // configs[2] if each CU took its own stream's jobs)
  const uint64_t per_cu = rbytes / region;  // region slots per wave / CU region
  const uint64_t nreg = (16ull << 30) / rbytes;
  const uint64_t slot = SCATTER == 1 ? ((uint64_t)id * 40503u) % nslots
                      : SCATTER == 2 ? blockIdx.x * per_cu + ((uint64_t)threadIdx.x * 97u) % per_cu
                      : SCATTER == 3 ? ((blockIdx.x + 64u * (threadIdx.x >> 6)) % nreg) * per_cu +
                                           ((uint64_t)(threadIdx.x & 63u) * 40503u) % per_cu
                                     : id;
  const uint8_t* base = d + slot * region + mis;  // misaligned like a chunk start
  const uint32_t sh = mis & 3u;
  const uint32_t sel = (sh << 24) | ((sh + 1) << 16) | ((sh + 2) << 8) | (sh + 3);
  Raw rb, rc;
  if (MEM) {
    load_raw(base, rb);
    if (AHEAD == 2) load_raw(base + 64, rc);
  }
  for (int b = 0; b < blocks; b += AHEAD) {
    uint32_t W[16];
    if (MEM) {
#pragma unroll
      for (int i = 0; i < 16; ++i) W[i] = __builtin_amdgcn_perm(rb.r[i + 1], rb.r[i], sel);
      load_raw(base + 64ull * (b + AHEAD), rb);
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) W[i] = (id * 2654435761u) ^ (sel + 31u * (uint32_t)(b * 16 + i));
    }
    sha256_compress(st, W);
    if (AHEAD == 2) {
      if (MEM) {
#pragma unroll
        for (int i = 0; i < 16; ++i) W[i] = __builtin_amdgcn_perm(rc.r[i + 1], rc.r[i], sel);
        load_raw(base + 64ull * (b + 3), rc);
      }
      sha256_compress(st, W);
    }
  }
  uint32_t x = 0;
  for (int i = 0; i < 8; ++i) x ^= st[i];
  out[id] = x;
}

template <bool MEM, int SCATTER, int AHEAD>
void run(const uint8_t* d, uint64_t region, uint64_t nslots, int cus, int blocks,
         uint64_t rbytes = 64ull << 20) {
  uint32_t* out;
  (void)hipMalloc(&out, (size_t)cus * 256 * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((k_lanes_mem<MEM, SCATTER, AHEAD>), dim3(cus), dim3(256), 84 * 1024, 0, d,
                       region, nslots, out, blocks, 5u, rbytes);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  const double total = (double)cus * 256 * blocks;
  printf("[%5llu MiB] %s %s ahead %d: %d blocks/lane, %.3f ms, %.1f blocks/us chip-wide (%.1f GB/s), %.0f "
         "cycles per wave-block at 2.4 GHz\n", (unsigned long long)(rbytes >> 20), MEM ? "HBM message " : "register msg",
         SCATTER == 1 ? "scattered" : SCATTER == 2 ? "CU-local " : SCATTER == 3 ? "wave-local" : "adjacent ", AHEAD, blocks, best, total / (best * 1e3),
         total * 64 / (best * 1e6), best * 1e-3 * 2.4e9 / blocks);
  (void)hipFree(out);
}

int main() {
  int dev = 0; hipDeviceProp_t p; (void)hipGetDeviceProperties(&p, dev);
  const int cus = p.multiProcessorCount;
  const int blocks = 400;
  const uint64_t region = 64ull * (blocks + 4);
  const uint64_t lanes = (uint64_t)cus * 256;
  // scattered: 16 GiB of region slots (configs[2]'s footprint), lanes spread over all of it
  const uint64_t big = 16ull << 30;
  const uint64_t nslots = big / region;
  uint8_t* d;
  if (hipMalloc(&d, big + 4096) != hipSuccess) return 1;
  (void)hipMemset(d, 0x5a, big + 4096);
  (void)lanes;
  for (int rep = 0; rep < 2; ++rep) {
    run<false, 0, 1>(d, region, nslots, cus, blocks);
    run<true, 0, 1>(d, region, nslots, cus, blocks);
    run<true, 1, 1>(d, region, nslots, cus, blocks);
    run<true, 2, 1>(d, region, nslots, cus, blocks);
    for (uint64_t rb = 64ull << 20; rb <= (4ull << 30); rb *= 2)
      run<true, 3, 1>(d, region, nslots, cus, blocks, rb);
  }
  (void)hipFree(d);
  return 0;
}

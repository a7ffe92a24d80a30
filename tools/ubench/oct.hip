// Microbenchmark + check: the skewed octet (sha256_blocks_oct, 8 VALU/round, one chain per 8
// lanes) against the single-lane rounds (sha256_rounds_kw) and the skewed pair's block loop
// (sha256_blocks_skew, 9 VALU/round). One lone wave, K+W rows in LDS as in k_sha's wave mode;
// `blocks` chained blocks; prints cycles per block and whether the final state matches.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include "../../bs_amd/csrc/sha256_device.h"
using namespace bsg;

#define STAMP(t) asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory")
typedef uint32_t u32x4r __attribute__((ext_vector_type(4), aligned(16)));

template <int V>
__global__ __launch_bounds__(64) void kb(uint64_t* out, uint32_t* io, int blocks) {
  __shared__ __attribute__((aligned(16))) uint32_t rows[2][68];
  for (int i = threadIdx.x; i < 68; i += blockDim.x) { rows[0][i] = io[i] * 2654435761u + i; rows[1][i] = 1u; }
  __syncthreads();
  const uint32_t H0[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                          0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint32_t st[8];
  for (int i = 0; i < 8; ++i) st[i] = H0[i];
  uint64_t t0 = 0, t1 = 0;
  const int emap[4] = {6, 7, 4, 5};
  if (V == 0) {  // single lane
    STAMP(t0);
    for (int b = 0; b < blocks; ++b) {
      const u32x4r* r = reinterpret_cast<const u32x4r*>(rows[0]);
      uint32_t KW[64];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const u32x4r v = r[q];
        KW[4 * q] = v.x; KW[4 * q + 1] = v.y; KW[4 * q + 2] = v.z; KW[4 * q + 3] = v.w;
      }
      sha256_rounds_kw<true>(st, KW);
    }
    STAMP(t1);
    if (threadIdx.x == 0) for (int i = 0; i < 8; ++i) io[2000 + i] = st[i];
  } else if (V == 1) {  // skewed pair block loop
    const SkewLane sl = skew_lane();
    uint32_t hs[4];
    for (int k = 0; k < 4; ++k) hs[k] = sl.a_side ? st[k] : st[emap[k]];
    STAMP(t0);
    sha256_blocks_skew(hs, rows[sl.a_side ? 1 : 0], 0u, (uint32_t)blocks, blocks, sl);
    STAMP(t1);
    if (threadIdx.x == 0 || threadIdx.x == 1)
      for (int k = 0; k < 4; ++k) io[2000 + (threadIdx.x == 1 ? k : emap[k])] = hs[k];
  } else {  // skewed octet block loop; every lane of every octet checked
    const OctLane ol = oct_lane();
    uint32_t hs[4];
    for (int k = 0; k < 4; ++k) hs[k] = ol.a_side ? st[k] : st[emap[k]];
    STAMP(t0);
    if (V == 3)  // the solo loop (round 6): no exec update, no slot copies, no s_nop
      sha256_blocks_oct_solo(hs, rows[ol.a_side ? 1 : 0], 0u, (uint32_t)blocks, ol);
    else
      sha256_blocks_oct(hs, rows[ol.a_side ? 1 : 0], 0u, (uint32_t)blocks, blocks, ol);
    STAMP(t1);
    if (threadIdx.x == 0 || threadIdx.x == 4)
      for (int k = 0; k < 4; ++k) io[2000 + (threadIdx.x == 4 ? k : emap[k])] = hs[k];
    // all 64 lanes' states, to check that every lane of every quad agrees
    for (int k = 0; k < 4; ++k) io[3000 + 4 * threadIdx.x + k] = hs[k];
  }
  if (threadIdx.x == 0) out[0] = t1 - t0;
}

template <int V> bool run(const char* name, uint32_t* ref, int blocks) {
  uint64_t* d; uint32_t* io;
  (void)hipMalloc(&d, 16); (void)hipMalloc(&io, 8192 * 4);
  (void)hipMemset(io, 3, 8192 * 4);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(kb<V>, dim3(1), dim3(64), 0, 0, d, io, blocks);
    if (hipDeviceSynchronize() != hipSuccess) { printf("%s: launch failed\n", name); return false; }
  }
  uint64_t h; (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  uint32_t fin[8]; (void)hipMemcpy(fin, io + 2000, 32, hipMemcpyDeviceToHost);
  bool ok = true;
  if (V == 0) for (int i = 0; i < 8; ++i) ref[i] = fin[i];
  else for (int i = 0; i < 8; ++i) ok &= ref[i] == fin[i];
  if (V >= 2) {
    uint32_t all[256]; (void)hipMemcpy(all, io + 3000, 1024, hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; ++l)
      for (int k = 0; k < 4; ++k) ok &= all[4 * l + k] == all[4 * (l & 4) + k];
  }
  printf("%-40s blocks %4d %8.0f cycles/block %6.2f cycles/round  state %08x .. %08x %s\n",
         name, blocks, (double)h / blocks, (double)h / blocks / 64, fin[0], fin[7],
         ok ? "MATCH" : "MISMATCH");
  (void)hipFree(d); (void)hipFree(io);
  return ok;
}

int main() {
  uint32_t ref[8];
  bool ok = true;
  for (int blocks : {1, 2, 7, 400}) {
    run<0>("single lane (14 VALU/round)", ref, blocks);
    ok &= run<1>("skewed pair loop (9 VALU/round)", ref, blocks);
    ok &= run<2>("skewed octet loop (8 VALU/round)", ref, blocks);
    ok &= run<3>("skewed octet solo loop (round 6)", ref, blocks);
  }
  return ok ? 0 : 1;
}

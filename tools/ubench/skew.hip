// Microbenchmark + check: the skewed lane pair (sha256_rounds_skew, 9 VALU/round) against the
// single-lane rounds (sha256_rounds_kw) and the banked pair (sha256_rounds_bank), one lone
// wave, K+W rows in LDS as in k_sha's wave mode. Prints cycles per 64-round block and whether
// each pair's final state equals the single-lane state.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include "../../bs_amd/csrc/sha256_device.h"
#include "skew_variants.inc"
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
  uint64_t t0, t1;
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
  } else if (V == 1) {  // banked pair (lanes 3, 4)
    const BankLane bl = bank_lane();
    uint32_t hs[4];
    for (int k = 0; k < 4; ++k) hs[k] = bl.a_side ? st[k] : st[4 + k];
    STAMP(t0);
    for (int b = 0; b < blocks; ++b) sha256_rounds_bank(hs, rows[bl.a_side ? 1 : 0], bl, true);
    STAMP(t1);
    if (threadIdx.x == 3 || threadIdx.x == 4)
      for (int k = 0; k < 4; ++k) io[2000 + (threadIdx.x == 4 ? k : 4 + k)] = hs[k];
  } else if (V == 3) {  // skewed pair, whole block loop in one asm statement
    const SkewLane sl = skew_lane();
    uint32_t hs[4];
    const int emap[4] = {6, 7, 4, 5};
    for (int k = 0; k < 4; ++k) hs[k] = sl.a_side ? st[k] : st[emap[k]];
    STAMP(t0);
    sha256_blocks_skew(hs, rows[sl.a_side ? 1 : 0], 0u, (uint32_t)blocks, blocks, sl);
    STAMP(t1);
    if (threadIdx.x == 0 || threadIdx.x == 1)
      for (int k = 0; k < 4; ++k) io[2000 + (threadIdx.x == 1 ? k : emap[k])] = hs[k];
  } else if (V >= 10) {  // instruction-order variants of the skewed pair (tools/gen_skew_asm.py)
    const SkewLane sl = skew_lane();
    uint32_t hs[4];
    const int emap[4] = {6, 7, 4, 5};
    for (int k = 0; k < 4; ++k) hs[k] = sl.a_side ? st[k] : st[emap[k]];
    const uint64_t amask = 0xAAAAAAAAAAAAAAAAull;
    STAMP(t0);
    for (int b = 0; b < blocks; ++b) {
      uint32_t v2 = hs[2], v1 = hs[3], v0 = hs[0], v3 = hs[1];
      const uint32_t addr = (uint32_t)reinterpret_cast<uintptr_t>(
          (__attribute__((address_space(3))) const uint32_t*)rows[sl.a_side ? 1 : 0]);
#define VAR_ASM(X)                                                                          \
  asm volatile(X : [v0] "+v"(v0), [v1] "+v"(v1), [v2] "+v"(v2), [v3] "+v"(v3)              \
               : [row] "v"(addr), [xm] "v"(sl.xm), [s1] "v"(sl.rot1), [s2] "v"(sl.rot2),   \
                 [s3] "v"(sl.rot3), [amask] "s"(amask)                                     \
               : "memory", BSG_SKEW_BLOCK_CLOBBERS_A)
      if (V == 10) VAR_ASM(BSG_SKEW_BLOCK_ASM_A);
      if (V == 11) VAR_ASM(BSG_SKEW_BLOCK_ASM_B);
      if (V == 12) VAR_ASM(BSG_SKEW_BLOCK_ASM_C);
      if (V == 13) VAR_ASM(BSG_SKEW_BLOCK_ASM_D);
      if (V == 15) VAR_ASM(BSG_SKEW_BLOCK_ASM_E);
      if (V == 16) VAR_ASM(BSG_SKEW_BLOCK_ASM_F);
      if (V == 17)
        asm volatile(BSG_SKEW_BLOCK_ASM_P : [v0] "+v"(v0), [v1] "+v"(v1), [v2] "+v"(v2), [v3] "+v"(v3)
                     : [row] "v"(addr), [xm] "v"(sl.xm), [s1] "v"(sl.rot1), [s2] "v"(sl.rot2),
                       [s3] "v"(sl.rot3), [amask] "s"(amask)
                     : "memory", BSG_SKEW_BLOCK_CLOBBERS_P);
      if (V == 14)
        asm volatile(BSG_SKEW_BLOCK_ASM_H : [v0] "+v"(v0), [v1] "+v"(v1), [v2] "+v"(v2), [v3] "+v"(v3)
                     : [row] "v"(addr), [xm] "v"(sl.xm), [s1] "v"(sl.rot1), [s2] "v"(sl.rot2),
                       [s3] "v"(sl.rot3), [amask] "s"(amask)
                     : "memory", BSG_SKEW_BLOCK_CLOBBERS_H);
      hs[0] += v0; hs[1] += v3; hs[2] += v2; hs[3] += v1;
    }
    STAMP(t1);
    if (threadIdx.x == 0 || threadIdx.x == 1)
      for (int k = 0; k < 4; ++k) io[2000 + (threadIdx.x == 1 ? k : emap[k])] = hs[k];
  } else {  // skewed pair (lanes 2p E, 2p+1 A)
    const SkewLane sl = skew_lane();
    uint32_t hs[4];
    const int emap[4] = {6, 7, 4, 5};
    for (int k = 0; k < 4; ++k) hs[k] = sl.a_side ? st[k] : st[emap[k]];
    STAMP(t0);
    for (int b = 0; b < blocks; ++b) sha256_rounds_skew(hs, rows[sl.a_side ? 1 : 0], sl, true);
    STAMP(t1);
    if (threadIdx.x == 0 || threadIdx.x == 1)
      for (int k = 0; k < 4; ++k) io[2000 + (threadIdx.x == 1 ? k : emap[k])] = hs[k];
  }
  if (threadIdx.x == 0) out[0] = t1 - t0;
}

template <int V> void run(const char* name, uint32_t* ref) {
  uint64_t* d; uint32_t* io;
  (void)hipMalloc(&d, 16); (void)hipMalloc(&io, 8192 * 4);
  (void)hipMemset(io, 3, 8192 * 4);
  const int blocks = 400;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(kb<V>, dim3(1), dim3(64), 0, 0, d, io, blocks);
    (void)hipDeviceSynchronize();
  }
  uint64_t h; (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  uint32_t fin[8]; (void)hipMemcpy(fin, io + 2000, 32, hipMemcpyDeviceToHost);
  bool ok = true;
  if (V == 0) for (int i = 0; i < 8; ++i) ref[i] = fin[i];
  else for (int i = 0; i < 8; ++i) ok &= ref[i] == fin[i];
  printf("%-48s %8.0f cycles/block %6.2f cycles/round  state %08x .. %08x %s\n", name,
         (double)h / blocks, (double)h / blocks / 64, fin[0], fin[7], ok ? "MATCH" : "MISMATCH");
  (void)hipFree(d); (void)hipFree(io);
}

int main() {
  uint32_t ref[8];
  run<0>("single lane (14 VALU/round)", ref);
  run<1>("banked pair (10 VALU + s_nop)", ref);
  run<2>("skewed pair (9 VALU/round)", ref);
  run<3>("skewed pair, asm block loop", ref);
  run<10>("skew order A: xad al0 al1 dpp al2 bx xor3 ch", ref);
  run<11>("skew order B: xad dpp al0 al1 al2 bx xor3 ch", ref);
  run<12>("skew order C: al0 al1 al2 bx xad dpp xor3 ch", ref);
  run<13>("skew order D: al0 al1 al2 xad xor3 bx dpp ch", ref);
  run<15>("timing only: exchange as plain v_add", ref);
  run<16>("timing only: no exchange instruction (8/round)", ref);
  run<17>("skew, pipelined exchange (model-best order)", ref);
  run<14>("skew, bank-conflict-free regs (+24 movs/block)", ref);
  return 0;
}

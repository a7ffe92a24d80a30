// Microbenchmark: cycles per 64-round SHA-256 block for one lone wave, paired-lane variants
// vs the single-lane rounds (K+W rows in LDS as in k_sha's wave mode). Timing only: some
// variants deliberately compute wrong values to isolate one instruction's cost.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include "../../bs_amd/csrc/sha256_device.h"
using namespace bsg;

#define STAMP(t) asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory")

typedef uint32_t u32x4r __attribute__((ext_vector_type(4), aligned(16)));

// Paired lanes (even = E, odd = A) with a cndmask + quad_perm DPP exchange (11 VALU/round).
struct PairLane {
  uint32_t rot1, rot2, rot3, xm, pm;
  bool odd;
};
__device__ __forceinline__ PairLane pair_lane() {
  PairLane p;
  p.odd = (threadIdx.x & 1u) != 0;
  p.rot1 = p.odd ? 2u : 6u;
  p.rot2 = p.odd ? 13u : 11u;
  p.rot3 = p.odd ? 22u : 25u;
  p.xm = p.odd ? 0xffffffffu : 0u;
  p.pm = p.odd ? 0u : 0xffffffffu;
  return p;
}
__device__ __forceinline__ uint32_t swap_pair(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);
}

// V: 0 pair (DPP + cndmask), 1 pair without DPP (wrong values), 2 pair, Z = T (no cndmask),
//    3 pair with the exchange through ds_swizzle, 4 single-lane rounds_kw
template <int V>
__device__ __forceinline__ void round_v(uint32_t& r1, uint32_t& r2, uint32_t& r3, uint32_t& r4,
                                       uint32_t kw, const PairLane& p) {
  const uint32_t S = xor3(rotr(r1, p.rot1), rotr(r1, p.rot2), rotr(r1, p.rot3));
  const uint32_t x = bitop3<0x78>(r1, r3, p.xm);
  const uint32_t F = bitop3<0xCA>(x, r2, r3);
  const uint32_t P = (r4 & p.pm) + kw;
  const uint32_t T = F + S + P;
  uint32_t n;
  if (V == 0) {
    const uint32_t Z = p.odd ? r4 : T;
    n = T + swap_pair(Z);
  } else if (V == 1) {
    const uint32_t Z = p.odd ? r4 : T;
    n = T + Z;
  } else if (V == 2) {
    n = T + swap_pair(T);
  } else {
    const uint32_t Z = p.odd ? r4 : T;
    n = T + (uint32_t)__builtin_amdgcn_ds_swizzle((int)Z, 0x041F);  // xor lane 1
  }
  r4 = r3; r3 = r2; r2 = r1; r1 = n;
}

// Compiler-scheduled version of the banked pair (the header's bank_round is hand-scheduled).
__device__ __forceinline__ uint32_t xad(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_xad_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ void bank_round_c(uint32_t& r1, uint32_t& r2, uint32_t& r3, uint32_t& r4,
                                             uint32_t kwl, const BankLane& b) {
  const uint32_t S = xor3(rotr(r1, b.rot1), rotr(r1, b.rot2), rotr(r1, b.rot3));
  const uint32_t x = bitop3<0x78>(r1, r3, b.xm);
  const uint32_t F = bitop3<0xCA>(x, r2, r3);
  const uint32_t P = xad(r4, b.xm, kwl);
  const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r4, 0x101, 0xF, 0x5, false);
  const uint32_t Q = P + dn;
  const uint32_t U = F + S + Q;
  const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)U, 0x111, 0xF, 0xA, false);
  const uint32_t n = U + up;
  r4 = r3; r3 = r2; r2 = r1; r1 = n;
}

template <int V>
__global__ void kb(uint64_t* out, uint32_t* io, int blocks) {
  __shared__ __attribute__((aligned(16))) uint32_t rows[3][68];
  for (int i = threadIdx.x; i < 2 * 68; i += blockDim.x) rows[i / 68][i % 68] = io[i] + i;
  for (int i = threadIdx.x; i < 68; i += blockDim.x) rows[2][i] = 1u;
  __syncthreads();
  const BankLane bl = bank_lane();
  const PairLane p = pair_lane();
  uint32_t s[4], st[8];
  for (int i = 0; i < 4; ++i) s[i] = io[200 + i] + threadIdx.x;
  for (int i = 0; i < 8; ++i) st[i] = io[200 + i] * (uint32_t)(i + 1);
  if (V == 5 || V == 6)
    for (int i = 0; i < 4; ++i) s[i] = io[200 + i] * (uint32_t)((bl.a_side ? i : 4 + i) + 1);
  uint64_t t0, t1;
  STAMP(t0);
  for (int b = 0; b < blocks; ++b) {
    if (V == 6) {
      const u32x4r* r = reinterpret_cast<const u32x4r*>(rows[bl.a_side ? 2 : 0]);
      uint32_t r1 = s[0], r2 = s[1], r3 = s[2], r4 = s[3];
      u32x4r kw = r[0];
      uint32_t q = bank_q0(r4, kw.x, bl);
#pragma unroll
      for (int qd = 0; qd < 16; ++qd) {
        const u32x4r kn = r[qd < 15 ? qd + 1 : 15];
        bank_round(r1, r2, r3, r4, q, kw.y, bl);
        bank_round(r1, r2, r3, r4, q, kw.z, bl);
        bank_round(r1, r2, r3, r4, q, kw.w, bl);
        bank_round(r1, r2, r3, r4, q, kn.x, bl);  // last round: value unused
        kw = kn;
      }
      s[0] += r1; s[1] += r2; s[2] += r3; s[3] += r4;
    } else if (V == 5) {
      const u32x4r* r = reinterpret_cast<const u32x4r*>(rows[bl.a_side ? 2 : 0]);
      uint32_t r1 = s[0], r2 = s[1], r3 = s[2], r4 = s[3];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const u32x4r kw = r[q];
        bank_round_c(r1, r2, r3, r4, kw.x, bl);
        bank_round_c(r1, r2, r3, r4, kw.y, bl);
        bank_round_c(r1, r2, r3, r4, kw.z, bl);
        bank_round_c(r1, r2, r3, r4, kw.w, bl);
      }
      s[0] += r1; s[1] += r2; s[2] += r3; s[3] += r4;
    } else if (V < 4) {
      const u32x4r* r = reinterpret_cast<const u32x4r*>(rows[p.odd ? 1 : 0]);
      uint32_t r1 = s[0], r2 = s[1], r3 = s[2], r4 = s[3];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const u32x4r kw = r[q];
        round_v<V>(r1, r2, r3, r4, kw.x, p);
        round_v<V>(r1, r2, r3, r4, kw.y, p);
        round_v<V>(r1, r2, r3, r4, kw.z, p);
        round_v<V>(r1, r2, r3, r4, kw.w, p);
      }
      s[0] += r1; s[1] += r2; s[2] += r3; s[3] += r4;
    } else {
      const u32x4r* r = reinterpret_cast<const u32x4r*>(rows[0]);
      uint32_t KW[64];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const u32x4r v = r[q];
        KW[4 * q] = v.x; KW[4 * q + 1] = v.y; KW[4 * q + 2] = v.z; KW[4 * q + 3] = v.w;
      }
      sha256_rounds_kw<true>(st, KW);
    }
  }
  STAMP(t1);
  uint32_t x = 0;
  for (int i = 0; i < 4; ++i) x ^= s[i];
  for (int i = 0; i < 8; ++i) x ^= st[i];
  io[1000 + threadIdx.x] = x;
  if (threadIdx.x == 0) out[0] = t1 - t0;
  // final states for the correctness check: single lane (lane 0) vs banked pair (lanes 3, 4)
  if (V == 4 && threadIdx.x == 0)
    for (int i = 0; i < 8; ++i) io[2000 + i] = st[i];
  if ((V == 5 || V == 6) && (threadIdx.x == 3 || threadIdx.x == 4))
    for (int i = 0; i < 4; ++i) io[2000 + (threadIdx.x == 4 ? i : 4 + i)] = s[i];
}

template <int V> void run(const char* name) {
  uint64_t* d; uint32_t* io;
  (void)hipMalloc(&d, 16); (void)hipMalloc(&io, 8192 * 4);
  (void)hipMemset(io, 1, 8192 * 4);
  const int blocks = 400;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(kb<V>, dim3(1), dim3(64), 0, 0, d, io, blocks);
    (void)hipDeviceSynchronize();
  }
  uint64_t h; (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  uint32_t fin[8]; (void)hipMemcpy(fin, io + 2000, 32, hipMemcpyDeviceToHost);
  printf("%-52s %8.0f cycles/block %6.1f cycles/round  state %08x %08x .. %08x\n", name,
         (double)h / blocks, (double)h / blocks / 64, fin[0], fin[1], fin[7]);
  (void)hipFree(d); (void)hipFree(io);
}

int main() {
  run<4>("single lane rounds_kw (14 VALU/round)");
  run<5>("banked pair: xad + 2 masked DPP adds (10 VALU/round)");
  run<6>("banked pair, hand-scheduled asm round");
  run<0>("pair: cndmask + DPP add (11 VALU/round)");
  run<1>("pair, no DPP (timing only)");
  run<2>("pair, DPP of T, no cndmask (timing only)");
  run<3>("pair, ds_swizzle exchange");
  return 0;
}

// sha256_device.h — CDNA4 device primitives shared by the kernels and tools/ubench:
// rotates (v_alignbit_b32), 3-input bitwise ops (v_bitop3_b32) and the SHA-256 compression
// function (FIPS 180-4 §6.2.2) fully unrolled with variables rotated by renaming.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bsg {

__device__ __forceinline__ uint32_t rotl1(uint32_t h) { return __builtin_amdgcn_alignbit(h, h, 31); }
__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t r) {
  return __builtin_amdgcn_alignbit(x, x, r);
}
// 3-input XOR in one VALU op (gfx950 v_bitop3_b32, truth table 0x96); hipcc emits two v_xor
// for a ^ b ^ c. The compiler builtin, which the scheduler can move like any other instruction
// (round 1 used inline asm).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// ---------------------------------------------------------------------------------------------
static constexpr uint32_t kK256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4,
    0xab1c5ed5, 0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe,
    0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f,
    0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7,
    0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc,
    0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b,
    0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116,
    0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
    0xc67178f2};

template <uint32_t TT>
__device__ __forceinline__ uint32_t bitop3(uint32_t a, uint32_t b, uint32_t c) {
  // v_bitop3_b32: bit i of the result = TT[(a_i << 2) | (b_i << 1) | c_i]
  return __builtin_amdgcn_bitop3_b32(a, b, c, TT);
}

// One SHA-256 round, 14 VALU ops: 3+1 (Sigma1), Ch (bitop3 0xCA), h+K+W, add3, d += T1,
// 3+1 (Sigma0), Maj (bitop3 0xE8), add3. Variables rotate by renaming, not by moves.
#define SHA_ROUND(a, b, c, d, e, f, g, h, kw)                                 \
  do {                                                                         \
    const uint32_t s1_ = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));           \
    const uint32_t ch_ = bitop3<0xCA>(e, f, g);                                \
    const uint32_t t1_ = (h + (kw)) + s1_ + ch_;                               \
    d += t1_;                                                                  \
    const uint32_t s0_ = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));           \
    const uint32_t mj_ = bitop3<0xE8>(a, b, c);                                \
    h = t1_ + s0_ + mj_;                                                       \
  } while (0)

__device__ __forceinline__ void sha256_compress(uint32_t (&st)[8], uint32_t (&W)[16]) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6],
           h = st[7];
#pragma unroll
  for (int t = 0; t < 64; t += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = t + u;
      if (i >= 16) {
        const uint32_t w15 = W[(i - 15) & 15], w2 = W[(i - 2) & 15];
        const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
        const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
        W[i & 15] = (W[i & 15] + s0) + (W[(i - 7) & 15] + s1);
      }
    }
    SHA_ROUND(a, b, c, d, e, f, g, h, kK256[t + 0] + W[(t + 0) & 15]);
    SHA_ROUND(h, a, b, c, d, e, f, g, kK256[t + 1] + W[(t + 1) & 15]);
    SHA_ROUND(g, h, a, b, c, d, e, f, kK256[t + 2] + W[(t + 2) & 15]);
    SHA_ROUND(f, g, h, a, b, c, d, e, kK256[t + 3] + W[(t + 3) & 15]);
    SHA_ROUND(e, f, g, h, a, b, c, d, kK256[t + 4] + W[(t + 4) & 15]);
    SHA_ROUND(d, e, f, g, h, a, b, c, kK256[t + 5] + W[(t + 5) & 15]);
    SHA_ROUND(c, d, e, f, g, h, a, b, kK256[t + 6] + W[(t + 6) & 15]);
    SHA_ROUND(b, c, d, e, f, g, h, a, kK256[t + 7] + W[(t + 7) & 15]);
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d;
  st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}


// The same compression as one generated asm statement (tools/gen_lane_asm.py): every
// instruction 8 bytes and 8-byte aligned. hipcc's own schedule of sha256_compress mixes 4- and
// 8-byte encodings with about half its 8-byte instructions at 4 mod 8, and takes 235 VGPRs in
// k_sha against 188 with this one. A lone wave runs both at ~6,000 cycles per block
// (profiles/r05_lanes_align.log); in k_sha under the configs[2] load the asm form takes k_sha
// from 13.44 to 13.10 ms (profiles/r05_ab8.log). k_sha_blobs uses it; k_sha's per-lane mode
// uses sha256_compress_kv below (K from resident VGPRs).
#include "sha256_lane_asm.inc"
__device__ __forceinline__ void sha256_compress_aligned(uint32_t (&st)[8], uint32_t (&W)[16]) {
  uint32_t x0, x1, x2, x3, x4, x5, x6, x7, t0, t1, t2, t3, t4, t5, k;
  asm volatile(BSG_LANE_COMPRESS_ASM
               : [st0] "+v"(st[0]), [st1] "+v"(st[1]), [st2] "+v"(st[2]), [st3] "+v"(st[3]),
                 [st4] "+v"(st[4]), [st5] "+v"(st[5]), [st6] "+v"(st[6]), [st7] "+v"(st[7]),
                 [w0] "+v"(W[0]), [w1] "+v"(W[1]), [w2] "+v"(W[2]), [w3] "+v"(W[3]),
                 [w4] "+v"(W[4]), [w5] "+v"(W[5]), [w6] "+v"(W[6]), [w7] "+v"(W[7]),
                 [w8] "+v"(W[8]), [w9] "+v"(W[9]), [w10] "+v"(W[10]), [w11] "+v"(W[11]),
                 [w12] "+v"(W[12]), [w13] "+v"(W[13]), [w14] "+v"(W[14]), [w15] "+v"(W[15]),
                 [x0] "=&v"(x0), [x1] "=&v"(x1), [x2] "=&v"(x2), [x3] "=&v"(x3),
                 [x4] "=&v"(x4), [x5] "=&v"(x5), [x6] "=&v"(x6), [x7] "=&v"(x7),
                 [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3),
                 [t4] "=&v"(t4), [t5] "=&v"(t5), [k] "=&s"(k));
}

// The same with K from 64 VGPRs the caller keeps resident (sha256_k_regs): no s_mov per round,
// for a wave that runs alone on its SIMD and issues every instruction at ~4 cycles, VALU or
// not (k_sha's per-lane mode: 5,782 against 5,979 cycles per block, tools/ubench/lanes_align.hip,
// profiles/r05_lanes_v4.log).
__device__ __forceinline__ void sha256_k_regs(uint32_t (&kv)[64]) {
#pragma unroll
  for (int i = 0; i < 64; ++i)  // opaque moves: the values stay in registers, not rematerialised
    asm volatile("v_mov_b32 %0, %1" : "=v"(kv[i]) : "i"(kK256[i]));
}
__device__ __forceinline__ void sha256_compress_kv(uint32_t (&st)[8], uint32_t (&W)[16],
                                                   const uint32_t (&kv)[64]) {
  uint32_t x0, x1, x2, x3, x4, x5, x6, x7, t0, t1, t2, t3, t4, t5;
  asm volatile(BSG_LANE_COMPRESS_ASM_KV
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
               : [k0] "v"(kv[0]), [k1] "v"(kv[1]), [k2] "v"(kv[2]), [k3] "v"(kv[3]),
                 [k4] "v"(kv[4]), [k5] "v"(kv[5]), [k6] "v"(kv[6]), [k7] "v"(kv[7]),
                 [k8] "v"(kv[8]), [k9] "v"(kv[9]), [k10] "v"(kv[10]), [k11] "v"(kv[11]),
                 [k12] "v"(kv[12]), [k13] "v"(kv[13]), [k14] "v"(kv[14]), [k15] "v"(kv[15]),
                 [k16] "v"(kv[16]), [k17] "v"(kv[17]), [k18] "v"(kv[18]), [k19] "v"(kv[19]),
                 [k20] "v"(kv[20]), [k21] "v"(kv[21]), [k22] "v"(kv[22]), [k23] "v"(kv[23]),
                 [k24] "v"(kv[24]), [k25] "v"(kv[25]), [k26] "v"(kv[26]), [k27] "v"(kv[27]),
                 [k28] "v"(kv[28]), [k29] "v"(kv[29]), [k30] "v"(kv[30]), [k31] "v"(kv[31]),
                 [k32] "v"(kv[32]), [k33] "v"(kv[33]), [k34] "v"(kv[34]), [k35] "v"(kv[35]),
                 [k36] "v"(kv[36]), [k37] "v"(kv[37]), [k38] "v"(kv[38]), [k39] "v"(kv[39]),
                 [k40] "v"(kv[40]), [k41] "v"(kv[41]), [k42] "v"(kv[42]), [k43] "v"(kv[43]),
                 [k44] "v"(kv[44]), [k45] "v"(kv[45]), [k46] "v"(kv[46]), [k47] "v"(kv[47]),
                 [k48] "v"(kv[48]), [k49] "v"(kv[49]), [k50] "v"(kv[50]), [k51] "v"(kv[51]),
                 [k52] "v"(kv[52]), [k53] "v"(kv[53]), [k54] "v"(kv[54]), [k55] "v"(kv[55]),
                 [k56] "v"(kv[56]), [k57] "v"(kv[57]), [k58] "v"(kv[58]), [k59] "v"(kv[59]),
                 [k60] "v"(kv[60]), [k61] "v"(kv[61]), [k62] "v"(kv[62]), [k63] "v"(kv[63]));
}

// Variant for experiments (tools/ubench): plain C operators, left to hipcc's selection.
#define SHA_ROUND_C(a, b, c, d, e, f, g, h, kw)                               \
  do {                                                                         \
    const uint32_t s1_ = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);               \
    const uint32_t ch_ = (e & f) | (~e & g);                                   \
    const uint32_t t1_ = (h + (kw)) + s1_ + ch_;                               \
    d += t1_;                                                                  \
    const uint32_t s0_ = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);               \
    const uint32_t mj_ = (a & b) | (c & (a | b));                              \
    h = t1_ + s0_ + mj_;                                                       \
  } while (0)

template <bool ASM>
__device__ __forceinline__ void sha256_compress_v(uint32_t (&st)[8], uint32_t (&W)[16]) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6],
           h = st[7];
#pragma unroll
  for (int t = 0; t < 64; t += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = t + u;
      if (i >= 16) {
        const uint32_t w15 = W[(i - 15) & 15], w2 = W[(i - 2) & 15];
        uint32_t s0, s1;
        if (ASM) {
          s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
          s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
        } else {
          s0 = rotr(w15, 7) ^ rotr(w15, 18) ^ (w15 >> 3);
          s1 = rotr(w2, 17) ^ rotr(w2, 19) ^ (w2 >> 10);
        }
        W[i & 15] = (W[i & 15] + s0) + (W[(i - 7) & 15] + s1);
      }
    }
#define R_(...) do { if (ASM) SHA_ROUND(__VA_ARGS__); else SHA_ROUND_C(__VA_ARGS__); } while (0)
    R_(a, b, c, d, e, f, g, h, kK256[t + 0] + W[(t + 0) & 15]);
    R_(h, a, b, c, d, e, f, g, kK256[t + 1] + W[(t + 1) & 15]);
    R_(g, h, a, b, c, d, e, f, kK256[t + 2] + W[(t + 2) & 15]);
    R_(f, g, h, a, b, c, d, e, kK256[t + 3] + W[(t + 3) & 15]);
    R_(e, f, g, h, a, b, c, d, kK256[t + 4] + W[(t + 4) & 15]);
    R_(d, e, f, g, h, a, b, c, kK256[t + 5] + W[(t + 5) & 15]);
    R_(c, d, e, f, g, h, a, b, kK256[t + 6] + W[(t + 6) & 15]);
    R_(b, c, d, e, f, g, h, a, kK256[t + 7] + W[(t + 7) & 15]);
#undef R_
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d;
  st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// Rounds only, with K[t] + W[t] precomputed elsewhere (long-chain path experiments).
template <bool ASM>
__device__ __forceinline__ void sha256_rounds_kw(uint32_t (&st)[8], const uint32_t (&KW)[64]) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6],
           h = st[7];
#pragma unroll
  for (int t = 0; t < 64; t += 8) {
#define R_(...) do { if (ASM) SHA_ROUND(__VA_ARGS__); else SHA_ROUND_C(__VA_ARGS__); } while (0)
    R_(a, b, c, d, e, f, g, h, KW[t + 0]);
    R_(h, a, b, c, d, e, f, g, KW[t + 1]);
    R_(g, h, a, b, c, d, e, f, KW[t + 2]);
    R_(f, g, h, a, b, c, d, e, KW[t + 3]);
    R_(e, f, g, h, a, b, c, d, KW[t + 4]);
    R_(d, e, f, g, h, a, b, c, KW[t + 5]);
    R_(c, d, e, f, g, h, a, b, KW[t + 6]);
    R_(b, c, d, e, f, g, h, a, KW[t + 7]);
#undef R_
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d;
  st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// ---------------------------------------------------------------------------------------------
// Banked lane pair for one long chain (wave mode). A single chain is bound by one wave's issue
// rate (~4.5 cycles per instruction, dependent or not; an s_nop wait state costs the same), so
// what counts is instructions per round. The round is split over two lanes that run the same
// 10 instructions (14 for the whole round in one lane), the E lane holding (e,f,g,h) and the
// A lane (a,b,c,d):
//   S = Sigma(R1): 3 x v_alignbit with per-lane counts + xor3      E: Sigma1(e)     A: Sigma0(a)
//   x = R1 ^ (R3 & xm)          (xm = 0 on E, ~0 on A)             E: e             A: a^c
//   F = Ch(x, R2, R3)                                               E: Ch(e,f,g)     A: Maj(a,b,c)
//   U = S + F + Q                                                   E: T1 + d = e'   A: T2 - d
//   n = U + U(lane-1), written on A lanes only (DPP bank mask)     E: e'            A: T1 + T2 = a'
// with Q prepared during the previous round (in the DPP hazard shadow of U):
//   P = (R4 ^ xm) + kwl         (kwl = K+W on E, 1 on A)           E: h + KW        A: -d
//   Q = P + R4(lane+1), written on E lanes only                     E: h + KW + d    A: -d
// DPP bank masks pick lanes in groups of 4 (bank k of a 16-lane row = lanes 4k..4k+3), so the
// pair is (lane 3, lane 4) of every 8: E lanes are those with lane & 4 == 0. The other lanes
// compute garbage and are ignored. kwl comes from a per-lane LDS row (E lanes: the block's K+W
// row; A lanes: a row of ones).
struct BankLane {
  uint32_t rot1, rot2, rot3, xm;
  bool a_side;
};

__device__ __forceinline__ BankLane bank_lane() {
  BankLane b;
  b.a_side = (threadIdx.x & 4u) != 0u;
  b.rot1 = b.a_side ? 2u : 6u;
  b.rot2 = b.a_side ? 13u : 11u;
  b.rot3 = b.a_side ? 22u : 25u;
  b.xm = b.a_side ? 0xffffffffu : 0u;
  return b;
}
constexpr uint32_t kBankE = 3, kBankA = 4;  // the lanes holding (e,f,g,h) and (a,b,c,d)

// One round, hand-scheduled in one asm block (the compiler's own schedule left the DPP
// source hazards to s_nop). q in: this round's Q; out: the next round's (from kwn).
__device__ __forceinline__ void bank_round(uint32_t& r1, uint32_t& r2, uint32_t& r3,
                                           uint32_t& r4, uint32_t& q, uint32_t kwn,
                                           const BankLane& b) {
  uint32_t u, qn, t0, t1, t2, x;
  asm("v_alignbit_b32 %[t0], %[r1], %[r1], %[s1]\n\t"
      "v_alignbit_b32 %[t1], %[r1], %[r1], %[s2]\n\t"
      "v_alignbit_b32 %[t2], %[r1], %[r1], %[s3]\n\t"
      "v_bitop3_b32 %[x], %[r1], %[r3], %[xm] bitop3:0x78\n\t"
      "v_bitop3_b32 %[t0], %[t0], %[t1], %[t2] bitop3:0x96\n\t"
      "v_bitop3_b32 %[x], %[x], %[r2], %[r3] bitop3:0xca\n\t"
      "v_add3_u32 %[u], %[t0], %[x], %[q]\n\t"
      "v_xad_u32 %[qn], %[r3], %[xm], %[kwn]\n\t"
      "v_add_u32_dpp %[qn], %[r3], %[qn] row_shl:1 row_mask:0xf bank_mask:0x5\n\t"
      "v_add_u32_dpp %[u], %[u], %[u] row_shr:1 row_mask:0xf bank_mask:0xa"
      : [u] "=&v"(u), [qn] "=&v"(qn), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2),
        [x] "=&v"(x)
      : [r1] "v"(r1), [r2] "v"(r2), [r3] "v"(r3), [q] "v"(q), [kwn] "v"(kwn),
        [s1] "v"(b.rot1), [s2] "v"(b.rot2), [s3] "v"(b.rot3), [xm] "v"(b.xm));
  r4 = r3;
  r3 = r2;
  r2 = r1;
  r1 = u;
  q = qn;
}

// Q of round 0 of a block, from the block's starting state.
__device__ __forceinline__ uint32_t bank_q0(uint32_t r4, uint32_t kw0, const BankLane& b) {
  uint32_t q;
  asm("v_xad_u32 %[q], %[r4], %[xm], %[kw]\n\t"
      "s_nop 1\n\t"
      "v_add_u32_dpp %[q], %[r4], %[q] row_shl:1 row_mask:0xf bank_mask:0x5"
      : [q] "=&v"(q)
      : [r4] "v"(r4), [xm] "v"(b.xm), [kw] "v"(kw0));
  return q;
}

// 64 rounds on this lane's half state s[4] (E: H4..H7, A: H0..H3) from this lane's LDS row
// (16 x 16 B); adds the block result into s if `active` (lanes of finished chains keep theirs).
__device__ __forceinline__ void sha256_rounds_bank(uint32_t (&s)[4], const uint32_t* row,
                                                   const BankLane& b, bool active = true) {
  typedef uint32_t u32x4r __attribute__((ext_vector_type(4), aligned(16)));
  const u32x4r* r = reinterpret_cast<const u32x4r*>(row);
  uint32_t r1 = s[0], r2 = s[1], r3 = s[2], r4 = s[3];
  u32x4r kw = r[0];
  uint32_t q = bank_q0(r4, kw.x, b);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const u32x4r kn = r[i < 15 ? i + 1 : 15];
    bank_round(r1, r2, r3, r4, q, kw.y, b);
    bank_round(r1, r2, r3, r4, q, kw.z, b);
    bank_round(r1, r2, r3, r4, q, kw.w, b);
    bank_round(r1, r2, r3, r4, q, kn.x, b);  // after round 63 this Q is not used
    kw = kn;
  }
  // 64 rounds (a multiple of 4): the names are back in place, r1 = e|a ...
  s[0] = active ? s[0] + r1 : s[0];
  s[1] = active ? s[1] + r2 : s[1];
  s[2] = active ? s[2] + r3 : s[2];
  s[3] = active ? s[3] + r4 : s[3];
}

// ---------------------------------------------------------------------------------------------
// Skewed lane pair (wave mode, default). Same split of the state as the banked pair, but the
// E lane runs two rounds AHEAD of the A lane, and the two lanes of a pair (2p, 2p+1: E even,
// A odd) swap one register per round with quad_perm:[1,0,3,2], which needs no bank mask since
// both lanes keep the DPP result. Register slot V(j) holds e_{j+2} on E lanes and a_j on A
// lanes; iteration i (R1..R4 = V(i-1)..V(i-4)) computes V(i):
//   P = (R4 ^ xm) + kwl          E: e_{i-2} + KW_{i+1}          A: -a_{i-4}
//   Z = P + R2(other lane)       E: h + KW + d of round i+1      A: e_i - a_{i-4} = T1 of round i-1
//   S = Sigma(R1), F = Ch(R1 ^ (R3 & xm), R2, R3)               E: Sigma1, Ch    A: Sigma0, Maj
//   V(i) = S + F + Z             E: e_{i+2}                      A: a_i
// Each lane needs from the other only a value written two iterations earlier, so there is no
// DPP hazard to wait out: 9 VALU issue slots per round (the banked pair takes 10 + 1 s_nop).
// A block is iterations -1 .. 64: in -1 and 0 only the E lane's result is kept (the A lane's
// a_{-1}, a_0 are the chaining values), in 63 and 64 only the A lane's (the E lane keeps e_61,
// e_62). A lane's half state hs[4] is (H0,H1,H2,H3) on A lanes and (H6,H7,H4,H5) on E lanes, so
// that the feed-forward hs[k] += V(64-k) is the same instruction on both lanes.
struct SkewLane {
  uint32_t rot1, rot2, rot3, xm;
  bool a_side;
};

__device__ __forceinline__ SkewLane skew_lane() {
  SkewLane b;
  b.a_side = (threadIdx.x & 1u) != 0u;
  b.rot1 = b.a_side ? 2u : 6u;
  b.rot2 = b.a_side ? 13u : 11u;
  b.rot3 = b.a_side ? 22u : 25u;
  b.xm = b.a_side ? 0xffffffffu : 0u;
  return b;
}

// One block (64 rounds) on this lane's half state from its LDS row (E lanes: the block's 64
// K+W words; A lanes: 64 ones), 16-byte aligned; feed-forward only if `active`. The 66
// iterations are one generated asm statement (tools/gen_skew_asm.py documents the schedule):
// as separate asm blocks, each containing the DPP exchange, hipcc put an s_nop in front of
// every other one.
#include "sha256_skew_block.inc"
__device__ __forceinline__ void sha256_rounds_skew(uint32_t (&hs)[4], const uint32_t* row,
                                                   const SkewLane& b, bool active = true) {
  // slot s holds V(j), j = s (mod 4): V(-2) = H4|H2, V(-3) = H5|H3, V(-4) = H6|-, V(-5) = H7|H1
  uint32_t v2 = hs[2], v1 = hs[3], v0 = hs[0], v3 = hs[1];
  const uint32_t addr = (uint32_t)reinterpret_cast<uintptr_t>(
      (__attribute__((address_space(3))) const uint32_t*)row);
  const uint64_t amask = 0xAAAAAAAAAAAAAAAAull;  // A lanes: odd
  asm volatile(BSG_SKEW_BLOCK_ASM
               : [v0] "+v"(v0), [v1] "+v"(v1), [v2] "+v"(v2), [v3] "+v"(v3)
               : [row] "v"(addr), [xm] "v"(b.xm), [s1] "v"(b.rot1), [s2] "v"(b.rot2),
                 [s3] "v"(b.rot3), [amask] "s"(amask)
               : "memory", BSG_SKEW_BLOCK_CLOBBERS);
  if (active) {
    hs[0] += v0;  // A: a_64 -> H0 | E: e_62 -> H6
    hs[1] += v3;  // A: a_63 -> H1 | E: e_61 -> H7
    hs[2] += v2;  // A: a_62 -> H2 | E: e_64 -> H4
    hs[3] += v1;  // A: a_61 -> H3 | E: e_63 -> H5
  }
}

// `nblk` consecutive blocks (wave-uniform) of the skewed pairs, block k's K+W row at
// row + k * stride bytes (A lanes: stride 0 on their row of ones), as one asm loop
// (tools/gen_skew_asm.py, main_loop). A lane pair whose chain has only `lim` blocks left stops
// after them (exec-masked), keeping its final state in hs.
#include "sha256_skew_loop.inc"
__device__ __forceinline__ void sha256_blocks_skew(uint32_t (&hs)[4], const uint32_t* row,
                                                   uint32_t stride, uint32_t nblk, int32_t lim,
                                                   const SkewLane& b) {
  if (nblk == 0) return;
  // wave-uniform, but under register pressure hipcc may hold it in a VGPR, which the "s"
  // operand below does not stop (the loop's s_cmp then fails to assemble)
  nblk = (uint32_t)__builtin_amdgcn_readfirstlane((int)nblk);
  const uint32_t addr = (uint32_t)reinterpret_cast<uintptr_t>(
      (__attribute__((address_space(3))) const uint32_t*)row);
  const uint64_t amask = 0xAAAAAAAAAAAAAAAAull;  // A lanes: odd
  uint32_t cnt;
  uint64_t sexec;
  asm volatile(BSG_SKEW_LOOP_ASM
               : [h0] "+v"(hs[0]), [h1] "+v"(hs[1]), [h2] "+v"(hs[2]), [h3] "+v"(hs[3]),
                 [cnt] "=&s"(cnt), [sexec] "=&s"(sexec)
               : [addr] "v"(addr), [stride] "v"(stride), [nblk] "s"(nblk), [lim] "v"(lim),
                 [xm] "v"(b.xm), [s1] "v"(b.rot1), [s2] "v"(b.rot2), [s3] "v"(b.rot3),
                 [amask] "s"(amask)
               : "memory", BSG_SKEW_LOOP_CLOBBERS);
}

// ---------------------------------------------------------------------------------------------
// Skewed octet (wave mode, solo and group tickets): one chain per 8 lanes, E quad at octet
// positions 0-3, A quad at 4-7, every lane of a quad holding the same values. Same skew and
// slot convention as the pair; a Sigma is one per-lane-count rotate (quad positions rotate by
// 6, 11, 25, 6 on E, by 2, 13, 22, 2 on A) and two DPP xors within the quad, and the exchange
// reads the mirror lane of the half-row (always in the other quad): 8 VALU per round, 64
// bytes of code, against the pair's 9 and 72 (tools/gen_skew_asm.py, main_loop_oct).
struct OctLane {
  uint32_t rot, xm;
  bool a_side;
};

__device__ __forceinline__ OctLane oct_lane() {
  OctLane b;
  const uint32_t p = threadIdx.x & 7u;
  b.a_side = p >= 4u;
  const uint32_t q = p & 3u;
  // E: 6, 11, 25, 6   A: 2, 13, 22, 2
  const uint32_t re = q == 1u ? 11u : (q == 2u ? 25u : 6u);
  const uint32_t ra = q == 1u ? 13u : (q == 2u ? 22u : 2u);
  b.rot = b.a_side ? ra : re;
  b.xm = b.a_side ? 0xffffffffu : 0u;
  return b;
}

// `nblk` consecutive blocks (wave-uniform) of the skewed octets, block k's K+W row at
// row + k * stride bytes (A lanes: stride 0 on their row of ones); an octet whose chain has
// only `lim` blocks left stops after them (exec-masked). hs as for the pair: A lanes
// (H0,H1,H2,H3), E lanes (H6,H7,H4,H5).
#include "sha256_oct_loop.inc"
__device__ __forceinline__ void sha256_blocks_oct(uint32_t (&hs)[4], const uint32_t* row,
                                                  uint32_t stride, uint32_t nblk, int32_t lim,
                                                  const OctLane& b) {
  if (nblk == 0) return;
  // wave-uniform, but under register pressure hipcc may hold it in a VGPR, which the "s"
  // operand below does not stop (the loop's s_cmp then fails to assemble)
  nblk = (uint32_t)__builtin_amdgcn_readfirstlane((int)nblk);
  const uint32_t addr = (uint32_t)reinterpret_cast<uintptr_t>(
      (__attribute__((address_space(3))) const uint32_t*)row);
  const uint64_t amask = 0xF0F0F0F0F0F0F0F0ull;  // A lanes: octet positions 4-7
  uint32_t cnt;
  uint64_t sexec;
  asm volatile(BSG_OCT_LOOP_ASM
               : [h0] "+v"(hs[0]), [h1] "+v"(hs[1]), [h2] "+v"(hs[2]), [h3] "+v"(hs[3]),
                 [cnt] "=&s"(cnt), [sexec] "=&s"(sexec)
               : [addr] "v"(addr), [stride] "v"(stride), [nblk] "s"(nblk), [lim] "v"(lim),
                 [xm] "v"(b.xm), [s1] "v"(b.rot), [amask] "s"(amask)
               : "memory", BSG_OCT_LOOP_CLOBBERS);
}

// The same loop for a chain that runs alone in its wave (every octet the same chain: solo
// tickets, helped solo chains, k_early): no per-block exec update, no slot copies, K+W quads
// read eight at a time and no s_nop (tools/gen_skew_asm.py, main_loop_oct_solo): 560
// instructions per block against 570.
#include "sha256_oct_solo_loop.inc"
__device__ __forceinline__ void sha256_blocks_oct_solo(uint32_t (&hs)[4], const uint32_t* row,
                                                       uint32_t stride, uint32_t nblk,
                                                       const OctLane& b) {
  if (nblk == 0) return;
  nblk = (uint32_t)__builtin_amdgcn_readfirstlane((int)nblk);  // (see sha256_blocks_oct)
  const uint32_t addr = (uint32_t)reinterpret_cast<uintptr_t>(
      (__attribute__((address_space(3))) const uint32_t*)row);
  const uint64_t amask = 0xF0F0F0F0F0F0F0F0ull;  // A lanes: octet positions 4-7
  uint32_t cnt;
  asm volatile(BSG_OCT_SOLO_LOOP_ASM
               : [h0] "+v"(hs[0]), [h1] "+v"(hs[1]), [h2] "+v"(hs[2]), [h3] "+v"(hs[3]),
                 [cnt] "=&s"(cnt)
               : [addr] "v"(addr), [stride] "v"(stride), [nblk] "s"(nblk), [xm] "v"(b.xm),
                 [s1] "v"(b.rot), [amask] "s"(amask)
               : "memory", BSG_OCT_SOLO_LOOP_CLOBBERS);
}

}  // namespace bsg

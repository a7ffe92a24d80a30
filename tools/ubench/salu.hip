// Microbenchmark: lone-wave SALU issue rate and SALU/VALU co-issue (whole timed loop in asm).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int V>
__global__ void kb(uint64_t* out, uint32_t* sink, uint32_t seed) {
  uint64_t t0, t1, r0, r1;
  uint32_t v0 = threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7;
  uint32_t s0 = seed, s1 = seed * 3, s2 = seed * 5, s3 = seed * 7, cnt = 1000;
  asm volatile("s_memtime %0\n s_memrealtime %1\n s_waitcnt lgkmcnt(0)" : "=s"(t0), "=s"(r0) :: "memory");
  if (V == 0)  // 4 independent SALU add chains, 128 instrs per iteration
    asm volatile("1:\n .rept 32\n s_add_u32 %0, %0, %1\n s_add_u32 %1, %1, %2\n s_add_u32 %2, %2, %3\n s_add_u32 %3, %3, %0\n .endr\n s_sub_u32 %4, %4, 1\n s_cmp_lg_u32 %4, 0\n s_cbranch_scc1 1b"
                 : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(cnt) :: "scc");
  if (V == 1)  // dependent SALU chain
    asm volatile("1:\n .rept 128\n s_add_u32 %0, %0, %1\n .endr\n s_sub_u32 %4, %4, 1\n s_cmp_lg_u32 %4, 0\n s_cbranch_scc1 1b"
                 : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(cnt) :: "scc");
  if (V == 2)  // 64-bit shifts (rotate of a duplicated pair), 4 independent
    asm volatile("s_mov_b32 s60, %0\n s_mov_b32 s61, %0\n s_mov_b32 s62, %1\n s_mov_b32 s63, %1\n 1:\n .rept 32\n s_lshl_b64 s[60:61], s[60:61], 3\n s_lshl_b64 s[62:63], s[62:63], 5\n s_lshr_b64 s[64:65], s[60:61], 7\n s_lshr_b64 s[66:67], s[62:63], 9\n .endr\n s_sub_u32 %4, %4, 1\n s_cmp_lg_u32 %4, 0\n s_cbranch_scc1 1b"
                 : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(cnt) :: "scc", "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67");
  if (V == 3)  // VALU (indep) + SALU (indep) interleaved 1:1, 64 + 64 per iteration
    asm volatile("1:\n .rept 16\n v_add_u32 %5, %5, %6\n s_add_u32 %0, %0, %1\n v_add_u32 %6, %6, %7\n s_add_u32 %1, %1, %2\n v_add_u32 %7, %7, %8\n s_add_u32 %2, %2, %3\n v_add_u32 %8, %8, %5\n s_add_u32 %3, %3, %0\n .endr\n s_sub_u32 %4, %4, 1\n s_cmp_lg_u32 %4, 0\n s_cbranch_scc1 1b"
                 : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(cnt), "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3) :: "scc");
  if (V == 4)  // VALU : SALU = 1 : 2
    asm volatile("1:\n .rept 16\n v_add_u32 %5, %5, %6\n s_add_u32 %0, %0, %1\n s_add_u32 %1, %1, %2\n v_add_u32 %6, %6, %7\n s_add_u32 %2, %2, %3\n s_add_u32 %3, %3, %0\n .endr\n s_sub_u32 %4, %4, 1\n s_cmp_lg_u32 %4, 0\n s_cbranch_scc1 1b"
                 : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(cnt), "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3) :: "scc");
  if (V == 5)  // VALU only, same loop shape (64 per iteration)
    asm volatile("1:\n .rept 16\n v_add_u32 %5, %5, %6\n v_add_u32 %6, %6, %7\n v_add_u32 %7, %7, %8\n v_add_u32 %8, %8, %5\n .endr\n s_sub_u32 %4, %4, 1\n s_cmp_lg_u32 %4, 0\n s_cbranch_scc1 1b"
                 : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(cnt), "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3) :: "scc");
  asm volatile("s_memtime %0\n s_memrealtime %1\n s_waitcnt lgkmcnt(0)" : "=s"(t1), "=s"(r1) :: "memory");
  sink[threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ s0 ^ s1 ^ s2 ^ s3;
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = r1 - r0; }
}

template <int V> void run(const char* name, double instrs_per_iter) {
  uint64_t* d; uint32_t* s; hipMalloc(&d, 16); hipMalloc(&s, 4096);
  for (int k = 0; k < 2; ++k) { hipLaunchKernelGGL(kb<V>, dim3(1), dim3(64), 0, 0, d, s, 12345u); hipDeviceSynchronize(); }
  uint64_t h[2]; hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
  printf("%-44s %.2f cycles/instr  (%.2f GHz)\n", name, (double)h[0] / (1000.0 * instrs_per_iter), (double)h[0] / (h[1] * 10.0));
  hipFree(d); hipFree(s);
}
int main() {
  run<0>("SALU s_add, 4 indep chains", 128);
  run<1>("SALU s_add, dependent chain", 128);
  run<2>("SALU s_lshl/lshr_b64, 4 indep", 128);
  run<3>("VALU+SALU 1:1 (per instr, 128/iter)", 128);
  run<4>("VALU+SALU 1:2 (per instr, 96/iter)", 96);
  run<5>("VALU only (per instr, 64/iter)", 64);
  return 0;
}

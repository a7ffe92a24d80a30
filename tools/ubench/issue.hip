// Microbenchmark: lone-wave issue rates on gfx950 (cycles via s_memtime, clock via s_memrealtime).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define STAMP(t) asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory")
#define RSTAMP(t) asm volatile("s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory")

template <int V>
__global__ void kb(uint64_t* out, uint32_t* sink, int iters) {
  uint32_t a = threadIdx.x, b = a * 3, c = a * 5, d = a * 7, e = a + 11, f = a + 13, g = a + 17, h = a + 19;
  uint32_t sa = 1, sb = 2, sc = 3, sd = 4;
  uint64_t t0, t1, r0, r1;
  if (V == 1) asm volatile("s_mov_b32 exec_hi, 0" ::: "memory");           // 32 lanes
  if (V == 2) asm volatile("s_mov_b32 exec_hi, 0\n s_mov_b32 exec_lo, 1" ::: "memory");  // 1 lane
  STAMP(t0); RSTAMP(r0);
  for (int i = 0; i < iters; ++i) {
    if (V <= 2)  // 8 independent chains of v_add (VALU throughput)
      asm volatile(".rept 16\n v_add_u32 %0, %0, %1\n v_add_u32 %1, %1, %2\n v_add_u32 %2, %2, %3\n v_add_u32 %3, %3, %4\n v_add_u32 %4, %4, %5\n v_add_u32 %5, %5, %6\n v_add_u32 %6, %6, %7\n v_add_u32 %7, %7, %0\n .endr"
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h));
    if (V == 3)  // one dependent chain (latency)
      asm volatile(".rept 128\n v_add_u32 %0, %0, %1\n .endr" : "+v"(a) : "v"(b));
    if (V == 4)  // dependent chain of v_bitop3
      asm volatile(".rept 128\n v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96\n .endr" : "+v"(a) : "v"(b), "v"(c));
    if (V == 5)  // dependent chain of alignbit
      asm volatile(".rept 128\n v_alignbit_b32 %0, %0, %0, 7\n .endr" : "+v"(a));
    if (V == 6)  // SALU only (4 independent chains)
      asm volatile(".rept 32\n s_add_u32 %0, %0, %1\n s_add_u32 %1, %1, %2\n s_add_u32 %2, %2, %3\n s_add_u32 %3, %3, %0\n .endr"
                   : "+s"(sa), "+s"(sb), "+s"(sc), "+s"(sd));
    if (V == 7)  // VALU + SALU interleaved 1:1 (128 of each)
      asm volatile(".rept 16\n v_add_u32 %0, %0, %1\n s_add_u32 %8, %8, %9\n v_add_u32 %1, %1, %2\n s_add_u32 %9, %9, %10\n v_add_u32 %2, %2, %3\n s_add_u32 %10, %10, %11\n v_add_u32 %3, %3, %4\n s_add_u32 %11, %11, %8\n v_add_u32 %4, %4, %5\n s_add_u32 %8, %8, %9\n v_add_u32 %5, %5, %6\n s_add_u32 %9, %9, %10\n v_add_u32 %6, %6, %7\n s_add_u32 %10, %10, %11\n v_add_u32 %7, %7, %0\n s_add_u32 %11, %11, %8\n .endr"
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h), "+s"(sa), "+s"(sb), "+s"(sc), "+s"(sd));
    if (V == 8)  // 2 independent chains of alignbit->bitop3->add3 (SHA-like ILP 2)
      asm volatile(".rept 32\n v_alignbit_b32 %0, %0, %0, 7\n v_alignbit_b32 %1, %1, %1, 7\n v_bitop3_b32 %0, %0, %2, %3 bitop3:0x96\n v_bitop3_b32 %1, %1, %2, %3 bitop3:0x96\n v_add3_u32 %0, %0, %2, %3\n v_add3_u32 %1, %1, %2, %3\n .endr"
                   : "+v"(a), "+v"(b) : "v"(c), "v"(d));
  }
  STAMP(t1); RSTAMP(r1);
  if (V == 1 || V == 2) asm volatile("s_mov_b64 exec, -1" ::: "memory");
  sink[threadIdx.x] = a ^ b ^ c ^ d ^ e ^ f ^ g ^ h ^ sa ^ sb ^ sc ^ sd;
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = r1 - r0; }
}

template <int V> void run(const char* name, int instrs_per_iter, int waves_per_simd) {
  uint64_t* d; uint32_t* s; hipMalloc(&d, 16); hipMalloc(&s, 4096 * 4);
  int iters = 2000;
  // waves_per_simd waves in one WG: 4 SIMDs per CU, waves go to SIMDs round-robin
  int threads = 64 * (waves_per_simd == 1 ? 1 : 4 * waves_per_simd);
  hipLaunchKernelGGL(kb<V>, dim3(1), dim3(threads), 0, 0, d, s, iters);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(kb<V>, dim3(1), dim3(threads), 0, 0, d, s, iters);
  hipDeviceSynchronize();
  uint64_t h[2]; hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
  double cyc = (double)h[0] / ((double)iters * instrs_per_iter);
  double ghz = (double)h[0] / ((double)h[1] * 10.0);  // realtime = 100 MHz
  printf("%-44s waves/SIMD=%d  %.2f cycles/instr (clock %.2f GHz)\n", name, waves_per_simd, cyc, ghz);
  hipFree(d); hipFree(s);
}

int main() {
  run<0>("VALU v_add, 8 indep chains, 64 lanes", 128, 1);
  run<0>("VALU v_add, 8 indep chains, 64 lanes", 128, 2);
  run<1>("VALU v_add, 8 indep chains, 32 lanes", 128, 1);
  run<2>("VALU v_add, 8 indep chains, 1 lane", 128, 1);
  run<3>("VALU v_add dependent chain", 128, 1);
  run<4>("v_bitop3 dependent chain", 128, 1);
  run<5>("v_alignbit dependent chain", 128, 1);
  run<6>("SALU s_add 4 indep chains", 128, 1);
  run<7>("VALU+SALU interleaved (per VALU instr)", 128, 1);
  run<8>("alignbit->bitop3->add3 x2 chains", 192, 1);
  return 0;
}

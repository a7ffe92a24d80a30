#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define STAMP(t) asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory")
__global__ __launch_bounds__(64) void k0(uint64_t* out, uint32_t* sink, int iters) {
  uint32_t a = threadIdx.x, b = a * 3 + 1, c = a * 5 + 2, d = a * 7 + 3, x = a ^ 9, y = a + 5;
  uint32_t r = (threadIdx.x & 1) ? 13u : 7u;
  uint64_t t0, t1;
  STAMP(t0);
  for (int i = 0; i < iters; ++i)
    asm volatile(".rept 16\nv_add3_u32 %0, %0, %4, %5\nv_add3_u32 %1, %1, %4, %5\nv_add3_u32 %2, %2, %4, %5\nv_add3_u32 %3, %3, %4, %5\n.endr" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y), "v"(r) : "s0", "s1", "scc");
  STAMP(t1);
  sink[threadIdx.x] = a ^ b ^ c ^ d;
  if (threadIdx.x == 0) out[0] = t1 - t0;
}
__global__ __launch_bounds__(64) void k1(uint64_t* out, uint32_t* sink, int iters) {
  uint32_t a = threadIdx.x, b = a * 3 + 1, c = a * 5 + 2, d = a * 7 + 3, x = a ^ 9, y = a + 5;
  uint32_t r = (threadIdx.x & 1) ? 13u : 7u;
  uint64_t t0, t1;
  STAMP(t0);
  for (int i = 0; i < iters; ++i)
    asm volatile(".rept 16\nv_add3_u32 %0, %0, %4, 1\nv_add3_u32 %1, %1, %4, 1\nv_add3_u32 %2, %2, %4, 1\nv_add3_u32 %3, %3, %4, 1\n.endr" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y), "v"(r) : "s0", "s1", "scc");
  STAMP(t1);
  sink[threadIdx.x] = a ^ b ^ c ^ d;
  if (threadIdx.x == 0) out[0] = t1 - t0;
}
__global__ __launch_bounds__(64) void k2(uint64_t* out, uint32_t* sink, int iters) {
  uint32_t a = threadIdx.x, b = a * 3 + 1, c = a * 5 + 2, d = a * 7 + 3, x = a ^ 9, y = a + 5;
  uint32_t r = (threadIdx.x & 1) ? 13u : 7u;
  uint64_t t0, t1;
  STAMP(t0);
  for (int i = 0; i < iters; ++i)
    asm volatile(".rept 16\nv_add3_u32 %0, %0, 3, 1\nv_add3_u32 %1, %1, 3, 1\nv_add3_u32 %2, %2, 3, 1\nv_add3_u32 %3, %3, 3, 1\n.endr" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y), "v"(r) : "s0", "s1", "scc");
  STAMP(t1);
  sink[threadIdx.x] = a ^ b ^ c ^ d;
  if (threadIdx.x == 0) out[0] = t1 - t0;
}
__global__ __launch_bounds__(64) void k3(uint64_t* out, uint32_t* sink, int iters) {
  uint32_t a = threadIdx.x, b = a * 3 + 1, c = a * 5 + 2, d = a * 7 + 3, x = a ^ 9, y = a + 5;
  uint32_t r = (threadIdx.x & 1) ? 13u : 7u;
  uint64_t t0, t1;
  STAMP(t0);
  for (int i = 0; i < iters; ++i)
    asm volatile(".rept 16\nv_add_u32_e64 %0, %0, %4\nv_add_u32_e64 %1, %1, %4\nv_add_u32_e64 %2, %2, %4\nv_add_u32_e64 %3, %3, %4\n.endr" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y), "v"(r) : "s0", "s1", "scc");
  STAMP(t1);
  sink[threadIdx.x] = a ^ b ^ c ^ d;
  if (threadIdx.x == 0) out[0] = t1 - t0;
}
__global__ __launch_bounds__(64) void k4(uint64_t* out, uint32_t* sink, int iters) {
  uint32_t a = threadIdx.x, b = a * 3 + 1, c = a * 5 + 2, d = a * 7 + 3, x = a ^ 9, y = a + 5;
  uint32_t r = (threadIdx.x & 1) ? 13u : 7u;
  uint64_t t0, t1;
  STAMP(t0);
  for (int i = 0; i < iters; ++i)
    asm volatile(".rept 16\nv_add_u32 %0, %0, %4\nv_add_u32 %1, %1, %4\nv_add_u32 %2, %2, %4\nv_add_u32 %3, %3, %4\n.endr" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y), "v"(r) : "s0", "s1", "scc");
  STAMP(t1);
  sink[threadIdx.x] = a ^ b ^ c ^ d;
  if (threadIdx.x == 0) out[0] = t1 - t0;
}
__global__ __launch_bounds__(64) void k5(uint64_t* out, uint32_t* sink, int iters) {
  uint32_t a = threadIdx.x, b = a * 3 + 1, c = a * 5 + 2, d = a * 7 + 3, x = a ^ 9, y = a + 5;
  uint32_t r = (threadIdx.x & 1) ? 13u : 7u;
  uint64_t t0, t1;
  STAMP(t0);
  for (int i = 0; i < iters; ++i)
    asm volatile(".rept 16\nv_alignbit_b32 %0, %0, %0, 7\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %2, %2, %2, 7\nv_alignbit_b32 %3, %3, %3, 7\n.endr" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y), "v"(r) : "s0", "s1", "scc");
  STAMP(t1);
  sink[threadIdx.x] = a ^ b ^ c ^ d;
  if (threadIdx.x == 0) out[0] = t1 - t0;
}
__global__ __launch_bounds__(64) void k6(uint64_t* out, uint32_t* sink, int iters) {
  uint32_t a = threadIdx.x, b = a * 3 + 1, c = a * 5 + 2, d = a * 7 + 3, x = a ^ 9, y = a + 5;
  uint32_t r = (threadIdx.x & 1) ? 13u : 7u;
  uint64_t t0, t1;
  STAMP(t0);
  for (int i = 0; i < iters; ++i)
    asm volatile(".rept 16\nv_add3_u32 %0, %0, %4, %5\ns_add_u32 s0, s0, 1\nv_add3_u32 %1, %1, %4, %5\ns_add_u32 s1, s1, 1\n.endr" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y), "v"(r) : "s0", "s1", "scc");
  STAMP(t1);
  sink[threadIdx.x] = a ^ b ^ c ^ d;
  if (threadIdx.x == 0) out[0] = t1 - t0;
}
__global__ __launch_bounds__(64) void k7(uint64_t* out, uint32_t* sink, int iters) {
  uint32_t a = threadIdx.x, b = a * 3 + 1, c = a * 5 + 2, d = a * 7 + 3, x = a ^ 9, y = a + 5;
  uint32_t r = (threadIdx.x & 1) ? 13u : 7u;
  uint64_t t0, t1;
  STAMP(t0);
  for (int i = 0; i < iters; ++i)
    asm volatile(".rept 16\nv_add3_u32 %0, %0, %4, %5\nv_add_u32 %1, %1, %4\nv_add3_u32 %2, %2, %4, %5\nv_add_u32 %3, %3, %4\n.endr" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y), "v"(r) : "s0", "s1", "scc");
  STAMP(t1);
  sink[threadIdx.x] = a ^ b ^ c ^ d;
  if (threadIdx.x == 0) out[0] = t1 - t0;
}
__global__ __launch_bounds__(64) void k8(uint64_t* out, uint32_t* sink, int iters) {
  uint32_t a = threadIdx.x, b = a * 3 + 1, c = a * 5 + 2, d = a * 7 + 3, x = a ^ 9, y = a + 5;
  uint32_t r = (threadIdx.x & 1) ? 13u : 7u;
  uint64_t t0, t1;
  STAMP(t0);
  for (int i = 0; i < iters; ++i)
    asm volatile(".rept 16\nv_xor_b32 %0, %0, %4\nv_xor_b32 %1, %1, %4\nv_xor_b32 %2, %2, %4\nv_xor_b32 %3, %3, %4\n.endr" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y), "v"(r) : "s0", "s1", "scc");
  STAMP(t1);
  sink[threadIdx.x] = a ^ b ^ c ^ d;
  if (threadIdx.x == 0) out[0] = t1 - t0;
}
__global__ __launch_bounds__(64) void k9(uint64_t* out, uint32_t* sink, int iters) {
  uint32_t a = threadIdx.x, b = a * 3 + 1, c = a * 5 + 2, d = a * 7 + 3, x = a ^ 9, y = a + 5;
  uint32_t r = (threadIdx.x & 1) ? 13u : 7u;
  uint64_t t0, t1;
  STAMP(t0);
  for (int i = 0; i < iters; ++i)
    asm volatile(".rept 16\nv_add_u32 %0, %0, %4\n.endr" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y), "v"(r) : "s0", "s1", "scc");
  STAMP(t1);
  sink[threadIdx.x] = a ^ b ^ c ^ d;
  if (threadIdx.x == 0) out[0] = t1 - t0;
}
__global__ __launch_bounds__(64) void k10(uint64_t* out, uint32_t* sink, int iters) {
  uint32_t a = threadIdx.x, b = a * 3 + 1, c = a * 5 + 2, d = a * 7 + 3, x = a ^ 9, y = a + 5;
  uint32_t r = (threadIdx.x & 1) ? 13u : 7u;
  uint64_t t0, t1;
  STAMP(t0);
  for (int i = 0; i < iters; ++i)
    asm volatile(".rept 16\nv_add_u32 %0, %0, %4\nv_add_u32 %1, %1, %4\n.endr" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y), "v"(r) : "s0", "s1", "scc");
  STAMP(t1);
  sink[threadIdx.x] = a ^ b ^ c ^ d;
  if (threadIdx.x == 0) out[0] = t1 - t0;
}
__global__ __launch_bounds__(64) void k11(uint64_t* out, uint32_t* sink, int iters) {
  uint32_t a = threadIdx.x, b = a * 3 + 1, c = a * 5 + 2, d = a * 7 + 3, x = a ^ 9, y = a + 5;
  uint32_t r = (threadIdx.x & 1) ? 13u : 7u;
  uint64_t t0, t1;
  STAMP(t0);
  for (int i = 0; i < iters; ++i)
    asm volatile(".rept 16\nv_mov_b32_dpp %0, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %1, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %2, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\nv_mov_b32_dpp %3, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n.endr" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y), "v"(r) : "s0", "s1", "scc");
  STAMP(t1);
  sink[threadIdx.x] = a ^ b ^ c ^ d;
  if (threadIdx.x == 0) out[0] = t1 - t0;
}
__global__ __launch_bounds__(64) void k12(uint64_t* out, uint32_t* sink, int iters) {
  uint32_t a = threadIdx.x, b = a * 3 + 1, c = a * 5 + 2, d = a * 7 + 3, x = a ^ 9, y = a + 5;
  uint32_t r = (threadIdx.x & 1) ? 13u : 7u;
  uint64_t t0, t1;
  STAMP(t0);
  for (int i = 0; i < iters; ++i)
    asm volatile(".rept 16\nv_bitop3_b32 %0, %0, %4, %5 bitop3:0x96\nv_bitop3_b32 %1, %1, %4, %5 bitop3:0x96\nv_bitop3_b32 %2, %2, %4, %5 bitop3:0x96\nv_bitop3_b32 %3, %3, %4, %5 bitop3:0x96\n.endr" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y), "v"(r) : "s0", "s1", "scc");
  STAMP(t1);
  sink[threadIdx.x] = a ^ b ^ c ^ d;
  if (threadIdx.x == 0) out[0] = t1 - t0;
}
int main() {
  uint64_t* d; uint32_t* s; uint64_t h; const int iters = 2000;
  (void)hipMalloc(&d, 8); (void)hipMalloc(&s, 4096);
  for (int r = 0; r < 2; ++r) { hipLaunchKernelGGL(k0, dim3(1), dim3(64), 0, 0, d, s, iters); (void)hipDeviceSynchronize(); }
  (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  printf("%-32s %6.2f cycles/instr\n", "add3 4 chains (3 vgpr)", (double)h / iters / 64);
  for (int r = 0; r < 2; ++r) { hipLaunchKernelGGL(k1, dim3(1), dim3(64), 0, 0, d, s, iters); (void)hipDeviceSynchronize(); }
  (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  printf("%-32s %6.2f cycles/instr\n", "add3 4 chains (2 vgpr + const)", (double)h / iters / 64);
  for (int r = 0; r < 2; ++r) { hipLaunchKernelGGL(k2, dim3(1), dim3(64), 0, 0, d, s, iters); (void)hipDeviceSynchronize(); }
  (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  printf("%-32s %6.2f cycles/instr\n", "add3 4 chains (1 vgpr + 2 const)", (double)h / iters / 64);
  for (int r = 0; r < 2; ++r) { hipLaunchKernelGGL(k3, dim3(1), dim3(64), 0, 0, d, s, iters); (void)hipDeviceSynchronize(); }
  (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  printf("%-32s %6.2f cycles/instr\n", "add_u32_e64 4 chains (VOP3 enc)", (double)h / iters / 64);
  for (int r = 0; r < 2; ++r) { hipLaunchKernelGGL(k4, dim3(1), dim3(64), 0, 0, d, s, iters); (void)hipDeviceSynchronize(); }
  (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  printf("%-32s %6.2f cycles/instr\n", "add_u32 VOP2 4 chains", (double)h / iters / 64);
  for (int r = 0; r < 2; ++r) { hipLaunchKernelGGL(k5, dim3(1), dim3(64), 0, 0, d, s, iters); (void)hipDeviceSynchronize(); }
  (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  printf("%-32s %6.2f cycles/instr\n", "alignbit const shift 4 chains", (double)h / iters / 64);
  for (int r = 0; r < 2; ++r) { hipLaunchKernelGGL(k6, dim3(1), dim3(64), 0, 0, d, s, iters); (void)hipDeviceSynchronize(); }
  (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  printf("%-32s %6.2f cycles/instr\n", "add3 + s_add alternating", (double)h / iters / 64);
  for (int r = 0; r < 2; ++r) { hipLaunchKernelGGL(k7, dim3(1), dim3(64), 0, 0, d, s, iters); (void)hipDeviceSynchronize(); }
  (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  printf("%-32s %6.2f cycles/instr\n", "add3/add VOP2 alternating", (double)h / iters / 64);
  for (int r = 0; r < 2; ++r) { hipLaunchKernelGGL(k8, dim3(1), dim3(64), 0, 0, d, s, iters); (void)hipDeviceSynchronize(); }
  (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  printf("%-32s %6.2f cycles/instr\n", "xor VOP2 4 chains", (double)h / iters / 64);
  for (int r = 0; r < 2; ++r) { hipLaunchKernelGGL(k9, dim3(1), dim3(64), 0, 0, d, s, iters); (void)hipDeviceSynchronize(); }
  (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  printf("%-32s %6.2f cycles/instr\n", "add VOP2 chain", (double)h / iters / 16);
  for (int r = 0; r < 2; ++r) { hipLaunchKernelGGL(k10, dim3(1), dim3(64), 0, 0, d, s, iters); (void)hipDeviceSynchronize(); }
  (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  printf("%-32s %6.2f cycles/instr\n", "add VOP2 2 chains", (double)h / iters / 32);
  for (int r = 0; r < 2; ++r) { hipLaunchKernelGGL(k11, dim3(1), dim3(64), 0, 0, d, s, iters); (void)hipDeviceSynchronize(); }
  (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  printf("%-32s %6.2f cycles/instr\n", "dpp mov 4 indep", (double)h / iters / 64);
  for (int r = 0; r < 2; ++r) { hipLaunchKernelGGL(k12, dim3(1), dim3(64), 0, 0, d, s, iters); (void)hipDeviceSynchronize(); }
  (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  printf("%-32s %6.2f cycles/instr\n", "bitop3 4 chains, 3 vgpr", (double)h / iters / 64);
  return 0;
}

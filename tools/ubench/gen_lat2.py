#!/usr/bin/env python3
"""Generates lat2.hip: issue/latency probe for one lone wave64 on gfx950. Each kernel runs a
repeated instruction pattern; the printout is cycles per instruction."""
PATTERNS = {
    "add3 4 chains (3 vgpr)": ["v_add3_u32 %0, %0, %4, %5", "v_add3_u32 %1, %1, %4, %5",
                               "v_add3_u32 %2, %2, %4, %5", "v_add3_u32 %3, %3, %4, %5"],
    "add3 4 chains (2 vgpr + const)": ["v_add3_u32 %0, %0, %4, 1", "v_add3_u32 %1, %1, %4, 1",
                                       "v_add3_u32 %2, %2, %4, 1", "v_add3_u32 %3, %3, %4, 1"],
    "add3 4 chains (1 vgpr + 2 const)": ["v_add3_u32 %0, %0, 3, 1", "v_add3_u32 %1, %1, 3, 1",
                                         "v_add3_u32 %2, %2, 3, 1", "v_add3_u32 %3, %3, 3, 1"],
    "add_u32_e64 4 chains (VOP3 enc)": ["v_add_u32_e64 %0, %0, %4", "v_add_u32_e64 %1, %1, %4",
                                        "v_add_u32_e64 %2, %2, %4", "v_add_u32_e64 %3, %3, %4"],
    "add_u32 VOP2 4 chains": ["v_add_u32 %0, %0, %4", "v_add_u32 %1, %1, %4",
                              "v_add_u32 %2, %2, %4", "v_add_u32 %3, %3, %4"],
    "alignbit const shift 4 chains": ["v_alignbit_b32 %0, %0, %0, 7", "v_alignbit_b32 %1, %1, %1, 7",
                                      "v_alignbit_b32 %2, %2, %2, 7", "v_alignbit_b32 %3, %3, %3, 7"],
    "add3 + s_add alternating": ["v_add3_u32 %0, %0, %4, %5", "s_add_u32 s0, s0, 1",
                                 "v_add3_u32 %1, %1, %4, %5", "s_add_u32 s1, s1, 1"],
    "add3/add VOP2 alternating": ["v_add3_u32 %0, %0, %4, %5", "v_add_u32 %1, %1, %4",
                                  "v_add3_u32 %2, %2, %4, %5", "v_add_u32 %3, %3, %4"],
    "xor VOP2 4 chains": ["v_xor_b32 %0, %0, %4", "v_xor_b32 %1, %1, %4",
                          "v_xor_b32 %2, %2, %4", "v_xor_b32 %3, %3, %4"],
    "add VOP2 chain": ["v_add_u32 %0, %0, %4"],
    "add VOP2 2 chains": ["v_add_u32 %0, %0, %4", "v_add_u32 %1, %1, %4"],
    "dpp mov 4 indep": ["v_mov_b32_dpp %0, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf",
                        "v_mov_b32_dpp %1, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf",
                        "v_mov_b32_dpp %2, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf",
                        "v_mov_b32_dpp %3, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"],
    "bitop3 4 chains, 3 vgpr": ["v_bitop3_b32 %0, %0, %4, %5 bitop3:0x96", "v_bitop3_b32 %1, %1, %4, %5 bitop3:0x96",
                                "v_bitop3_b32 %2, %2, %4, %5 bitop3:0x96", "v_bitop3_b32 %3, %3, %4, %5 bitop3:0x96"],
}
src = ['#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <cstdint>',
       '#define STAMP(t) asm volatile("s_memtime %0\\n s_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory")']
names = list(PATTERNS)
for k, n in enumerate(names):
    body = "\\n".join(PATTERNS[n])
    src.append(f'''__global__ __launch_bounds__(64) void k{k}(uint64_t* out, uint32_t* sink, int iters) {{
  uint32_t a = threadIdx.x, b = a * 3 + 1, c = a * 5 + 2, d = a * 7 + 3, x = a ^ 9, y = a + 5;
  uint32_t r = (threadIdx.x & 1) ? 13u : 7u;
  uint64_t t0, t1;
  STAMP(t0);
  for (int i = 0; i < iters; ++i)
    asm volatile(".rept 16\\n{body}\\n.endr" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y), "v"(r) : "s0", "s1", "scc");
  STAMP(t1);
  sink[threadIdx.x] = a ^ b ^ c ^ d;
  if (threadIdx.x == 0) out[0] = t1 - t0;
}}''')
src.append('int main() {\n  uint64_t* d; uint32_t* s; uint64_t h; const int iters = 2000;\n'
           '  (void)hipMalloc(&d, 8); (void)hipMalloc(&s, 4096);')
for k, n in enumerate(names):
    cnt = 16 * len(PATTERNS[n])
    src.append(f'  for (int r = 0; r < 2; ++r) {{ hipLaunchKernelGGL(k{k}, dim3(1), dim3(64), 0, 0, d, s, iters); (void)hipDeviceSynchronize(); }}\n'
               f'  (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);\n'
               f'  printf("%-32s %6.2f cycles/instr\\n", "{n}", (double)h / iters / {cnt});')
src.append('  return 0;\n}')
open("lat2.hip", "w").write("\n".join(src) + "\n")

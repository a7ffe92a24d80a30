#!/usr/bin/env python3
"""Generate tools/ubench/scanload.hip: k_scan's per-byte pattern WITH its HBM stream, on the
whole chip, at 2, 3 and 4 waves per SIMD (one workgroup per CU, as k_scan), to price a
three-wave k_scan before building one.

Per lane: 2 KiB strips, whole 128-byte lines loaded one line ahead (8 x global_load_dwordx4
into two 32-register line buffers, as k_scan), after 16 lines the next strip of the grid.
Per byte: v_perm (LDS address byte*256 + lane*4), ds_read_b32 into a 16-deep lookup ring
(lgkmcnt(14)), v_alignbit (rotl 1), v_bitop3 (xor3); per two bytes one v_min3_u16.
Variants: full; no loads (words stay in registers); no LDS (a v_mov instead of the lookup); lines
requested two ahead (three line buffers); a strip restart every 2 KiB (drain, history load,
lookups, hash warm-up). Every variant runs twice: the first pass warms the clock up (its first
launches ran at 1.5-1.7 GHz), the second pass is the one to read.
Output: TB/s, the time for 16 GiB (configs[2]; k_scan: 3.7 ms) and the launch's clock.
"""
import os

RING = 16


def line_body(buf: int, lds: bool) -> list[str]:
    L = []
    for k in range(128):
        w = buf + (k >> 2)
        L.append(f"v_perm_b32 v40, v{w}, v12, s{8 + (k & 3)}")
        t_new = 16 + (k % RING)
        t_use = 16 + ((k + 1) % RING)
        if lds:
            L.append(f"ds_read_b32 v{t_new}, v40")
            L.append("s_waitcnt lgkmcnt(14)")
        else:
            L.append(f"v_mov_b32 v{t_new}, v40")
        h, h0 = ("v1", "v2") if k % 2 == 0 else ("v2", "v1")
        L.append(f"v_alignbit_b32 {h}, {h0}, {h0}, 31")
        L.append(f"v_bitop3_b32 {h}, {h}, v{t_use}, v{32 + (k % 8)} bitop3:0x96")
        if k % 2 == 1:
            L.append("v_min3_u16 v3, v3, v1, v2")
    return L


AD = 108  # line address v[AD:AD+1]: v[108:109] with two line buffers, v[140:141] with three


def loads(buf: int) -> list[str]:
    # line address in v[AD:AD+1]; advance by s14 (128, or the strip jump every 16th line)
    L = [f"global_load_dwordx4 v[{buf + 4 * q}:{buf + 4 * q + 3}], v[{AD}:{AD + 1}], off offset:{16 * q}"
         for q in range(8)]
    L += ["s_add_u32 s16, s16, 1", "s_and_b32 s17, s16, 15", "s_cmp_eq_u32 s17, 0",
          "s_cselect_b32 s14, s15, 128",
          f"v_add_co_u32 v{AD}, vcc, s14, v{AD}", f"v_addc_co_u32 v{AD + 1}, vcc, 0, v{AD + 1}, vcc"]
    return L


def restart(hist: int) -> list[str]:
    """k_scan's per-strip start: drain, load the 64 history bytes, look them up, fold the hash."""
    L = ["s_waitcnt vmcnt(0) lgkmcnt(0)"]
    L += [f"global_load_dwordx4 v[{hist + 4 * q}:{hist + 4 * q + 3}], v[{AD}:{AD + 1}], off offset:{16 * q}"
          for q in range(4)]
    L += ["s_waitcnt vmcnt(0)"]
    for k in range(64):
        L.append(f"v_perm_b32 v40, v{hist + (k >> 2)}, v12, s{8 + (k & 3)}")
        L.append(f"ds_read_b32 v{16 + (k % RING)}, v40")
        L.append("s_waitcnt lgkmcnt(14)")
    L += ["s_waitcnt lgkmcnt(0)"]
    for k in range(64):
        L.append("v_alignbit_b32 v1, v1, v1, 31")
        L.append(f"v_xor_b32 v1, v1, v{16 + (k % RING)}")
    return L


def kernel(name: str, load: bool, lds: bool, ahead: int = 1, every: int = 0) -> list[str]:
    global AD
    AD = 108 if ahead == 1 else 140  # (<= 128 VGPRs with two buffers: 4 waves per SIMD fit)
    A, B, C = 44, 76, 108
    body, pro = [], []
    if ahead == 1:
        body += line_body(A, lds)
        if load:
            body += ["s_waitcnt vmcnt(0)"] + loads(A)
        body += line_body(B, lds)
        if load:
            body += ["s_waitcnt vmcnt(0)"] + loads(B)
        if load:
            pro += loads(A) + ["s_waitcnt vmcnt(0)"] + loads(B)
    else:  # two lines in flight while one is hashed: three line buffers in rotation
        pro += loads(A) + loads(B)
        for cur, nxt in ((A, C), (B, A), (C, B)):
            body += loads(nxt) + ["s_waitcnt vmcnt(16)"] + line_body(cur, lds)
    if every:  # a strip restart every `every` iterations (s18 counts them)
        hist = AD + 2
        body = (["s_add_u32 s18, s18, 1", f"s_cmp_eq_u32 s18, {every}", "s_cbranch_scc0 .Lnors%=",
                 "s_mov_b32 s18, 0"] + restart(hist) + [".Lnors%=:"] + body)
    asm = "\\n".join(pro + ["s_mov_b32 s18, 0", ".Lloop%=:"] + body +
                     ["s_sub_u32 s13, s13, 1", "s_cmp_lg_u32 s13, 0", "s_cbranch_scc1 .Lloop%="])
    regs = ["v1", "v2", "v3", "v12", "v40", f"v{AD}", f"v{AD + 1}"] + \
        [f"v{r}" for r in range(16, 40)] + [f"v{r}" for r in range(44, AD)] + \
        ([f"v{r}" for r in range(AD + 2, AD + 18)] if every else [])
    clob = ", ".join(f'"{r}"' for r in regs)
    return [
        f'__global__ __launch_bounds__(1024) void k_{name}(const uint8_t* buf, uint32_t* sink, int iters, uint32_t jump, uint64_t* clk) {{',
        '  extern __shared__ uint32_t tab[];',
        '  for (int i = threadIdx.x; i < 16384; i += blockDim.x) tab[i] = i * 2654435761u;',
        '  __syncthreads();',
        '  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;',
        '  const uint8_t* p = buf + gid * 2048;',
        '  uint32_t o;',
        '  uint64_t t0, r0, t1, r1;',
        '  asm volatile("s_memtime %0\\n s_memrealtime %1\\n s_waitcnt lgkmcnt(0)" : "=s"(t0), "=s"(r0) :: "memory");',
        '  asm volatile(',
        '    "v_mov_b32 v1, %1\\n v_mov_b32 v2, %1\\n v_mov_b32 v3, -1\\n"',
        '    "v_lshlrev_b32 v12, 2, %1\\n v_and_b32 v12, 0xfc, v12\\n"',
        f'    "v_mov_b32 v{AD}, %4\\n v_mov_b32 v{AD + 1}, %5\\n"',
        '    "s_mov_b32 s8, 0x0c0c0400\\n s_mov_b32 s9, 0x0c0c0500\\n s_mov_b32 s10, 0x0c0c0600\\n s_mov_b32 s11, 0x0c0c0700\\n"',
        '    "s_mov_b32 s13, %2\\n s_mov_b32 s15, %3\\n s_mov_b32 s16, 0\\n s_mov_b32 s14, 128\\n"',
        f'    "{asm}\\n"',
        '    "s_waitcnt vmcnt(0) lgkmcnt(0)\\n v_xor_b32 %0, v3, v44\\n"',
        '    : "=v"(o) : "v"(threadIdx.x), "s"(iters), "s"(jump), "v"((uint32_t)(uintptr_t)p), "v"((uint32_t)((uintptr_t)p >> 32))',
        f'    : "memory", "vcc", "s8", "s9", "s10", "s11", "s13", "s14", "s15", "s16", "s17", "s18", {clob});',
        '  asm volatile("s_memtime %0\\n s_memrealtime %1\\n s_waitcnt lgkmcnt(0)" : "=s"(t1), "=s"(r1) :: "memory");',
        '  sink[gid & 1023] = o;',
        '  if (gid == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }',
        '}', '']


src = ['// Generated by gen_scanload.py: k_scan per-byte pattern with its HBM stream, whole chip.',
       '#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <cstdint>', '']
VARIANTS = (("full", True, True, 1, 0), ("noload", False, True, 1, 0), ("nolds", True, False, 1, 0),
            ("full2a", True, True, 2, 0), ("nolds2a", True, False, 2, 0),
            ("full_rs", True, True, 1, 8), ("full2a_rs", True, True, 2, 5))
for name, load, lds, ahead, every in VARIANTS:
    src += kernel(name, load, lds, ahead, every)
src += [
    'template <typename K> void run(K k, const char* name, int wps, const uint8_t* buf, uint32_t* s, int lpi = 2) {',
    '  const int grid = 256, threads = 64 * 4 * wps;',
    '  const uint64_t lanes = (uint64_t)grid * threads;',
    '  // each iteration = 2 lines (256 B) per lane; a strip = 8 iterations; ~4 GiB per launch',
    '  int iters = (int)((4ull << 30) / (lanes * 128 * lpi)) & ~7;',
    '  const uint32_t jump = (uint32_t)(lanes * 2048 - 15 * 128);',
    '  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);',
    '  uint64_t* clk; hipMalloc(&clk, 16);',
    '  hipLaunchKernelGGL(k, dim3(grid), dim3(threads), 98304, 0, buf, s, iters, jump, clk);',
    '  hipEventRecord(a);',
    '  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(threads), 98304, 0, buf, s, iters, jump, clk);',
    '  hipEventRecord(b); hipEventSynchronize(b);',
    '  float ms = 0; hipEventElapsedTime(&ms, a, b); ms /= 3;',
    '  const double bytes = (double)lanes * iters * 128 * lpi;',
    '  uint64_t c[2]; hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost); hipFree(clk);',
    '  printf("%-9s waves/SIMD=%d  %.2f TB/s  -> 16 GiB in %.2f ms  (%.1f MiB per launch, %.3f ms, clock %.2f GHz)\\n", name, wps,',
    '         bytes / (ms * 1e-3) / 1e12, (16.0 * (1ull << 30)) / (bytes / (ms * 1e-3)) * 1e3, bytes / 1048576.0, ms,',
    '         c[1] ? (double)c[0] / ((double)c[1] * 10.0) : 0.0);',
    '}',
    'int main() {',
    '  uint8_t* buf; uint32_t* s;',
    '  const size_t n = (5ull << 30) + (64u << 20);',
    '  hipMalloc(&buf, n); hipMalloc(&s, 4096); hipMemset(buf, 0x5a, n);',
    '  // pass 0 warms the clocks and the buffer up (the first launches over a fresh 5 GiB buffer',
    '  // ran ~20 % slower than the same kernel later in the run); pass 1 is the one to read',
    '  for (int pass = 0; pass < 2; ++pass) {',
    '    printf("pass %d\\n", pass);',
    '    for (int w : {2, 3, 4}) run(k_full, "full", w, buf, s);',
    '    for (int w : {2, 3, 4}) run(k_noload, "noload", w, buf, s);',
    '    for (int w : {2, 3, 4}) run(k_nolds, "nolds", w, buf, s);',
    '    for (int w : {2, 3}) run(k_full2a, "full2a", w, buf, s, 3);',
    '    for (int w : {2, 3}) run(k_nolds2a, "nolds2a", w, buf, s, 3);',
    '    for (int w : {2}) run(k_full_rs, "full_rs", w, buf, s);',
    '    for (int w : {2}) run(k_full2a_rs, "full2a_rs", w, buf, s, 3);',
    '  }',
    '  hipFree(buf); hipFree(s);',
    '  return 0;',
    '}']
open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "scanload.hip"), "w").write("\n".join(src) + "\n")

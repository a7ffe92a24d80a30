"""Generate tools/ubench/issue2.hip: lone-wave VALU issue cost of straight-line sequences
(every source written >= 8 instructions earlier unless the pattern says otherwise)."""
import os

N = 256          # instructions per pattern body


def pat_add():
    return [f"v_add_u32 v{40 + i % 32}, v{40 + (i + 9) % 32}, v{40 + (i + 17) % 32}" for i in range(N)]


def pat_mov():
    return [f"v_mov_b32 v{40 + i % 32}, v{40 + (i + 9) % 32}" for i in range(N)]


def pat_alignbit():
    return [f"v_alignbit_b32 v{40 + i % 32}, v{40 + (i + 9) % 32}, v{40 + (i + 9) % 32}, 7" for i in range(N)]


def pat_alignbit_v():
    return [f"v_alignbit_b32 v{40 + i % 32}, v{40 + (i + 9) % 32}, v{40 + (i + 9) % 32}, v{40 + (i + 17) % 32}" for i in range(N)]


def pat_bitop3():
    return [f"v_bitop3_b32 v{40 + i % 32}, v{40 + (i + 9) % 32}, v{40 + (i + 17) % 32}, v{40 + (i + 25) % 32} bitop3:0x96" for i in range(N)]


def pat_add3():
    return [f"v_add3_u32 v{40 + i % 32}, v{40 + (i + 9) % 32}, v{40 + (i + 17) % 32}, v{40 + (i + 25) % 32}" for i in range(N)]


def pat_xad():
    return [f"v_xad_u32 v{40 + i % 32}, v{40 + (i + 9) % 32}, v{40 + (i + 17) % 32}, v{40 + (i + 25) % 32}" for i in range(N)]


def pat_dpp():
    return [f"v_add_u32_dpp v{40 + i % 32}, v{40 + (i + 9) % 32}, v{40 + (i + 17) % 32} quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" for i in range(N)]


def pat_perm_s():
    return [f"v_perm_b32 v{40 + i % 32}, v{40 + (i + 9) % 32}, v{40 + (i + 17) % 32}, s8" for i in range(N)]


def pat_cndmask():
    return [f"v_cndmask_b32_e64 v{40 + i % 32}, v{40 + (i + 9) % 32}, v{40 + (i + 17) % 32}, s[10:11]" for i in range(N)]


def skew_round(base, i):
    """One skewed SHA round on a private register set (base..base+11), as in the kernel."""
    S = [base + k for k in range(4)]           # state slots
    P, Z, T0, T1, T2, X = (base + 4 + k for k in range(6))
    XM, KW = base + 10, base + 11
    r1, r2, r3, r4 = S[(i - 1) % 4], S[(i - 2) % 4], S[(i - 3) % 4], S[(i - 4) % 4]
    out = S[i % 4]
    return [
        f"v_xad_u32 v{P}, v{r4}, v{XM}, v{KW}",
        f"v_alignbit_b32 v{T0}, v{r1}, v{r1}, v{XM}",
        f"v_alignbit_b32 v{T1}, v{r1}, v{r1}, v{KW}",
        f"v_add_u32_dpp v{Z}, v{r2}, v{P} quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf",
        f"v_alignbit_b32 v{T2}, v{r1}, v{r1}, v{XM}",
        f"v_bitop3_b32 v{X}, v{r1}, v{r3}, v{XM} bitop3:0x78",
        f"v_bitop3_b32 v{T0}, v{T0}, v{T1}, v{T2} bitop3:0x96",
        f"v_bitop3_b32 v{X}, v{X}, v{r2}, v{r3} bitop3:0xca",
        f"v_add3_u32 v{out}, v{T0}, v{X}, v{Z}",
    ]


def pat_skew1():
    L = []
    for i in range(N // 9 + 1):
        L += skew_round(40, i)
    return L[:N - N % 9]


def pat_skew2():
    """two independent chains, rounds interleaved instruction by instruction"""
    L = []
    for i in range(N // 18 + 1):
        a, b = skew_round(40, i), skew_round(56, i)
        for x, y in zip(a, b):
            L += [x, y]
    return L[:N - N % 18]


def pat_skew_nodpp():
    L = []
    for i in range(N // 9 + 1):
        L += [x.replace("v_add_u32_dpp", "v_add_u32").split(" quad_perm")[0] for x in skew_round(40, i)]
    return L[:N - N % 9]


def pat_alignbit_ab():
    return [f"v_alignbit_b32 v{40 + i % 32}, v{40 + (i + 9) % 32}, v{40 + (i + 13) % 32}, 7" for i in range(N)]


def pat_mix_align_add():
    return [(f"v_alignbit_b32 v{40 + i % 32}, v{40 + (i + 9) % 32}, v{40 + (i + 9) % 32}, 7" if i % 2 == 0
             else f"v_add_u32 v{40 + i % 32}, v{40 + (i + 9) % 32}, v{40 + (i + 17) % 32}") for i in range(N)]


def pat_mix_align_add3():
    return [(f"v_alignbit_b32 v{40 + i % 32}, v{40 + (i + 9) % 32}, v{40 + (i + 9) % 32}, 7" if i % 2 == 0
             else f"v_add3_u32 v{40 + i % 32}, v{40 + (i + 9) % 32}, v{40 + (i + 17) % 32}, v{40 + (i + 25) % 32}") for i in range(N)]


def pat_mix_vop3_vop2():
    return [(f"v_add3_u32 v{40 + i % 32}, v{40 + (i + 9) % 32}, v{40 + (i + 17) % 32}, v{40 + (i + 25) % 32}" if i % 2 == 0
             else f"v_add_u32 v{40 + i % 32}, v{40 + (i + 9) % 32}, v{40 + (i + 17) % 32}") for i in range(N)]


def pat_lshl_add_2src():
    return [f"v_lshl_add_u32 v{40 + i % 32}, v{40 + (i + 9) % 32}, 3, v{40 + (i + 17) % 32}" for i in range(N)]


def pat_bitop3_2src():
    return [f"v_bitop3_b32 v{40 + i % 32}, v{40 + (i + 9) % 32}, v{40 + (i + 17) % 32}, 0 bitop3:0x96" for i in range(N)]


def pat_skew_noalign():
    L = []
    for i in range(N // 9 + 1):
        for x in skew_round(40, i):
            if x.startswith("v_alignbit_b32"):
                d, a, _, sh = [t.strip() for t in x[len("v_alignbit_b32 "):].split(",")]
                x = f"v_bitop3_b32 {d}, {a}, {a}, {sh} bitop3:0x96"
            L.append(x)
    return L[:N - N % 9]


def pat_skew_constshift():
    L = []
    for i in range(N // 9 + 1):
        for x in skew_round(40, i):
            if x.startswith("v_alignbit_b32"):
                x = x.rsplit(",", 1)[0] + ", 7"
            L.append(x)
    return L[:N - N % 9]


def skew_round_v(base, i, split_xor3=False, split_add3=False):
    L = []
    for x in skew_round(base, i):
        if split_xor3 and "bitop3:0x96" in x:
            d, a, b, c = [t.strip() for t in x[len("v_bitop3_b32 "):].split(" bitop3")[0].split(",")]
            L += [f"v_xor_b32 {d}, {a}, {b}", f"v_xor_b32 {d}, {c}, {d}"]
        elif split_add3 and x.startswith("v_add3_u32"):
            d, a, b, c = [t.strip() for t in x[len("v_add3_u32 "):].split(",")]
            # V = T0 + X + Z: first Z += X (Z is free after), then V = T0 + Z
            L += [f"v_add_u32 {c}, {b}, {c}", f"v_add_u32 {d}, {a}, {c}"]
        else:
            L.append(x)
    return L


def mk(split_xor3, split_add3):
    def f():
        L = []
        i = 0
        while len(L) < N:
            L += skew_round_v(40, i, split_xor3, split_add3)
            i += 1
        return L
    return f


def skew_xchg(base, i, mode):
    L = []
    for x in skew_round(base, i):
        if "v_add_u32_dpp" in x:
            d, a, b = [t.strip() for t in x[len("v_add_u32_dpp "):].split(" quad_perm")[0].split(",")]
            T = f"v{base + 12}"
            if mode == "movdpp":
                L.insert(0, f"v_mov_b32_dpp {T}, {a} quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
                L.append(f"v_add_u32 {d}, {T}, {b}")
            elif mode == "swap":
                L.insert(0, f"v_mov_b32 {T}, {a}")
                L.insert(1, f"v_alignbit_b32 v{base + 13}, v{base + 14}, v{base + 14}, 7")  # filler for the 2 wait states
                L.insert(2, f"v_permlane32_swap_b32 {T}, {T}")
                L.append(f"v_add_u32 {d}, {T}, {b}")
            elif mode == "swap_nofill":
                L.insert(0, f"v_mov_b32 {T}, {a}")
                L.insert(1, "s_nop 1")
                L.insert(2, f"v_permlane32_swap_b32 {T}, {T}")
                L.append(f"v_add_u32 {d}, {T}, {b}")
        else:
            L.append(x)
    return L


def mkx(mode):
    def f():
        L = []
        i = 0
        while len(L) < N:
            L += skew_xchg(40, i, mode)
            i += 1
        return L
    return f


def skew_order(base, i, order):
    """mov_dpp exchange; order: names from xad al0 al1 al2 bx xor3 ch add3 mdpp zadd;
    'mdppN' = the exchange for the NEXT round issued here (reads V(i-1))."""
    S = [base + k for k in range(4)]
    P, Z, T0, T1, T2, X = (base + 4 + k for k in range(6))
    XM, KW = base + 10, base + 11
    T = base + 12 + (i % 2)         # exchange register, double-buffered for mdppN
    TN = base + 12 + ((i + 1) % 2)
    r1, r2, r3, r4 = S[(i - 1) % 4], S[(i - 2) % 4], S[(i - 3) % 4], S[(i - 4) % 4]
    out = S[i % 4]
    ins = {
        "xad": f"v_xad_u32 v{P}, v{r4}, v{XM}, v{KW}",
        "al0": f"v_alignbit_b32 v{T0}, v{r1}, v{r1}, v{XM}",
        "al1": f"v_alignbit_b32 v{T1}, v{r1}, v{r1}, v{KW}",
        "al2": f"v_alignbit_b32 v{T2}, v{r1}, v{r1}, v{XM}",
        "bx": f"v_bitop3_b32 v{X}, v{r1}, v{r3}, v{XM} bitop3:0x78",
        "xor3": f"v_bitop3_b32 v{T0}, v{T0}, v{T1}, v{T2} bitop3:0x96",
        "ch": f"v_bitop3_b32 v{X}, v{X}, v{r2}, v{r3} bitop3:0xca",
        "add3": f"v_add3_u32 v{out}, v{T0}, v{X}, v{Z}",
        "mdpp": f"v_mov_b32_dpp v{T}, v{r2} quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf",
        "mdppN": f"v_mov_b32_dpp v{TN}, v{r1} quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf",
        "zadd": f"v_add_u32 v{Z}, v{T}, v{P}",
    }
    return [ins[k] for k in order.split()]


def mko(order):
    def f():
        L = []
        i = 0
        while len(L) < N:
            L += skew_order(40, i, order)
            i += 1
        return L
    return f


ORDERS_X = ["mdpp xad al0 al1 al2 bx xor3 ch zadd add3",
            "mdpp xad al0 al1 zadd al2 bx xor3 ch add3",
            "xad al0 mdpp al1 al2 zadd bx xor3 ch add3",
            "xad al0 al1 zadd al2 bx xor3 ch add3 mdppN",
            "xad al0 zadd al1 al2 bx mdppN xor3 ch add3",
            "al0 al1 al2 bx xad zadd xor3 ch add3 mdppN"]


PATS = [(f"order {k}: {o}", mko(o)) for k, o in enumerate(ORDERS_X)] + [
("skew, exchange = mov_dpp + VOP2 add", mkx("movdpp")),
        ("skew, exchange = mov + swap32 + add (+filler)", mkx("swap")),
        ("skew, exchange = mov + s_nop1 + swap32 + add", mkx("swap_nofill")),
("skew round, xor3 -> 2 VOP2 xor", mk(True, False)), ("skew round, add3 -> 2 VOP2 add", mk(False, True)),
        ("skew round, both split", mk(True, True)),
("alignbit a,b,const", pat_alignbit_ab), ("alignbit/add alternating", pat_mix_align_add),
        ("alignbit/add3 alternating", pat_mix_align_add3), ("add3/add alternating", pat_mix_vop3_vop2),
        ("lshl_add 2 vgpr + const", pat_lshl_add_2src), ("bitop3 2 vgpr + const", pat_bitop3_2src),
        ("skew round, alignbit -> bitop3", pat_skew_noalign), ("skew round, const shifts", pat_skew_constshift),
("add VOP2", pat_add), ("mov", pat_mov), ("alignbit const", pat_alignbit),
        ("alignbit vgpr shift", pat_alignbit_v), ("bitop3 3 vgpr", pat_bitop3),
        ("add3 3 vgpr", pat_add3), ("xad 3 vgpr", pat_xad), ("add_dpp", pat_dpp),
        ("perm sgpr sel", pat_perm_s), ("cndmask e64", pat_cndmask),
        ("skew round, 1 chain", pat_skew1), ("skew round, 2 chains interleaved", pat_skew2),
        ("skew round, 1 chain, no dpp", pat_skew_nodpp)]

src = ['// Generated by gen_issue2.py', '#include <hip/hip_runtime.h>', '#include <cstdio>',
       '#include <cstdint>', '',
       '#define STAMP(t) asm volatile("s_memtime %0\\n s_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory")', '']
for idx, (name, f) in enumerate(PATS):
    body = f()
    src += [f'__global__ void k{idx}(uint64_t* out, int iters) {{',
            '  uint64_t t0, t1;',
            '  for (int w = 0; w < 2; ++w) {',
            '  STAMP(t0);',
            '  asm volatile("s_mov_b32 s8, 0x05040100\\n s_mov_b64 s[10:11], -1\\n s_mov_b32 s12, %0\\n"',
            '    ".Lloop%=:\\n"',
            '    "' + "\\n".join(body) + '\\n"',
            '    "s_sub_u32 s12, s12, 1\\n s_cmp_lg_u32 s12, 0\\n s_cbranch_scc1 .Lloop%=\\n"',
            '    :: "s"(iters) : "s8", "s10", "s11", "s12", "scc", ' + ", ".join(f'"v{r}"' for r in range(40, 72)) + ');',
            '  __syncthreads();',
            '  STAMP(t1);',
            '  }',
            f'  if (threadIdx.x == 0) {{ out[0] = t1 - t0; out[1] = {len(body)}; }}',
            '}', '']
src += ['int main() {', '  uint64_t* d; (void)hipMalloc(&d, 16); uint64_t h[2]; const int iters = 400;']
MULTI = {"add3 3 vgpr", "add VOP2", "skew round, 1 chain", "bitop3 3 vgpr"}
for idx, (name, f) in enumerate(PATS):
    if name in MULTI:
        for w in (1, 2, 4):
            src += [f'  hipLaunchKernelGGL(k{idx}, dim3(1), dim3({256 * w}), 0, 0, d, iters); (void)hipDeviceSynchronize();',
                    '  (void)hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);',
                    f'  printf("%-44s {w} waves/SIMD: %.2f cycles per instr per SIMD\\n", "{name}", (double)h[0] / ((double)iters * h[1] * {w}));']
    src += [f'  hipLaunchKernelGGL(k{idx}, dim3(1), dim3(64), 0, 0, d, iters); (void)hipDeviceSynchronize();',
            '  (void)hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);',
            f'  printf("%-44s %.2f cycles/instr  %u instrs\\n", "{name}", (double)h[0] / ((double)iters * h[1]), (unsigned)h[1]);']
src += ['  return 0;', '}']
open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "issue2.hip"), "w").write("\n".join(src) + "\n")

#!/usr/bin/env python3
"""Per-lane SHA-256 compression (FIPS 180-4, one message block per lane) as one generated
inline-asm statement, every instruction 8 bytes (VOP3, or VOP2 + a 32-bit literal for K + W)
and the statement 8-byte aligned (.p2align 3), so no 8-byte instruction starts at 4 mod 8: the
round-5 octet measurements (tools/gen_oct_variants.py, profiles/r05_oct_var_alignment.log) cost
each such instruction ~10 cycles of a lone wave, and k_sha's per-lane waves run one per SIMD.
Writes bs_amd/csrc/sha256_lane_asm.inc: BSG_LANE_COMPRESS_ASM (operands st0..st7, w0..w15
read-write, x0..x7, t0..t5 and the SGPR k scratch) and BSG_LANE_COMPRESS_ASM_KV (the same with
K read from the VGPR inputs k0..k63 instead of the SGPR: no s_mov per round)."""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "bs_amd", "csrc", "sha256_lane_asm.inc")
K = [0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4,
     0xab1c5ed5, 0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe,
     0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f,
     0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7,
     0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc,
     0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b,
     0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116,
     0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
     0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
     0xc67178f2]


def body(nomov=False, sgprk=False, vgprk=False):
    """The statement's instruction lines. nomov: rounds 0-3 write their new a and e into the
    x registers instead of copying st into x first (8 moves fewer); sgprk: K goes through an
    SGPR (s_mov, then one v_add3 of h, K and W) instead of a VOP2 literal add (64 VALU fewer,
    64 SALU more). Returns (lines, VALU count)."""
    L = [".p2align 3"]
    e = L.append
    T = [f"%[t{i}]" for i in range(6)]
    W = [f"%[w{i}]" for i in range(16)]
    X = [f"%[x{i}]" for i in range(8)]
    ST = [f"%[st{i}]" for i in range(8)]
    # working variables a..h by register name, rotated by renaming each round
    if nomov:
        regs = ST + X          # a..h start in st (read only), rounds 0-3 write x0..x7
        names = list(range(8))
    else:
        for i in range(8):
            e(f"v_mov_b32_e64 {X[i]}, {ST[i]}")
        regs = X
        names = list(range(8))
    fresh = 8                  # next x register for nomov's first four rounds

    def sched(i):  # W[i & 15] for round i >= 16
        w15, w2, w7, w16 = W[(i - 15) & 15], W[(i - 2) & 15], W[(i - 7) & 15], W[i & 15]
        e(f"v_alignbit_b32 {T[0]}, {w15}, {w15}, 7")
        e(f"v_alignbit_b32 {T[1]}, {w2}, {w2}, 17")
        e(f"v_alignbit_b32 {T[2]}, {w15}, {w15}, 18")
        e(f"v_alignbit_b32 {T[3]}, {w2}, {w2}, 19")
        e(f"v_lshrrev_b32_e64 {T[5]}, 10, {w2}")
        e(f"v_lshrrev_b32_e64 {T[4]}, 3, {w15}")
        e(f"v_bitop3_b32 {T[1]}, {T[1]}, {T[3]}, {T[5]} bitop3:0x96")
        e(f"v_bitop3_b32 {T[0]}, {T[0]}, {T[2]}, {T[4]} bitop3:0x96")
        e(f"v_add3_u32 {w16}, {w16}, {T[1]}, {w7}")
        e(f"v_add_u32_e64 {w16}, {w16}, {T[0]}")

    for i in range(64):
        if i >= 16:
            sched(i)
        a, b, c, d, ee, f, g, h = (regs[names[k]] for k in range(8))
        if nomov and i < 4:
            nd, nh = fresh, fresh + 1   # new e, new a into x registers; st stays intact
            fresh += 2
        else:
            nd, nh = names[3], names[7]
        od, oh = regs[nd], regs[nh]
        if sgprk and not vgprk:
            e(f"s_mov_b32 %[k], 0x{K[i]:08x}")
        e(f"v_alignbit_b32 {T[0]}, {ee}, {ee}, 6")
        e(f"v_alignbit_b32 {T[1]}, {ee}, {ee}, 11")
        e(f"v_alignbit_b32 {T[2]}, {ee}, {ee}, 25")
        e(f"v_bitop3_b32 {T[4]}, {ee}, {f}, {g} bitop3:0xca")
        if vgprk:
            e(f"v_add3_u32 {T[5]}, {h}, %[k{i}], {W[i & 15]}")
        elif sgprk:
            e(f"v_add3_u32 {T[5]}, {h}, %[k], {W[i & 15]}")
        else:
            e(f"v_add_u32_e32 {T[5]}, 0x{K[i]:08x}, {W[i & 15]}")
        e(f"v_bitop3_b32 {T[0]}, {T[0]}, {T[1]}, {T[2]} bitop3:0x96")
        e(f"v_alignbit_b32 {T[1]}, {a}, {a}, 2")
        e(f"v_alignbit_b32 {T[2]}, {a}, {a}, 13")
        if sgprk or vgprk:
            e(f"v_add3_u32 {T[5]}, {T[5]}, {T[0]}, {T[4]}")
        else:
            e(f"v_add3_u32 {T[5]}, {h}, {T[5]}, {T[0]}")
        e(f"v_alignbit_b32 {T[3]}, {a}, {a}, 22")
        if not (sgprk or vgprk):
            e(f"v_add_u32_e64 {T[5]}, {T[5]}, {T[4]}")
        e(f"v_bitop3_b32 {T[4]}, {a}, {b}, {c} bitop3:0xe8")
        e(f"v_bitop3_b32 {T[1]}, {T[1]}, {T[2]}, {T[3]} bitop3:0x96")
        e(f"v_add_u32_e64 {od}, {d}, {T[5]}")
        e(f"v_add3_u32 {oh}, {T[5]}, {T[1]}, {T[4]}")
        # rename: (a..h) <- (h', a, b, c, d', e, f, g)
        names = [nh, names[0], names[1], names[2], nd, names[4], names[5], names[6]]
    for k in range(8):
        e(f"v_add_u32_e64 {ST[k]}, {ST[k]}, {regs[names[k]]}")
    return L, sum(1 for ln in L if ln.startswith("v_"))


def macro(name, lines, n_valu, what):
    text = " \\\n".join(f'  "{ln}\\n"' for ln in lines)
    return (f"// Per-lane SHA-256 compression{what}: {n_valu} VALU, every instruction 8 bytes, 8-aligned.\n"
            f"#define {name} \\\n{text}\n")


def gen():
    L, n = body(nomov=True, sgprk=True)
    L4, n4 = body(nomov=True, vgprk=True)
    with open(OUT, "w") as f:
        f.write("// GENERATED by tools/gen_lane_asm.py -- do not edit.\n")
        f.write(macro("BSG_LANE_COMPRESS_ASM", L, n, " (K through an SGPR)"))
        f.write(macro("BSG_LANE_COMPRESS_ASM_KV", L4, n4, " (K from 64 resident VGPRs k0..k63)"))
    print(f"wrote {OUT}: {n} / {n4} VALU")
    # the round-5 variants side by side for tools/ubench/lanes_align.hip
    out = os.path.join(ROOT, "tools", "ubench", "lane_variants.inc")
    with open(out, "w") as f:
        f.write("// GENERATED by tools/gen_lane_asm.py -- do not edit.\n")
        for nm, kw in (("LANE_V1", {}), ("LANE_V2", {"nomov": True}),
                       ("LANE_V3", {"nomov": True, "sgprk": True}),
                       ("LANE_V4", {"nomov": True, "vgprk": True})):
            L, n = body(**kw)
            f.write(macro(nm, L, n, f" ({kw})"))
            print(f"{nm} {kw}: {n} VALU")


if __name__ == "__main__":
    gen()

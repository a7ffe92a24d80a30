#!/usr/bin/env python3
"""EXPERIMENT: the octet chain loop of tools/gen_skew_asm.py (main_loop_oct)
with other K+W load / wait schedules, into tools/ubench/oct_variants.inc for
tools/ubench/oct_var.hip. The SQ counters on the real loop (profiles/r05_octet_loop_pass2_valu_pmc.json)
put 15.6 % of its cycles in SQ_WAIT_ANY (s_waitcnt) and none in instruction-issue stalls, so
these vary only where and how often the loop waits for its K+W quads:
  base    one ds_read_b128 per quad, s_waitcnt lgkmcnt(1) before it (the product loop)
  pair    two quads per wait: at every second quad lgkmcnt(0), then the next two quads
  far     quads four ahead (8 buffers), lgkmcnt(3) before each load
  quad4   four quads per wait (8 buffers): lgkmcnt(0) every fourth quad, then four loads
  nowait  base without any s_waitcnt in the loop (timing only: results are wrong)
  *_a     the same with an s_nop 0 wherever an 8-byte instruction would start at 4 mod 8 from
          the loop label, and the label 8-byte aligned (.p2align 3); *_a32: label 32-byte
          aligned; *_m: every 8-byte instruction deliberately at 4 mod 8 (the opposite)
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "ubench", "oct_variants.inc")


def size_of(ins):
    op = ins.split()[0]
    if op.startswith("s_") or op.startswith("L_") or op.endswith(":"):
        return 0 if op.endswith(":") or op.startswith(".") else 4
    if op in ("v_mov_b32", "v_add_u32", "v_cmp_lt_i32") and "_e64" not in op:
        return 4
    return 8


def gen(name, policy, align=None):
    S = ["v64", "v65", "v66", "v67"]
    P_, Z_, T_, S_, X_, ROT = ("v72", "v73", "v74", "v75", "v77", "v76")
    ADDR, NADDR = "v80", "v81"
    nbuf = 8 if policy in ("far", "quad4") else 4
    KB = [84 + 4 * k for k in range(nbuf)]
    clob = S + [P_, Z_, T_, S_, X_, ROT, ADDR, NADDR] + [f"v{r}" for r in range(84, 84 + 4 * nbuf)]
    L = []
    off = [0]  # bytes from the loop label (alignment variants)

    def e(ins):
        sz = size_of(ins)
        if align in ("a", "a32") and off[0] is not None and sz == 8 and off[0] % 8 == 4:
            L.append("s_nop 0")
            off[0] += 4
        if align == "m" and off[0] is not None and sz == 8 and off[0] % 8 == 0:
            L.append("s_nop 0")
            off[0] += 4
        L.append(ins)
        if off[0] is not None:
            off[0] += sz

    def kreg(word):
        q, c = divmod(word, 4)
        return f"v{KB[q % nbuf] + c}"

    def load(q):
        b = KB[q % nbuf]
        base, off = (ADDR, q) if q < 16 else (NADDR, q - 16)
        e(f"ds_read_b128 v[{b}:{b + 3}], {base} offset:{16 * off}")

    def sl(j):
        return S[j % 4]

    e("s_waitcnt lgkmcnt(0)")
    e("s_mov_b64 %[sexec], exec")
    e("s_mov_b32 %[cnt], 0")
    e(f"v_mov_b32 {ADDR}, %[addr]")
    ahead = {"base": 2, "pair": 2, "nowait": 2, "far": 4, "quad4": 4}[policy]
    for q in range(ahead):
        load(q)
    if align == "a":
        L.append(".p2align 3")
    elif align in ("a32", "m"):
        L.append(".p2align 5")
    L.append("L_oct_loop_%=:")
    off[0] = 0
    e("v_cmp_lt_i32 vcc, %[cnt], %[lim]")
    e("s_and_b64 exec, exec, vcc")
    e(f"v_mov_b32 {S[2]}, %[h2]")
    e(f"v_mov_b32 {S[1]}, %[h3]")
    e(f"v_mov_b32 {S[0]}, %[h0]")
    e(f"v_mov_b32 {S[3]}, %[h1]")
    e(f"v_add_u32 {NADDR}, {ADDR}, %[stride]")
    seen = set()
    for i in range(-1, 65):
        w = min(i + 1, 63)
        q = w // 4
        if q not in seen:
            seen.add(q)
            if policy == "base":
                e("s_waitcnt lgkmcnt(1)")
                load(q + 2)
            elif policy == "nowait":
                load(q + 2)
            elif policy == "pair":
                if q % 2 == 0:
                    e("s_waitcnt lgkmcnt(0)")
                    load(q + 2)
                    load(q + 3)
            elif policy == "far":
                e("s_waitcnt lgkmcnt(3)")
                load(q + 4)
            elif policy == "quad4":
                if q % 4 == 0:
                    e("s_waitcnt lgkmcnt(0)")
                    for k in range(4):
                        load(q + 4 + k)
        r1, r2, r3, r4 = sl(i - 1), sl(i - 2), sl(i - 3), sl(i - 4)
        out = sl(i)
        keep_a = i in (-1, 0)
        keep_e = i in (63, 64)
        dst = Z_ if (keep_a or keep_e) else out
        e(f"v_alignbit_b32 {ROT}, {r1}, {r1}, %[s1]")
        e(f"v_bitop3_b32 {X_}, {r1}, {r3}, %[xm] bitop3:0x78")
        e(f"v_xad_u32 {P_}, {r4}, %[xm], {kreg(w)}")
        e(f"v_xor_b32_dpp {T_}, {ROT}, {ROT} quad_perm:[1,2,0,1] row_mask:0xf bank_mask:0xf")
        e(f"v_bitop3_b32 {X_}, {X_}, {r2}, {r3} bitop3:0xca")
        e(f"v_xor_b32_dpp {S_}, {ROT}, {T_} quad_perm:[2,0,1,2] row_mask:0xf bank_mask:0xf")
        e(f"v_add_u32_dpp {Z_}, {r2}, {P_} row_half_mirror row_mask:0xf bank_mask:0xf")
        e(f"v_add3_u32 {dst}, {S_}, {X_}, {Z_}")
        if keep_a:
            e(f"v_cndmask_b32_e64 {out}, {Z_}, {out}, %[amask]")
        if keep_e:
            e(f"v_cndmask_b32_e64 {out}, {out}, {Z_}, %[amask]")
    e(f"v_add_u32 %[h0], %[h0], {S[0]}")
    e(f"v_add_u32 %[h1], %[h1], {S[3]}")
    e(f"v_add_u32 %[h2], %[h2], {S[2]}")
    e(f"v_add_u32 %[h3], %[h3], {S[1]}")
    e(f"v_mov_b32 {ADDR}, {NADDR}")
    e("s_add_u32 %[cnt], %[cnt], 1")
    e("s_cmp_lt_u32 %[cnt], %[nblk]")
    e("s_cbranch_scc1 L_oct_loop_%=")
    e("s_waitcnt lgkmcnt(0)")
    e("s_mov_b64 exec, %[sexec]")
    body = " \\\n".join(f'  "{ln}\\n"' for ln in L)
    cl = ", ".join(f'"{c}"' for c in clob)
    return f"#define OCTV_{name.upper()} \\\n{body}\n#define OCTV_{name.upper()}_CLOB {cl}, \"vcc\", \"scc\"\n"


def main():
    with open(OUT, "w") as f:
        f.write("// GENERATED by tools/gen_oct_variants.py -- experiment, not in the build.\n")
        for p in ("base", "pair", "far", "quad4", "nowait"):
            f.write(gen(p, p))
            for al in ("a", "a32", "m"):
                f.write(gen(f"{p}_{al}", p, al))
    print(OUT)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Generates bs_amd/csrc/scan_block_loop.inc: k_scan's fast pass over one lane's strip
(split_bits >= 16 pre-filter) as ONE inline-asm statement with every 8-byte instruction 8-byte
aligned.

Why again: rounds 1 and 2 wrote this loop in asm twice (tools/gen_scan_asm.py, history in its
docstring) and neither beat the compiled loop. Round 5 then found that on gfx950 an 8-byte
instruction starting at 4 mod 8 costs a lone wave ~10 cycles, and the replay of
this loop with every 8-byte instruction aligned ran 5 % faster with its loads (16 % without,
profiles/r05_scanalign.log). hipcc's k_scan<true> loop has 536 of its 1,559 instructions per
four blocks at 4 mod 8.

The statement covers what scan_span<true> did: the window history (the 64 bytes before the
strip) and the strip's first line are loaded, the history's table values looked up and folded
into the hash, block 0 looked up, then every full block hashed byte by byte. Output: one bit per
block whose pre-filter fires (the exact pass rescans it). Per byte k of block cb (h = the hash
after byte k-1; HIN = table values of block cb-1 = the out-going bytes, HCUR = those of block cb,
looked up one block earlier; W = the words of block cb+1):
    v_alignbit  H0, H, H, 31                 rotl 1
    v_perm      A, W[k/4], lane4, sel[k%4]   LDS address of block cb+1's byte k (byte*256+lane*4)
    v_bitop3    H0, H0, HIN[k], HCUR[k]      3-way xor (0x96)
    ds_read_b32 HIN[k], A                    HIN[k] is free once consumed: block cb+1's value
and the odd byte the same into H, then v_min3_u16 M, M, H0, H. HIN/HCUR swap roles every block
and the two line buffers every line, so the loop (four blocks) carries no moves. Lines (two
blocks) are requested one line ahead, both halves back to back, addresses clamped to the strip's
last full block. Lanes whose strip has fewer blocks drop out by exec mask. At most 15 LDS reads
are in flight (lgkmcnt is 4 bits): a wait before every 8th read; each consumed lookup was issued
64 reads earlier, so it has landed. Fixed registers v40..v247; the compiler keeps what lives
across the statement in v0..v39 and v248..v255.
"""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "bs_amd", "csrc", "scan_block_loop.inc")
MC = "/opt/rocm/lib/llvm/bin/llvm-mc"

H, H0, M, A0, A1, HITS, NM1, T = (f"v{40 + i}" for i in range(8))
TPAIR, TLO = "v[48:49]", "v48"        # (clamped block * 64, 0) for the 64-bit address add
ADDR = "v[50:51]"
LB = (56, 88)                          # two line buffers of 32 words (block 2j: +0, 2j+1: +16)
HA, HB = 120, 184                      # 64 + 64 table values
CLOBBER = (40, 248)


def wreg(x, k):
    """VGPR holding byte k's word of block x (x = -1: the window history, in line buffer 1's
    odd half, free until line 1 is requested)."""
    if x < 0:
        return f"v{LB[1] + 16 + (k >> 2)}"
    return f"v{LB[(x // 2) % 2] + 16 * (x % 2) + (k >> 2)}"


def gen():
    L = []
    e = L.append

    def lds_read(dst, addr, k):
        if k % 8 == 0:
            e("s_waitcnt lgkmcnt(7)")      # <= 15 LDS reads in flight
        e(f"ds_read_b32 v{dst}, {addr}")

    def set_addr(block_expr):
        e(f"v_min_u32 {TLO}, {block_expr}, {NM1}")
        e(f"v_lshlrev_b32 {TLO}, 6, {TLO}")
        e(f"v_lshl_add_u64 {ADDR}, {TPAIR}, 0, %[base]")

    def load_words(x, addr):
        r0 = int(wreg(x, 0)[1:])
        for q in range(4):
            e(f"global_load_dwordx4 v[{r0 + 4 * q}:{r0 + 4 * q + 3}], {addr}, off offset:{16 * q}")

    def lookups(x, dst):
        for k in range(64):
            a = A0 if k % 2 == 0 else A1
            e(f"v_perm_b32 {a}, {wreg(x, k)}, %[lane4], %[sel{k & 3}]")
            lds_read(dst + k, a, k)

    # ---- prologue: history, line 0 (blocks 0 and min(1, last)) ----
    e("s_mov_b64 %[sexec], exec")
    e(f"v_mov_b32 {HITS}, 0")
    e(f"v_add_u32 {NM1}, -1, %[nfull]")
    e("v_mov_b32 v49, 0")
    load_words(-1, "%[pre]")
    load_words(0, "%[base]")
    set_addr("1")
    load_words(1, ADDR)
    e("s_waitcnt vmcnt(8) lgkmcnt(0)")     # the history landed (and the compiler's LDS reads)
    lookups(-1, HA)                        # HA = table values of the history bytes
    e("s_waitcnt vmcnt(4)")                # block 0 landed
    lookups(0, HB)                         # HB = table values of block 0
    e("s_waitcnt lgkmcnt(8)")              # every history value landed (older than HB's)
    e(f"v_mov_b32 {H}, 0")
    for k in range(64):                    # h = hash of the history window
        e(f"v_alignbit_b32 {H}, {H}, {H}, 31")
        e(f"v_xor_b32 {H}, {H}, v{HA + k}")
    e("s_mov_b32 %[b], 0")

    def block(i):
        # block cb = b + i (b a multiple of 4)
        hin, hcur = (HA, HB) if i % 2 == 0 else (HB, HA)
        if i == 0:
            e("v_cmp_lt_u32 vcc, %[b], %[nfull]")
        else:
            e(f"s_add_u32 %[sb], %[b], {i}")
            e("v_cmp_lt_u32 vcc, %[sb], %[nfull]")
        e("s_and_b64 exec, exec, vcc")
        e("s_cbranch_execz L_scan_done_%=")
        if i % 2 == 0:
            # line (cb+2, cb+3) into the other buffer (its words were last read by block cb-2)
            e(f"s_add_u32 %[sb], %[b], {i + 2}")
            set_addr("%[sb]")
            load_words(i + 2, ADDR)
            e(f"s_add_u32 %[sb], %[b], {i + 3}")
            set_addr("%[sb]")
            load_words(i + 3, ADDR)
            e("s_waitcnt vmcnt(8)")        # block cb+1 (this line's odd half) landed
        else:
            e("s_waitcnt vmcnt(4)")        # block cb+1 (the next line's even half) landed
        e(f"v_mov_b32 {M}, -1")
        for k in range(0, 64, 2):
            for j, (dst, src) in enumerate(((H0, H), (H, H0))):
                kk = k + j
                a = A0 if j == 0 else A1
                e(f"v_alignbit_b32 {dst}, {src}, {src}, 31")
                e(f"v_perm_b32 {a}, {wreg(i + 1, kk)}, %[lane4], %[sel{kk & 3}]")
                e(f"v_bitop3_b32 {dst}, {dst}, v{hin + kk}, v{hcur + kk} bitop3:0x96")
                lds_read(hin + kk, a, kk)
            e(f"v_min3_u16 {M}, {M}, {H0}, {H}")
        e(f"v_cmp_eq_u16 vcc, 0, {M}")
        e(f"s_lshl_b32 %[sb], {1 << i}, %[b]")
        e(f"v_mov_b32 {T}, %[sb]")
        e(f"v_cndmask_b32 {T}, 0, {T}, vcc")
        e(f"v_or_b32 {HITS}, {HITS}, {T}")

    loop = []
    L_pro = L
    L = loop
    e = L.append
    for i in range(4):
        block(i)
    e("s_add_u32 %[b], %[b], 4")
    e("s_branch L_scan_loop_%=")
    tail = ["L_scan_done_%=:", "s_mov_b64 exec, %[sexec]", "s_waitcnt vmcnt(0) lgkmcnt(0)",
            f"v_mov_b32 %[hits], {HITS}"]
    return L_pro, loop, tail


def sizes(lines):
    text = "\n".join(re.sub(r"%\[(\w+)\]", lambda m: OPS[m.group(1)], l.replace("%=", "0"))
                     for l in lines) + "\n"
    out = subprocess.run([MC, "-arch=amdgcn", "-mcpu=gfx950", "-show-encoding"], input=text,
                         capture_output=True, text=True, check=True).stdout
    enc = [len(m.group(1).split(",")) for m in re.finditer(r"encoding: \[([^\]]*)\]", out)]
    res, k = [], 0
    for l in lines:
        s = l.strip()
        if not s or s.endswith(":") or s.startswith("."):
            res.append(0)
        else:
            res.append(enc[k])
            k += 1
    assert k == len(enc), (k, len(enc))
    return res


# stand-ins of the operands' register classes, for sizing only
OPS = {"sexec": "s[20:21]", "b": "s22", "sb": "s23", "nfull": "v0", "lane4": "v1",
       "sel0": "s24", "sel1": "s25", "sel2": "s26", "sel3": "s27", "pre": "v[2:3]",
       "base": "v[4:5]", "hits": "v6"}


def align8(lines):
    """An s_nop 0 before every 8-byte instruction that would start at 4 mod 8 (the loop label is
    .p2align 3)."""
    out, off = [], 0
    for l, n in zip(lines, sizes(lines)):
        if n == 8 and off % 8 == 4:
            out.append("s_nop 0")
            off += 4
        out.append(l)
        off += n
    return out


def main():
    pro, loop, tail = gen()
    loop = align8(loop)
    sz = sizes(loop)
    mis, off = 0, 0
    for n in sz:
        mis += n == 8 and off % 8 == 4
        off += n
    n_ins = sum(1 for n in sz if n)
    n_nop = sum(1 for l in loop if l == "s_nop 0")
    body = pro + [".p2align 3", "L_scan_loop_%=:"] + loop + tail
    nvalu = sum(1 for l in loop if l.startswith("v_"))
    with open(OUT, "w") as f:
        f.write("// GENERATED by tools/gen_scan_loop.py -- do not edit.\n")
        f.write(f"// k_scan fast pass (split_bits >= 16): loop of 4 blocks = {n_ins} instructions "
                f"({nvalu} VALU, {n_nop} s_nop), {off} bytes, {mis} 8-byte ones at 4 mod 8.\n")
        f.write("#define BSG_SCAN_LOOP_ASM \\\n")
        for l in body:
            f.write(f'  "{l}\\n" \\\n')
        f.write('  ""\n')
        lo, hi = CLOBBER
        f.write("#define BSG_SCAN_LOOP_CLOBBERS " +
                ", ".join(f'"v{r}"' for r in range(lo, hi)) + ', "vcc", "scc", "memory"\n')
    print(OUT, f"loop: {n_ins} instructions, {nvalu} VALU, {n_nop} s_nop, {mis} misaligned")


if __name__ == "__main__":
    main()

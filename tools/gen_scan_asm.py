#!/usr/bin/env python3
"""ROUNDS 1-2 EXPERIMENT, NOT IN THE BUILD; the product form since round 6 is
tools/gen_scan_loop.py (the same loop with every 8-byte instruction aligned). Here: k_scan's rolling buzhash32 over all full
64-byte blocks of one lane's strip (split_bits >= 16 pre-filter) as ONE inline-asm statement.
It was wired in as `scan_blocks_asm(pre, base, nfull, lane4, h, hits)` (outputs: the hash after
the last full block and one bit per pre-filter hit; a k_scan<ASM> template so the compiled loop
kept its own register budget), passed the GPU parity tests in every form below, and measured
per 16 GiB (configs[2]): VGPR-staged loads one block ahead 4.16-4.45 ms (the compiled loop:
4.09-4.42 on the same boxes); + an L2 touch two or four blocks ahead 5.2-5.4 ms; a progressive
quad ring (each 16-B quad refilled as soon as consumed) 5.65 ms; LDS-DMA staging in a 3-slot
ring per wave (`gen_dma`, 160 KiB LDS per workgroup) 5.15 ms; the asm loop without loads
3.0 ms (compiled: 3.35). So the schedule was not what held the loop back; the compiled loop
stays.

Why asm was tried: hipcc's schedule of the same loop issued ~30 cycles per byte-step per SIMD,
against 21 for this per-byte pattern in tools/ubench/scanlike.hip; here the order is fixed.

Per byte k of block b (h = hash after byte k-1; HIN = table values of block b-1 = the out-going
bytes, HCUR = those of block b, looked up one block earlier; W = words of block b+1):
    v_alignbit  H0, H, H, 31              rotl 1
    v_perm      A, W[k/4], lane4, sel[k%4]   LDS address of block b+1's byte k (byte*256+lane*4)
    v_bitop3    H0, H0, HIN[k], HCUR[k]   3-way xor (0x96)
    ds_read_b32 HIN[k], A                 HIN[k] is free once consumed: it becomes block b+1's
... the odd byte the same into H, then
    v_perm      PK, H, H0, 0x05040100     lo16 of the two hashes
    v_pk_min_u16 M, M, PK
After the block, M's halves hold the minimum low 16 bits of its 64 hashes; a zero marks the
block in HITS (bit b) for the exact re-scan. HIN and HCUR swap roles every block, W and WN
(the prefetch of block b+2) too, so a 2-block iteration carries no moves.

Lanes whose strip has fewer blocks drop out by exec mask. LDS reads are throttled to at most 15
in flight (lgkmcnt is 4 bits); every consumed lookup was issued 64 reads earlier, so it has
landed whenever at most 15 are outstanding.
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "bs_amd", "variants", "scan_block_loop_r01.inc")  # not the product include

# fixed registers (the compiler keeps everything else in v0-v71 and v244-v255)
H, H0, M, PK, A0, A1, T = (f"v{72 + i}" for i in range(7))   # v79: JUNK
HITS = "v80"
NM1 = "v81"                 # nfull - 1
TPAIR = "v[82:83]"          # (clamped block index, 0) for the 64-bit address add
TLO = "v82"
ADDR = "v[84:85]"           # address of the block being loaded
PADDR = "v[86:87]"          # address of the block being touched
JUNK = "v79"                # destination of the L2 touches
PREFETCH = int(os.environ.get("BSG_SCAN_TOUCH", "2"))  # touch this many blocks beyond the loads
W0, WN0 = 88, 104           # 16 + 16 word registers
HA0, HB0 = 120, 184         # 64 + 64 table-value registers
CLOBBER_RANGE = (72, 248)


def w(base, k):
    return f"v{base + (k >> 2)}"


def hv(base, k):
    return f"v{base + k}"


def gen(noload=False, coal=False):
    L = []
    e = L.append

    def lds_read(dst, addr, k):
        # a wait before every 8th read of a block keeps <= 15 reads in flight across blocks
        if k % 8 == 0:
            e("s_waitcnt lgkmcnt(7)")
        e(f"ds_read_b32 {dst}, {addr}")

    # Word registers: W (v88..v103) and WN (v104..v119) alternate: the words of block x are in
    # W when x is even, in WN when x is odd; the window history counts as block -1.
    def wreg(x):
        return W0 if x % 2 == 0 else WN0

    def load_block(x, addr):
        r0 = wreg(x)
        for j in range(4):
            r = r0 + 4 * j
            if coal:
                e(f"global_load_dwordx4 v[{r}:{r + 3}], {addr}, off offset:{1024 * j}")
            elif noload:
                for i in range(4):
                    e(f"v_xor_b32 v{r + i}, v84, v{r + i}")
            else:
                e(f"global_load_dwordx4 v[{r}:{r + 3}], {addr}, off offset:{16 * j}")

    def touch(addr):
        # L2 warm-up: one dword of a block PREFETCH blocks ahead, into a junk register; the block's
        # own loads, issued two blocks later, then hit L2 instead of waiting on HBM
        if PREFETCH and not noload:
            e(f"global_load_dword {JUNK}, {addr}, off")

    def lookups_of(x, dst_base):
        for k in range(64):
            a = A0 if k % 2 == 0 else A1
            e(f"v_perm_b32 {a}, v{wreg(x) + (k >> 2)}, %[lane4], %[sel{k & 3}]")
            lds_read(hv(dst_base, k), a, k)

    def set_addr(sblock_expr, reg=ADDR, coal_shift=False):
        e(f"v_min_u32 {TLO}, {sblock_expr}, {NM1}")
        e(f"v_lshlrev_b32 {TLO}, {12 if (coal and coal_shift) else 6}, {TLO}")
        e(f"v_lshl_add_u64 {reg}, {TPAIR}, 0, %[{'coal' if (coal and coal_shift) else 'base'}]")

    # ---- prologue: window history (64 bytes before the strip) and blocks 0, 1 ----
    e("s_waitcnt vmcnt(0) lgkmcnt(0)")
    e("s_mov_b64 %[sexec], exec")
    e(f"v_mov_b32 {HITS}, 0")
    e(f"v_add_u32 {NM1}, -1, %[nfull]")
    e("v_mov_b32 v83, 0")
    load_block(-1, "%[pre]")
    load_block(0, "%[base]")
    e("s_waitcnt vmcnt(4)")
    lookups_of(-1, HA0)                    # HA = table values of the history bytes
    set_addr("1")
    load_block(1, ADDR)
    for x in range(2, 2 + PREFETCH):
        set_addr(str(x), reg=PADDR)
        touch(PADDR)
    e(f"s_waitcnt vmcnt({4 + (PREFETCH if not noload else 0)})")
    lookups_of(0, HB0)                     # HB = table values of block 0
    e("s_waitcnt lgkmcnt(0)")
    e(f"v_mov_b32 {H}, 0")
    for k in range(64):                    # h = hash of the history window
        e(f"v_alignbit_b32 {H}, {H}, {H}, 31")
        e(f"v_xor_b32 {H}, {H}, {hv(HA0, k)}")
    e("s_mov_b32 %[b], 0")

    def block(hin, hcur, parity):
        # block cb = b + parity: its lookups read block cb+1's words; block cb+2 is loaded now
        if parity == 0:
            e("v_cmp_lt_u32 vcc, %[b], %[nfull]")
        else:
            e("s_add_u32 %[sb], %[b], 1")
            e("v_cmp_lt_u32 vcc, %[sb], %[nfull]")
        e("s_and_b64 exec, exec, vcc")
        e("s_cbranch_execz L_scan_done_%=")
        e(f"s_add_u32 %[sb], %[b], {2 + parity}")
        set_addr("%[sb]", coal_shift=True)
        load_block(parity, ADDR)               # block cb+2 has cb's parity
        if PREFETCH and not noload:
            e(f"s_add_u32 %[sb], %[b], {2 + PREFETCH + parity}")
            set_addr("%[sb]", reg=PADDR)
            touch(PADDR)
        # block cb+1's words: all but the youngest loads (cb+2's and the two touches issued since)
        e(f"s_waitcnt vmcnt({6 if (PREFETCH and not noload) else 4})")
        words = wreg(1 + parity)
        e(f"v_mov_b32 {M}, -1")
        for k in range(0, 64, 2):
            for j, (dst, src) in enumerate(((H0, H), (H, H0))):
                kk = k + j
                a = A0 if j == 0 else A1
                e(f"v_alignbit_b32 {dst}, {src}, {src}, 31")
                e(f"v_perm_b32 {a}, v{words + (kk >> 2)}, %[lane4], %[sel{kk & 3}]")
                e(f"v_bitop3_b32 {dst}, {dst}, {hv(hin, kk)}, {hv(hcur, kk)} bitop3:0x96")
                lds_read(hv(hin, kk), a, kk)
            e(f"v_perm_b32 {PK}, {H}, {H0}, %[selpk]")
            e(f"v_pk_min_u16 {M}, {M}, {PK}")
        # hit: either half of M is zero
        e(f"v_lshrrev_b32 {T}, 16, {M}")
        e(f"v_min_u16 {T}, {M}, {T}")
        e(f"v_cmp_eq_u16 vcc, 0, {T}")
        if parity == 0:
            e("s_lshl_b32 %[sb], 1, %[b]")
        else:
            e("s_lshl_b32 %[sb], 2, %[b]")
        e(f"v_mov_b32 {PK}, %[sb]")
        e(f"v_cndmask_b32 {T}, 0, {PK}, vcc")
        e(f"v_or_b32 {HITS}, {HITS}, {T}")

    e("L_scan_loop_%=:")
    block(HA0, HB0, 0)
    block(HB0, HA0, 1)
    e("s_add_u32 %[b], %[b], 2")
    e("s_branch L_scan_loop_%=")
    e("L_scan_done_%=:")
    e("s_mov_b64 exec, %[sexec]")
    e("s_waitcnt vmcnt(0) lgkmcnt(0)")
    e(f"v_mov_b32 %[h], {H}")
    e(f"v_mov_b32 %[hits], {HITS}")
    return L


def gen_dma():
    """The same block loop, with each lane's next blocks staged by LDS-DMA
    (global_load_lds_dwordx4) into a 3-slot ring per wave after the 64 KiB table
    (slot = 4 KiB: quad q of lane l at q*1024 + l*16): two blocks in flight per lane without
    VGPRs, so a CU keeps ~64-96 KiB of reads in flight (the VGPR-staged loop: 32 KiB)."""
    L = []
    e = L.append
    LR = "v79"          # lane's read address in its wave's ring: ring + lane*16
    QADDR = "v[86:87]"

    def lds_read(dst, addr, k):
        if k % 8 == 0:
            e("s_waitcnt lgkmcnt(7)")
        e(f"ds_read_b32 {dst}, {addr}")

    def lookups(dst_base):
        for k in range(64):
            a = A0 if k % 2 == 0 else A1
            e(f"v_perm_b32 {a}, v{W0 + (k >> 2)}, %[lane4], %[sel{k & 3}]")
            lds_read(hv(dst_base, k), a, k)

    def dma(slot, addr):
        # quad q of every lane's block -> ring slot: LDS = M0 + lane*16 (M0 = slot base + q*1024)
        for q in range(4):
            if q:
                e(f"v_lshl_add_u64 {QADDR}, {addr}, 0, {16 * q}")
            e(f"s_add_u32 m0, %[ring], {slot * 4096 + q * 1024}")
            e("s_nop 0")
            e(f"global_load_lds_dwordx4 {addr if q == 0 else QADDR}, off")

    def read_words(slot):
        for q in range(4):
            e(f"ds_read_b128 v[{W0 + 4 * q}:{W0 + 4 * q + 3}], {LR} offset:{slot * 4096 + q * 1024}")

    def set_addr(sblock_expr):
        e(f"v_min_u32 {TLO}, {sblock_expr}, {NM1}")
        e(f"v_lshlrev_b32 {TLO}, 6, {TLO}")
        e(f"v_lshl_add_u64 {ADDR}, {TPAIR}, 0, %[base]")

    e("s_waitcnt vmcnt(0) lgkmcnt(0)")
    e("s_mov_b64 %[sexec], exec")
    e("s_mov_b32 %[keep], m0")
    e(f"v_mov_b32 {HITS}, 0")
    e(f"v_add_u32 {NM1}, -1, %[nfull]")
    e("v_mov_b32 v83, 0")
    e(f"v_lshl_add_u32 {LR}, %[lane4], 2, %[ring]")
    # window history (block -1) -> slot 2, blocks 0, 1 -> slots 0, 1
    dma(2, "%[pre]")
    dma(0, "%[base]")
    set_addr("1")
    dma(1, ADDR)
    e("s_waitcnt vmcnt(8)")
    read_words(2)
    e("s_waitcnt lgkmcnt(0)")
    lookups(HA0)                           # HA = table values of the history bytes
    e("s_waitcnt vmcnt(4)")
    read_words(0)
    e("s_waitcnt lgkmcnt(0)")
    lookups(HB0)                           # HB = table values of block 0
    set_addr("2")
    dma(2, ADDR)
    e("s_waitcnt lgkmcnt(0)")
    e(f"v_mov_b32 {H}, 0")
    for k in range(64):
        e(f"v_alignbit_b32 {H}, {H}, {H}, 31")
        e(f"v_xor_b32 {H}, {H}, {hv(HA0, k)}")
    e("s_mov_b32 %[b], 0")

    def block(i):
        # block cb = b + i (b a multiple of 6): hin/hcur by parity, ring slots by cb mod 3
        hin, hcur = (HA0, HB0) if i % 2 == 0 else (HB0, HA0)
        if i == 0:
            e("v_cmp_lt_u32 vcc, %[b], %[nfull]")
        else:
            e(f"s_add_u32 %[sb], %[b], {i}")
            e("v_cmp_lt_u32 vcc, %[sb], %[nfull]")
        e("s_and_b64 exec, exec, vcc")
        e("s_cbranch_execz L_scan_done_%=")
        e("s_waitcnt vmcnt(4)")            # block cb+1 has landed in its slot
        read_words((i + 1) % 3)
        e("s_waitcnt lgkmcnt(0)")
        e(f"s_add_u32 %[sb], %[b], {i + 3}")
        set_addr("%[sb]")
        dma(i % 3, ADDR)                   # block cb+3 into block cb's slot (read a block ago)
        e(f"v_mov_b32 {M}, -1")
        for k in range(0, 64, 2):
            for j, (dst, src) in enumerate(((H0, H), (H, H0))):
                kk = k + j
                a = A0 if j == 0 else A1
                e(f"v_alignbit_b32 {dst}, {src}, {src}, 31")
                e(f"v_perm_b32 {a}, v{W0 + (kk >> 2)}, %[lane4], %[sel{kk & 3}]")
                e(f"v_bitop3_b32 {dst}, {dst}, {hv(hin, kk)}, {hv(hcur, kk)} bitop3:0x96")
                lds_read(hv(hin, kk), a, kk)
            e(f"v_perm_b32 {PK}, {H}, {H0}, %[selpk]")
            e(f"v_pk_min_u16 {M}, {M}, {PK}")
        e(f"v_lshrrev_b32 {T}, 16, {M}")
        e(f"v_min_u16 {T}, {M}, {T}")
        e(f"v_cmp_eq_u16 vcc, 0, {T}")
        e(f"s_lshl_b32 %[sb], {1 << i}, %[b]")
        e(f"v_mov_b32 {PK}, %[sb]")
        e(f"v_cndmask_b32 {T}, 0, {PK}, vcc")
        e(f"v_or_b32 {HITS}, {HITS}, {T}")

    e("L_scan_loop_%=:")
    for i in range(6):
        block(i)
    e("s_add_u32 %[b], %[b], 6")
    e("s_branch L_scan_loop_%=")
    e("L_scan_done_%=:")
    e("s_mov_b64 exec, %[sexec]")
    e("s_waitcnt vmcnt(0) lgkmcnt(0)")
    e("s_mov_b32 m0, %[keep]")
    e(f"v_mov_b32 %[h], {H}")
    e(f"v_mov_b32 %[hits], {HITS}")
    return L


def main():
    write(gen_dma(), OUT.replace(".inc", "_dma.inc"), "BSG_SCAN_LOOP_ASM")
    write(gen(), OUT, "BSG_SCAN_LOOP_ASM")
    write(gen(noload=True), OUT.replace(".inc", "_noload.inc"), "BSG_SCAN_LOOP_ASM")
    write(gen(coal=True), OUT.replace(".inc", "_coal.inc"), "BSG_SCAN_LOOP_ASM")


def write(L, path, name):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    nvalu = sum(1 for l in L if l.startswith("v_"))
    with open(path, "w") as f:
        f.write("// GENERATED by tools/gen_scan_asm.py -- do not edit.\n")
        f.write(f"// k_scan full-block loop (split_bits >= 16): {len(L)} lines, {nvalu} VALU.\n")
        f.write(f"#define {name} \\\n")
        for l in L:
            f.write(f'  "{l}\\n" \\\n')
        f.write('  ""\n')
        lo, hi = CLOBBER_RANGE
        f.write("#define BSG_SCAN_LOOP_CLOBBERS " +
                ", ".join(f'"v{r}"' for r in range(lo, hi)) + ', "vcc", "scc"\n')
    print(path, len(L), "lines")




# ---------------------------------------------------------------------------------------------
# Round 2 EXPERIMENT, NOT IN THE BUILD: the block loop with whole lines requested TWO lines
# ahead (a first replay run, tools/ubench/gen_scanload.py, showed 3.73 -> 3.06 ms per 16 GiB;
# that was the GPU clock ramping up during the first launches, at full clock both take ~3.0 ms;
# the compiled form needs ~284 VGPRs). Wired into k_scan<true> as scan_lines2() it passed the GPU
# parity tests (test_gpu_parity, test_gpu_configs, test_gpu_params: 90 tests), but a same-box A/B
# gave configs[2]'s k_scan 3.68 / 3.82 ms against 3.71 / 3.69 for the compiled loop
# (profiles/r02_scan_asm2_ab.log), as the clock-corrected replay predicts. Fixed registers
# v22..v255; the compiler keeps what lives across the statement in v0..v21.
#   line j = blocks 2j, 2j+1 -> line buffer LB[j % 3] (lo half = block 2j); the 64 history bytes
#   are block -1 (line -1, hi half). Block cb hashes with hin (out-going) / hcur (in-coming) and
#   looks up block cb+1's bytes into hin; at the start of an even block cb = 2j, line j+2 is
#   requested into the buffer line j-1 has left, so line j+1's words (first read at block 2j+1)
#   were requested three blocks before they are used.
# Per byte: rotl1 (alignbit), perm (LDS address byte*256 + lane*4), xor3 (bitop3), ds_read_b32;
# per two bytes one v_min3_u16 of the low 16 bits (split_bits >= 16 pre-filter).
L2_H, L2_H0, L2_M, L2_A, L2_HITS, L2_NM1 = (f"v{22 + i}" for i in range(6))
L2_A0 = L2_A1 = L2_T = L2_A  # a DS / VMEM instruction reads its address VGPRs at issue
L2_TPAIR, L2_TLO = "v[28:29]", "v28"
L2_ADDR = "v[30:31]"
L2_LB = (32, 64, 96)
L2_HA, L2_HB = 128, 192
L2_OUT = os.path.join(ROOT, "bs_amd", "csrc", "scan_lines2_loop.inc")


def gen_lines2():
    L = []
    e = L.append

    def wreg(x, k):  # VGPR holding byte k's word of block x
        j = x // 2
        return f"v{L2_LB[j % 3] + 16 * (x % 2) + (k >> 2)}"

    def lds_read(dst, addr, k):
        if k % 8 == 0:
            e("s_waitcnt lgkmcnt(7)")  # at most 15 LDS reads in flight (lgkmcnt has 4 bits)
        e(f"ds_read_b32 v{dst}, {addr}")

    def set_addr(reg, block_sgpr):
        e(f"v_min_u32 {L2_TLO}, {block_sgpr}, {L2_NM1}")
        e(f"v_lshlrev_b32 {L2_TLO}, 6, {L2_TLO}")
        e(f"v_lshl_add_u64 {reg}, {L2_TPAIR}, 0, %[base]")

    def load_half(x, addr):
        r0 = L2_LB[(x // 2) % 3] + 16 * (x % 2)
        for q in range(4):
            e(f"global_load_dwordx4 v[{r0 + 4 * q}:{r0 + 4 * q + 3}], {addr}, off offset:{16 * q}")

    def load_line(first_block_sgpr_expr, x_even):
        # blocks x, x+1 (clamped to the strip), both halves back to back: the line is fetched once
        e(f"s_add_u32 %[sb], %[b], {first_block_sgpr_expr}")
        set_addr(L2_ADDR, "%[sb]")
        load_half(x_even, L2_ADDR)
        e("s_add_u32 %[sb], %[sb], 1")
        set_addr(L2_ADDR, "%[sb]")      # (the loads above read their address at issue)
        load_half(x_even + 1, L2_ADDR)

    def lookups(x, dst):
        for k in range(64):
            a = L2_A0 if k % 2 == 0 else L2_A1
            e(f"v_perm_b32 {a}, {wreg(x, k)}, %[lane4], %[sel{k & 3}]")
            lds_read(dst + k, a, k)

    # ---- prologue: history (block -1), line 0, line 1 ----
    e("s_waitcnt vmcnt(0) lgkmcnt(0)")
    e("s_mov_b64 %[sexec], exec")
    e(f"v_mov_b32 {L2_HITS}, 0")
    e(f"v_add_u32 {L2_NM1}, -1, %[nfull]")
    e("v_mov_b32 v29, 0")
    e("s_mov_b32 %[b], 0")
    hist = L2_LB[2] + 16
    for q in range(4):
        e(f"global_load_dwordx4 v[{hist + 4 * q}:{hist + 4 * q + 3}], %[pre], off offset:{16 * q}")
    load_line(0, 0)
    load_line(2, 2)
    e("s_waitcnt vmcnt(16)")                   # the history landed
    lookups(-1, L2_HA)                        # HA = table values of the history bytes
    e("s_waitcnt vmcnt(8)")                    # line 0 landed
    lookups(0, L2_HB)                         # HB = table values of block 0
    e("s_waitcnt lgkmcnt(0)")
    e(f"v_mov_b32 {L2_H}, 0")
    for k in range(64):                       # h = hash of the history window
        e(f"v_alignbit_b32 {L2_H}, {L2_H}, {L2_H}, 31")
        e(f"v_xor_b32 {L2_H}, {L2_H}, v{L2_HA + k}")

    def block(i):
        # block cb = b + i (b a multiple of 6); its words are those of block i mod 6's slot
        hin, hcur = (L2_HA, L2_HB) if i % 2 == 0 else (L2_HB, L2_HA)
        if i == 0:
            e(f"v_cmp_lt_u32 vcc, %[b], %[nfull]")
        else:
            e(f"s_add_u32 %[sb], %[b], {i}")
            e("v_cmp_lt_u32 vcc, %[sb], %[nfull]")
        e("s_and_b64 exec, exec, vcc")
        e("s_cbranch_execz L_scan2_done_%=")
        e("s_waitcnt vmcnt(8)")                # this block's lookups read block cb+1's words
        if i % 2 == 0:                        # start of line j = cb/2: request line j+2
            load_line(i + 4, i + 4)
        e(f"v_mov_b32 {L2_M}, -1")
        for k in range(0, 64, 2):
            for j, (dst, src) in enumerate(((L2_H0, L2_H), (L2_H, L2_H0))):
                kk = k + j
                a = L2_A0 if j == 0 else L2_A1
                e(f"v_alignbit_b32 {dst}, {src}, {src}, 31")
                e(f"v_perm_b32 {a}, {wreg(i + 1, kk)}, %[lane4], %[sel{kk & 3}]")
                e(f"v_bitop3_b32 {dst}, {dst}, v{hin + kk}, v{hcur + kk} bitop3:0x96")
                lds_read(hin + kk, a, kk)
            e(f"v_min3_u16 {L2_M}, {L2_M}, {L2_H0}, {L2_H}")
        e(f"v_cmp_eq_u16 vcc, 0, {L2_M}")
        e(f"s_lshl_b32 %[sb], {1 << i}, %[b]")
        e(f"v_mov_b32 {L2_T}, %[sb]")
        e(f"v_cndmask_b32 {L2_T}, 0, {L2_T}, vcc")
        e(f"v_or_b32 {L2_HITS}, {L2_HITS}, {L2_T}")

    e("L_scan2_loop_%=:")
    for i in range(6):
        block(i)
    e("s_add_u32 %[b], %[b], 6")
    e("s_branch L_scan2_loop_%=")
    e("L_scan2_done_%=:")
    e("s_mov_b64 exec, %[sexec]")
    e("s_waitcnt vmcnt(0) lgkmcnt(0)")
    e(f"v_mov_b32 %[hits], {L2_HITS}")
    nvalu = sum(1 for l in L if l.startswith("v_"))
    with open(L2_OUT, "w") as f:
        f.write("// GENERATED by tools/gen_scan_asm.py (gen_lines2) -- do not edit.\n")
        f.write(f"// k_scan full-block loop, lines requested two ahead: {len(L)} lines, {nvalu} VALU.\n")
        f.write("#define BSG_SCAN_LINES2_ASM \\\n")
        for l in L:
            f.write(f'  "{l}\\n" \\\n')
        f.write('  ""\n')
        f.write("#define BSG_SCAN_LINES2_CLOBBERS " +
                ", ".join(f'"v{r}"' for r in range(22, 256)) + ', "vcc", "scc"\n')
    print(L2_OUT, len(L), "lines", nvalu, "VALU")


if __name__ == "__main__":
    import sys
    if len(sys.argv) > 1 and sys.argv[1] == "lines2":
        gen_lines2()
    else:
        main()

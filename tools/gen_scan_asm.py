#!/usr/bin/env python3
"""EXPERIMENT, NOT IN THE BUILD: k_scan's rolling buzhash32 over all full
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
OUT = os.path.join(ROOT, "bs_amd", "csrc", "scan_block_loop.inc")

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


if __name__ == "__main__":
    main()

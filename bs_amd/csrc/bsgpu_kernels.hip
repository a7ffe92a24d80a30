// bsgpu_kernels.hip — CDNA4 (gfx950) kernels for BS's hashsplit chunker + SHA-256 refs.
//
// Pipeline for one run over a batch of stream segments (see bsgpu_internal.h):
//   k_scan      rolling buzhash32 over every byte position, one lane per 2 KiB strip,
//               64-byte window history kept in VGPRs, 64-way replicated table in LDS
//               (conflict-free ds_read_b32), candidates (tz >= split_bits) into per-strip slots
//   scan_*      exclusive prefix sums (strip counts -> candidate offsets; flags -> chunk index)
//   k_compact   slots -> one sorted candidate list (re-scans the rare overflowing strips)
//   k_select    MinSize greedy as independent walks between "sync points"
//   k_chunks    boundary list; k_tally per-stream counts
//   k_sha       batched variable-length SHA-256, one lane per chunk, dynamic per-lane queue
//
// Reference semantics being reproduced: hashsplit.Splitter as wired by split.NewWriter
// (/root/reference/split/split.go:85-89) and bs.Blob.Ref = sha256 (/root/reference/bs.go:24-26).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "bsgpu_internal.h"
#include "bsgpu_launch.h"
#include "sha256_device.h"
#include "scan_block_loop.inc"

// Wave-mode rounds run split over lanes: skewed pairs (9 VALU per round, 2,941 cycles per
// block on MI355X) and skewed octets (8 VALU, 2,330 at round 5); one lane running the whole
// round takes 14 VALU (4,021 cycles; tools/ubench/skew.hip, oct.hip).
// Wave-mode tiers (k_bucket_scan), in percent of the longest job's blocks: jobs of at least
// BSG_TLEN_PCT run on solo / group tickets (the kSolo longest one per wave, then 8 per wave),
// jobs of BSG_PAIR_PCT up to that on pair tickets (32 per wave, one skewed lane pair each, ring
// fills every 2 blocks), the rest per lane. A pair job's block takes ~2.27 us under load
// against the solo chain's 1.19, so pair jobs above ~0.52 of the longest end after it; with
// the faster per-lane mode (regions, round 2) per-lane jobs may reach 0.34 of it. Measured on
// configs[2]: 50 / 34 with 16 solo tickets 888 GiB/s, 56 / 30 with 8 (the
// earlier setting) 831 on the same box; configs[1] unchanged. Round 5: with the octet chain at
// 2,330 cycles per block (a group ticket ~3x the per-lane wave-cycles per block) and the pair
// at about the per-lane cost, 53 / 56 / 58 gave 982-991 / 987-999 / 962-969 GiB/s and 50 gave
// 977-978 (profiles/r05_ab29_c2.log, r05_ab30_c2.log): 55, a step below the 58 cliff where pair
// jobs end after the longest chain.
#ifndef BSG_TLEN_PCT
#define BSG_TLEN_PCT 55
#endif
#ifndef BSG_PAIR_PCT
#define BSG_PAIR_PCT 34
#endif
// With the octet chains (round 2) a lightly loaded launch — all its blocks are less than a
// tenth of what the chip's lanes hash while the longest chain runs — ends on the pair tickets
// unless the group tier reaches further down: configs[1] 88.2 GiB/s at 56 %, 93.1 at 48 %
// (same chain end), while configs[2] (loaded, per-lane throughput decides) is best at 56 %.
#ifndef BSG_TLEN_PCT_LIGHT
#define BSG_TLEN_PCT_LIGHT 48
#endif
#ifndef BSG_PAIR_PCT_LIGHT
#define BSG_PAIR_PCT_LIGHT 30
#endif

namespace bsg {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(16)));

__device__ __forceinline__ uint32_t tz32(uint32_t h) { return h ? (uint32_t)__builtin_ctz(h) : 32u; }

typedef const __attribute__((address_space(1))) u32x4* g_u32x4p;

// All stream data is in device global memory; the explicit address space keeps these global
// loads (vmcnt only) even where hipcc cannot infer it (e.g. after ScanArgs went through a call),
// instead of flat loads that also count against lgkmcnt, the LDS lookups' counter.
__device__ __forceinline__ void load16(const uint8_t* p, uint32_t (&w)[16]) {
  g_u32x4p q = (g_u32x4p)(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    u32x4 v = q[i];
    w[4 * i + 0] = v.x;
    w[4 * i + 1] = v.y;
    w[4 * i + 2] = v.z;
    w[4 * i + 3] = v.w;
  }
}

// LDS byte address of table row `byte k of word w` in this lane's replica: byte*256 + lane*4,
// built by one v_perm_b32: D.b0 = lane4, D.b1 = w.b[k], D.b2 = D.b3 = 0.
__device__ __forceinline__ uint32_t tab_addr(uint32_t w, uint32_t lane4, int k) {
  // k is a compile-time constant after unrolling, so the selector is an inline literal
  return __builtin_amdgcn_perm(w, lane4, 0x0c0c0400u | ((4u + (uint32_t)(k & 3)) << 8));
}
__device__ __forceinline__ uint32_t lds_u32(const uint32_t* tab, uint32_t byte_addr) {
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(tab) + byte_addr);
}
__device__ __forceinline__ uint32_t lookup(const uint32_t* tab, uint32_t w, uint32_t lane4,
                                           int k) {
  return lds_u32(tab, tab_addr(w, lane4, k));
}

// Called by k_scan (kScanThreads) and k_rescan (kScanWG) workgroups. 256 rows x 64 replicas;
// each uint4 store writes 4 replicas of one row. A thread issues all of its loads before its
// stores: as a load-store loop, each of the 8 iterations waited for its global load (~8
// dependent L2 round trips at the start of every workgroup, before any scanning).
template <uint32_t NT = kScanWG>
__device__ __forceinline__ void load_table(uint32_t* tab, const uint32_t* __restrict__ T) {
  constexpr uint32_t kVec = kTabRows * kTabRep / 4;
  constexpr uint32_t kPer = kVec / NT;
  static_assert(kVec % NT == 0, "table stores per thread");
  u32x4a* t4 = reinterpret_cast<u32x4a*>(tab);
  uint32_t v[kPer];
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) v[k] = T[(threadIdx.x + k * NT) >> 4];
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) t4[threadIdx.x + k * NT] = u32x4a{v[k], v[k], v[k], v[k]};
}

template <class P>
__device__ __forceinline__ uint32_t find_stream(P strip0, uint32_t n, uint64_t strip) {
  // largest s in [0, n) with strip0[s] <= strip (zero-length streams are skipped)
  uint32_t lo = 0, hi = n;  // invariant: strip0[lo] <= strip < strip0[hi]
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if (strip0[mid] <= strip) lo = mid;
    else hi = mid;
  }
  return lo;
}

// ---------------------------------------------------------------------------------------------
// Rolling scan of one strip.
// h(p) = XOR_{k<64} rotl(T[x[p-k]], k mod 32): after warming the window with the 64 bytes
// before the strip (stream history / zeros), each byte costs one LDS lookup, one rotate and
// one 3-way xor; the outgoing byte's table value comes from the 64-entry VGPR history.
// ---------------------------------------------------------------------------------------------
struct StripCtx {
  uint32_t stream;
  uint64_t start;      // segment offset of the strip
  uint32_t count;      // candidates found so far
  uint64_t wbase;      // WRITE mode: first output index
};

template <bool WRITE>
__device__ __forceinline__ void emit(const ScanArgs& a, StripCtx& c, uint64_t strip,
                                     uint64_t seg_off, bool force, uint32_t tz) {
  if (WRITE) {
    uint64_t idx = c.wbase + c.count;
    if (idx < a.cand_cap) a.cand[idx] = cand_pack(c.stream, seg_off, force, tz);
  } else {
    if (c.count < (uint32_t)kSlotCap)
      a.slots[strip * kSlotCap + c.count] = slot_pack((uint32_t)(seg_off - c.start), force, tz);
  }
  c.count++;
}

// Exact scan of `n` (<= 64) positions starting at a 64-aligned segment offset: the hash before
// them is rebuilt from the 64 bytes that precede them (the window property: h depends only on
// those bytes), then each position gets the exact test tz >= bits (equivalent to the fast
// pass's mask test for bits <= 32; Bits > 32 never splits, hashsplit's tz >= SplitBits with
// tz <= 32). Loads are whole 64-byte blocks (BSG_READ_SLACK makes the tail block readable).
// Returns the hash at the last position scanned. FULL (n == 64, every hit block): the lookups of
// each group of kExactGroup positions are issued together before its steps; with a per-position
// `k < n` test every step was its own basic block and waited for its own two LDS reads (the
// exact pass, then the k_refine kernel, ~26 us on 16 K strips).
constexpr int kExactGroup = 8;
template <bool WRITE, bool FULL>
__device__ __forceinline__ uint32_t exact_block(const ScanArgs& a, const uint32_t* tab,
                                                uint32_t lane4, const uint8_t* blk,
                                                const uint8_t* prev, uint32_t n, StripCtx& c,
                                                uint64_t strip, uint64_t off) {
  uint32_t w[16], pw[16];
  load16(blk, w);
  load16(prev, pw);
  uint32_t h = 0;
#pragma unroll
  for (int k = 0; k < 64; ++k) h = rotl1(h) ^ lookup(tab, pw[k >> 2], lane4, k);
  const uint32_t bits = a.p.split_bits;
  if constexpr (FULL) {
#pragma unroll
    for (int q = 0; q < 64; q += kExactGroup) {
      uint32_t tin[kExactGroup], tout[kExactGroup];
#pragma unroll
      for (int k = 0; k < kExactGroup; ++k) {
        tin[k] = lookup(tab, w[(q + k) >> 2], lane4, q + k);
        tout[k] = lookup(tab, pw[(q + k) >> 2], lane4, q + k);
      }
#pragma unroll
      for (int k = 0; k < kExactGroup; ++k) {
        h = xor3(rotl1(h), tout[k], tin[k]);
        const uint32_t tz = tz32(h);
        if (tz >= bits) emit<WRITE>(a, c, strip, off + q + k, false, tz);
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < 64; ++k) {
      if ((uint32_t)k < n) {
        const uint32_t tin = lookup(tab, w[k >> 2], lane4, k);
        const uint32_t tout = lookup(tab, pw[k >> 2], lane4, k);
        h = xor3(rotl1(h), tout, tin);
        const uint32_t tz = tz32(h);
        if (tz >= bits) emit<WRITE>(a, c, strip, off + k, false, tz);
      }
    }
  }
  return h;
}

// k_scan / k_compact allocate no LDS but the dynamic table, so the table starts at LDS
// address 0 and tab_addr()'s result is the address itself (through the generic pointer the
// compiler keeps one v_add of the base per lookup). table_at_lds0() guards the assumption; it
// folds to a constant.
typedef const __attribute__((address_space(3))) uint32_t* lds_u32p;
__device__ __forceinline__ uint32_t lds_at(const uint32_t*, uint32_t byte_addr) {
  return *reinterpret_cast<lds_u32p>(static_cast<uintptr_t>(byte_addr));
}
__device__ __forceinline__ bool table_at_lds0(const uint32_t* tab) {
  return (uint32_t)(uintptr_t)((lds_u32p)tab) == 0u;
}

// One 64-byte block of the compiled fast loop (the narrow pre-filter, split_bits < 16; the
// WIDE form is the asm statement of scan_span), software-pipelined: hin[] holds the table values
// of the previous block (the out-going bytes), hcur[] those of this block (looked up one block
// earlier). As soon as step k has consumed hin[k], the lookup of byte k of the NEXT block is
// issued into that register, so ~64 LDS reads are in flight behind the hash chain instead of
// sitting in front of it, and the two arrays swap roles every block (no register moves).
// Candidate pre-filter per block: min3 of (h & mask); a block whose pre-filter hits is re-scanned
// exactly by k_scan's exact pass.
template <bool LOAD>
__device__ __forceinline__ bool chain64(const uint32_t* tab, const uint32_t (&wnext)[16],
                                        uint32_t (&hin)[64], const uint32_t (&hcur)[64],
                                        uint32_t& h, uint32_t lane4, uint32_t mask) {
  uint32_t m = 0xffffffffu;
#pragma unroll
  for (int k = 0; k < 64; ++k) {
    h = xor3(rotl1(h), hin[k], hcur[k]);
    if (LOAD) hin[k] = lds_at(tab, tab_addr(wnext[k >> 2], lane4, k));
    m = min(m, h & mask);
  }
  return m == 0;
}

__device__ __forceinline__ void lookup64(const uint32_t* tab, const uint32_t (&w)[16],
                                         uint32_t (&t)[64], uint32_t lane4) {
#pragma unroll
  for (int k = 0; k < 64; ++k) t[k] = lds_at(tab, tab_addr(w[k >> 2], lane4, k));
}

// All full 64-byte blocks of a strip. On entry hA = table values of the 64 bytes before the
// strip, h = the hash there, and w0 / w1 = the strip's first line (blocks 0 and 1, loaded by
// the caller beside the history block). Blocks whose pre-filter hits are only marked here (one
// bit each); k_scan's exact pass scans them afterwards, in block order, so the fast loop holds
// nothing but the two histories, two word blocks and the hash (no call, no scratch).
static_assert(kStrip / 64 <= 32, "one 32-bit hit mask per strip (kStrip <= 2 KiB)");

__device__ __forceinline__ uint32_t scan_full_blocks(const ScanArgs& a, const uint32_t* tab,
                                                     uint32_t lane4, const uint8_t* base,
                                                     uint32_t nfull, uint32_t& h,
                                                     uint32_t (&hA)[64], uint32_t (&w0)[16],
                                                     uint32_t (&w1)[16]) {
  const uint32_t mask = a.p.mask;
  uint32_t hB[64];
  // Blocks are loaded in pairs, the two 64-byte halves of one 128-byte line back to back, so
  // the line is fetched once: loaded one block apart, the second half often found its line
  // evicted from L2 and fetched it again (k_scan read 1.5x its input on configs[1]).
  uint32_t n0[16], n1[16];
  uint32_t hits = 0;
  lookup64(tab, w0, hB, lane4);                         // hB = block 0
  uint32_t b = 0;
  for (; b + 1 < nfull; b += 2) {
    load16(base + 64ull * min(b + 2, nfull - 1), n0);  // the next line (clamped, branch-free)
    load16(base + 64ull * min(b + 3, nfull - 1), n1);
    // block b: out-going hA, in-coming hB; looks up block b+1 into hA
    hits |= chain64<true>(tab, w1, hA, hB, h, lane4, mask) ? 1u << b : 0u;
    // block b+1: out-going hB, in-coming hA; looks up block b+2 into hB
    hits |= chain64<true>(tab, n0, hB, hA, h, lane4, mask) ? 1u << (b + 1) : 0u;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      w0[i] = n0[i];
      w1[i] = n1[i];
    }
  }
  if (b < nfull) {  // odd block count: the last block, then its values back into hA
    hits |= chain64<false>(tab, w1, hA, hB, h, lane4, mask) ? 1u << b : 0u;
#pragma unroll
    for (int k = 0; k < 64; ++k) hA[k] = hB[k];
  }
  return hits;
}

// strip0 (the streams' first strips) cached in LDS after the table, when it fits: the stream
// of a strip is a binary search over it, one dependent load per step, at every strip start.
constexpr uint32_t kStrip0Lds = 2048;
typedef const __attribute__((address_space(3))) uint64_t* lds_u64p;

__device__ __forceinline__ lds_u64p cache_strip0(uint32_t* lds_after, const ScanArgs& a,
                                                 uint32_t cap = kStrip0Lds) {
  if (a.nstreams + 1 > cap) return nullptr;
  uint64_t* s0 = reinterpret_cast<uint64_t*>(lds_after);
  for (uint32_t i = threadIdx.x; i <= a.nstreams; i += blockDim.x) s0[i] = a.strip0[i];
  return (lds_u64p)(s0);  // generic -> LDS address space
}

// Where a strip lies: its stream (binary search over the streams' first strips) and segment.
struct StripLoc {
  uint32_t stream;
  uint64_t start;     // segment offset of the strip
  uint32_t len;       // bytes in the strip
  bool last;          // the segment's last strip
};

__device__ __forceinline__ StripLoc locate(const ScanArgs& a, uint64_t strip, lds_u64p s0) {
  StripLoc l;
  uint64_t first;
  if (s0) {
    l.stream = find_stream(s0, a.nstreams, strip);
    first = s0[l.stream];
  } else {
    l.stream = find_stream(a.strip0, a.nstreams, strip);
    first = a.strip0[l.stream];
  }
  const uint64_t seglen = a.streams[l.stream].len;
  l.start = (strip - first) * (uint64_t)kStrip;
  l.len = (uint32_t)min((uint64_t)kStrip, seglen - l.start);
  l.last = l.start + l.len == seglen;
  return l;
}

// Where a strip's bytes are and what its segment needs, for the fast pass: located and read from
// the stream descriptor one strip AHEAD of its scan (k_scan's loop), so the binary search and the
// descriptor loads run behind the current strip's scan instead of stalling both waves of every
// SIMD at each strip start.
struct StripJob {
  const uint8_t* d;    // the segment's first byte
  const uint8_t* pre;  // the 64 bytes before the strip (the segment history for its first strip)
  uint64_t start;      // segment offset of the strip
  uint32_t len;        // bytes in the strip
  bool tail;           // the exact pass has the segment's < 64-byte tail or the final flush here
  bool fin;            // the segment ends its stream (Splitter.Close's flush at its last byte)
  uint64_t seglen;     // the segment's length
};

__device__ __forceinline__ StripJob strip_job(const ScanArgs& a, uint64_t strip, lds_u64p s0) {
  const StripLoc l = locate(a, strip, s0);
  const StreamDesc* sd = a.streams + l.stream;
  StripJob j;
  j.d = a.data + sd->data_off;
  j.pre = l.start >= 64 ? j.d + l.start - 64 : sd->hist;
  j.start = l.start;
  j.len = l.len;
  j.tail = (l.len & 63u) != 0 || (l.last && sd->finalize);
  j.fin = sd->finalize;
  j.seglen = sd->len;
  return j;
}

// Fast pass over one strip: the rolling hash at every position of its full 64-byte blocks, a
// hit bit per block whose pre-filter fires. The strip's first line is loaded with its history
// block (one HBM round trip per strip start instead of two; a short strip reads within
// kReadSlack), then the window is warmed on the history in the running form h = rotl1(h) ^ t.
// WIDE (split_bits >= 16, every default run): one generated asm statement
// (tools/gen_scan_loop.py, scan_block_loop.inc) with every 8-byte instruction 8-byte aligned,
// 324 instructions per block against hipcc's 390 (536 of its 1,559 per four blocks started at
// 4 mod 8): configs[2]'s k_scan 3.49-3.55 -> 3.22-3.30 ms (round 6,
// profiles/r06_c8_*). The narrow pre-filter keeps the compiled loop (scan_full_blocks).
// (Round 5 measured and dropped: the warm-up as independent rotates folded by xor3, and chained
// strips — lane l continuing lane l-1's strip so that the history block is not read again —
// which cut k_scan's reads from 1.069x to 1.007x of its input but ran 4-7 % longer,
// profiles/r05_ab20_*.log: the loop is not bound by HBM bytes alone.)
template <bool WIDE>
__device__ __forceinline__ uint32_t scan_span(const ScanArgs& a, const uint32_t* tab,
                                              uint32_t lane4, const StripJob& j) {
  const uint32_t nfull = j.len >> 6;
  const uint8_t* base = j.d + j.start;
  if (WIDE) {
    // operands: the LDS address selectors of tab_addr() for bytes 0-3 of a word; the statement
    // owns v40-v247 (histories, two line buffers, hash, addresses) and restores exec
    uint32_t hits, b, sb;
    uint64_t sexec;
    asm volatile(BSG_SCAN_LOOP_ASM
                 : [hits] "=v"(hits), [sexec] "=&s"(sexec), [b] "=&s"(b), [sb] "=&s"(sb)
                 : [nfull] "v"(nfull), [lane4] "v"(lane4), [pre] "v"(j.pre), [base] "v"(base),
                   [sel0] "s"(0x0c0c0400u), [sel1] "s"(0x0c0c0500u), [sel2] "s"(0x0c0c0600u),
                   [sel3] "s"(0x0c0c0700u)
                 : BSG_SCAN_LOOP_CLOBBERS);
    return hits;
  }
  uint32_t w[16], w0[16], w1[16], hist[64];
  load16(j.pre, w);
  load16(base, w0);
  load16(base + 64ull * min(1u, nfull - 1), w1);
  __builtin_amdgcn_sched_barrier(0);
  uint32_t h = 0;
#pragma unroll
  for (int k = 0; k < 64; ++k) {
    uint32_t t = lds_at(tab, tab_addr(w[k >> 2], lane4, k));
    h = rotl1(h) ^ t;
    hist[k] = t;
  }
  return nfull ? scan_full_blocks(a, tab, lane4, base, nfull, h, hist, w0, w1) : 0u;
}

// Appends the flagged strips of a wave to its workgroup's refine list (refine + blockIdx.x *
// list_cap): entry = strip << 32 | hit mask. The list's count is an LDS word, so the append is a
// returning LDS atomic (a returning global one's vmcnt(0) wait also drained the next strip's
// prefetched lines); the workgroup stores its count at exit.
__device__ __forceinline__ void refine_append(const ScanArgs& a, bool flag, uint64_t strip,
                                              uint32_t hits, uint32_t* lds_cnt) {
  const uint64_t m = __ballot(flag);
  if (!m) return;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t leader = (uint32_t)__builtin_ctzll(m);
  uint32_t b = 0;
  if (lane == leader) b = atomicAdd(lds_cnt, (uint32_t)__builtin_popcountll(m));
  const uint64_t base = (uint64_t)blockIdx.x * a.list_cap + (uint32_t)__shfl((int)b, (int)leader);
  if (flag) {
    const uint64_t below = m & ((1ull << lane) - 1ull);
    a.refine[base + (uint64_t)__builtin_popcountll(below)] = (strip << 32) | hits;
  }
}

// Calls f(entry) for this thread's share of the refine lists: workgroup g of the consumer
// (k_compact, k_rescan; their grids are ScanArgs::lists) walks k_scan workgroup g's list, whose
// length is about the same for every list.
template <class F>
__device__ __forceinline__ void for_refine(const ScanArgs& a, uint32_t threads, F f) {
  for (uint32_t g = blockIdx.x; g < a.lists; g += gridDim.x) {
    const uint64_t n = a.list_cnt[g];
    const uint64_t* list = a.refine + (uint64_t)g * a.list_cap;
    for (uint64_t i = threadIdx.x; i < n; i += threads) f(list[i]);
  }
}

// Exact candidates of one strip flagged by the fast pass, in position order: its hit blocks,
// then the segment's tail (< 64 bytes), then Splitter.Close()'s flush of the final chunk (a
// forced candidate at the last byte, level from the same check). WRITE = false: the first
// kSlotCap into the strip's slots; true: all of them straight into the candidate list at wbase.
template <bool WRITE>
__device__ __forceinline__ uint32_t refine_strip(const ScanArgs& a, const uint32_t* tab,
                                                 uint32_t lane4, uint64_t strip, uint32_t hits,
                                                 uint64_t wbase, lds_u64p s0) {
  const StripLoc l = locate(a, strip, s0);
  const StreamDesc* sd = a.streams + l.stream;
  const uint8_t* d = a.data + sd->data_off;
  StripCtx c;
  c.stream = l.stream;
  c.start = l.start;
  c.count = 0;
  c.wbase = wbase;
  while (hits) {
    const uint64_t off = l.start + 64ull * (uint32_t)__builtin_ctz(hits);
    hits &= hits - 1;
    exact_block<WRITE, true>(a, tab, lane4, d + off, off >= 64 ? d + off - 64 : sd->hist, 64u, c,
                       strip, off);
  }
  const uint32_t rem = l.len & 63u;
  const bool flush = l.last && sd->finalize;
  if (rem || flush) {
    // the hash entering the tail (or, with no tail, at the segment's last byte) is rebuilt
    // from the 64 bytes before the tail's 64-aligned start
    const uint64_t off = l.start + (l.len & ~63u);
    const uint32_t h = exact_block<WRITE, false>(a, tab, lane4, d + off,
                                          off >= 64 ? d + off - 64 : sd->hist, rem, c, strip, off);
    if (flush) emit<WRITE>(a, c, strip, l.start + l.len - 1, true, tz32(h));
  }
  return c.count;
}

// k_scan's workgroup: 256 threads (one wave per SIMD), a strip each per iteration, two
// workgroups per CU, so a CU's next workgroup starts when one ends instead of when the CU's only
// one does (its slowest wave ends ~10 % after the average, profiles/r05_scan_stamps*); 512-thread
// workgroups, one per CU, measured the same (profiles/r05_ab38_c1.log). Dynamic LDS: the table
// (at address 0), strip0 (two entries short of kStrip0Lds, so that two workgroups fit the CU's
// 160 KiB), the list count and two ticket slots.
// The grid is what the chip holds at once (two workgroups per CU) and each workgroup takes its
// next strip group from a ticket counter (Counters::scan_ticket) instead of a fixed stride, so
// the workgroups of slow CUs take fewer groups and all end together. With the fixed stride,
// 1,024 workgroups ran as two rounds of 512 and the step ended with the slowest workgroup of the
// second round: wave life 1.61 ms on average, 2.05 at most, the kernel 3.6 ms on configs[2]
// (profiles/r05_scan_stamps5_w256.log). A workgroup takes at most kScanDynShare times its even
// share, which bounds its refine list.
constexpr uint64_t kScanDynShare = 2;
constexpr uint32_t kScanThreads = 256;
constexpr uint32_t kScanGroup = kScanThreads;  // strips per workgroup iteration
constexpr uint32_t kScanStrip0Cap = kStrip0Lds - 2;
constexpr uint32_t kScanLdsStrip0 = kTabRows * kTabRep * 4;
constexpr uint32_t kScanLdsCnt = kScanLdsStrip0 + kScanStrip0Cap * 8;
constexpr uint32_t kScanLds = kScanLdsCnt + 16u;  // the list count, 2 ticket slots
static_assert(2 * kScanLds <= 160 * 1024, "two k_scan workgroups per CU");

// WIDE (split_bits >= 16, the packed 16-bit pre-filter) and the narrow form are separate
// kernels, so each holds one copy of the fast loop and its registers.
template <bool WIDE>
__global__ __launch_bounds__(kScanThreads, 2) void k_scan(ScanArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t tab[];
  if (!table_at_lds0(tab)) {
    if (threadIdx.x == 0) atomicOr(reinterpret_cast<unsigned long long*>(&a.ctr->error), 2ull);
    return;
  }
  uint32_t* lds_cnt = tab + kScanLdsCnt / 4;
  if (threadIdx.x == 0) *lds_cnt = 0u;
  load_table<kScanThreads>(tab, a.table);
  const lds_u64p s0 = cache_strip0(tab + kScanLdsStrip0 / 4, a, kScanStrip0Cap);
  __syncthreads();
  const uint32_t lane4 = (threadIdx.x & 63u) << 2;
  uint64_t g = blockIdx.x;
  StripJob job{};
  if (g * kScanGroup + threadIdx.x < a.nstrips) job = strip_job(a, g * kScanGroup + threadIdx.x, s0);
  // group tickets: the first group is blockIdx.x, later ones gridDim.x + the counter's value.
  // Thread 0 takes the ticket after next while the current group is scanned; it reaches the
  // others through LDS slot (iteration & 1) behind the iteration's barrier (a slot is written
  // again two iterations later, after every thread has passed the barrier that follows its reads).
  const uint64_t ngroups = (a.nstrips + kScanGroup - 1) / kScanGroup;
  const uint64_t max_groups = a.list_cap / kScanGroup;  // the refine list's bound
  uint32_t* tslot = lds_cnt + 1;
  uint64_t taken = 1;
  uint64_t gnext = ~0ull;
  if (threadIdx.x == 0) {
    const uint64_t t = taken < max_groups
        ? gridDim.x + atomicAdd(reinterpret_cast<unsigned long long*>(&a.ctr->scan_ticket), 1ull)
        : ~0ull;
    tslot[0] = (uint32_t)min(t, (uint64_t)0xffffffffu);
  }
  __syncthreads();
  gnext = tslot[0];
  taken += gnext < ngroups;
  for (uint32_t it = 1; g < ngroups; ++it) {
    const uint64_t strip = g * kScanGroup + threadIdx.x;
    const StripJob cur = job;
    const uint64_t next = gnext < ngroups ? gnext * kScanGroup + threadIdx.x : ~0ull;
    if (next < a.nstrips) job = strip_job(a, next, s0);  // used one iteration later
    uint64_t tk = ~0ull;
    if (threadIdx.x == 0 && gnext < ngroups && taken < max_groups)
      tk = gridDim.x + atomicAdd(reinterpret_cast<unsigned long long*>(&a.ctr->scan_ticket), 1ull);
    bool flag = false;
    uint32_t hits = 0;
    const bool in = strip < a.nstrips;
    if (in) {
      hits = scan_span<WIDE>(a, tab, lane4, cur);
      a.counts[strip] = 0u;
      flag = hits || cur.tail;
    }
    refine_append(a, flag, strip, hits, lds_cnt);
    if (threadIdx.x == 0) tslot[it & 1u] = (uint32_t)min(tk, (uint64_t)0xffffffffu);
    __syncthreads();
    g = gnext;
    gnext = g < ngroups ? tslot[it & 1u] : ~0ull;
    taken += gnext < ngroups;
  }
  __syncthreads();
  const uint32_t nlist = *lds_cnt;
  if (threadIdx.x == 0) a.list_cnt[blockIdx.x] = nlist;
  // The exact pass over this workgroup's own list, here, with the table and strip0 already in
  // LDS: no dispatch, no table load, and a workgroup that ends early refines while the others
  // still scan. (The list entries are this workgroup's own stores, ordered by the barrier
  // above.)
  const uint64_t* list = a.refine + (uint64_t)blockIdx.x * a.list_cap;
  for (uint32_t i = threadIdx.x; i < nlist; i += kScanThreads) {
    const uint64_t e = list[i];
    const uint64_t strip = e >> 32;
    const uint32_t n = refine_strip<false>(a, tab, lane4, strip, (uint32_t)e, 0, s0);
    a.counts[strip] = n;
    if (n > (uint32_t)kSlotCap)
      atomicAdd(reinterpret_cast<unsigned long long*>(&a.ctr->rescan), 1ull);
  }
}

// Slots -> the sorted candidate list, one lane per strip. No table and no re-scan registers,
// so many waves per SIMD hide the loads; strips whose candidates overflowed their slots are
// left to k_rescan.
__global__ __launch_bounds__(256) void k_compact(ScanArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  if (a.ctr->overflow) return;
  const lds_u64p s0 = cache_strip0(lds, a);
  __syncthreads();
  // only strips on k_scan's refine list can hold candidates (every other count is 0)
  for_refine(a, blockDim.x, [&](uint64_t e) {
    const uint64_t strip = e >> 32;
    const uint32_t cnt = a.counts[strip];
    if (cnt == 0 || cnt > (uint32_t)kSlotCap) return;
    const uint64_t base = a.cand_off[strip];
    uint32_t st;
    uint64_t first;
    if (s0) {
      st = find_stream(s0, a.nstreams, strip);
      first = s0[st];
    } else {
      st = find_stream(a.strip0, a.nstreams, strip);
      first = a.strip0[st];
    }
    const uint64_t start = (strip - first) * (uint64_t)kStrip;  // segment-relative
    for (uint32_t i = 0; i < cnt; ++i) {
      const uint32_t v = a.slots[strip * kSlotCap + i];
      if (base + i < a.cand_cap)
        a.cand[base + i] = cand_pack(st, start + (v >> 8), (v & 0x80u) != 0, v & 63u);
    }
  });
}

// Strips with more candidates than slots (k_scan counted them in ctr->rescan) are scanned
// again, writing straight into the candidate list. Exits at once when there are none.
__global__ __launch_bounds__(kScanWG, 2) void k_rescan(ScanArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t tab[];
  if (a.ctr->overflow || !a.ctr->rescan) return;
  if (!table_at_lds0(tab)) {
    if (threadIdx.x == 0) atomicOr(reinterpret_cast<unsigned long long*>(&a.ctr->error), 2ull);
    return;
  }
  load_table(tab, a.table);
  __syncthreads();
  const uint32_t lane4 = (threadIdx.x & 63u) << 2;
  for_refine(a, kScanWG, [&](uint64_t e) {
    const uint64_t strip = e >> 32;
    if (a.counts[strip] > (uint32_t)kSlotCap)
      refine_strip<true>(a, tab, lane4, strip, (uint32_t)e, a.cand_off[strip], nullptr);
  });
}

// ---------------------------------------------------------------------------------------------
// Exclusive prefix sum u32 -> u64 (k_prefix1). n is min(n_bound, *n_dev) when n_dev != null.
// ---------------------------------------------------------------------------------------------
constexpr int kScanT = 256, kScanItems = 8, kScanTile = kScanT * kScanItems;

__device__ __forceinline__ uint64_t scan_n(const PrefixArgs& a) {
  uint64_t n = a.n_bound;
  if (a.n_dev) n = min(n, *a.n_dev);
  return n;
}

// Single-pass exclusive prefix (round 5; decoupled look-back): one dispatch instead of a
// reduce -> top -> down sequence of three, each of which cost a kernel boundary and a pass over
// the input on the way to the early chains (configs[2]: 48 us for the strip counts). Workgroup t
// takes tile t, publishes its tile's sum, and wave 0 looks back over the preceding tiles 64 at a
// time, summing published tile sums until it meets a tile's published inclusive prefix. Tiles go
// by blockIdx, not by a ticket counter: one counter hands out ≈ 88 tickets per us
// (MI355X_MICROARCH.md, dequeue), 47 us for configs[2]'s 4,096 tiles, which made this kernel
// slower than the three it replaced (profiles/r05_ab2.log). A status word carries its value with
// its flag (the value in the low 62 bits), so one relaxed agent-scope (sc1) store publishes it and
// one such load reads it: no payload to fence. k_start zeroes the status words.
// Forward progress rests on in-order dispatch: the command processor hands out a grid's
// workgroups in blockIdx order, each XCD's share in order too, so every tile a workgroup waits
// for has been dispatched before it (it is resident or has finished) and a waiting workgroup never
// holds back the one it waits for. Should that ever fail, the bounded poll (kPfxPolls sleeps,
// ~1 s) ends the wait and flags device error 32 instead of hanging the GPU.
constexpr uint64_t kPfxAgg = 1ull << 62, kPfxInc = 2ull << 62, kPfxVal = kPfxAgg - 1;
constexpr uint32_t kPfxPolls = 1u << 22;

__device__ __forceinline__ uint64_t pfx_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void pfx_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kScanT) void k_prefix1(PrefixArgs a) {
  __shared__ uint64_t wsum[kScanT / 64];
  __shared__ uint64_t sh_excl;
  if (a.skip_if && *a.skip_if) return;
  const uint64_t n = scan_n(a);
  uint64_t* status = a.partials;
  const uint64_t t = blockIdx.x;
  const uint64_t base = t * (uint64_t)kScanTile;
  if (base >= n && t != 0) return;  // past the data: nobody looks back at this tile
  const uint64_t first = base + (uint64_t)threadIdx.x * kScanItems;
  uint32_t v[kScanItems];
  uint64_t sum = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    v[i] = (first + i < n) ? a.in[first + i] : 0u;
    sum += v[i];
  }
  uint64_t x = sum;  // inclusive wave scan
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(x, o);
    if ((threadIdx.x & 63) >= (uint32_t)o) x += y;
  }
  if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = x;
  __syncthreads();
  uint64_t pre = x - sum;
  const uint32_t w = threadIdx.x >> 6;
  for (uint32_t k = 0; k < w; ++k) pre += wsum[k];
  const uint64_t agg = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  if (w == 0) {
    const uint32_t lane = threadIdx.x & 63u;
    uint64_t excl = 0;
    if (t == 0) {
      if (lane == 0) pfx_store(status, kPfxInc | agg);
    } else {
      if (lane == 0) pfx_store(status + t, kPfxAgg | agg);
      int64_t p = (int64_t)t - 1;  // the window's newest tile
      bool done = false;
      uint32_t polls = 0;
      while (!done) {
        const int64_t q = p - (int64_t)lane;  // this lane's predecessor
        uint64_t st = q >= 0 ? pfx_load(status + q) : kPfxInc;  // (before tile 0: nothing)
        while (__ballot(st == 0)) {  // someone's predecessor has not published yet
          if (++polls > kPfxPolls) {
            if (lane == 0 && a.error) atomicOr(reinterpret_cast<unsigned long long*>(a.error), 32ull);
            st = kPfxInc;  // give up (the run is flagged)
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          if (st == 0) st = pfx_load(status + q);
        }
        // the nearest predecessor with an inclusive prefix ends the look-back
        const uint64_t inc = __ballot((st & kPfxInc) != 0);
        const uint32_t stop = inc ? (uint32_t)__builtin_ctzll(inc) : 64u;
        uint64_t part = (lane <= stop) ? (st & kPfxVal) : 0ull;
        for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
        excl += part;
        done = inc != 0;
        p -= 64;
      }
      if (lane == 0) pfx_store(status + t, kPfxInc | (excl + agg));
    }
    if (lane == 0) {
      sh_excl = excl;
      if (n == 0 || (base < n && n <= base + kScanTile)) {  // the last tile: the total
        *a.total = excl + agg;
        if (a.overflow && excl + agg > a.cap) *a.overflow = 1;
      }
    }
  }
  __syncthreads();
  pre += sh_excl;
  // Offsets are only read where the input is non-zero (k_compact / k_rescan for strips with
  // candidates, k_chunks for flagged candidates), so only those are written: on configs[2]
  // this is ~250 K of 8 M strip offsets.
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    if (first + i < n && v[i]) a.out[first + i] = pre;
    pre += v[i];
  }
}

// ---------------------------------------------------------------------------------------------
// MinSize greedy selection. A candidate whose distance to its predecessor (or to the open
// chunk's start) is >= MinSize is a boundary whatever came before ("sync point"), so the
// greedy chain restarts there: one lane walks each run of candidates between sync points.
// ---------------------------------------------------------------------------------------------

__global__ __launch_bounds__(256) void k_select(SelArgs a) {
  if (a.ctr->overflow) return;
  const uint64_t total = a.ctr->ncand;
  const uint64_t minsz = a.p.min_size;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const uint64_t c = a.cand[i];
    const uint32_t s = cand_stream(c);
    // Candidate positions are segment-relative (40 bits: a segment is < 2^40 bytes of device
    // memory); the open chunk's start and the boundaries are absolute stream offsets (u64), so
    // a stream may run past 2^40 bytes, as split.Writer.Write allows (split/split.go:99-101).
    const uint64_t Er = cand_pos(c) + 1;  // segment-relative end if this candidate is a boundary
    const bool first = (i == 0) || cand_stream(a.cand[i - 1]) != s;
    if (!first) {
      const uint64_t pEr = cand_pos(a.cand[i - 1]) + 1;
      if (Er - pEr < minsz) continue;  // not a sync point: covered by an earlier walk
    }
    const uint64_t sb = a.streams[s].seg_base;
    uint64_t last, j;
    if (first) {
      last = a.streams[s].open_start;
      j = i;
    } else {
      a.flags[i] = 1;
      last = sb + Er;
      j = i + 1;
    }
    uint64_t prevEr = first ? 0 : Er;
    for (; j < total; ++j) {
      const uint64_t cj = a.cand[j];
      if (cand_stream(cj) != s) break;
      const uint64_t Ejr = cand_pos(cj) + 1;
      if (j > i && Ejr - prevEr >= minsz) break;  // next sync point starts its own walk
      const uint64_t Ej = sb + Ejr;
      const bool f = cand_force(cj) ? (Ej > last) : (Ej - last >= minsz);
      a.flags[j] = f ? 1u : 0u;
      if (f) last = Ej;
      prevEr = Ejr;
    }
  }
}

__global__ __launch_bounds__(256) void k_chunks(ChunkArgs a) {
  if (a.ctr->overflow) return;
  const uint64_t total = a.ctr->ncand;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint32_t bits = a.p.split_bits;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    if (!a.flags[i]) continue;
    const uint64_t c = a.cand[i];
    const uint64_t k = a.fidx[i];
    const uint32_t s = cand_stream(c);
    const uint32_t tz = cand_tz(c);
    const uint32_t level = tz >= bits ? tz - bits : 0u;
    const uint64_t E = a.streams[s].seg_base + cand_pos(c) + 1;  // absolute stream offset
    if (k >= a.chunk_cap) {  // cannot happen if selection is right (chunks >= MinSize)
      atomicOr(reinterpret_cast<unsigned long long*>(&a.ctr->error), 1ull);
      continue;
    }
    a.bnd_end[k] = E;
    a.bnd_info[k] = ((uint64_t)s << 32) | level;
  }
}

// Per-stream chunk count and end of the last chunk. The boundary list is stream-major, so a
// stream's chunks are one contiguous range found by binary search (no contended atomics: with
// one stream, 16 K same-address atomics cost ~200 us).
__device__ __forceinline__ uint64_t first_chunk_of(const uint64_t* info, uint64_t M, uint32_t s) {
  uint64_t lo = 0, hi = M;  // first k with stream(k) >= s
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if ((uint32_t)(info[mid] >> 32) < s) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(256) void k_tally(ChunkArgs a, uint32_t nstreams) {
  if (a.ctr->overflow || a.ctr->error) return;
  const uint64_t M = min(a.ctr->nchunks, a.chunk_cap);
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nstreams;
       s += gridDim.x * blockDim.x) {
    const uint64_t lo = first_chunk_of(a.bnd_info, M, s);
    const uint64_t hi = first_chunk_of(a.bnd_info, M, s + 1);
    a.scount[s] = hi - lo;
    if (hi > lo) a.last_end[s] = a.bnd_end[hi - 1];  // else k_start's open_start stays
  }
}

// bsg_engine_hash: every stream of the batch is one blob, hashed whole as one final chunk of
// level 0 (no scan, no selection); k_lens / k_order / k_sha then run as for a split batch, so
// the longest blobs get the wave-mode chains and the rest the per-lane LPT queues.
__global__ __launch_bounds__(256) void k_blob_jobs(ChunkArgs a, const StreamDesc* streams,
                                                   uint32_t nstreams) {
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nstreams;
       s += gridDim.x * blockDim.x) {
    const uint64_t L = streams[s].len;
    a.bnd_end[s] = L;
    a.bnd_info[s] = (uint64_t)s << 32;
    a.scount[s] = 1;
    a.last_end[s] = L;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    a.ctr->nchunks = nstreams;
    a.ctr->ncand = nstreams;
  }
}

__global__ __launch_bounds__(256) void k_start(StartArgs a) {
  const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  static_assert(sizeof(StreamDesc) % 16 == 0, "descriptors copy as 16-byte words");
  const uint64_t n4 = (uint64_t)a.nstreams * (sizeof(StreamDesc) / 16);
  const u32x4a* s4 = reinterpret_cast<const u32x4a*>(a.src);
  u32x4a* d4 = reinterpret_cast<u32x4a*>(a.streams);
  for (uint64_t i = t0; i < n4; i += stride) d4[i] = s4[i];
  if (a.src_strip0)
    for (uint64_t i = t0; i <= a.nstreams; i += stride) a.strip0[i] = a.src_strip0[i];
  for (uint64_t i = t0; i < a.nzero0; i += stride) a.zero0[i] = 0u;
  for (uint64_t i = t0; i < a.nzero1; i += stride) a.zero1[i] = 0u;
  for (uint64_t i = t0; i < a.nzero2; i += stride) a.zero2[i] = 0u;
  for (uint64_t i = t0; i < a.nzero3; i += stride) a.zero3[i] = 0u;
  for (uint64_t s = t0; s < a.nstreams; s += stride) {
    a.last_end[s] = a.src[s].open_start;
    a.scount[s] = 0;
    a.carry[s].valid = 0;
  }
}

// ---------------------------------------------------------------------------------------------
// Batched variable-length SHA-256 (FIPS 180-4). One lane = one chunk at a time; lanes pull
// jobs from a device queue as they finish, so a wave stays full whatever the length mix.
// Jobs [0, M) are finished chunks; jobs [M, M + nstreams) are the open chunks of non-final
// segments (hash whole blocks only, export the midstate).
// Job info from k_lens (jinfo): nblocks | eligible << 31; kNoJob for ids without a job.
constexpr uint32_t kNoJob = 0xffffffffu;
constexpr uint32_t kJobElig = 0x80000000u;

struct ShaJob {
  uint64_t id;          // job index
  uint64_t start, end;  // stream offsets [start, end)
  const uint8_t* dbase; // first data byte of this launch's part of the message
  const uint8_t* hist;  // prefix bytes (the open chunk's unhashed head), prefix_len of them
  uint64_t L;           // message bytes available this launch (prefix + data)
  uint64_t consumed;    // bytes already folded into the init state
  uint32_t prefix;
  uint32_t nblocks;
  uint32_t fin;
  uint32_t level;
  uint32_t stream;
};

__device__ bool sha_setup(const ShaArgs& a, uint64_t j, uint64_t M, ShaJob& jb,
                          uint32_t (&st)[8]) {
  uint32_t s;
  if (j < M) {
    const uint64_t info = a.bnd_info[j];
    s = (uint32_t)(info >> 32);
    jb.level = (uint32_t)info;
    jb.end = a.bnd_end[j];
    const StreamDesc* sd = a.streams + s;
    jb.start = (j > 0 && (uint32_t)(a.bnd_info[j - 1] >> 32) == s) ? a.bnd_end[j - 1]
                                                                  : sd->open_start;
    jb.fin = 1;
  } else {
    s = (uint32_t)(j - M);
    const StreamDesc* sd = a.streams + s;
    if (sd->finalize) return false;
    jb.start = a.last_end[s];
    jb.end = sd->seg_base + sd->len;
    // a short open chunk is carried to the next segment as bytes, not as a midstate
    if (jb.end - jb.start <= sd->carry_cap) return false;
    jb.level = 0;
    jb.fin = 0;
  }
  const StreamDesc* sd = a.streams + s;
  jb.id = j;
  jb.stream = s;
  int64_t dstart;  // negative: the open chunk's head precedes the segment in device memory
  if (jb.start < sd->seg_base && !(sd->flags & kDescOpenInDevice)) {
    // continues the open chunk of the previous segment from its midstate
    jb.prefix = sd->prefix_len;
    jb.consumed = sd->consumed;
#pragma unroll
    for (int i = 0; i < 8; ++i) st[i] = sd->mid[i];
    dstart = 0;
  } else {
    jb.prefix = 0;
    jb.consumed = 0;
    st[0] = 0x6a09e667; st[1] = 0xbb67ae85; st[2] = 0x3c6ef372; st[3] = 0xa54ff53a;
    st[4] = 0x510e527f; st[5] = 0x9b05688c; st[6] = 0x1f83d9ab; st[7] = 0x5be0cd19;
    dstart = (int64_t)jb.start - (int64_t)sd->seg_base;
  }
  jb.dbase = a.data + (int64_t)sd->data_off + dstart;
  jb.hist = sd->hist + 64 - jb.prefix;
  if (jb.end < jb.start || jb.end > sd->seg_base + sd->len || jb.start < sd->open_start) {
    atomicOr(reinterpret_cast<unsigned long long*>(&a.ctr->error), 2ull);  // bug guard
    return false;
  }
  jb.L = jb.prefix + (uint64_t)((int64_t)(jb.end - sd->seg_base) - dstart);
  jb.nblocks = jb.fin ? (uint32_t)((jb.L + 8) / 64 + 1) : (uint32_t)(jb.L / 64);
  return true;
}

// Raw (unaligned) 64-byte block: 17 aligned dwords + a v_perm_b32 selector that both realigns
// and byte-swaps, plus the number of valid message bytes in the block (<64 only at a chunk's
// end). Issued one block ahead so the load latency hides under the compression.
struct RawBlock {
  uint32_t r[17];
  uint32_t sel;
  int32_t valid;  // message bytes of this block that are data: 64 (full), 0..63 (tail), -1 (pad)
};

typedef __attribute__((address_space(1))) const uint32_t gu32;
typedef __attribute__((address_space(1))) const u32x4 gu32x4;

// Block at message offset o0 (>= prefix) of a job whose data bytes are dbase[o - prefix].
// Branch-free on purpose (the same five loads into the same registers every time, so the
// compiler never drains a prefetch at a control-flow join) and wide (4 x dwordx4 + 1 dword:
// every load instruction touches one cache line per lane, so fewer instructions = less
// TA/L1 work when four waves share a CU). Reads may run up to kReadSlack bytes past the end of
// the data; the engine requires that much readable memory after every stream
// (bsg_engine_run checks the allocation), and pad_words masks whatever is read there.
__device__ __forceinline__ void raw_load(const uint8_t* dbase, uint64_t o0, uint32_t prefix,
                                         uint64_t L, RawBlock& rb) {
  const uint8_t* p = dbase + (o0 - prefix);
  const int64_t vv = (int64_t)L - (int64_t)o0;
  rb.valid = vv < 0 ? -1 : (vv >= 64 ? 64 : (int32_t)vv);
  const uintptr_t addr = reinterpret_cast<uintptr_t>(p);
  const uint32_t sh = (uint32_t)(addr & 3u);
  gu32* al = reinterpret_cast<gu32*>(addr & ~(uintptr_t)3);
  rb.sel = (sh << 24) | ((sh + 1) << 16) | ((sh + 2) << 8) | (sh + 3);
  gu32x4* q = reinterpret_cast<gu32x4*>(al);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const u32x4 x = q[i];
    rb.r[4 * i] = x.x; rb.r[4 * i + 1] = x.y; rb.r[4 * i + 2] = x.z; rb.r[4 * i + 3] = x.w;
  }
  rb.r[16] = al[16];
}

// N consecutive blocks from p (message offset o0 of a job of L message bytes): one aligned base
// and one selector for all of them (p + 64 b keeps p's low two bits), the blocks at immediate
// offsets of that base (per-lane mode, round 5: the address and selector math ran once per
// block before; sel = the low two bits replicated into every byte by one v_perm, + 0x00010203).
template <int N>
__device__ __forceinline__ void raw_load_n(const uint8_t* p, uint64_t o0, uint64_t L,
                                           RawBlock (&rb)[N]) {
  const uintptr_t addr = reinterpret_cast<uintptr_t>(p);
  const uint32_t sh = (uint32_t)(addr & 3u);
  const uint32_t sel = __builtin_amdgcn_perm(0u, sh, 0u) + 0x00010203u;
  gu32* al = reinterpret_cast<gu32*>(addr & ~(uintptr_t)3);
#pragma unroll
  for (int b = 0; b < N; ++b) {
    const int64_t vv = (int64_t)L - (int64_t)(o0 + 64ull * b);
    rb[b].valid = vv < 0 ? -1 : (vv >= 64 ? 64 : (int32_t)vv);
    rb[b].sel = sel;
    gu32x4* q = reinterpret_cast<gu32x4*>(al + 16 * b);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const u32x4 x = q[i];
      rb[b].r[4 * i] = x.x; rb[b].r[4 * i + 1] = x.y; rb[b].r[4 * i + 2] = x.z; rb[b].r[4 * i + 3] = x.w;
    }
    rb[b].r[16] = al[16 * b + 16];
  }
}

__device__ __forceinline__ void raw_to_words(const RawBlock& rb, uint32_t (&W)[16]) {
#pragma unroll
  for (int i = 0; i < 16; ++i) W[i] = __builtin_amdgcn_perm(rb.r[i + 1], rb.r[i], rb.sel);
}

// Tail block: keep the valid bytes, append 0x80, zero the rest (FIPS 180-4 §5.1.1).
__device__ __forceinline__ void pad_words(int32_t valid, uint32_t (&W)[16]) {
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int32_t k = valid - 4 * q;  // valid bytes in word q
    const uint32_t keep = k >= 4 ? 0xffffffffu : (k <= 0 ? 0u : (0xffffffffu << (32 - 8 * k)));
    const uint32_t pad = (k >= 0 && k < 4) ? (0x80u << (24 - 8 * k)) : 0u;
    W[q] = (W[q] & keep) | pad;
  }
}

__device__ __forceinline__ void sha_load_slow(const ShaJob& jb, uint32_t blk, uint32_t (&W)[16]) {
  const uint64_t o0 = 64ull * blk;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    uint32_t word = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint64_t o = o0 + 4 * q + r;
      uint32_t byte;
      if (o < jb.prefix) byte = jb.hist[o];
      else if (o < jb.L) byte = jb.dbase[o - jb.prefix];
      else byte = (o == jb.L) ? 0x80u : 0u;
      word = (word << 8) | byte;
    }
    W[q] = word;
  }
  if (jb.fin && blk + 1 == jb.nblocks) {
    const uint64_t bits = (jb.consumed + jb.L) * 8ull;
    W[14] = (uint32_t)(bits >> 32);
    W[15] = (uint32_t)bits;
  }
}

__device__ void sha_finish(const ShaArgs& a, const ShaJob& jb, const uint32_t (&st)[8]) {
  if (jb.fin) {
    ChunkRec* r = a.out + jb.id;
    r->offset = jb.start;
    r->len = jb.end - jb.start;
    r->level = jb.level;
    r->stream = jb.stream;
    uint32_t* ref = reinterpret_cast<uint32_t*>(r->ref);
#pragma unroll
    for (int i = 0; i < 8; ++i) ref[i] = __builtin_bswap32(st[i]);
  } else {
    CarryOut* co = a.carry + jb.stream;
#pragma unroll
    for (int i = 0; i < 8; ++i) co->mid[i] = st[i];
    co->consumed = jb.consumed + 64ull * jb.nblocks;
    co->open_start = jb.start;
    co->prefix_len = (uint32_t)(jb.L & 63u);
    co->valid = 1;
  }
}

#ifndef BSG_LANE_LEAD
#define BSG_LANE_LEAD 4  // iterations before a job's end at which its successor is popped
#endif
// Blocks per per-lane iteration: the job-switch and queue logic runs once per this many
// compressions (3 and 4 measured slower, round 5).
constexpr int kLaneBPI = 2;

// Tail block, cheaper form for the per-lane loop: words before the one holding byte `valid`
// stay, that word keeps its valid bytes and gets the 0x80, later words are zero (valid -1: a
// block of padding only).
__device__ __forceinline__ void pad_words_lane(int32_t valid, uint32_t (&W)[16]) {
  const int32_t q0 = valid >> 2;  // arithmetic: -1 for valid == -1
  const uint32_t b = 8u * ((uint32_t)valid & 3u);
  const uint32_t keep = ~(0xffffffffu >> b), pad = 0x80000000u >> b;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const uint32_t t = (W[q] & keep) | pad;
    W[q] = q < q0 ? W[q] : (q == q0 ? t : 0u);
  }
}

// The message words of block `blk` of the current job (rb holds it, prefetched). Idle lanes
// (act false) skip the tail handling: their rb is a past-the-end block, and taking the tail
// branch for them would run it for the whole wave in nearly every iteration.
// Per-lane mode's rare per-lane branches (a job's head or tail block, a job's end, a job switch,
// the pipeline steps, the record store) sit behind a wave-uniform test (a ballot), so the common
// iteration, where no lane takes them, runs no exec-mask bookkeeping for them: without it the
// loop issued 46 SALU and 11 branches per block (round 5, profiles/r05_lane_mix.json).
#define LANE_ANY(cond) (__ballot(cond))

__device__ __forceinline__ void lane_words(const ShaJob& jb, uint32_t blk, const RawBlock& rb,
                                           bool act, uint32_t (&W)[16]) {
  raw_to_words(rb, W);
  const bool slow = 64ull * blk < jb.prefix;
  const bool tail = act && rb.valid < 64;
  if (__ballot(slow || tail)) {
    if (slow) {
      sha_load_slow(jb, blk, W);  // head block of a continued chunk (once per segment)
    } else if (tail) {
      pad_words_lane(rb.valid, W);
      if (jb.fin && blk + 1 == jb.nblocks) {
        const uint64_t bits = (jb.consumed + jb.L) * 8ull;
        W[14] = (uint32_t)(bits >> 32);
        W[15] = (uint32_t)bits;
      }
    }
  }
}

// A region's pop counter: the jobs taken from it so far (longest first) in its low word, a
// region holding fewer than 2^32 jobs; the high word stays zero (round 5 counted jobs taken from
// the region's tail there, for an experiment since dropped), and is kept in the test below and in
// sha_lane_mode's pop: without it the per-lane loop compiled to a different layout and ran 3 %
// slower per block (6,400-6,500 against 6,290 cycles, profiles/r06_c3_c2_*.log).
// Returns hd, or n when no job is left (the jobs left are rorder[off + hd .. off + n)).
__device__ __forceinline__ uint64_t reg_head(const ShaArgs& a, uint32_t r, uint64_t n) {
  const uint64_t v = __hip_atomic_load(&a.reg->head[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t hd = (uint32_t)v, hi = v >> 32;
  return hd + hi < n ? hd : n;
}

// The region whose next job is the longest (longest-first across regions, so the last jobs
// anywhere are short ones; ties: the first from `start` on), or R if every region is empty.
// Called by a whole wave (some lanes may have left per-lane mode already); three dependent
// loads per region, a few times per wave. (Picking the region with the most jobs left instead
// ended configs[2]'s per-lane mode 2.3 ms after the median wave: regions left with few but
// long jobs were found last.)
__device__ uint32_t pick_region(const ShaArgs& a, uint32_t R, uint32_t start) {
  const uint64_t act = __ballot(1);
  const uint32_t nact = (uint32_t)__popcll(act);
  const uint32_t rank =
      __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
  start %= R;
  uint64_t key = 0;
  for (uint32_t r = rank; r < R; r += nact) {
    const uint64_t o = a.reg->off[r], n = a.reg->off[r + 1] - o;
    const uint64_t h = reg_head(a, r, n);
    if (h < n) {
      const uint32_t len = (a.jinfo[a.rorder[o + h]] & ~kJobElig) + 1u;
      const uint64_t dist = (r + R - start) % R;
      const uint64_t k = ((uint64_t)len << 8) | (255u - dist);
      key = k > key ? k : key;
    }
  }
  uint64_t best = 0;
  for (uint64_t m = act; m; m &= m - 1) {  // max over the active lanes
    const int l = (int)__builtin_ctzll(m);
    const uint64_t v =
        ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(key >> 32), l) << 32) |
        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)key, l);
    best = v > best ? v : best;
  }
  return best ? (uint32_t)((start + 255u - (uint32_t)(best & 255u)) % R) : R;
}

#ifndef BSG_REGION_POLL
#define BSG_REGION_POLL 8      // a wave compares its region's progress with the others' every
#endif                         // this many pops (0: only when its region runs dry)
#ifndef BSG_REGION_LEN_LAG
#define BSG_REGION_LEN_LAG 25  // ... moving if another region's next job is this many % longer
#endif
// The region whose next job is the longest, if that job is more than BSG_REGION_LEN_LAG % longer
// than `cur`'s next one, else `cur`. Regions are drained longest first, so this keeps the waves
// close to one global longest-first order, and the per-lane waves end together: on configs[2]
// the poll by share taken let them end over ~0.35 ms, the last ones ~0.18 ms after the longest
// chain; by length they end with it (+1 %, profiles/r04_region_len_ab.log).
__device__ uint32_t longer_region(const ShaArgs& a, uint32_t R, uint32_t cur) {
  const uint64_t act = __ballot(1);
  const uint32_t nact = (uint32_t)__popcll(act);
  const uint32_t rank =
      __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
  uint64_t key = 0;   // next job's blocks << 8 | (255 - distance from cur)
  uint32_t mine = 0;  // cur's next job's blocks (0: dry), on the lane that read it
  bool has_mine = false;
  for (uint32_t r = rank; r < R; r += nact) {
    const uint64_t o = a.reg->off[r], n = a.reg->off[r + 1] - o;
    const uint64_t h = reg_head(a, r, n);
    uint32_t len = 0;
    if (h < n) len = (a.jinfo[a.rorder[o + h]] & ~kJobElig) + 1u;
    if (r == cur) {
      mine = len;
      has_mine = true;
    }
    if (len) {
      const uint64_t k = ((uint64_t)len << 8) | (255u - (r + R - cur) % R);
      key = k > key ? k : key;
    }
  }
  uint64_t best = 0;
  uint32_t cur_len = 0;
  for (uint64_t m = act; m; m &= m - 1) {
    const int l = (int)__builtin_ctzll(m);
    const uint64_t v =
        ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(key >> 32), l) << 32) |
        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)key, l);
    best = v > best ? v : best;
    if (__builtin_amdgcn_readlane((int)has_mine, l)) cur_len = (uint32_t)__builtin_amdgcn_readlane((int)mine, l);
  }
  if (!best) return cur;
  const uint64_t best_len = best >> 8;
  if (best_len * 100 <= (uint64_t)cur_len * (100 + BSG_REGION_LEN_LAG)) return cur;
  return (cur + 255u - (uint32_t)(best & 255u)) % R;
}

// Per-lane mode: each lane hashes one chunk at a time, longest first within the address region
// its wave works on (Regions). An iteration hashes kLaneBPI blocks per lane. Starting the
// next job is pipelined per lane, one memory step per iteration, so no iteration waits for
// more than what the one before issued:
//   BSG_LANE_LEAD iterations before its job ends a lane pops a slot of its wave's region
//   (one atomic per wave) -> loads the job id (rorder) -> loads its LaneJob (k_lens) -> in its
//   last iteration prefetches the new job's first blocks instead of past-the-end ones and
//   switches jobs in registers; the finished job's record is stored one iteration later.
// The loop waits once per iteration, at its top, for everything the previous one issued (a
// whole compression earlier). Round 2 first popped and set up the next job only when the last
// one ended, and the whole wave waited for that atomic and ~4 dependent loads whenever any
// lane switched. A job too short for the pipeline idles only its own lane until its successor
// is ready; continued and open chunks (streaming) still take the synchronous sha_setup path.
// The compressions are one generated asm statement (sha256_compress_kv, sha256_lane_asm.inc)
// with K in 64 resident VGPRs: k_sha runs one wave per SIMD, so it has VGPRs to spare.
__device__ void sha_lane_mode(const ShaArgs& a, uint64_t M) {
  constexpr int kBPI = kLaneBPI;  // blocks per iteration (per lane)
  const uint32_t lane = threadIdx.x & 63u;
  ShaJob jb;
  jb.dbase = a.data;  // a readable address for the idle prefetch before the first job
  jb.L = 0;
  jb.prefix = 0;
  jb.consumed = 0;
  jb.nblocks = 0;
  jb.fin = 1;
  uint32_t st[8] = {};
  uint32_t kv[64];  // K, resident for the whole loop
  sha256_k_regs(kv);
  RawBlock rb[kBPI];
#pragma unroll
  for (int b = 0; b < kBPI; ++b) {
#pragma unroll
    for (int i = 0; i < 17; ++i) rb[b].r[i] = 0;
    rb[b].sel = 0;
    rb[b].valid = 0;
  }
  bool act = false;
  uint32_t blk = 0;
  // next-job pipeline: 0 nothing, 1 slot popped (q next iteration), 2 job id loading (nj),
  // 5 descriptor loading (ldn, job nj_d), 3 descriptor ready (ld, job ld_id), 4 queue exhausted
  uint32_t stage = 0;
  uint64_t q = 0, nj = 0, nj_d = 0, ld_id = 0;
  // the descriptor as two 16-byte vectors (a struct got its words shuffled right after the
  // load, which made the whole wave wait for it)
  u32x4 ld0 = {0, 0, 0, 0}, ld1 = {0, 0, 0, 0}, ldn0 = ld0, ldn1 = ld0;
  // a pop is one atomic per wave (the first active lane's); its result stays in that lane's
  // register until the next iteration, where each popping lane adds its rank
  uint64_t pop_base = 0;
  uint32_t pop_leader = 0, pop_rank = 0;
  // the record of the last job that ended, stored in the next iteration
  bool pend = false;
  uint64_t p_id = 0, p_start = 0, p_len = 0;
  uint32_t p_level = 0, p_stream = 0, pst[8] = {};
  uint64_t tm0 = 0, tr0 = 0;
  bool stamp = false;
  // The wave's region (wave-uniform): its workgroup's (= its CU's) first, then, whenever it
  // runs dry, the one whose next job is the longest. pop_off / pop_n: the last pop's region.
  const uint32_t R = (uint32_t)a.reg->nregions;
  uint32_t reg = blockIdx.x % R;
  uint64_t reg_off = a.reg->off[reg], reg_n = a.reg->off[reg + 1] - reg_off;
  uint64_t pop_off = reg_off, pop_n = reg_n;
  bool all_done = false;
  uint32_t npops = 0;     // pops by this wave (wave-uniform)
  bool poll = false;
  for (;;) {
    // Everything the last iteration issued (block prefetch, pipeline loads, the pop, the
    // record store) has had a whole compression to land: wait for all of it here, once, so
    // the compiler needs no wait further down.
    __builtin_amdgcn_s_waitcnt(0xF70);  // vmcnt(0)
    uint32_t W[kBPI][16];
#pragma unroll
    for (int b = 0; b < kBPI; ++b)  // garbage on idle lanes and past a job's end (never used)
      lane_words(jb, blk + b, rb[b], act && blk + b < jb.nblocks, W[b]);
    // pipeline steps whose loads landed (the wait above): 5 -> 3, 2 -> 5, 1 -> 2 / 0
    bool dry = false;
    if (LANE_ANY(stage == 5 || stage == 2 || stage == 1)) {
    if (stage == 5) {
      ld0 = ldn0;
      ld1 = ldn1;
      ld_id = nj_d;
      stage = 3;
    } else if (stage == 2) {
      nj_d = nj;  // its descriptor is loaded below
      stage = 5;
    } else if (stage == 1) {
      // the region's pop count before this pop (reg_head: low word; the high word is zero)
      const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)pop_base, pop_leader);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(pop_base >> 32), pop_leader);
      const uint64_t local = (uint64_t)lo + pop_rank;
      dry = local + hi >= pop_n;
      q = pop_off + local;
      stage = dry ? 0u : 2u;  // its job id is loaded below; else the region ran dry
    }
    }
    if (__ballot(dry) && !all_done && pop_off == reg_off) {
      // the current region ran dry: move to the one with the most jobs left (wave-uniform,
      // synchronous; a few times per wave)
      reg = pick_region(a, R, reg + 1);
      if (reg >= R) {
        all_done = true;
      } else {
        reg_off = a.reg->off[reg];
        reg_n = a.reg->off[reg + 1] - reg_off;
      }
    }
    if (BSG_REGION_POLL && poll && !all_done && R > 1) {
      // keep the waves on one global longest-first order: move to the region whose next job is
      // well longer than this one's
      poll = false;
      const uint32_t r2 = longer_region(a, R, reg);
      if (r2 != reg) {
        reg = r2;
        reg_off = a.reg->off[reg];
        reg_n = a.reg->off[reg + 1] - reg_off;
      }
    }
    const bool ld_ready = stage == 3;
    bool need = stage == 0 && (!act || blk + kBPI * BSG_LANE_LEAD >= jb.nblocks);
    if (all_done) {  // every region is empty: lanes wanting a job are done
      if (need) stage = 4;
      need = false;
    }
    // The two lookups run on every lane, every iteration (lanes with nothing to look up
    // re-read entry 0 or their last one): a load under a per-lane condition into a
    // loop-carried value made hipcc merge the old and the new value by register copies that
    // waited for the load at once.
    {
      const gu32x4* pd = reinterpret_cast<const gu32x4*>(reinterpret_cast<uintptr_t>(a.jdesc + nj_d));
      ldn0 = pd[0];
      ldn1 = pd[1];
      nj = a.rorder[stage == 2 ? q : 0ull];
    }
    const uint64_t nm = __ballot(need);
    if (nm) {  // wave-uniform
      const uint32_t leader = __builtin_amdgcn_readfirstlane(lane);
      if (lane == leader) {
        // an address the compiler cannot prove uniform, so that its atomic optimiser leaves
        // this one-lane atomic alone (it would broadcast the result at once, i.e. wait for it)
        uint32_t z;
        asm volatile("v_mov_b32 %0, 0" : "=v"(z));
        pop_base = atomicAdd(reinterpret_cast<unsigned long long*>(&a.reg->head[reg]) + z,
                             (unsigned long long)__popcll(nm));
      }
      pop_leader = leader;
      pop_off = reg_off;
      pop_n = reg_n;
      if (BSG_REGION_POLL && ++npops % (BSG_REGION_POLL ? BSG_REGION_POLL : 1) == 0) poll = true;
      if (need) {
        pop_rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(nm >> 32),
                                             __builtin_amdgcn_mbcnt_lo((uint32_t)nm, 0u));
        stage = 1;
      }
    }
    if (LANE_ANY(pend) && pend) {
      ChunkRec* r = a.out + p_id;
      r->offset = p_start;
      r->len = p_len;
      r->level = p_level;
      r->stream = p_stream;
      uint32_t* ref = reinterpret_cast<uint32_t*>(r->ref);
#pragma unroll
      for (int i = 0; i < 8; ++i) ref[i] = __builtin_bswap32(pst[i]);
      pend = false;
    }
    // prefetch: the current job's next blocks, or in its last iteration (or when idle) the
    // next job's first ones; otherwise past-the-end blocks (slack, never used)
    const bool cont = act && blk + kBPI < jb.nblocks;
    // LaneJob words: dptr (0, 1), start (2, 3), len (4, 5), stream (6), meta (7)
    const uint64_t ld_dptr = ((uint64_t)ld0.y << 32) | ld0.x;
    const uint64_t ld_start = ((uint64_t)ld0.w << 32) | ld0.z;
    const uint64_t ld_len = ((uint64_t)ld1.y << 32) | ld1.x;
    const bool take = !cont && ld_ready && !(ld1.w & kLaneJobSlow);
    {  // both blocks of the iteration from one aligned base and byte selector (raw_load_n)
      const uint64_t o0 = take ? 0ull : 64ull * (blk + kBPI);
      const uint8_t* p0 = take ? reinterpret_cast<const uint8_t*>(ld_dptr)
                               : jb.dbase + (o0 - jb.prefix);
      raw_load_n<kBPI>(p0, o0, take ? ld_len : jb.L, rb);
    }
#pragma unroll
    for (int b = 0; b < kBPI; ++b)
      if (act && blk + b < jb.nblocks) sha256_compress_kv(st, W[b], kv);
    blk += kBPI;
    if (LANE_ANY(act && blk >= jb.nblocks) && act && blk >= jb.nblocks) {
      act = false;
      if (jb.fin) {
        pend = true;
        p_id = jb.id;
        p_start = jb.start;
        p_len = jb.end - jb.start;
        p_level = jb.level;
        p_stream = jb.stream;
#pragma unroll
        for (int i = 0; i < 8; ++i) pst[i] = st[i];
      } else {
        sha_finish(a, jb, st);  // open chunk: midstate carry (streaming, one per stream)
      }
      if (stamp) {
        a.ctr->diag2[1] = __builtin_amdgcn_s_memtime();
        a.ctr->diag2[3] = __builtin_amdgcn_s_memrealtime();
        a.ctr->diag2[0] = tm0;
        a.ctr->diag2[2] = tr0;
        a.ctr->diag2[4] = jb.nblocks;
        stamp = false;
      }
    }
    if (LANE_ANY(!act) && !act) {
      if (take) {  // its first block is on its way into rb
        jb.id = ld_id;
        jb.start = ld_start;
        jb.end = ld_start + ld_len;
        jb.dbase = reinterpret_cast<const uint8_t*>(ld_dptr);
        jb.L = ld_len;
        jb.consumed = 0;
        jb.prefix = 0;
        jb.fin = 1;
        jb.level = ld1.w & ~kLaneJobSlow;
        jb.stream = ld1.z;
        jb.nblocks = (uint32_t)((ld_len + 8) / 64 + 1);
        st[0] = 0x6a09e667; st[1] = 0xbb67ae85; st[2] = 0x3c6ef372; st[3] = 0xa54ff53a;
        st[4] = 0x510e527f; st[5] = 0x9b05688c; st[6] = 0x1f83d9ab; st[7] = 0x5be0cd19;
        blk = 0;
        act = true;
        stage = 0;
        stamp = (q == 0);  // diagnostic timing of region 0's longest per-lane job
        if (stamp) {
          tm0 = __builtin_amdgcn_s_memtime();
          tr0 = __builtin_amdgcn_s_memrealtime();
        }
      } else if (ld_ready) {  // continued or open chunk: the full setup, synchronously (rare)
        stage = 0;
        if (sha_setup(a, ld_id, M, jb, st)) {
          blk = 0;
          if (jb.nblocks == 0) {
            sha_finish(a, jb, st);
          } else {
            act = true;
#pragma unroll
            for (int b = 0; b < kBPI; ++b)  // block 0 of a continued chunk: sha_load_slow
              if (64u * b >= jb.prefix) raw_load(jb.dbase, 64ull * b, jb.prefix, jb.L, rb[b]);
          }
        }
      } else if (stage == 4 && !pend) {
        break;
      }
    }
  }
}


// ---------------------------------------------------------------------------------------------
// Wave-per-chunk path for the longest chunks. A SHA-256 chain is serial, so a batch's wall time
// is its longest chunk's chain; a lone lane of a mostly finished wave issues at ~5.2 cycles per
// VALU op, a full wave at ~4.1. Here one 64-lane wave owns one long chunk: all lanes build the
// message schedule (K+W) of 64 consecutive blocks at once into an LDS ring, then the wave runs
// the 64 rounds of each block uniformly (~14 VALU per round) reading K+W by broadcast
// ds_read_b128. Jobs with >= long_thresh blocks (max(1024, longest/2)) take this path.
// ---------------------------------------------------------------------------------------------
// Job ordering: long jobs -> long_list; the rest counting-sorted on nblocks, longest first
// (LPT), so the lanes of one wave hold chunks of similar length and finish together.
__device__ __forceinline__ uint32_t lpt_bucket(const Counters* ctr, uint32_t nblocks) {
  const uint64_t mx = ctr->max_nblocks;
  const uint64_t d = mx > nblocks ? mx - nblocks : 0;
  const uint64_t b = d / ctr->bucket_width;
  return b < (uint64_t)kLptBuckets ? (uint32_t)b : (uint32_t)(kLptBuckets - 1);
}

// Region (0 .. R-1) of a per-lane job by the address of its first data byte.
__device__ __forceinline__ uint32_t job_region(const ShaArgs& a, uint64_t dptr, uint32_t R) {
  const int64_t o = (int64_t)(dptr - reinterpret_cast<uint64_t>(a.data));
  if (o <= 0 || R <= 1) return 0;
  const uint64_t r = ((uint64_t)o * R) / (a.span ? a.span : 1);
  return r < R ? (uint32_t)r : R - 1;
}


// Counting sort of the jobs on their LPT bucket, aggregated in LDS: pass 1 (SCATTER = false)
// counts jobs (and wave-eligible jobs) per bucket, one global atomic per non-empty bucket per
// workgroup; pass 2 gives each job its slot — a rank within its workgroup's bucket from an LDS
// atomic plus the workgroup's base, reserved with one global atomic per non-empty bucket — in
// the long list (eligible, bucket < long_buckets) or the per-lane order. Round 1 ran
// sha_setup for every job in both passes and one same-address global atomic per job (92 and
// 94 us on configs[2], 258 K jobs).
template <bool SCATTER>
__global__ __launch_bounds__(256) void k_order(ShaArgs a) {
  __shared__ uint32_t h0[kLptBuckets], h1[kLptBuckets];  // counts / ranks (all | eligible)
  if (a.ctr->overflow || a.ctr->error) return;
  const uint64_t M = a.ctr->nchunks;
  if (M > a.chunk_cap) return;
  const uint64_t njobs = M + a.nstreams;
  const uint64_t nlb = a.ctr->long_buckets;  // valid in the SCATTER pass
  for (uint64_t tile = (uint64_t)blockIdx.x * blockDim.x; tile < njobs;
       tile += (uint64_t)gridDim.x * blockDim.x) {
    for (uint32_t i = threadIdx.x; i < (uint32_t)kLptBuckets; i += blockDim.x) h0[i] = h1[i] = 0;
    __syncthreads();
    const uint64_t j = tile + threadIdx.x;
    const uint32_t info = j < njobs ? a.jinfo[j] : kNoJob;
    uint32_t b = 0, rank = 0;
    bool is_long = false;
    if (info != kNoJob) {
      b = lpt_bucket(a.ctr, info & ~kJobElig);
      const bool elig = (info & kJobElig) != 0;
      if (!SCATTER) {
        atomicAdd(&h0[b], 1u);
        if (elig) atomicAdd(&h1[b], 1u);
      } else {
        is_long = elig && b < nlb;
        rank = atomicAdd(is_long ? &h1[b] : &h0[b], 1u);
      }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < (uint32_t)kLptBuckets; i += blockDim.x) {
      const uint32_t c0 = h0[i], c1 = h1[i];
      if (!SCATTER) {
        if (c0) atomicAdd(a.bucket_cnt + i, c0);
        if (c1) atomicAdd(a.bucket_elig + i, c1);
      } else {  // the workgroup's base in each bucket replaces its count
        if (c0) h0[i] = atomicAdd(a.bucket_off + i, c0);
        if (c1) h1[i] = atomicAdd(a.bucket_loff + i, c1);
      }
    }
    __syncthreads();
    if (SCATTER && info != kNoJob) {
      if (is_long) {
        a.long_list[h1[b] + rank] = j;
      } else {
        a.order[h0[b] + rank] = j;
        if (a.span > kRegionBytes)
          a.oreg[h0[b] + rank] = (uint8_t)job_region(a, a.jdesc[j].dptr, (uint32_t)a.reg->nregions);
      }
    }
    __syncthreads();
  }
}

// Exclusive scan of 4 values per thread over a 1024-thread block; returns the total.
__device__ __forceinline__ uint32_t block_scan4(uint32_t (&v)[4], uint32_t (&pre)[4],
                                                uint32_t* wsum) {
  const uint32_t t = threadIdx.x;
  const uint32_t sum = v[0] + v[1] + v[2] + v[3];
  uint32_t x = sum;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if ((t & 63) >= (uint32_t)o) x += y;
  }
  __syncthreads();
  if ((t & 63) == 63) wsum[t >> 6] = x;
  __syncthreads();
  uint32_t p = 0, total = 0;
  for (uint32_t w = 0; w < 16; ++w) {
    if (w < (t >> 6)) p += wsum[w];
    total += wsum[w];
  }
  p += x - sum;
#pragma unroll
  for (int i = 0; i < 4; ++i) { pre[i] = p; p += v[i]; }
  return total;
}

// ---- per-lane jobs regrouped by region, longest first within each (see Regions) ----------
// The LPT order (a.order, nshort jobs) is cut into kRegionSegs segments; k_rcount counts each
// segment's jobs per region, k_rscan turns the counts into each segment's offset within its
// region, k_rtotal lays the regions out, and k_rscatter moves every job to
// rorder[off[region] + its segment's offset + its rank], walking its segment in order, so each
// region keeps the LPT order (up to the order inside one 256-job tile).
__device__ __forceinline__ uint64_t seg_len(uint64_t n) {
  return (n + kRegionSegs - 1) / kRegionSegs;
}

__global__ __launch_bounds__(256) void k_rcount(ShaArgs a) {
  __shared__ uint32_t hist[kMaxRegions];
  if (a.ctr->overflow || a.ctr->error || a.ctr->nchunks > a.chunk_cap) return;
  const uint64_t n = a.ctr->nshort, L = seg_len(n);
  const uint32_t t = threadIdx.x;
  hist[t] = 0;
  __syncthreads();
  const uint64_t lo = blockIdx.x * L, hi = min(n, lo + L);
  for (uint64_t i = lo + t; i < hi; i += 256) atomicAdd(&hist[a.oreg[i]], 1u);
  __syncthreads();
  a.reg->cnt[blockIdx.x * kMaxRegions + t] = hist[t];
}

__global__ __launch_bounds__(kRegionSegs) void k_rscan(ShaArgs a) {
  __shared__ uint32_t wsum[kRegionSegs / 64];
  if (a.ctr->overflow || a.ctr->error || a.ctr->nchunks > a.chunk_cap) return;
  const uint32_t r = blockIdx.x, t = threadIdx.x;  // region r, segment t
  if (r >= a.reg->nregions) return;
  uint32_t* c = a.reg->cnt + t * kMaxRegions + r;
  const uint32_t v = *c;
  uint32_t x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if ((t & 63) >= (uint32_t)o) x += y;
  }
  if ((t & 63) == 63) wsum[t >> 6] = x;
  __syncthreads();
  uint32_t base = 0, tot = 0;
  for (uint32_t w = 0; w < kRegionSegs / 64; ++w) {
    if (w < (t >> 6)) base += wsum[w];
    tot += wsum[w];
  }
  *c = base + x - v;  // exclusive: segment t's offset within region r
  if (t == 0) a.reg->head[r] = tot;  // the region's size, until k_rtotal
}

__global__ __launch_bounds__(kMaxRegions) void k_rtotal(ShaArgs a) {
  __shared__ uint64_t wsum[kMaxRegions / 64];
  if (a.ctr->overflow || a.ctr->error || a.ctr->nchunks > a.chunk_cap) return;
  const uint32_t t = threadIdx.x;
  const uint32_t R = (uint32_t)a.reg->nregions;
  const uint64_t v = t < R ? a.reg->head[t] : 0;
  uint64_t x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(x, o);
    if ((t & 63) >= (uint32_t)o) x += y;
  }
  if ((t & 63) == 63) wsum[t >> 6] = x;
  __syncthreads();
  uint64_t base = 0;
  for (uint32_t w = 0; w < (t >> 6); ++w) base += wsum[w];
  __syncthreads();
  a.reg->off[t] = t < R ? base + x - v : a.ctr->nshort;
  if (t == 0) {
    a.reg->off[kMaxRegions] = a.ctr->nshort;
    a.reg->rr = 0;
  }
  a.reg->head[t] = 0;
}

__global__ __launch_bounds__(256) void k_rscatter(ShaArgs a) {
  __shared__ uint64_t base[kMaxRegions];
  __shared__ uint32_t tc[kMaxRegions];
  if (a.ctr->overflow || a.ctr->error || a.ctr->nchunks > a.chunk_cap) return;
  const uint64_t n = a.ctr->nshort, L = seg_len(n);
  const uint32_t t = threadIdx.x;
  base[t] = a.reg->off[t] + a.reg->cnt[blockIdx.x * kMaxRegions + t];
  tc[t] = 0;
  __syncthreads();
  const uint64_t lo = blockIdx.x * L, hi = min(n, lo + L);
  for (uint64_t tile = lo; tile < hi; tile += 256) {
    const uint64_t i = tile + t;
    uint32_t r = 0, rank = 0;
    uint64_t j = 0;
    if (i < hi) {
      r = a.oreg[i];
      j = a.order[i];
      rank = atomicAdd(&tc[r], 1u);
    }
    __syncthreads();
    if (i < hi) a.rorder[base[r] + rank] = j;
    __syncthreads();
    base[t] += tc[t];
    tc[t] = 0;
    __syncthreads();
  }
}

// Splits the jobs between the SHA-256 paths and lays out both queues, longest first.
// Bucket b (LPT, b = 0 longest) of wave-eligible jobs goes to solo / group tickets iff its
// longest length is >= tlen (BSG_TLEN_PCT of the longest, and the per-lane work share) and
// those tickets stay <= half the waves; the next buckets down to tlen2 (BSG_PAIR_PCT) go to
// pair tickets within the rest of that budget. A per-lane job takes ~2.5x the time per block
// of a skewed-pair one under load (~7,650 vs ~3,030 cycles; ~4,250 with a pair ticket's ring
// fills), so the longest per-lane job, not the longest chain, would otherwise end the launch.
__global__ __launch_bounds__(1024) void k_bucket_scan(ShaArgs a) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t nok;
  const uint32_t t = threadIdx.x;
  if (t == 0) nok = 0;
  const uint64_t mx = a.ctr->max_nblocks, w = a.ctr->bucket_width;
  const bool light = a.ctr->total_blocks * 10ull < mx * 64ull * a.waves;
  uint64_t tlen = (mx * (light ? BSG_TLEN_PCT_LIGHT : BSG_TLEN_PCT)) / 100;
  const uint64_t share = (a.ctr->total_blocks * 9) / (10ull * 64ull * a.waves);
  tlen = max(max(tlen, share), (uint64_t)kLongMinBlocks);
  uint64_t cap = kSolo + (uint64_t)kGroup * (a.waves / 2 > kSolo ? a.waves / 2 - kSolo : 0);
  if (a.long_mode == 2) { tlen = 0; cap = ~0ull; }
  uint32_t e[4], pe[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) e[i] = a.bucket_elig[4 * t + i];
  block_scan4(e, pe, wsum);
  uint32_t ok = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint64_t b = 4 * t + i;
    const uint64_t top = mx > b * w ? mx - b * w : 0;  // longest length in bucket b
    ok += (a.long_mode != 1 && top >= tlen && (uint64_t)pe[i] + e[i] <= cap) ? 1u : 0u;
  }
  __syncthreads();
  atomicAdd(&nok, ok);  // monotone in b: the eligible buckets are a prefix
  __syncthreads();
  const uint32_t nlb8 = nok;
  uint32_t lv[4], lo[4], sv[4], so[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) lv[i] = (4 * t + i < nlb8) ? e[i] : 0u;
  const uint32_t n8 = block_scan4(lv, lo, wsum);
  const uint64_t t8 = n8 <= kSolo ? n8 : kSolo + (n8 - kSolo + kGroup - 1) / kGroup;
  uint32_t nlb = nlb8;
  const uint64_t pair_pct = light ? BSG_PAIR_PCT_LIGHT : BSG_PAIR_PCT;
  if (pair_pct > 0 && a.long_mode == 0) {
    // the next buckets, down to pair_pct % of the longest, on pair tickets within the
    // remaining half-of-the-waves ticket budget
    const uint64_t tlen2 = max((mx * pair_pct) / 100, (uint64_t)kLongMinBlocks);
    const uint64_t tb = a.waves / 2 > t8 ? a.waves / 2 - t8 : 0;
    const uint64_t cap2 = tb * kPairGroup;
    uint32_t ok2 = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint64_t b = 4 * t + i;
      const uint64_t top = mx > b * w ? mx - b * w : 0;
      ok2 += (b >= nlb8 && top >= tlen2 && (uint64_t)pe[i] + e[i] - n8 <= cap2) ? 1u : 0u;
    }
    __syncthreads();
    if (t == 0) nok = 0;
    __syncthreads();
    atomicAdd(&nok, ok2);
    __syncthreads();
    nlb = nlb8 + nok;
#pragma unroll
    for (int i = 0; i < 4; ++i) lv[i] = (4 * t + i < nlb) ? e[i] : 0u;
  }
  const uint32_t nlong = block_scan4(lv, lo, wsum);
#pragma unroll
  for (int i = 0; i < 4; ++i) sv[i] = a.bucket_cnt[4 * t + i] - lv[i];
  const uint32_t nshort = block_scan4(sv, so, wsum);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a.bucket_loff[4 * t + i] = lo[i];
    a.bucket_off[4 * t + i] = so[i];
  }
  if (t == 0) {
    a.ctr->long_buckets = nlb;
    a.ctr->nlong = nlong;
    a.ctr->nshort = nshort;
    // regions of <= kRegionBytes (one per several CUs), each with enough jobs to balance
    const uint64_t rmax = min((uint64_t)kMaxRegions, max((uint64_t)a.waves / 16, (uint64_t)1));
    const uint64_t rspan = (a.span + kRegionBytes - 1) / kRegionBytes;
    a.reg->nregions = min(min(rmax, rspan), max((uint64_t)nshort / kMinRegionJobs, (uint64_t)1));
    if (a.span <= kRegionBytes) {  // one region: the k_r* kernels are not launched, and
      a.reg->off[0] = 0;           // per-lane mode reads the LPT order itself (rorder = order)
      a.reg->off[1] = nshort;
      a.reg->head[0] = 0;
    }
    a.ctr->long_thresh = mx > (uint64_t)nlb * w ? mx - (uint64_t)nlb * w : 0;  // diagnostic
    a.ctr->nlong_grp = n8;
    a.ctr->tickets_grp = t8;
    // lightly loaded: the solo tickets run with helper waves (k_sha<true>), the queue after them
    const uint64_t helped = (light && a.long_mode == 0)
                                ? min(min((uint64_t)n8, (uint64_t)kSolo), (uint64_t)a.waves / 2)
                                : 0;
    a.ctr->helped = helped;
    a.ctr->long_head = helped;
    a.ctr->ntickets = t8 + (nlong - n8 + kPairGroup - 1) / kPairGroup;
  }
}

// The chunk k_pick chose for early chain k: its stream and [start, end) (k_lens, k_early).
__device__ __forceinline__ bool early_key(const ShaArgs& a, int k, uint32_t* s, uint64_t* start,
                                          uint64_t* end) {
  const uint64_t top = a.early->top[k];
  if (!top) return false;
  const uint64_t c = a.cand[(uint32_t)top], cn = a.cand[(uint32_t)top + 1];
  *s = cand_stream(c);
  const uint64_t sb = a.streams[*s].seg_base;
  *start = sb + cand_pos(c) + 1;
  *end = sb + cand_pos(cn) + 1;
  return true;
}

__global__ __launch_bounds__(256) void k_lens(ShaArgs a) {
  if (a.ctr->overflow || a.ctr->error) return;
  const uint64_t M = a.ctr->nchunks;
  if (M > a.chunk_cap) return;
  const uint64_t njobs = M + a.nstreams;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint32_t st[8];
  ShaJob jb;
  uint64_t mx = 0, tot = 0;
  // early chains: the chunks k_early hashes leave k_sha's queues (they still count in the
  // longest job and the total, so the tiers are those of the whole run)
  uint32_t es[kEarly] = {~0u, ~0u};
  uint64_t e0[kEarly] = {0, 0}, e1[kEarly] = {0, 0};
  if (a.early)
    for (int k = 0; k < kEarly; ++k)
      if (!early_key(a, k, &es[k], &e0[k], &e1[k])) es[k] = ~0u;
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < njobs; j += stride) {
    uint32_t info = kNoJob;
    if (sha_setup(a, j, M, jb, st)) {
      tot += jb.nblocks;
      // continued chunks (a head from hist) stay per-lane
      if (jb.prefix == 0) mx = max(mx, (uint64_t)jb.nblocks);
      bool early = false;
      if (j < M && jb.fin && jb.prefix == 0 && jb.consumed == 0)
        for (int k = 0; k < kEarly; ++k)
          if (jb.stream == es[k] && jb.start == e0[k] && jb.end == e1[k]) {
            a.early->idx[k] = j + 1;
            early = true;
          }
      if (early) {
        a.jinfo[j] = kNoJob;
        continue;
      }
      info = min(jb.nblocks, ~kJobElig) | (jb.prefix == 0 ? kJobElig : 0u);
      LaneJob d;
      d.dptr = reinterpret_cast<uint64_t>(jb.dbase);
      d.start = jb.start;
      d.len = jb.L;
      d.stream = jb.stream;
      // per-lane mode starts a fresh final chunk from this alone; a continued chunk (midstate,
      // head bytes) or an open one (midstate out) takes sha_setup
      d.meta = jb.level | ((jb.fin && jb.prefix == 0 && jb.consumed == 0) ? 0u : kLaneJobSlow);
      a.jdesc[j] = d;
    }
    a.jinfo[j] = info;
  }
  // one atomic pair per workgroup, not per wave: the 4,096 waves' same-address atomics cost ~25 us
  // of the kernel's 57-70 on configs[2] (now 28-40; the launch is one job per thread,
  // profiles/r06_c16_*)
  __shared__ uint64_t wmx[4], wtot[4];
  for (int o = 32; o > 0; o >>= 1) {
    mx = max(mx, (uint64_t)__shfl_down(mx, o));
    tot += (uint64_t)__shfl_down(tot, o);
  }
  if ((threadIdx.x & 63) == 0) {
    wmx[threadIdx.x >> 6] = mx;
    wtot[threadIdx.x >> 6] = tot;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) {
      mx = max(mx, wmx[w]);
      tot += wtot[w];
    }
    if (mx) atomicMax(reinterpret_cast<unsigned long long*>(&a.ctr->max_nblocks), (unsigned long long)mx);
    if (tot) atomicAdd(reinterpret_cast<unsigned long long*>(&a.ctr->total_blocks), (unsigned long long)tot);
  }
}

__global__ void k_thresh(Counters* ctr, int mode) {
  (void)mode;
  const uint64_t w = (ctr->max_nblocks + kLptBuckets) / kLptBuckets;
  ctr->bucket_width = w ? w : 1;
}

// Orders one wave's LDS ring writes before its reads (and reads before the next writes). The
// ring is private to the wave, and a wave's LDS operations are executed in order, so only the
// compiler has to be kept from reordering: a wave-scope fence, no s_barrier (the other waves
// of the workgroup run independent jobs).
__device__ __forceinline__ void ring_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
  return v;
}

// Wave mode: ticket t of the long list (LPT order). Tickets [0, kSolo) are one job each, the
// rest kGroup consecutive jobs each. The wave expands the message schedule of 64 blocks at a
// time into its LDS ring (G chains x 64/G blocks; lane l expands block l % B of chain l / B),
// then the skewed lane pairs of octet c (lanes 8c+2p: E, 8c+2p+1: A) run the rounds of chain
// c, 9 VALU per round (sha256_rounds_skew); a solo job's chain is run by every pair alike.
__device__ void sha_wave_job(const ShaArgs& a, uint64_t M, uint64_t t, uint64_t nlong,
                             uint32_t* ring) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t n8 = a.ctr->nlong_grp, t8 = a.ctr->tickets_grp;
  const bool pairs = t >= t8;                  // pair tickets follow the solo / group ones
  const bool solo = !pairs && t < kSolo;
  const uint64_t j0 = solo ? t : pairs ? n8 + (t - t8) * kPairGroup : kSolo + (t - kSolo) * kGroup;
  const uint64_t jend = pairs ? nlong : n8;    // a group ticket never reaches into the pair jobs
  const uint32_t G = solo ? 1u : pairs ? kPairGroup : kGroup;
  const uint32_t B = 64u / G;                  // blocks per chain per ring fill
  const uint32_t cA = lane / B;                // chain this lane expands (phase A)
  const uint32_t cR = cA;                      // chain this lane's pair runs (phase B)
  // phase-A job
  ShaJob ja;
  uint32_t sta[8];
  const bool va = j0 + cA < jend && sha_setup(a, a.long_list[j0 + cA], M, ja, sta);
  if (!va) {  // empty slot of the last group: expand readable bytes, never used
    ja.dbase = a.data;
    ja.L = 0;
    ja.fin = 0;
    ja.consumed = 0;
  }
  const uint32_t na = va ? ja.nblocks : 0u;
  // phase-B job (also the one this lane's pair finishes)
  ShaJob jb;
  uint32_t st[8];
  const bool vb = j0 + cR < jend && sha_setup(a, a.long_list[j0 + cR], M, jb, st);
  const uint32_t nb = vb ? jb.nblocks : 0u;
  uint64_t tm0 = 0, tr0 = 0;
  // timing stamps of the longest job (read back as Counters::diag), unless k_early ran it
  const bool stamp = t == 0 && !(a.early && a.early->top[0]);
  if (stamp) {
    tm0 = __builtin_amdgcn_s_memtime();
    tr0 = __builtin_amdgcn_s_memrealtime();
  }
  const uint32_t nmax = __builtin_amdgcn_readfirstlane(wave_max(nb));
  // Pair tickets: skewed lane pairs (2p: E, 2p+1: A). Solo and group tickets: skewed octets
  // (one chain per 8 lanes, E quad at positions 0-3, A quad at 4-7; 8 VALU per round against
  // the pair's 9). Half states A: H0..H3, E: H6, H7, H4, H5.
  const SkewLane bl = skew_lane();
  const OctLane ol = oct_lane();
  const bool a_side = pairs ? bl.a_side : ol.a_side;
  uint32_t hs[4];
  hs[0] = a_side ? st[0] : st[6];
  hs[1] = a_side ? st[1] : st[7];
  hs[2] = a_side ? st[2] : st[4];
  hs[3] = a_side ? st[3] : st[5];
  // Each ring fill's message block is requested one fill ahead, before the chain runs on the
  // current fill, so a fill never waits for HBM (a pair ticket fills every 2 blocks).
  RawBlock rb;
  raw_load(ja.dbase, 64ull * min(lane % B, max(na, 1u) - 1u), 0, ja.L, rb);
  for (uint32_t base = 0; base < nmax; base += B) {
    // phase A: block base + lane % B of chain cA into LDS row `lane`; past a chain's last
    // block (or for an empty slot) the last block is re-expanded, so no load leaves the slack
    const uint32_t blk = min(base + lane % B, max(na, 1u) - 1u);
    uint32_t W[16];
    raw_to_words(rb, W);
    const int32_t valid = rb.valid;
    raw_load(ja.dbase, 64ull * min(base + B + lane % B, max(na, 1u) - 1u), 0, ja.L, rb);
    if (valid < 64) {
      pad_words(valid, W);
      if (ja.fin && blk + 1 == na) {
        const uint64_t bits = (ja.consumed + ja.L) * 8ull;
        W[14] = (uint32_t)(bits >> 32);
        W[15] = (uint32_t)bits;
      }
    }
    u32x4a* row = reinterpret_cast<u32x4a*>(ring + lane * kLongRow);
#pragma unroll
    for (int tt = 0; tt < 64; tt += 4) {
      uint32_t kw[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = tt + u;
        if (i >= 16) {
          const uint32_t w15 = W[(i - 15) & 15], w2 = W[(i - 2) & 15];
          const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
          const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
          W[i & 15] = (W[i & 15] + s0) + (W[(i - 7) & 15] + s1);
        }
        kw[u] = kK256[i] + W[i & 15];
      }
      row[tt / 4] = u32x4a{kw[0], kw[1], kw[2], kw[3]};
    }
    ring_sync();
    // phase B: blocks base .. base+B-1 of every chain
    const uint32_t steps = min(B, nmax - base);
    const uint32_t* ones = ring + 64 * kLongRow;
    const uint32_t* krow = a_side ? ones : ring + cR * B * kLongRow;
    const uint32_t stride = a_side ? 0u : 4u * kLongRow;
    if (pairs)
      sha256_blocks_skew(hs, krow, stride, steps, (int32_t)nb - (int32_t)base, bl);
    else
      sha256_blocks_oct(hs, krow, stride, steps, (int32_t)nb - (int32_t)base, ol);
    ring_sync();
  }
  // each lane collects its chain's state: H0..H3 from an A lane (the pair's odd lane, the
  // octet's position 4), H4..H7 from its E lane
  const int pe = (int)(lane & ~(B - 1u)), pa = (int)((lane & ~(B - 1u)) | (pairs ? 1u : 4u));
#pragma unroll
  for (int k = 0; k < 4; ++k) st[k] = (uint32_t)__shfl((int)hs[k], pa);
  st[6] = (uint32_t)__shfl((int)hs[0], pe);
  st[7] = (uint32_t)__shfl((int)hs[1], pe);
  st[4] = (uint32_t)__shfl((int)hs[2], pe);
  st[5] = (uint32_t)__shfl((int)hs[3], pe);
  if (vb && (lane & (B - 1u)) == 0) {
    sha_finish(a, jb, st);
    if (stamp) {
      a.ctr->diag[1] = __builtin_amdgcn_s_memtime();
      a.ctr->diag[3] = __builtin_amdgcn_s_memrealtime();
      a.ctr->diag[0] = tm0;
      a.ctr->diag[2] = tr0;
      a.ctr->diag[4] = jb.nblocks;
    }
  }
}

// Wave-uniform queue pop: lane 0 takes the ticket, every lane gets it as an SGPR value.
__device__ __forceinline__ uint64_t pop_uniform(uint64_t* head) {
  uint32_t lo = 0, hi = 0;
  if ((threadIdx.x & 63u) == 0) {
    const uint64_t t = atomicAdd(reinterpret_cast<unsigned long long*>(head), 1ull);
    lo = (uint32_t)t;
    hi = (uint32_t)(t >> 32);
  }
  lo = __builtin_amdgcn_readlane(lo, 0);
  hi = __builtin_amdgcn_readlane(hi, 0);
  return ((uint64_t)hi << 32) | lo;
}

// Solo tickets of a lightly loaded launch, with a helper wave. A solo chain's
// wave otherwise stops every 64 blocks to expand the next 64 message schedules into its ring:
// ~50 of its ~2,720 cycles per block, on the launch's critical path. Here the first workgroups
// to start (k_sha<true>) take solo tickets in pairs: waves 0 and 1 run the two chains, waves 2
// and 3 fill their rings, two halves of 64 K+W rows per chain, handed over by sequence numbers
// in LDS (fill f goes to half f & 1; the filler publishes fill_seq = f / 2 + 1 after writing
// its rows, the chain publishes done_seq = f / 2 + 1 after running them). The waves of a
// workgroup are resident together, so the hand-off depends on nothing outside the workgroup;
// every wait is bounded.
constexpr uint32_t kHelpHalfWords = 64 * kLongRow;
constexpr uint32_t kHelpOnes = 4 * kHelpHalfWords;     // the A lanes' row of ones
constexpr uint32_t kHelpFlags = kHelpOnes + kLongRow;  // fill_seq[2][2], then done_seq[2][2]
constexpr uint32_t kHelpWords = kHelpFlags + 8;
constexpr uint32_t kHelpSlot = 4 * kRingWords;         // the workgroup's pair index (past all rings)

__device__ __forceinline__ uint32_t lds_seq_load(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_seq_store(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);  // rows land first
}
// Waits until *p == want (wave-uniform). Bounded (a.seq_wait_limit polls, ~1 s); a timeout,
// never expected, flags a device error so that the run fails instead of hanging.
__device__ bool lds_seq_wait(const ShaArgs& a, uint32_t* p, uint32_t want) {
  for (uint32_t i = 0; i < a.seq_wait_limit; ++i) {
    if ((uint32_t)__builtin_amdgcn_readfirstlane((int)lds_seq_load(p)) == want) return true;
    __builtin_amdgcn_s_sleep(1);
  }
  if ((threadIdx.x & 63u) == 0)
    atomicOr(reinterpret_cast<unsigned long long*>(&a.ctr->error), 8ull);
  return false;
}

// The chain wave of a helped solo chain c of the workgroup: sha_wave_job's octet loop over the
// filler's halves, from the state st of a job of nb blocks. Returns the final state in st (every
// lane) and false if a handshake timed out (the device error flag is set then).
__device__ __forceinline__ bool solo_chain_blocks(const ShaArgs& a, uint32_t nb, uint32_t (&st)[8],
                                                  uint32_t* lds, uint32_t c) {
  const uint32_t lane = threadIdx.x & 63u;
  const OctLane ol = oct_lane();
  uint32_t hs[4];
  hs[0] = ol.a_side ? st[0] : st[6];
  hs[1] = ol.a_side ? st[1] : st[7];
  hs[2] = ol.a_side ? st[2] : st[4];
  hs[3] = ol.a_side ? st[3] : st[5];
  uint32_t* fill_seq = lds + kHelpFlags + 2 * c;
  uint32_t* done_seq = lds + kHelpFlags + 4 + 2 * c;
  const uint32_t* ones = lds + kHelpOnes;
  uint32_t f = 0;
  for (uint32_t base = 0; base < nb; base += 64, ++f) {
    const uint32_t h = f & 1u;
    if (!lds_seq_wait(a, fill_seq + h, f / 2 + 1)) return false;
    const uint32_t* krow = ol.a_side ? ones : lds + (2 * c + h) * kHelpHalfWords;
    const uint32_t stride = ol.a_side ? 0u : 4u * kLongRow;
    sha256_blocks_oct_solo(hs, krow, stride, min(64u, nb - base), ol);
    if (lane == 0) lds_seq_store(done_seq + h, f / 2 + 1);
  }
  // H0..H3 from octet position 4 (an A lane), H4..H7 from position 0 (an E lane)
#pragma unroll
  for (int k = 0; k < 4; ++k) st[k] = (uint32_t)__shfl((int)hs[k], 4);
  st[6] = (uint32_t)__shfl((int)hs[0], 0);
  st[7] = (uint32_t)__shfl((int)hs[1], 0);
  st[4] = (uint32_t)__shfl((int)hs[2], 0);
  st[5] = (uint32_t)__shfl((int)hs[3], 0);
  return true;
}

// The chain wave of helped solo ticket t (the workgroup's chain c).
__device__ void sha_solo_chain(const ShaArgs& a, uint64_t M, uint64_t t, uint32_t* lds,
                               uint32_t c) {
  const uint32_t lane = threadIdx.x & 63u;
  ShaJob jb;
  uint32_t st[8];
  const bool vb = sha_setup(a, a.long_list[t], M, jb, st);
  const uint32_t nb = __builtin_amdgcn_readfirstlane(vb ? jb.nblocks : 0u);  // one job: uniform
  // timing stamps of the longest job (read back as Counters::diag), unless an early chain
  // (k_early) ran the longest jobs and stamps them
  const bool stamp = t == 0 && !(a.early && a.early->top[0]);
  uint64_t tm0 = 0, tr0 = 0;
  if (stamp) {
    tm0 = __builtin_amdgcn_s_memtime();
    tr0 = __builtin_amdgcn_s_memrealtime();
  }
  if (!solo_chain_blocks(a, nb, st, lds, c)) return;
  if (vb && lane == 0) {
    sha_finish(a, jb, st);
    if (stamp) {
      a.ctr->diag[1] = __builtin_amdgcn_s_memtime();
      a.ctr->diag[3] = __builtin_amdgcn_s_memrealtime();
      a.ctr->diag[0] = tm0;
      a.ctr->diag[2] = tr0;
      a.ctr->diag[4] = jb.nblocks;
    }
  }
}

// The filler wave of helped solo chain c: fill f is the K+W rows of blocks 64f .. 64f+63 (lane
// l: block 64f + l, the last block again past the end), into half f & 1 once the chain has run
// that half's previous fill. Each fill's block is requested one fill ahead.
__device__ __forceinline__ void solo_fill_blocks(const ShaArgs& a, ShaJob ja, bool va,
                                                 uint32_t* lds, uint32_t c) {
  const uint32_t lane = threadIdx.x & 63u;
  if (!va) {
    ja.dbase = a.data;
    ja.L = 0;
    ja.fin = 0;
    ja.consumed = 0;
  }
  const uint32_t na = __builtin_amdgcn_readfirstlane(va ? ja.nblocks : 0u);
  uint32_t* fill_seq = lds + kHelpFlags + 2 * c;
  uint32_t* done_seq = lds + kHelpFlags + 4 + 2 * c;
  RawBlock rb;
  raw_load(ja.dbase, 64ull * min(lane, max(na, 1u) - 1u), 0, ja.L, rb);
  uint32_t f = 0;
  for (uint32_t base = 0; base < na; base += 64, ++f) {
    const uint32_t h = f & 1u;
    if (f >= 2 && !lds_seq_wait(a, done_seq + h, f / 2)) return;
    const uint32_t blk = min(base + lane, max(na, 1u) - 1u);
    uint32_t W[16];
    raw_to_words(rb, W);
    const int32_t valid = rb.valid;
    raw_load(ja.dbase, 64ull * min(base + 64u + lane, max(na, 1u) - 1u), 0, ja.L, rb);
    if (valid < 64) {
      pad_words(valid, W);
      if (ja.fin && blk + 1 == na) {
        const uint64_t bits = (ja.consumed + ja.L) * 8ull;
        W[14] = (uint32_t)(bits >> 32);
        W[15] = (uint32_t)bits;
      }
    }
    u32x4a* row = reinterpret_cast<u32x4a*>(lds + (2 * c + h) * kHelpHalfWords + lane * kLongRow);
#pragma unroll
    for (int tt = 0; tt < 64; tt += 4) {
      uint32_t kw[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = tt + u;
        if (i >= 16) {
          const uint32_t w15 = W[(i - 15) & 15], w2 = W[(i - 2) & 15];
          const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
          const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
          W[i & 15] = (W[i & 15] + s0) + (W[(i - 7) & 15] + s1);
        }
        kw[u] = kK256[i] + W[i & 15];
      }
      row[tt / 4] = u32x4a{kw[0], kw[1], kw[2], kw[3]};
    }
    if (lane == 0) lds_seq_store(fill_seq + h, f / 2 + 1);
  }
}

// The filler wave of helped solo ticket t.
__device__ void sha_solo_fill(const ShaArgs& a, uint64_t M, uint64_t t, uint32_t* lds,
                              uint32_t c) {
  ShaJob ja;
  uint32_t sta[8];
  const bool va = sha_setup(a, a.long_list[t], M, ja, sta);
  solo_fill_blocks(a, ja, va, lds, c);
}

// The SHA-256 kernel. One 256-thread workgroup per CU (its LDS request admits only one), so
// each of the 4 waves owns a SIMD: one wave saturates a SIMD's integer VALU (~4.2 cycles per
// wave-instruction; a second wave on the SIMD only runs in the first one's gaps), so stacking
// waves gains nothing and would stall the latency-critical wave-mode chains. Every wave first
// drains the long-job queue in wave mode, then turns to per-lane mode (longest-first order).
// (Measured and dropped: 8 waves per workgroup, two per SIMD — the chains kept their speed but
// the longest per-lane jobs, sharing a SIMD, took 1.5x as long (round 2); and four more per-lane
// waves taking each region's shortest jobs beside waves 0-3 (round 5, profiles/r05_ab21_*.log:
// configs[2] 886-902 against 914-970 GiB/s; the chip's clock fell from 2.32-2.34 to 2.23-2.24 GHz
// under the extra issue, slowing the chains by 4 % at the same cycles per block).)
constexpr uint32_t kShaWaves = 4;
constexpr uint32_t kShaBlock = 64 * kShaWaves;

// Two instantiations, launched back to back; the one that does not match the launch (helped
// solo tickets or not, k_bucket_scan) returns at once. k_sha<false> holds no helper code, so
// its per-lane loop keeps its register allocation: k_sha sits at the SGPR limit, and the
// helper code in the same kernel made hipcc spill SGPRs inside that loop (configs[2] 880 ->
// 760-840 GiB/s). k_sha<true> runs only lightly loaded launches, where per-lane mode is short.
template <bool HELP>
__global__ __launch_bounds__(kShaBlock, 1) void k_sha(ShaArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  if (a.ctr->overflow || a.ctr->error) return;
  if ((a.ctr->helped != 0) != HELP) return;
  const uint64_t M = a.ctr->nchunks;
  if (M > a.chunk_cap) return;  // k_chunks flagged the error
  const uint64_t nlong = a.ctr->nlong;
  if ((threadIdx.x & 63u) == 0) {  // diagnostic timeline: when the kernel's first wave started
    const uint64_t rt = __builtin_amdgcn_s_memrealtime();
    if (atomicAdd(reinterpret_cast<unsigned long long*>(&a.ctr->sha_arrivals), 1ull) == 0)
      a.ctr->sha_start_rt = rt;
  }
  const uint64_t ntickets = a.ctr->ntickets;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t* ring = lds + wv * kRingWords;
  uint64_t t = ~0ull;
  bool helper_wg = false;
  if constexpr (HELP) {  // the first workgroups to start take the helped solo pairs
    if (threadIdx.x == 0)
      lds[kHelpSlot] = (uint32_t)atomicAdd(reinterpret_cast<unsigned long long*>(&a.ctr->help_wg), 1ull);
    __syncthreads();
    const uint64_t helped = a.ctr->helped, hw = lds[kHelpSlot];
    if (hw * 2 < helped) {  // workgroup-uniform
      helper_wg = true;
      for (uint32_t i = threadIdx.x; i < (uint32_t)kLongRow; i += blockDim.x) lds[kHelpOnes + i] = 1u;
      if (threadIdx.x < 8) lds[kHelpFlags + threadIdx.x] = 0u;
      __syncthreads();
      const uint32_t c = wv & 1u;
      const uint64_t ht = hw * 2 + c;
      if (ht < helped) {
        __builtin_amdgcn_s_setprio(3);
        if (wv < 2) sha_solo_chain(a, M, ht, lds, c);
        else sha_solo_fill(a, M, ht, lds, c);
        __builtin_amdgcn_s_setprio(0);
      }
    }
  }
  if (!helper_wg) {
    // row of ones after each wave's 64 K+W rows (the A lanes' kw in sha256_rounds_bank)
    for (uint32_t i = threadIdx.x & 63u; i < (uint32_t)kLongRow; i += 64) ring[64 * kLongRow + i] = 1u;
    // A plain pre-tested loop on a scalar ticket: a `for (;;) { if (lane == 0) atomic; ...;
    // break; }` form was restructured by hipcc into a nested loop that re-entered job 0 forever.
    t = pop_uniform(&a.ctr->long_head);
  }
  if (t < ntickets) {
    // A long chain is the launch's critical path. When another kernel's waves share its SIMD
    // (the streaming pipeline runs the next tile's scan beside this k_sha), the arbiter should
    // issue the chain's instructions first.
    __builtin_amdgcn_s_setprio(3);
    while (t < ntickets) {
      sha_wave_job(a, M, t, nlong, ring);
      t = pop_uniform(&a.ctr->long_head);
    }
    __builtin_amdgcn_s_setprio(0);
  }
  sha_lane_mode(a, M);
  if ((threadIdx.x & 63u) == 0)
    atomicMax(reinterpret_cast<unsigned long long*>(&a.ctr->lane_end_rt),
              (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

// ---------------------------------------------------------------------------------------------
// Early chains (see Early in bsgpu_internal.h).
// ---------------------------------------------------------------------------------------------
// k_pick: the two longest chunks (E_i, E_i+1] whose both ends are sure boundaries, i.e. c_i is
// a sync point (E_i - E_i-1 >= MinSize: k_select makes it a boundary whatever came before) and
// c_i+1 is one too or is the forced final flush. Chunks below the wave-mode floor are not worth
// the second stream. Keys are (blocks << 32 | i), so all keys differ.
// Such a chunk always satisfies k_lens's match (fin, prefix == 0, consumed == 0): it starts at
// the boundary c_i, after c_i-1 of the same segment, so it is never a segment's first chunk —
// the only one that can hold head bytes or a midstate carried in (prefix, consumed) — and it
// ends at a boundary, so it is never the open chunk a non-final segment leaves (fin). A pick
// that k_lens still does not match is a selection bug, flagged by k_early_fix (device error 16).
// (Engine runs start every stream fresh, open_start == seg_base == 0; streaming engines, whose
// segments carry open chunks, never run early chains: early_ok() requires !snapshot.)
__device__ __forceinline__ uint64_t pick_key(const uint64_t* __restrict__ cand, uint64_t n,
                                             uint64_t i, uint64_t minsz) {
  if (i == 0 || i + 1 >= n) return 0;
  const uint64_t c = cand[i];
  const uint64_t cp = cand[i - 1], cn = cand[i + 1];
  const uint32_t s = cand_stream(c);
  if (cand_stream(cp) != s || cand_stream(cn) != s) return 0;
  const uint64_t E = cand_pos(c) + 1, Ep = cand_pos(cp) + 1, En = cand_pos(cn) + 1;
  if (E - Ep < minsz) return 0;                        // c_i is not a sync point
  if (!cand_force(cn) && En - E < minsz) return 0;     // c_i+1 not sure
  if (cand_force(c)) return 0;                         // (a flush ends its stream)
  const uint64_t nb = (En - E + 8) / 64 + 1;
  if (nb < kLongMinBlocks || nb >= (1ull << 31)) return 0;
  return (nb << 32) | i;
}

// The two largest of (b1 >= b2) over the wave, in every lane.
__device__ __forceinline__ void top2_wave(uint64_t& b1, uint64_t& b2) {
  uint64_t m1 = b1;
  for (int o = 32; o > 0; o >>= 1) m1 = max(m1, (uint64_t)__shfl_xor((long long)m1, o));
  uint64_t m2 = b1 == m1 ? b2 : b1;  // the best of all but m1's lane's first
  for (int o = 32; o > 0; o >>= 1) m2 = max(m2, (uint64_t)__shfl_xor((long long)m2, o));
  b1 = m1;
  b2 = m2;
}

// A small grid (kPickWGs workgroups of 1024 for up to 4 M candidates) reduces to one key pair per workgroup, so top[] sees
// few atomics (same-address atomics from thousands of waves cost ~0.1 ms). Each workgroup
// submits its pair: top[0] keeps the maximum, and whatever a submission displaces or loses goes
// to top[1], which so ends with the largest key other than top[0]'s.
constexpr uint32_t kPickWGs = 64;
__global__ __launch_bounds__(1024) void k_pick(const uint64_t* __restrict__ cand, Counters* ctr,
                                               uint32_t min_size, Early* e) {
  __shared__ uint64_t wp[2 * 16];
  if (ctr->overflow || ctr->error) return;
  const uint64_t n = ctr->ncand;
  if (n >= (1ull << 32)) return;  // the key carries i in 32 bits
  uint64_t b1 = 0, b2 = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t key = pick_key(cand, n, i, min_size);
    b2 = max(b2, min(key, b1));
    b1 = max(b1, key);
  }
  top2_wave(b1, b2);
  const uint32_t w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63u) == 0) {
    wp[2 * w] = b1;
    wp[2 * w + 1] = b2;
  }
  __syncthreads();
  if (w != 0) return;
  const uint32_t l = threadIdx.x;
  b1 = l < 2 * nw ? wp[l] : 0;  // one key per lane: the pairs' members
  b2 = 0;
  top2_wave(b1, b2);
  if (l == 0 && b1) {
    unsigned long long* t = reinterpret_cast<unsigned long long*>(e->top);
    const uint64_t old = atomicMax(t, (unsigned long long)b1);
    if (old < b1) {
      if (old) atomicMax(t + 1, (unsigned long long)old);
      if (b2) atomicMax(t + 1, (unsigned long long)b2);
    } else {
      atomicMax(t + 1, (unsigned long long)b1);
    }
  }
}

// k_early: one workgroup on the second stream, laid out as a helped solo pair of k_sha<true>:
// waves 0 and 1 run the chains of the picked chunks 0 and 1, waves 2 and 3 fill their rings.
__global__ __launch_bounds__(256, 1) void k_early(ShaArgs a, uint32_t split_bits) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  if (a.ctr->overflow || a.ctr->error) return;
  Early* e = a.early;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63u;
  for (uint32_t i = threadIdx.x; i < (uint32_t)kLongRow; i += blockDim.x) lds[kHelpOnes + i] = 1u;
  if (threadIdx.x < 8) lds[kHelpFlags + threadIdx.x] = 0u;
  __syncthreads();
  const uint32_t c = wv & 1u;
  ShaJob jb;
  uint32_t s;
  if (!early_key(a, (int)c, &s, &jb.start, &jb.end)) return;  // no such pick: the wave leaves
  const uint64_t cn = a.cand[(uint32_t)e->top[c] + 1];
  const StreamDesc* sd = a.streams + s;
  jb.id = c;
  jb.stream = s;
  jb.level = cand_tz(cn) >= split_bits ? cand_tz(cn) - split_bits : 0u;
  jb.fin = 1;
  jb.prefix = 0;
  jb.consumed = 0;
  jb.dbase = a.data + sd->data_off + (jb.start - sd->seg_base);
  jb.hist = sd->hist + 64;
  jb.L = jb.end - jb.start;
  jb.nblocks = (uint32_t)((jb.L + 8) / 64 + 1);
  __builtin_amdgcn_s_setprio(3);
  if (wv >= 2) {
    solo_fill_blocks(a, jb, true, lds, c);
    return;
  }
  uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                    0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  const uint64_t tm0 = __builtin_amdgcn_s_memtime(), tr0 = __builtin_amdgcn_s_memrealtime();
  const uint32_t nb = __builtin_amdgcn_readfirstlane(jb.nblocks);
  if (!solo_chain_blocks(a, nb, st, lds, c)) return;
  if (lane == 0) {
    ChunkRec* r = e->rec + c;
    r->offset = jb.start;
    r->len = jb.L;
    r->level = jb.level;
    r->stream = jb.stream;
    uint32_t* ref = reinterpret_cast<uint32_t*>(r->ref);
#pragma unroll
    for (int i = 0; i < 8; ++i) ref[i] = __builtin_bswap32(st[i]);
    if (c == 0) {
      e->diag[1] = __builtin_amdgcn_s_memtime();
      e->diag[3] = __builtin_amdgcn_s_memrealtime();
      e->diag[0] = tm0;
      e->diag[2] = tr0;
      e->diag[4] = jb.nblocks;
    }
  }
}

// After k_sha and k_early: the early chunks' records into their places (k_lens matched them to
// their job indices), and the longest one's timing stamps into the counters.
// A pick that k_lens did not match was hashed by k_sha as usual, but it means the pick rule and
// the selection disagree about a chunk: a bug, flagged as a device error (bit 16) so that no
// test passes over it.
__global__ void k_early_fix(Early* e, ChunkRec* out, Counters* ctr) {
  if (ctr->overflow || ctr->error) return;
  const int k = threadIdx.x;
  if (k < kEarly && e->top[k] && e->idx[k]) out[e->idx[k] - 1] = e->rec[k];
  if (k < kEarly && e->top[k] && !e->idx[k])
    atomicOr(reinterpret_cast<unsigned long long*>(&ctr->error), 16ull);
  if (k == 0 && e->top[0] && e->idx[0])
    for (int i = 0; i < 5; ++i) ctr->diag[i] = e->diag[i];
}

// ---------------------------------------------------------------------------------------------
// Standalone batched SHA-256 over (offset, length) blobs (bsg_sha256_batch).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_sha_blobs(BlobShaArgs a) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
    ShaJob jb;
    jb.id = i;
    jb.start = 0;
    jb.end = a.len[i];
    jb.dbase = a.base + a.off[i];
    jb.hist = nullptr;
    jb.L = a.len[i];
    jb.consumed = 0;
    jb.prefix = 0;
    jb.fin = 1;
    jb.nblocks = (uint32_t)((jb.L + 8) / 64 + 1);
    uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                      0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    RawBlock rb;
    raw_load(jb.dbase, 0, 0, jb.L, rb);
    for (uint32_t blk = 0; blk < jb.nblocks; ++blk) {
      uint32_t W[16];
      raw_to_words(rb, W);
      if (rb.valid < 64) {
        pad_words(rb.valid, W);
        if (blk + 1 == jb.nblocks) {
          const uint64_t bits = jb.L * 8ull;
          W[14] = (uint32_t)(bits >> 32);
          W[15] = (uint32_t)bits;
        }
      }
      raw_load(jb.dbase, 64ull * (blk + 1), 0, jb.L, rb);
      sha256_compress_aligned(st, W);
    }
    uint32_t* ref = reinterpret_cast<uint32_t*>(a.refs + 32 * i);
#pragma unroll
    for (int k = 0; k < 8; ++k) ref[k] = __builtin_bswap32(st[k]);
  }
}

// ---------------------------------------------------------------------------------------------
// Synthetic input (bench/test utility, not on the hot path): word i = splitmix64(seed+(i+1)*G)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_fill_splitmix(uint8_t* p, uint64_t n, uint64_t seed) {
  const uint64_t nw = (n + 7) / 8;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += stride) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    if (8 * i + 8 <= n) {
      *reinterpret_cast<uint64_t*>(p + 8 * i) = z;
    } else {
      for (uint64_t b = 0; 8 * i + b < n; ++b) p[8 * i + b] = (uint8_t)(z >> (8 * b));
    }
  }
}

hipError_t launch_fill_splitmix(uint8_t* p, uint64_t n, uint64_t seed, hipStream_t s,
                                int num_cus) {
  const uint32_t grid = (uint32_t)std::min<uint64_t>((n / 8 + 255) / 256 + 1, 16ull * num_cus);
  hipLaunchKernelGGL(k_fill_splitmix, dim3(grid), dim3(256), 0, s, p, n, seed);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------------------------
static inline uint32_t grid_for(uint64_t items, uint32_t per_block, uint32_t cap) {
  uint64_t g = (items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  return (uint32_t)(g < cap ? g : cap);
}

uint32_t scan_lists(uint64_t nstrips, int num_cus) {
  const uint64_t groups = (nstrips + kScanGroup - 1) / kScanGroup;
  return grid_for(groups, 1, 2u * (uint32_t)num_cus);  // two k_scan workgroups per CU
}

uint64_t scan_list_cap(uint64_t nstrips, uint32_t lists) {
  const uint64_t groups = (nstrips + kScanGroup - 1) / kScanGroup;
  const uint64_t share = lists ? (groups + lists - 1) / lists : 0;
  return min(groups, kScanDynShare * share) * (uint64_t)kScanGroup;
}

hipError_t launch_scan(const ScanArgs& a, hipStream_t s, int num_cus) {
  const uint32_t grid = scan_lists(a.nstrips, num_cus);
  if (grid != a.lists) return hipErrorInvalidValue;  // the refine lists assume this grid
  static_assert(kScanLds <= 160 * 1024, "k_scan LDS");
  if (a.p.split_bits >= 16)
    hipLaunchKernelGGL(k_scan<true>, dim3(grid), dim3(kScanThreads), kScanLds, s, a);
  else
    hipLaunchKernelGGL(k_scan<false>, dim3(grid), dim3(kScanThreads), kScanLds, s, a);
  return hipGetLastError();
}

// The refine-list consumers run one workgroup per k_scan workgroup's list.
hipError_t launch_compact(const ScanArgs& a, hipStream_t s, int) {
  hipLaunchKernelGGL(k_compact, dim3(a.lists), dim3(256), kStrip0Lds * 8, s, a);
  return hipGetLastError();
}

hipError_t launch_rescan(const ScanArgs& a, hipStream_t s, int) {
  hipLaunchKernelGGL(k_rescan, dim3(a.lists), dim3(kScanWG), kTabRows * kTabRep * 4, s, a);
  return hipGetLastError();
}

uint64_t prefix_partials_needed(uint64_t n_bound) {
  const uint64_t nb = (n_bound + kScanTile - 1) / kScanTile;
  return nb ? nb : 1;  // a status word per tile (an empty input still runs tile 0)
}

hipError_t launch_prefix(const PrefixArgs& a, hipStream_t s) {
  // status words [0, nb), zeroed by k_start (prefix_partials_needed)
  const uint64_t nb = prefix_partials_needed(a.n_bound);
  hipLaunchKernelGGL(k_prefix1, dim3((uint32_t)nb), dim3(kScanT), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_select(const SelArgs& a, uint64_t cand_bound, hipStream_t s, int num_cus) {
  const uint32_t grid = grid_for(cand_bound, 256, 8u * (uint32_t)num_cus);
  hipLaunchKernelGGL(k_select, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_chunks(const ChunkArgs& a, uint64_t cand_bound, uint32_t nstreams, hipStream_t s,
                         int num_cus) {
  const uint32_t grid = grid_for(cand_bound, 256, 8u * (uint32_t)num_cus);
  hipLaunchKernelGGL(k_chunks, dim3(grid), dim3(256), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_tally, dim3(grid_for(nstreams, 256, 1024)), dim3(256), 0, s, a, nstreams);
  return hipGetLastError();
}

hipError_t launch_blob_jobs(const ChunkArgs& a, const StreamDesc* streams, uint32_t nstreams,
                            hipStream_t s, int num_cus) {
  const uint32_t grid = grid_for(nstreams, 256, 4u * (uint32_t)num_cus);
  hipLaunchKernelGGL(k_blob_jobs, dim3(grid), dim3(256), 0, s, a, streams, nstreams);
  return hipGetLastError();
}

hipError_t launch_start(const StartArgs& a, hipStream_t s) {
  const uint64_t work = std::max<uint64_t>(
      std::max<uint64_t>((uint64_t)a.nstreams * (sizeof(StreamDesc) / 16), a.nstreams + 1ull),
      std::max(std::max(a.nzero0, a.nzero1), std::max(a.nzero2, a.nzero3)));
  hipLaunchKernelGGL(k_start, dim3(grid_for(work, 256, 1024)), dim3(256), 0, s, a);
  return hipGetLastError();
}

constexpr uint32_t kShaLds = 84 * 1024;  // > 80 KiB: one k_sha workgroup per CU (160 KiB LDS)
static_assert(4 * kRingWords * 4 <= kShaLds, "wave rings fit");
static_assert(kHelpWords <= kHelpSlot && (kHelpSlot + 1) * 4 <= kShaLds,
              "helped solo rings and the pair slot fit");

hipError_t launch_sha(const ShaArgs& a, uint64_t job_bound, hipStream_t s, int num_cus) {
  (void)job_bound;  // persistent: one workgroup per CU, waves loop over the job queues
  hipLaunchKernelGGL(k_sha<true>, dim3((uint32_t)num_cus), dim3(kShaBlock), kShaLds, s, a);
  hipLaunchKernelGGL(k_sha<false>, dim3((uint32_t)num_cus), dim3(kShaBlock), kShaLds, s, a);
  return hipGetLastError();
}

hipError_t launch_pick(const uint64_t* cand, uint64_t cand_cap, Counters* ctr, uint32_t min_size,
                       Early* e, hipStream_t s, int num_cus) {
  // ~64 candidates per thread at most, unless that takes more than 4 workgroups per CU
  const uint64_t g = std::min<uint64_t>(std::max<uint64_t>(kPickWGs, cand_cap >> 16),
                                        4ull * (uint32_t)num_cus);
  hipLaunchKernelGGL(k_pick, dim3((uint32_t)g), dim3(1024), 0, s, cand, ctr, min_size, e);
  return hipGetLastError();
}

hipError_t launch_early(const ShaArgs& a, uint32_t split_bits, hipStream_t s) {
  hipLaunchKernelGGL(k_early, dim3(1), dim3(256), kShaLds, s, a, split_bits);
  return hipGetLastError();
}

hipError_t launch_early_fix(Early* e, ChunkRec* out, Counters* ctr, hipStream_t s) {
  hipLaunchKernelGGL(k_early_fix, dim3(1), dim3(64), 0, s, e, out, ctr);
  return hipGetLastError();
}

hipError_t launch_longlist(const ShaArgs& a, uint64_t job_bound, hipStream_t s, int num_cus) {
  const uint32_t grid = grid_for(job_bound, 256, 4u * (uint32_t)num_cus);
  hipLaunchKernelGGL(k_lens, dim3(grid), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_thresh, dim3(1), dim3(1), 0, s, a.ctr, a.long_mode);
  hipLaunchKernelGGL(k_order<false>, dim3(grid), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_bucket_scan, dim3(1), dim3(1024), 0, s, a);
  hipLaunchKernelGGL(k_order<true>, dim3(grid), dim3(256), 0, s, a);
  if (a.span > kRegionBytes) {  // else one region (k_bucket_scan) over the LPT order itself
    hipLaunchKernelGGL(k_rcount, dim3(kRegionSegs), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_rscan, dim3(kMaxRegions), dim3(kRegionSegs), 0, s, a);
    hipLaunchKernelGGL(k_rtotal, dim3(1), dim3(kMaxRegions), 0, s, a);
    hipLaunchKernelGGL(k_rscatter, dim3(kRegionSegs), dim3(256), 0, s, a);
  }
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_copy_out(const uint32_t* __restrict__ src,
                                                  uint32_t* __restrict__ dst, uint64_t words) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride)
    dst[i] = src[i];
}

hipError_t launch_copy_out(const void* src, void* dst, uint64_t bytes, hipStream_t s) {
  // every caller copies whole structs of 4-byte multiples (ChunkRec, Counters, u64 arrays)
  const uint64_t words = bytes / 4;
  if (words == 0) return hipSuccess;
  const uint32_t grid = grid_for(words, 256, 64);
  hipLaunchKernelGGL(k_copy_out, dim3(grid), dim3(256), 0, s,
                     static_cast<const uint32_t*>(src), static_cast<uint32_t*>(dst), words);
  return hipGetLastError();
}

hipError_t launch_sha_blobs(const BlobShaArgs& a, hipStream_t s, int num_cus) {
  const uint32_t grid = grid_for(a.n, 256, 8u * (uint32_t)num_cus);
  hipLaunchKernelGGL(k_sha_blobs, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace bsg

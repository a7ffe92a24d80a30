// bsgpu_internal.h — device data layout shared by the HIP kernels and the host engine.
//
// One launch ("run") processes a batch of stream SEGMENTS. A segment is a contiguous range of
// one byte stream that lives in device memory. Fresh streams (the batch API) have zero history,
// IV hash state and finalize=1. Streaming continuation (split.Writer over many Write calls,
// reference split/split.go:99-126) carries a 64-byte window history, the open chunk's start
// and its SHA-256 midstate from one segment to the next.
#pragma once
#include <stdint.h>

namespace bsg {

constexpr int kScanWG = 512;       // threads per rolling-scan workgroup (8 waves)
#ifndef BSG_STRIP
#define BSG_STRIP 2048
#endif
constexpr int kStrip = BSG_STRIP;  // bytes per lane-strip in the rolling scan
constexpr int kSlotCap = 4;        // candidates kept per strip in the first scan pass
constexpr int kTabRows = 256;      // buzhash32 table rows
constexpr int kTabRep = 64;        // one replica per lane: LDS address = byte*256 + lane*4

// Candidate record (u64): | stream:16 | pos:40 | force:1 | unused:1 | tz:6 |
constexpr int kCandPosShift = 8;
constexpr uint64_t kCandPosMask = (1ull << 40) - 1;
constexpr uint64_t kCandForce = 1ull << 7;

__host__ __device__ inline uint64_t cand_pack(uint32_t stream, uint64_t pos, bool force,
                                              uint32_t tz) {
  return ((uint64_t)stream << 48) | ((pos & kCandPosMask) << kCandPosShift) |
         (force ? kCandForce : 0ull) | (uint64_t)(tz & 63u);
}
__host__ __device__ inline uint32_t cand_stream(uint64_t c) { return (uint32_t)(c >> 48); }
__host__ __device__ inline uint64_t cand_pos(uint64_t c) {
  return (c >> kCandPosShift) & kCandPosMask;
}
__host__ __device__ inline bool cand_force(uint64_t c) { return (c & kCandForce) != 0; }
__host__ __device__ inline uint32_t cand_tz(uint64_t c) { return (uint32_t)(c & 63u); }

// Per-strip slot record (u32): | local_off:24 | force:1 | unused:1 | tz:6 |
__host__ __device__ inline uint32_t slot_pack(uint32_t local, bool force, uint32_t tz) {
  return (local << 8) | (force ? 0x80u : 0u) | (tz & 63u);
}

struct StreamDesc {            // 160 bytes, 16-byte aligned
  uint64_t data_off;           // device byte offset of the segment's first byte
  uint64_t len;                // segment length (bytes)
  uint64_t strip0;             // first global strip index of this segment
  uint64_t seg_base;           // stream offset of the segment's first byte
  uint64_t open_start;         // stream offset where the open (unfinished) chunk starts
  uint64_t consumed;           // open-chunk bytes already folded into mid[] (multiple of 64)
  uint32_t finalize;           // 1: flush the tail as the final chunk (Splitter.Close)
  uint32_t prefix_len;         // open-chunk bytes held in hist[64-prefix_len..63], < 64
  uint32_t mid[8];             // SHA-256 midstate of the open chunk (IV when consumed == 0)
  uint32_t carry_cap;          // non-final segment: leave an open chunk of <= carry_cap bytes
                               // unhashed (the next segment re-hashes it from device memory)
  uint32_t flags;              // kDescOpenInDevice: the open chunk's bytes [open_start, seg_base)
                               // sit in device memory right before data_off (consumed == 0)
  uint8_t hist[64];            // the 64 stream bytes before seg_base (zeros before offset 0)
};
constexpr uint32_t kDescOpenInDevice = 1;
static_assert(sizeof(StreamDesc) == 160, "StreamDesc layout");

struct CarryOut {              // open chunk state after a non-final segment
  uint32_t mid[8];
  uint64_t consumed;           // bytes folded into mid (multiple of 64)
  uint64_t open_start;         // stream offset of the open chunk
  uint32_t prefix_len;         // trailing open-chunk bytes not yet hashed (< 64)
  uint32_t valid;
};

struct ChunkRec {              // == bsg_chunk (include/bsgpu.h)
  uint64_t offset;
  uint64_t len;
  uint32_t level;
  uint32_t stream;
  uint8_t ref[32];
};
static_assert(sizeof(ChunkRec) == 56, "ChunkRec layout");

struct Params {
  uint32_t split_bits;         // trailing-zero bits for a boundary (>= 1; > 32 never splits)
  uint32_t min_size;           // minimum chunk size (>= 1)
  uint32_t mask;               // (1 << split_bits) - 1, all ones for split_bits >= 32
  uint32_t pad_;
};

// Device counters, zeroed at the start of every run (one hipMemsetAsync).
struct Counters {
  uint64_t ncand;              // total candidates (from the strip-count scan)
  uint64_t nchunks;            // total boundaries = finalized chunks
  uint64_t help_wg;            // k_sha workgroups arrived (the first helped/2 run helped solo pairs)
  uint64_t overflow;           // candidate buffer too small (host grows and re-runs)
  uint64_t error;              // device-side sanity check failed (bug guard; run is invalid)
  uint64_t max_nblocks;        // longest SHA-256 job in blocks (k_lens)
  uint64_t long_thresh;        // jobs with >= this many blocks run on the wave-per-chunk path
  uint64_t nlong;              // number of such jobs (k_longlist)
  uint64_t long_head;          // k_sha_long work queue head
  uint64_t nshort;             // jobs on the per-lane path (k_bucket_scatter)
  uint64_t bucket_width;       // LPT bucket width in blocks
  uint64_t diag[5];            // k_sha_long job 0: memtime0/1, realtime0/1, nblocks (diagnostic)
  uint64_t diag2[5];           // k_sha per-lane job order[0]: same fields
  uint64_t rescan;             // strips with more candidates than slots (k_compact re-scans)
  uint64_t total_blocks;       // SHA-256 blocks over all jobs (k_lens)
  uint64_t long_buckets;       // LPT buckets [0, long_buckets) of wave-eligible jobs -> wave mode
  uint64_t ntickets;           // wave-mode work items: kSolo single jobs, then groups of kGroup
  uint64_t sha_arrivals;       // k_sha waves started (diagnostic)
  uint64_t sha_start_rt;       // s_memrealtime of the first k_sha wave (diagnostic)
  uint64_t lane_end_rt;        // latest s_memrealtime at which a wave left per-lane mode
  uint64_t nlong_grp;          // long jobs on solo / kGroup tickets; the rest of the long list
  uint64_t tickets_grp;        //   runs on pair tickets (kPairGroup jobs, one lane pair each)
  uint64_t nrefine;            // strips k_scan listed for its exact pass
  uint64_t helped;             // solo tickets [0, helped) run with a helper wave (k_sha)
  uint64_t scan_ticket;        // k_scan's strip groups handed out past the first (BSG_SCAN_DYN)
  uint64_t pad[7];
};
static_assert(sizeof(Counters) == 320, "Counters layout");

// Per-lane job descriptor (k_lens writes one per job): per-lane mode prefetches it a few blocks
// before its current job ends, so starting the next job costs no dependent loads.
struct LaneJob {
  uint64_t dptr;               // first data byte of the message (device address)
  uint64_t start;              // stream offset of the chunk (record offset)
  uint64_t len;                // message bytes = chunk length (fast jobs)
  uint32_t stream;
  uint32_t meta;               // level | kLaneJobSlow
};
static_assert(sizeof(LaneJob) == 32, "LaneJob layout");
constexpr uint32_t kLaneJobSlow = 0x80000000u;  // continued or open chunk: full sha_setup path

// Per-lane job queues by address region (k_sha per-lane mode). A lane's loads go to its own
// chunk, so the 64 lanes of a wave touch 64 places in HBM per load. With a CU's lanes spread
// over 16 GiB, 97 % of those loads miss the CU's address-translation cache (UTCL1) and a block
// costs ~60 % more than with the CU's lanes inside 2 GiB (tools/ubench/lanes_mem.hip,
// profiles/r02_lanes_tlb.log). The per-lane jobs are therefore regrouped, longest first within
// each region, into regions of at most kRegionBytes of address span, and all waves of a k_sha
// workgroup (one per CU) take their jobs from the same region until it runs dry.
constexpr uint32_t kMaxRegions = 256;
constexpr uint32_t kRegionSegs = 256;        // segments of the LPT order counted separately
constexpr uint32_t kMinRegionJobs = 4096;    // fewer per-lane jobs per region: fewer regions
constexpr uint64_t kRegionBytes = 1ull << 30;
struct Regions {
  uint64_t nregions;                         // R (k_bucket_scan), 1 .. kMaxRegions
  uint64_t rr;                               // round-robin start region of entering waves
  uint64_t pad_[6];
  uint64_t head[kMaxRegions];                // pop counters (zeroed by k_rtotal)
  uint64_t off[kMaxRegions + 1];             // region r's jobs: rorder[off[r] .. off[r + 1])
  uint64_t pad2_[7];
  uint32_t cnt[kRegionSegs * kMaxRegions];   // per segment and region: count, then offset
};

// Early chains (round 4). A step is bound by its longest chunks' serial SHA-256 chains, and
// in k_sha they start only after the whole selection (k_select .. k_order, ~0.1-0.3 ms of small
// dispatches). The sorted candidates already fix the chunks whose both ends are sync points
// (sure boundaries): on a second stream k_pick takes the kEarly longest of them and k_early
// hashes them (a helped pair: two chains, two ring fillers) while selection runs; k_lens takes the chunks (same stream, start and end) out of
// k_sha's queues and k_early_fix writes their records. A pick k_lens does not match is hashed
// by k_sha as usual.
constexpr int kEarly = 2;
struct Early {
  uint64_t top[kEarly];      // k_pick: (blocks << 32) | i for the chunk (E_i, E_i+1]; 0 = none
  uint64_t idx[kEarly];      // k_lens: 1 + the chunk's job index (0: not matched)
  uint64_t diag[5];          // k_early: timing stamps of top[0]'s chain (as Counters::diag)
  uint64_t pad_;
  ChunkRec rec[kEarly];      // k_early: the chunks' records
};
static_assert(sizeof(Early) % 16 == 0, "Early layout");

constexpr uint32_t kLongMinBlocks = 1024;  // never use the wave path below 64 KiB
#ifndef BSG_SOLO
#define BSG_SOLO 16  // configs[2]: the 9th-16th longest jobs on group tickets (1.40 us per
#endif           // block against 1.19 solo) ended 0.5 ms after the longest
constexpr uint32_t kSolo = BSG_SOLO;  // wave mode: the kSolo longest jobs run one per wave,
constexpr uint32_t kGroup = 8;   // the next ones kGroup per wave (one banked lane pair each)
constexpr uint32_t kPairGroup = 32;  // then (optionally) 32 per wave, one lane pair each
constexpr int kLongRow = 68;               // LDS words per K+W row (64 + pad: conflict-free b128)
constexpr int kRingWords = 65 * kLongRow;  // per wave: 64 K+W rows + one row of ones
constexpr int kLptBuckets = 4096;          // longest-first job order: counting sort on nblocks
constexpr uint64_t kReadSlack = 256;       // readable bytes required after every stream's data

}  // namespace bsg

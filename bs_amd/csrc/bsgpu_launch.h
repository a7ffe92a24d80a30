// bsgpu_launch.h — kernel argument blocks and launchers (host <-> bsgpu_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bsgpu_internal.h"

namespace bsg {

struct ScanArgs {
  const uint8_t* data;
  const StreamDesc* streams;
  const uint64_t* strip0;   // nstreams + 1 cumulative strip counts
  uint32_t nstreams;
  uint64_t nstrips;
  const uint32_t* table;    // 256 buzhash32 entries
  Params p;
  uint32_t* counts;         // [nstrips]
  uint64_t* refine;         // [lists * list_cap] strips k_scan's exact pass must scan: strip << 32
                            // | the fast pass's hit mask (one bit per 64-byte block); k_scan
                            // workgroup g appends to refine + g * list_cap
  uint32_t* slots;          // [nstrips * kSlotCap]
  const uint64_t* cand_off; // [nstrips] exclusive candidate offsets (compact)
  uint64_t* cand;           // [cand_cap]
  uint64_t cand_cap;
  Counters* ctr;
  uint32_t lists;           // k_scan's grid = the number of refine lists (scan_lists())
  uint64_t list_cap;        // entries per list: the strips one k_scan workgroup scans, at most
  uint32_t* list_cnt;       // [lists] each list's length, stored by its workgroup at exit
};
// k_scan's grid for nstrips strips (its workgroups take 256-strip groups by ticket) and the length
// bound of each workgroup's refine list; the host sizes ScanArgs::refine with them.
uint32_t scan_lists(uint64_t nstrips, int num_cus);
uint64_t scan_list_cap(uint64_t nstrips, uint32_t lists);

struct PrefixArgs {
  const uint32_t* in;
  uint64_t* out;
  uint64_t* partials;
  uint64_t n_bound;         // host bound on n
  const uint64_t* n_dev;    // optional device-side n (min with n_bound)
  uint64_t* total;          // receives the sum
  uint64_t* overflow;       // optional: set to 1 when total > cap
  uint64_t cap;
  const uint64_t* skip_if;  // optional: skip when *skip_if != 0
  uint64_t* error;          // k_prefix1: Counters::error (|= 32: a look-back poll timed out)
};

struct SelArgs {
  const uint64_t* cand;
  const StreamDesc* streams;
  uint32_t* flags;
  Params p;
  Counters* ctr;
};

struct ChunkArgs {
  const uint64_t* cand;
  const uint32_t* flags;
  const uint64_t* fidx;
  uint64_t* bnd_end;
  uint64_t* bnd_info;
  uint64_t* scount;
  uint64_t* last_end;
  uint64_t chunk_cap;
  Params p;
  Counters* ctr;
  const StreamDesc* streams;  // k_chunks: seg_base turns relative candidates into offsets
};

// k_start: a run's set-up in one dispatch (it was two H2D copies, two memsets and k_init): the
// descriptors (and the streams' first strips) from kernel-visible pinned host memory into
// device memory, the counters and the LPT bucket counts zeroed, each stream's open-chunk start
// and carry state initialised.
struct StartArgs {
  const StreamDesc* src;        // the run's descriptors, pinned host memory (device address)
  const uint64_t* src_strip0;   // nstreams + 1 first strips, pinned host memory; null: none
  StreamDesc* streams;
  uint64_t* strip0;
  uint32_t nstreams;
  uint64_t* last_end;
  uint64_t* scount;
  CarryOut* carry;
  uint32_t* zero0;              // Counters (+ Early), zeroed
  uint32_t nzero0;              // words
  uint32_t* zero1;              // LPT bucket counts, zeroed
  uint32_t nzero1;              // words
  uint32_t* zero2;              // the two prefixes' status words (k_prefix1), zeroed
  uint32_t nzero2;              // words
  uint32_t* zero3;
  uint32_t nzero3;
};

struct ShaArgs {
  const uint8_t* data;
  const StreamDesc* streams;
  uint32_t nstreams;
  const uint64_t* bnd_end;
  const uint64_t* bnd_info;
  const uint64_t* last_end;
  Counters* ctr;
  ChunkRec* out;
  CarryOut* carry;
  uint64_t chunk_cap;
  uint64_t* long_list;      // [chunk_cap + nstreams] job ids for the wave-per-chunk path
  uint64_t* order;          // [chunk_cap + nstreams] per-lane jobs, longest first
  uint32_t* bucket_cnt;     // [kLptBuckets] all jobs per LPT bucket, zeroed per run
  uint32_t* bucket_elig;    // [kLptBuckets] wave-eligible jobs per bucket, zeroed per run
  uint32_t* bucket_off;     // [kLptBuckets] per-lane order offsets
  uint32_t* bucket_loff;    // [kLptBuckets] long-list offsets
  uint32_t* jinfo;          // [chunk_cap + nstreams] per job, from k_lens: nblocks | eligible
                            // << 31, or kNoJob (no job: a short open chunk carried as bytes)
  LaneJob* jdesc;           // [chunk_cap + nstreams] per job, from k_lens: what per-lane mode
                            // needs to start it without sha_setup's dependent loads
  Regions* reg;             // per-lane region queues (see Regions)
  uint8_t* oreg;            // [chunk_cap + nstreams] region of order[i] (k_order)
  uint64_t* rorder;         // [chunk_cap + nstreams] per-lane jobs by region, longest first
  uint64_t span;            // bytes from data to the end of the last stream (regions)
  int long_mode;            // 0 auto, 1 per-lane only, 2 wave mode only (experiments)
  uint32_t waves;           // waves of the k_sha grid (4 per CU)
  uint32_t seq_wait_limit;  // polls before a helper-wave handshake flags a device error
                            // (~1 s; BSG_DEBUG_SEQ_WAIT overrides it, 0: fail at once, tests)
  const uint64_t* cand;     // early chains: the sorted candidates (k_lens decodes the picks)
  Early* early;             // early chains of this run, or nullptr
};

struct BlobShaArgs {
  const uint8_t* base;
  const uint64_t* off;
  const uint64_t* len;
  uint64_t n;
  uint8_t* refs;            // [n * 32]
};

hipError_t launch_scan(const ScanArgs& a, hipStream_t s, int num_cus);
hipError_t launch_compact(const ScanArgs& a, hipStream_t s, int num_cus);
hipError_t launch_rescan(const ScanArgs& a, hipStream_t s, int num_cus);
uint64_t prefix_partials_needed(uint64_t n_bound);
hipError_t launch_prefix(const PrefixArgs& a, hipStream_t s);
hipError_t launch_select(const SelArgs& a, uint64_t cand_bound, hipStream_t s, int num_cus);
hipError_t launch_chunks(const ChunkArgs& a, uint64_t cand_bound, uint32_t nstreams, hipStream_t s,
                         int num_cus);
hipError_t launch_start(const StartArgs& a, hipStream_t s);
hipError_t launch_blob_jobs(const ChunkArgs& a, const StreamDesc* streams, uint32_t nstreams,
                            hipStream_t s, int num_cus);
hipError_t launch_sha(const ShaArgs& a, uint64_t job_bound, hipStream_t s, int num_cus);
hipError_t launch_longlist(const ShaArgs& a, uint64_t job_bound, hipStream_t s, int num_cus);
hipError_t launch_sha_blobs(const BlobShaArgs& a, hipStream_t s, int num_cus);
// Early chains (see Early): picked and hashed on a second stream from k_compact on (k_lens waits
// for the picks), the records' fix-up on the engine stream after k_sha (it waits for the chains).
hipError_t launch_pick(const uint64_t* cand, uint64_t cand_cap, Counters* ctr, uint32_t min_size,
                       Early* e, hipStream_t s, int num_cus);
hipError_t launch_early(const ShaArgs& a, uint32_t split_bits, hipStream_t s);
hipError_t launch_early_fix(Early* e, ChunkRec* out, Counters* ctr, hipStream_t s);
// Device -> pinned host bytes by a kernel on stream s (dst: the device alias of a hipHostMalloc
// buffer). Unlike hipMemcpyAsync D2H, a kernel waiting in its own stream for the work before
// it holds no place in the shared copy-engine queue, so it cannot stall other streams' H2D.
hipError_t launch_copy_out(const void* src, void* dst, uint64_t bytes, hipStream_t s);
hipError_t launch_fill_splitmix(uint8_t* p, uint64_t n, uint64_t seed, hipStream_t s,
                                int num_cus);

}  // namespace bsg

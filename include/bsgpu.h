/*
 * bsgpu.h — C ABI of libbsgpu, the MI355X (gfx950) ingest path for BS's hashsplit chunker and
 * SHA-256 blob refs. Plain pointers and sizes only; no C++ exceptions cross this boundary.
 *
 * Reference interfaces replaced (paths relative to the bobg/bs tree):
 *   bsg_open / bsg_write / bsg_close / bsg_drain
 *       -> split.NewWriter(ctx, st, opts...)            split/split.go:44-96
 *          (*split.Writer).Write([]byte) (int, error)   split/split.go:99-101
 *          (*split.Writer).Close() error                split/split.go:104-126
 *          options Bits / MinSize / Fanout               split/split.go:137,148,161
 *       The per-byte loop they replace is hashsplit.Splitter.Write/Close (github.com/bobg/hashsplit
 *       v1.1.1, go.mod:9) with buzhash32 (github.com/chmduquesne/rollinghash v4.0.0, go.sum:61-62).
 *       The chunk records carry the ref that st.Put would compute (split/split.go:72 ->
 *       store/mem/mem.go:67 -> bs.go:24-26); the caller still calls its own Store.Put.
 *   bsg_sha256_batch
 *       -> bs.Blob.Ref() = sha256.Sum256(b)              bs.go:24-26 (many blobs at once)
 *   bsg_engine_* (device-resident batch of independent streams)
 *       -> N concurrent split.Writers, e.g. fs.Dir.AddDir's per-file writers (fs/dir.go:157-174)
 *
 * Threading: one bsg_ctx / bsg_engine per thread at a time; different contexts are
 * independent (each owns a HIP stream) and may run concurrently. Every entry point makes the
 * context's device current (hipSetDevice) so callers may migrate between OS threads.
 *
 * Errors: functions return BSG_OK (0) or a negative code; bsg_errstr() describes it.
 */
#ifndef BSGPU_H
#define BSGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BSG_OK 0
#define BSG_EINVAL (-22)   /* bad argument (null pointer, unaligned stream offset, ...) */
#define BSG_ENOMEM (-12)   /* host or device allocation failed */
#define BSG_EDEVICE (-5)   /* HIP runtime / kernel error */
#define BSG_ESTATE (-71)   /* Write after Close, etc. */
#define BSG_ENODEV (-19)   /* no such HIP device */
#define BSG_ENOTFOUND (-2) /* bs.ErrNotFound (store.go:63) */
#define BSG_ECORRUPT (-74) /* a fetched blob does not hash to its ref (reader verify) */
#define BSG_EIO (-1001)    /* filesystem error (store/file) */

/* split.Writer options. Zero fields take hashsplit's own defaults (SplitBits 13, MinSize 64);
 * bsg_params_default() gives split.NewWriter's defaults (16 / 1024 / fanout 8,
 * split/split.go:48,88-89). Like split.Bits / split.MinSize (split/split.go:137-152, which
 * store the value unchecked), every value is accepted: MinSize 1..63 lets the 64-byte window
 * span a boundary (allowed, only discouraged by split.go:146), and Bits > 32 never splits
 * (TrailingZeros32 is at most 32), so the whole stream is one final chunk of level 0. A cgo
 * caller maps MinSize(n <= 0) to 0 (hashsplit's default) and clamps Bits to 2^32-1. */
typedef struct bsg_params {
  uint32_t split_bits; /* Bits(n): trailing zero bits for a boundary (0 = 13) */
  uint32_t min_size;   /* MinSize(n): minimum chunk size (0 = 64) */
  uint32_t fanout;     /* Fanout(n): tree level divisor (host tree only; 0 = 8) */
  uint32_t reserved;
} bsg_params;

/* One chunk: the bytes [offset, offset+len) of a stream, its hashsplit level (trailing zeros
 * minus split_bits, NOT yet divided by fanout; split/split.go:86 divides) and its ref. */
typedef struct bsg_chunk {
  uint64_t offset;
  uint64_t len;
  uint32_t level;
  uint32_t stream;
  uint8_t ref[32];
} bsg_chunk; /* 56 bytes */

const char* bsg_errstr(int err);
bsg_params bsg_params_default(void);
/* The buzhash32 table used when callers pass table == NULL: rollinghash's GenerateHashes(1). */
void bsg_default_table(uint32_t out[256]);
int bsg_device_count(void);
/* Optional, once per process: makes `device` current, creates its HIP context and a few HIP
 * streams (kept in the library's stream pool), initialises the copy engines, loads every kernel
 * of the split and hash paths (one tiny split and hash) and starts the host copy threads — the
 * one-time cost (~50 ms) that the first Writer of a process pays otherwise. A server calls it
 * at start-up. */
int bsg_init(int device);

/* ---- streaming split.Writer (bytes arrive from host memory) ---- */
typedef struct bsg_ctx bsg_ctx;
bsg_ctx* bsg_open(int device, const bsg_params* params, const uint32_t* table /* 256 or NULL */,
                  int* err);
/* Copies p[0..n) into pinned staging (the caller keeps ownership of p); full tiles are split
 * and hashed on the device as they fill. A stream has no length limit, as split.Writer.Write
 * (split/split.go:99-101): stream offsets are 64-bit throughout; only positions inside one
 * device tile (< 2^40 bytes of device memory) travel in 40-bit fields. */
int bsg_write(bsg_ctx* ctx, const uint8_t* p, size_t n);
/* Zero-copy Write: *p / *cap = the free rest of the current pinned staging buffer (at most
 * 64 MiB and never more than the rest of the tile; a stream's first buffer grows from 4 MiB,
 * so early windows are smaller); the caller fills up to *cap bytes there (e.g. an io.Reader
 * reads straight into it) and commits n of them. Same stream semantics as bsg_write; the
 * window is valid until the next call on ctx. */
int bsg_write_window(bsg_ctx* ctx, uint8_t** p, size_t* cap);
int bsg_write_commit(bsg_ctx* ctx, size_t n);
/* Page-locks host memory the caller owns (hipHostRegister) so that bsg_write_pinned can copy
 * from it to the device without a staging copy; bsg_host_unregister undoes it. */
int bsg_host_register(void* p, size_t n);
int bsg_host_unregister(void* p);
/* bsg_write from memory registered with bsg_host_register: the H2D reads p[0..n) directly and
 * asynchronously, so the caller keeps those bytes unchanged and registered until the chunks
 * covering them have been drained (at the latest, until bsg_close / bsg_reset returns). Same
 * stream semantics as bsg_write. */
int bsg_write_pinned(bsg_ctx* ctx, const uint8_t* p, size_t n);
/* Flushes the final chunk (hashsplit Splitter.Close). Idempotent. */
int bsg_close(bsg_ctx* ctx);
/* bsg_close in steps, so that a caller can Put the chunks of earlier tiles while the last ones
 * finish: bsg_close_begin submits the final segment without waiting (the stream is closed);
 * each bsg_close_step waits for the oldest tile still on the device and makes its chunks
 * drainable, storing the number of tiles still on the device in *left (0: as after bsg_close). */
int bsg_close_begin(bsg_ctx* ctx);
int bsg_close_step(bsg_ctx* ctx, size_t* left);
/* Number of finished chunks not yet drained, and drain up to cap of them (stream order). */
size_t bsg_pending(const bsg_ctx* ctx);
size_t bsg_drain(bsg_ctx* ctx, bsg_chunk* out, size_t cap);
/* Device tile size in bytes (default 256 MiB); call before the first write. Three tiles are
 * processed at once (BSG_STREAM_SLOTS overrides): tile i+1's split starts as soon as tile i's
 * boundaries are known, while tile i's SHA-256 is still running. Host bytes pass through a
 * ring of four pinned staging buffers of min(tile, 64 MiB), each copied to the device as soon
 * as it is full, into one of four device data slots (BSG_DATA_SLOTS). */
int bsg_set_tile(bsg_ctx* ctx, size_t tile_bytes);
/* Longest open chunk carried between tiles as bytes on the device (default 8 MiB); a longer
 * one is carried as a SHA-256 midstate, which makes the next tile wait for this tile's hashes.
 * 0 = always midstate (tests). Call before the first write. */
int bsg_set_carry_cap(bsg_ctx* ctx, size_t bytes);
/* Tests: the stream's first byte has stream offset `base` (records carry offsets from it, the
 * split is unchanged), so that offsets past 2^40 can be exercised without writing 1 TiB. Call
 * before the first write; bsg_reset goes back to 0. */
int bsg_set_stream_base(bsg_ctx* ctx, uint64_t base);
/* Start a new stream on the same context (its device and pinned buffers are kept), as a
 * pool of split.Writers would; undrained chunks of the previous stream are discarded. */
int bsg_reset(bsg_ctx* ctx);
void bsg_free(bsg_ctx* ctx);
/* Where a stream's host-to-device time went, since bsg_open / the last bsg_reset (a diagnostic:
 * an io.Copy into split.Writer is bound by the host copy, the PCIe copy or the device). Waits
 * for the context's copy stream. */
typedef struct bsg_stream_stats {
  uint64_t host_bytes;         /* bytes bsg_write copied into pinned staging */
  uint64_t host_copy_ns;       /* wall time of those copies (all copy threads together) */
  uint64_t stage_wait_ns;      /* time Writes waited for a stage's previous H2D copy */
  uint64_t h2d_bytes;          /* bytes copied host-to-device from the stages */
  uint64_t h2d_copies;         /* number of those copies */
  uint64_t h2d_busy_ns;        /* sum of their durations (HIP events on the copy stream) */
  uint64_t h2d_span_ns;        /* the first one's start to the last one's end */
  uint64_t copy_bytes_node[4]; /* host copy bytes by NUMA node of the copying thread's CPU */
  uint64_t last_tile_ns;       /* the final tile's kernels on the device (bsg_close's tail) */
  uint64_t tail_ns;            /* the last H2D copy's end to the final tile's records in host
                                * memory */
  int32_t gpu_node;            /* NUMA node of the device (sysfs; -1 unknown) */
  uint32_t stage_nodes;        /* bit mask of the NUMA nodes the pinned stages' pages are on */
  uint32_t src_nodes;          /* bit mask of the nodes of the Write sources' first pages */
  uint32_t copy_nt;            /* 1: the copies used non-temporal stores */
} bsg_stream_stats;
int bsg_stream_stats_get(bsg_ctx* ctx, bsg_stream_stats* out);

/* ---- device-resident batch of independent streams ---- */
typedef struct bsg_engine bsg_engine;
bsg_engine* bsg_engine_create(int device, const uint32_t* table /* 256 or NULL */, int* err);
void bsg_engine_destroy(bsg_engine* eng);
/* Enqueue split + hash of nstreams streams d_data[off[i] .. off[i]+len[i]) (device memory,
 * off[i] % 16 == 0; off/len are host arrays; at most 65,535 streams of < 2^40 bytes each, a
 * device-memory bound: one stream of a run lies whole in device memory).
 * Asynchronous on the engine's stream (a run of >= 256 MiB hashes its two longest chunks on a
 * second pooled stream, which the engine's stream waits for before the run completes; see
 * BSG_KNOB_EARLY).
 * The allocation holding d_data must extend at least BSG_READ_SLACK bytes past the end of the
 * last stream (the SHA-256 loader reads whole 64-byte blocks and masks the excess). */
#define BSG_READ_SLACK 256
int bsg_engine_run(bsg_engine* eng, const uint8_t* d_data, const uint64_t* off,
                   const uint64_t* len, uint32_t nstreams, const bsg_params* params);
/* Enqueue SHA-256 of nblobs whole blobs d_data[off[i] .. off[i]+len[i]) (bs.Blob.Ref,
 * bs.go:24-26, for many blobs at once: the read-side verification of split.Reader, a store's
 * batched Puts): same constraints as bsg_engine_run (device memory, off[i] % 16 == 0, at most
 * 65,535 blobs, BSG_READ_SLACK readable bytes after the last); no splitting, record i (after
 * bsg_engine_finish) carries blob i's ref, offset 0 and len[i]. Asynchronous. */
int bsg_engine_hash(bsg_engine* eng, const uint8_t* d_data, const uint64_t* off,
                    const uint64_t* len, uint32_t nblobs);
/* Wait for the run; handles candidate-buffer growth (re-runs once if needed). Returns the
 * total chunk count in *nchunks. */
int bsg_engine_finish(bsg_engine* eng, uint64_t* nchunks);
/* Device pointer to the run's chunk records (stream-major, offset order); valid until the
 * next run. */
const bsg_chunk* bsg_engine_chunks_device(const bsg_engine* eng);
/* Copy records / per-stream counts to host. */
int bsg_engine_copy_chunks(bsg_engine* eng, bsg_chunk* out, uint64_t cap);
int bsg_engine_copy_counts(bsg_engine* eng, uint64_t* counts, uint32_t nstreams);
/* The engine's HIP stream (hipStream_t), e.g. for event timing. */
void* bsg_engine_stream(bsg_engine* eng);
/* Per-stage HIP event timing of later runs, and the last finished run's stage durations in
 * ms: [0] rolling scan (k_scan), [1] prefix/compact/select/chunks, [2] SHA-256 (k_sha, and the
 * early chains' tail). Timed on the engine's own stream. enable: 0 off, 1 every stage (four
 * events per run), 2 the SHA-256 stage only (two events; [0] and [1] read -1). Each event on
 * the stream costs the run time. */
int bsg_engine_profile(bsg_engine* eng, int enable);
int bsg_engine_stage_ms(const bsg_engine* eng, float out[3]);
/* Diagnostics of the last run: [0] jobs on the wave-per-chunk path, [1] its block threshold,
 * [2] longest job (blocks), [3..7] one long job's s_memtime start/end, s_memrealtime
 * start/end (100 MHz) and block count, [8..12] the same for the longest per-lane job,
 * [13] per-lane job count. */
int bsg_engine_diag(const bsg_engine* eng, uint64_t out[16]);
/* Diagnostic timeline of the last run's k_sha, in 100 MHz s_memrealtime ticks: first wave
 * started, longest wave-mode job started / ended, last wave left per-lane mode. */
int bsg_engine_timeline(const bsg_engine* eng, uint64_t out[4]);
/* Last run's candidate count (diagnostics). */
uint64_t bsg_engine_candidates(const bsg_engine* eng);

/* Convenience: split + hash host-resident streams (copies to the device), results to host.
 * Any number of streams: they run in groups of at most 65,535 streams and ~8 GiB. Records are
 * in stream order, `stream` = the index in this call; at most cap are written, *nchunks is the
 * total. */
int bsg_split_hash_batch(int device, const uint8_t* host_data, const uint64_t* off,
                         const uint64_t* len, uint32_t nstreams, const bsg_params* params,
                         const uint32_t* table, bsg_chunk* out, uint64_t cap, uint64_t* counts,
                         uint64_t* nchunks);

/* Batched SHA-256 of n blobs base[off[i] .. off[i]+len[i]); base may be host or device memory;
 * refs receives n*32 bytes (host). */
int bsg_sha256_batch(int device, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                     uint32_t n, uint8_t* refs);

/* The same with persistent device buffers and a HIP stream of its own (one per thread at a
 * time), for callers that hash many small batches (tree nodes, store Puts). */
typedef struct bsg_hasher bsg_hasher;
bsg_hasher* bsg_hasher_new(int device);
int bsg_hasher_sum(bsg_hasher* h, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                   uint32_t n, uint8_t* refs);
/* The same for scattered blobs: blob i is ptrs[i][0 .. len[i]) (host memory), e.g. the chunks a
 * store holds separately. Large batches (>= 16 blobs and 4 MiB) are packed into pinned staging
 * and hashed in bsg_engine_hash mode; small ones by one blob per lane. */
int bsg_hasher_sum_ptrs(bsg_hasher* h, const uint8_t* const* ptrs, const uint64_t* len,
                        uint32_t n, uint8_t* refs);
void bsg_hasher_free(bsg_hasher* h);
/* Diagnostics: bytes of pinned host memory the hasher holds (its small-batch buffer, its
 * metadata and record buffers, its large-batch staging). A large blob hashed through the
 * small-batch path is copied from pageable memory and does not grow it. */
size_t bsg_hasher_pinned_bytes(const bsg_hasher* h);

/* Device memory helpers (so callers need no second HIP runtime): kind 0 = H2D, 1 = D2H,
 * 2 = D2D. */
void* bsg_device_malloc(int device, size_t bytes);
int bsg_device_free(int device, void* p);
int bsg_memcpy(int device, void* dst, const void* src, size_t n, int kind);
int bsg_device_synchronize(int device);

/* Utility (benchmarks/tests, not part of the reference surface): fill device memory with the
 * SplitMix64 counter stream of bs_amd/synth.py (word i = splitmix64(seed + (i+1)*0x9E37...)). */
int bsg_fill_splitmix(int device, uint8_t* d_ptr, uint64_t nbytes, uint64_t seed, void* stream);

/* ---- C++ host mirror of split.Writer / split.Reader / store/mem (bs_split.hpp), exposed for
 * C callers and tests ---- */
typedef struct bsg_store bsg_store;   /* a bs.Store; every Put's ref comes from the GPU */
bsg_store* bsg_memstore_new(int device);   /* store/mem  (store/mem/mem.go:17-124) */
/* store/file (store/file/file.go:20-154): blobs at <root>/blobs/<hex[:2]>/<hex[:4]>/<hex>. */
bsg_store* bsg_filestore_new(const char* root, int device);
void bsg_store_free(bsg_store* s);
size_t bsg_store_count(const bsg_store* s);
/* store/file writes split.Writer's chunks behind (bs::FileStore::PutBlob): at most `bytes` of
 * accepted, unwritten blobs are pending before a Put waits (default 1 GiB). BSG_EINVAL for
 * store/mem. */
int bsg_filestore_set_write_behind(bsg_store* s, uint64_t bytes);
/* Bytes of host memory a store/mem keeps alive: its own blob copies plus, once each, the Write
 * pieces its chunks alias (split.Writer hands chunks over without copying). 0 for store/file. */
size_t bsg_store_held_bytes(const bsg_store* s);
/* Get: copies min(cap, len) bytes, *n = blob length; returns BSG_ENOTFOUND if absent. */
int bsg_store_get(bsg_store* s, const uint8_t ref[32], uint8_t* out, size_t cap, size_t* n);
int bsg_store_put(bsg_store* s, const uint8_t* data, size_t n, uint8_t ref_out[32], int* added);
/* Put with a ref the caller already has (a chunk record's ref): no hash is computed, the store
 * trusts the ref (bs::RefPutter in bs_split.hpp). Needs no GPU. */
int bsg_store_put_ref(bsg_store* s, const uint8_t ref[32], const uint8_t* data, size_t n,
                      int* added);
/* ListRefs(start, f) (store.go:13-24; mem.go:39-59, file.go:83-160): refs > start in lexicographic order, up to cap of them
 * into refs (32 bytes each); returns the total count after start. */
size_t bsg_store_list_from(bsg_store* s, const uint8_t start[32], uint8_t* refs, size_t cap);
/* All refs in lexicographic order (32 bytes each, up to cap); returns the total count. */
size_t bsg_store_list(bsg_store* s, uint8_t* refs, size_t cap);
/* bs.DeleterStore.Delete (store.go:50-54) for store/mem (mem.go:79-85): absent refs are not an
 * error. BSG_EINVAL for store/file, which is not a DeleterStore in the reference. */
int bsg_store_delete(bsg_store* s, const uint8_t ref[32]);
/* split.Protect (split/split.go:306-322), gc's traversal of a split tree: the children of the
 * Node stored at ref, child nodes first (traverse[i] = 1: protect them recursively), then its
 * leaves (traverse[i] = 0). Up to cap refs (32 bytes each); *n = the number of children. */
int bsg_split_protect(bsg_store* s, const uint8_t ref[32], uint8_t* refs, uint8_t* traverse,
                      size_t cap, size_t* n);

typedef struct bsg_writer bsg_writer; /* split.NewWriter / Write / Close / Root */
bsg_writer* bsg_writer_new(int device, bsg_store* s, const bsg_params* params, size_t tile,
                           int* err);
int bsg_writer_write(bsg_writer* w, const uint8_t* p, size_t n);
int bsg_writer_close(bsg_writer* w);
/* Tests: bsg_set_stream_base for the Writer's context, before the first bsg_writer_write; the
 * Writer's tree and Root are unchanged (tree offsets start at 0, as split.Writer's). */
int bsg_writer_set_stream_base(bsg_writer* w, uint64_t base);
int bsg_writer_root(const bsg_writer* w, uint8_t out[32]);
/* Where the Writer's time went, in seconds: [0] Write copies (into its pieces and pinned
 * staging), [1] chunk records processed on its background thread (store Puts + the tree,
 * overlapping the copies), [2] Writes and Close waiting for that thread, [3] tree-node hashes
 * on the GPU, [4] Close, [5] of which waiting for the last tiles on the device, [6] tree-node
 * hash calls. */
int bsg_writer_timings(const bsg_writer* w, double out[7]);
void bsg_writer_free(bsg_writer* w);

typedef struct bsg_reader bsg_reader; /* split.NewReader / Read / Seek / Size */
bsg_reader* bsg_reader_new(bsg_store* s, const uint8_t root[32], int* err);
/* flags: BSG_READER_VERIFY = check every fetched chunk's SHA-256 against its ref: a window of
 * leaf nodes (up to 256 MiB; BSG_VERIFY_WINDOW bytes if set) per batched GPU call, the next
 * window verified in the background while this one is read; a read that needs a chunk of a
 * window that failed returns BSG_ECORRUPT. */
#define BSG_READER_VERIFY 1
bsg_reader* bsg_reader_open(bsg_store* s, const uint8_t root[32], int flags, int device,
                            int* err);
int64_t bsg_reader_read(bsg_reader* r, uint8_t* buf, size_t n); /* bytes; 0 at EOF; <0 error */
int64_t bsg_reader_seek(bsg_reader* r, int64_t off, int whence);
uint64_t bsg_reader_size(const bsg_reader* r);
/* Verify-mode diagnostics: out[0] windows verified on the reading thread, out[1] windows taken
 * from the background read-ahead, out[2] bytes verified, out[3] read-ahead windows dropped (a
 * seek made them stale). */
int bsg_reader_stats(const bsg_reader* r, uint64_t out[4]);
void bsg_reader_free(bsg_reader* r);

/* ---- test and debug knobs (process-wide; each starts from its environment variable) ---- */
#define BSG_KNOB_SEQ_WAIT 1      /* BSG_DEBUG_SEQ_WAIT: polls of a k_sha helper handshake before
                                  * it flags a device error (0: fail at once; tests) */
#define BSG_KNOB_LONG_MODE 2     /* BSG_LONG_MODE: wave-mode tiers 0 auto, 1 off, 2 all */
#define BSG_KNOB_VERIFY_WINDOW 3 /* BSG_VERIFY_WINDOW: split::Reader verify window in bytes
                                  * (0: 256 MiB), read when a Reader is opened */
#define BSG_KNOB_EARLY 4         /* BSG_EARLY: 1 (default) hashes the two longest chunks whose
                                  * ends are sure boundaries on a second stream from right after
                                  * candidate compaction (engine runs of >= 256 MiB); 0 off */
#define BSG_KNOB_POLL 5          /* BSG_POLL: 1 (default) makes bsg_engine_finish poll its stream
                                  * (with a CPU pause between queries, for at most 100 ms, then it
                                  * blocks: no interrupt wake-up latency on a step-sized run); 0
                                  * blocks in hipStreamSynchronize at once */
#define BSG_KNOB_COPY_NT 6       /* BSG_COPY_NT: 1 (default) copies Write bytes into pinned
                                  * staging (and the Writer's pieces) with non-temporal stores;
                                  * 0 uses memcpy */
#define BSG_KNOB_LIGHT_BYTES 7  /* engine runs of at most this many bytes (default 4 GiB) keep
                                  * their early chains on the engine stream and move selection
                                  * and k_sha to the second stream; larger runs the other way
                                  * (tests run one input both ways) */
#define BSG_KNOB_LAST BSG_KNOB_LIGHT_BYTES
int bsg_debug_set(int knob, int64_t value);
int64_t bsg_debug_get(int knob); /* -1 for an unknown knob */

#ifdef __cplusplus
}
#endif
#endif /* BSGPU_H */

/*
 * bsoracle.h — CPU ORACLE (test infrastructure only).
 *
 * A plain-C restatement of the reference's hashsplit + SHA-256 ref path, used ONLY as the
 * checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg. Nothing in the
 * product path (bs_amd/, libbsgpu) links, loads or calls this code.
 *
 * What it restates (see bsoracle.c for per-function citations):
 *   - bs.Blob.Ref()            = sha256.Sum256          /root/reference/bs.go:24-26
 *   - split.NewWriter defaults  MinSize=1024, SplitBits=16, fanout=8
 *                                                       /root/reference/split/split.go:48,88-89
 *   - hashsplit.Splitter (github.com/bobg/hashsplit v1.1.1, go.mod:9) and buzhash32
 *     (github.com/chmduquesne/rollinghash v4.0.0+incompatible, go.sum:61-62). Neither module's
 *     source is in /root/reference; their algorithms are restated from their published source
 *     (recalled) — see DESIGN.md "Oracle and parity status".
 *   - buzhash32 default table = GenerateHashes(1) = Go math/rand (rngSource, seed 1):
 *     reproduced from Go's published algorithm. Pinned by known-answer values of Go's
 *     rand.New(rand.NewSource(1)).Int63() (tests/golden/go_rand_kat.json).
 */
#ifndef BSORACLE_H
#define BSORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct bso_chunk {
    uint64_t offset;  /* stream offset of the first byte */
    uint64_t len;     /* chunk length in bytes */
    uint32_t level;   /* hashsplit level (trailing zeros - split_bits), before /fanout */
    uint32_t stream;  /* stream index (multi-stream API) */
    uint8_t ref[32];  /* SHA-256 of the chunk bytes */
} bso_chunk;          /* 56 bytes, identical layout to bsg_chunk in include/bsgpu.h */

/* ---- Go math/rand restatement ---- */
void bso_gorand_seed(int64_t seed);      /* rand.NewSource(seed) (global oracle instance) */
int64_t bso_gorand_int63(void);          /* Source.Int63() */

/* ---- buzhash32 ---- */
void bso_buzhash32_generate(int64_t seed, uint32_t out[256]); /* rollinghash GenerateHashes */
/* h(p) for every position p of x (window 64, zero-primed): out[p] */
void bso_rolling_sums(const uint32_t table[256], const uint8_t* x, size_t n, uint32_t* out);

/* ---- SHA-256 (FIPS 180-4) ---- */
void bso_sha256(const uint8_t* data, size_t n, uint8_t out[32]);
/* Which compression bso_sha256 uses: 1 = x86 SHA extensions (detected by cpuid, the default
 * when present, as Go's crypto/sha256 does on amd64), 0 = portable scalar C. */
int bso_sha256_impl(void);
/* Select it (want_ni = 0 forces scalar); returns the implementation now in use. */
int bso_sha256_use(int want_ni);

/* ---- hashsplit Splitter restatement (per byte, literal) ----
 * Returns the number of chunks; writes at most `cap` chunk records (offset/len/level, and the
 * SHA-256 ref when with_refs != 0). Call with cap=0 to count. */
size_t bso_split(const uint32_t table[256], const uint8_t* x, size_t n, unsigned split_bits,
                 unsigned min_size, int with_refs, bso_chunk* out, size_t cap);

/* Multi-stream split+ref with `threads` worker threads (one stream per task). Streams are
 * [base+off[i], base+off[i]+len[i]). Chunks are written stream-major into out (cap records);
 * counts[i] receives stream i's chunk count. Returns the total chunk count. */
size_t bso_split_streams(const uint32_t table[256], const uint8_t* base, const uint64_t* off,
                         const uint64_t* len, uint32_t nstreams, unsigned split_bits,
                         unsigned min_size, int threads, bso_chunk* out, size_t cap,
                         uint64_t* counts);

/* split.Writer end to end: Splitter, TreeBuilder (level / fanout), F, PutProto, Close ->
 * root = Writer.Root (bs.Zero for no input). keep_copies != 0 also copies every blob as a
 * store/mem Put of Go's appended chunk would (the "full Writer" CPU baseline); returns the
 * number of blobs put (with keep_copies) or 0. The TreeBuilder rules are recalled
 * (Go-unpinned), the same as oracle.py's py_tree_root. */
size_t bso_writer_root(const uint32_t table[256], const uint8_t* x, size_t n, unsigned split_bits,
                       unsigned min_size, unsigned fanout, int keep_copies, uint8_t root[32]);
size_t bso_writer_root_fold(const uint32_t table[256], const uint8_t* x, size_t n,
                            unsigned split_bits, unsigned min_size, unsigned fanout,
                            int keep_copies, int fold_mode, uint8_t root[32]);

#ifdef __cplusplus
}
#endif
#endif

/*
 * bsoracle.c — CPU ORACLE (test infrastructure only; see bsoracle.h).
 *
 * Plain scalar C restatement of the reference's split + ref path. It is the CHECKER for the
 * HIP path and the "port" CPU baseline in bench.py. It is never linked into libbsgpu.
 *
 * Provenance of each piece (the reference is Go; the per-byte loop lives in two third-party
 * modules that are NOT in /root/reference):
 *   gorand_*     Go stdlib math/rand rngSource (rng.go: seedrand, Seed, Uint64/Int63) and the
 *                rngCooked table, which Go generates with gen_cooked.go (ALFG run 7.8e12
 *                steps from srand(1)). We regenerate rngCooked by polynomial jump-ahead of the
 *                lagged-Fibonacci recurrence. Pinned: rand.NewSource(1).Int63() must yield
 *                5577006791947779410, 8674665223082153551, ... (tests/golden/go_rand_kat.json).
 *   buzhash32_*  github.com/chmduquesne/rollinghash v4.0.0+incompatible, buzhash32:
 *                GenerateHashes(seed) (uint32(rand.Int63()), skipping duplicates), New() uses
 *                GenerateHashes(1); Write(window) primes; Roll(c):
 *                  sum = rotl(sum,1) ^ rotl(T[oldest], len(window) % 32) ^ T[c].   [recalled]
 *   split_*      github.com/bobg/hashsplit v1.1.1 Splitter: NewSplitter writes 64 zero bytes
 *                into the buzhash (window 64); Write appends each byte, Rolls it, and once
 *                len(chunk) >= MinSize checks tz = TrailingZeros32(Sum32()); tz >= SplitBits
 *                => emit (chunk, level = tz - SplitBits), chunk = nil, no reset (Reset=false).
 *                Close emits the non-empty remainder with level from the same check (0 if the
 *                check fails).                                                      [recalled]
 *                BS wiring: split/split.go:85-89 (callback, MinSize 1024, SplitBits 16).
 *   sha256       FIPS 180-4; bs.Blob.Ref (bs.go:24-26) = crypto/sha256.Sum256. Scalar, or with
 *                the x86 SHA extensions when the host has them (as Go's amd64 crypto/sha256).
 */
#include "bsoracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------
 * Go math/rand (rngSource) restatement.
 * ---------------------------------------------------------------------------------------- */
#define RNG_LEN 607
#define RNG_TAP 273
#define INT32MAX 2147483647

static int32_t gorand_seedrand(int32_t x) { /* x[n+1] = 48271 * x[n] mod (2**31 - 1) */
    const int32_t A = 48271, Q = 44488, R = 3399;
    int32_t hi = x / Q, lo = x % Q;
    x = A * lo - R * hi;
    if (x < 0) x += INT32MAX;
    return x;
}

/* p(x) = x^607 - x^334 - 1 over Z/2^64: the characteristic polynomial of
 * y[n] = y[n-607] + y[n-273] (the ALFG output sequence). out = a*b mod p. */
static void gorand_polymulmod(const uint64_t* a, const uint64_t* b, uint64_t* out) {
    uint64_t t[2 * RNG_LEN];
    memset(t, 0, sizeof t);
    for (int i = 0; i < RNG_LEN; i++) {
        if (!a[i]) continue;
        for (int j = 0; j < RNG_LEN; j++) t[i + j] += a[i] * b[j];
    }
    for (int k = 2 * RNG_LEN - 2; k >= RNG_LEN; k--) {
        uint64_t c = t[k];
        if (!c) continue;
        t[k] = 0;
        t[k - RNG_LEN + 334] += c;
        t[k - RNG_LEN] += c;
    }
    memcpy(out, t, RNG_LEN * sizeof(uint64_t));
}

static uint64_t g_cooked[RNG_LEN];
static int g_cooked_ready;
static pthread_mutex_t g_cooked_mu = PTHREAD_MUTEX_INITIALIZER;

/* gen_cooked.go: srand(1) with (<<20, <<10) mixing, then 7.8e12 vrand() calls; rngCooked is
 * the resulting 607-word feedback register. Computed here by jump-ahead (milliseconds). */
static void gorand_make_cooked(void) {
    pthread_mutex_lock(&g_cooked_mu);
    if (g_cooked_ready) { pthread_mutex_unlock(&g_cooked_mu); return; }
    uint64_t vec[RNG_LEN];
    int tap = 0, feed = RNG_LEN - RNG_TAP;
    int32_t x = 1;
    for (int i = -20; i < RNG_LEN; i++) {
        x = gorand_seedrand(x);
        if (i >= 0) {
            uint64_t u = (uint64_t)(int64_t)x << 20;
            x = gorand_seedrand(x);
            u ^= (uint64_t)(int64_t)x << 10;
            x = gorand_seedrand(x);
            u ^= (uint64_t)(int64_t)x;
            vec[i] = u;
        }
    }
    uint64_t y[RNG_LEN]; /* first 607 outputs: the basis of the recurrence */
    for (int i = 0; i < RNG_LEN; i++) {
        if (--tap < 0) tap += RNG_LEN;
        if (--feed < 0) feed += RNG_LEN;
        vec[feed] += vec[tap];
        y[i] = vec[feed];
    }
    const uint64_t M = 7800000000000ULL; /* calls made by gen_cooked.go */
    uint64_t e = M - RNG_LEN;
    uint64_t c[RNG_LEN], b[RNG_LEN], tmp[RNG_LEN];
    memset(c, 0, sizeof c); c[0] = 1;  /* c = x^0 */
    memset(b, 0, sizeof b); b[1] = 1;  /* b = x^1 */
    while (e) {
        if (e & 1) { gorand_polymulmod(c, b, tmp); memcpy(c, tmp, sizeof c); }
        e >>= 1;
        if (e) { gorand_polymulmod(b, b, tmp); memcpy(b, tmp, sizeof b); }
    }
    /* outputs M-607 .. M-1; output n was stored at vec[(334 - (n+1)) mod 607] */
    for (int j = 0; j < RNG_LEN; j++) {
        uint64_t v = 0;
        for (int i = 0; i < RNG_LEN; i++) v += c[i] * y[i];
        uint64_t n = M - RNG_LEN + (uint64_t)j;
        int idx = (int)(((int64_t)334 - (int64_t)((n + 1) % RNG_LEN) + 2 * RNG_LEN) % RNG_LEN);
        g_cooked[idx] = v;
        uint64_t top = c[RNG_LEN - 1]; /* c *= x (mod p) */
        memmove(c + 1, c, (RNG_LEN - 1) * sizeof(uint64_t));
        c[0] = top;
        c[334] += top;
    }
    g_cooked_ready = 1;
    pthread_mutex_unlock(&g_cooked_mu);
}

typedef struct { int tap, feed; uint64_t vec[RNG_LEN]; } gorand_src;

static void gorand_src_seed(gorand_src* r, int64_t seed) { /* rng.go rngSource.Seed */
    gorand_make_cooked();
    r->tap = 0;
    r->feed = RNG_LEN - RNG_TAP;
    seed = seed % INT32MAX;
    if (seed < 0) seed += INT32MAX;
    if (seed == 0) seed = 89482311;
    int32_t x = (int32_t)seed;
    for (int i = -20; i < RNG_LEN; i++) {
        x = gorand_seedrand(x);
        if (i >= 0) {
            uint64_t u = (uint64_t)(int64_t)x << 40;
            x = gorand_seedrand(x);
            u ^= (uint64_t)(int64_t)x << 20;
            x = gorand_seedrand(x);
            u ^= (uint64_t)(int64_t)x;
            u ^= g_cooked[i];
            r->vec[i] = u;
        }
    }
}

static int64_t gorand_src_int63(gorand_src* r) { /* rngSource.Uint64() & rngMask */
    if (--r->tap < 0) r->tap += RNG_LEN;
    if (--r->feed < 0) r->feed += RNG_LEN;
    uint64_t x = r->vec[r->feed] + r->vec[r->tap];
    r->vec[r->feed] = x;
    return (int64_t)(x & 0x7fffffffffffffffULL);
}

static gorand_src g_src;
void bso_gorand_seed(int64_t seed) { gorand_src_seed(&g_src, seed); }
int64_t bso_gorand_int63(void) { return gorand_src_int63(&g_src); }

/* ------------------------------------------------------------------------------------------
 * buzhash32 (rollinghash v4.0.0) restatement.
 * ---------------------------------------------------------------------------------------- */
void bso_buzhash32_generate(int64_t seed, uint32_t out[256]) { /* GenerateHashes(seed) */
    gorand_src r;
    gorand_src_seed(&r, seed);
    for (int i = 0; i < 256; i++) {
        uint32_t x;
        for (;;) { /* `for used[x] { x = uint32(random.Int63()) }` */
            x = (uint32_t)gorand_src_int63(&r);
            int dup = 0;
            for (int j = 0; j < i; j++) dup |= (out[j] == x);
            if (!dup) break;
        }
        out[i] = x;
    }
}

static inline uint32_t rotl32(uint32_t x, unsigned r) {
    r &= 31;
    return r ? (x << r) | (x >> (32 - r)) : x;
}

typedef struct { /* Buzhash32 with a 64-byte window */
    uint32_t sum;
    uint8_t window[64];
    int oldest;
    unsigned nrotate; /* len(window) % 32 */
    const uint32_t* T;
} buzhash32;

static void buzhash32_init_zero(buzhash32* d, const uint32_t* T) {
    /* NewSplitter: rs := buzhash32.New(); rs.Write(zeroes[:64]) */
    d->T = T;
    d->sum = 0;
    memset(d->window, 0, sizeof d->window);
    d->oldest = 0;
    for (int i = 0; i < 64; i++) d->sum = rotl32(d->sum, 1) ^ T[0];
    d->nrotate = 64 % 32;
}

static inline void buzhash32_roll(buzhash32* d, uint8_t c) {
    uint32_t hn = d->T[c];
    uint32_t h0 = d->T[d->window[d->oldest]];
    d->window[d->oldest] = c;
    if (++d->oldest >= 64) d->oldest = 0;
    d->sum = rotl32(d->sum, 1) ^ rotl32(h0, d->nrotate) ^ hn;
}

void bso_rolling_sums(const uint32_t table[256], const uint8_t* x, size_t n, uint32_t* out) {
    buzhash32 d;
    buzhash32_init_zero(&d, table);
    for (size_t p = 0; p < n; p++) {
        buzhash32_roll(&d, x[p]);
        out[p] = d.sum;
    }
}

/* ------------------------------------------------------------------------------------------
 * SHA-256, FIPS 180-4 §6.2.
 * ---------------------------------------------------------------------------------------- */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static inline uint32_t rotr32(uint32_t x, unsigned r) { return (x >> r) | (x << (32 - r)); }

static void sha256_block(uint32_t st[8], const uint8_t* p) {
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
        w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) |
               ((uint32_t)p[4 * i + 2] << 8) | p[4 * i + 3];
    for (int i = 16; i < 64; i++) {
        uint32_t s0 = rotr32(w[i - 15], 7) ^ rotr32(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = rotr32(w[i - 2], 17) ^ rotr32(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 64; i++) {
        uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
        uint32_t ch = (e & f) ^ (~e & g);
        uint32_t t1 = h + S1 + ch + K256[i] + w[i];
        uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
        uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        uint32_t t2 = S0 + mj;
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

/* The same compression with the x86 SHA extensions (SHA-NI), when the host has them. Go's
 * crypto/sha256 (bs.go:25) uses them on amd64 (sha256block_amd64.s), so the CPU baseline uses
 * them too; both implementations are checked against each other and the FIPS/hashlib vectors.
 * The state is kept as the instructions want it: ABEF in one register, CDGH in the other.
 * Group g of four rounds adds K[4g..4g+3] to message words W[4g..4g+3]; W[16..63] come from
 * sha256msg1 (sigma0 part, issued three groups ahead) and sha256msg2 (sigma1 part). */
#if defined(__x86_64__)
#include <cpuid.h>
#include <immintrin.h>
__attribute__((target("sha,sse4.1,ssse3")))
static void sha256_blocks_ni(uint32_t st[8], const uint8_t* p, size_t nblocks) {
    const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
    __m128i t = _mm_loadu_si128((const __m128i*)&st[0]);    /* A B C D (low to high) */
    __m128i s1 = _mm_loadu_si128((const __m128i*)&st[4]);   /* E F G H */
    t = _mm_shuffle_epi32(t, 0xB1);                          /* B A D C */
    s1 = _mm_shuffle_epi32(s1, 0x1B);                        /* H G F E */
    __m128i s0 = _mm_alignr_epi8(t, s1, 8);                  /* F E B A = "ABEF" */
    s1 = _mm_blend_epi16(s1, t, 0xF0);                       /* H G D C = "CDGH" */
    for (size_t b = 0; b < nblocks; b++, p += 64) {
        const __m128i save0 = s0, save1 = s1;
        __m128i m[4];
        for (int i = 0; i < 4; i++)
            m[i] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(p + 16 * i)), bswap);
        for (int g = 0; g < 16; g++) {
            __m128i k = _mm_add_epi32(m[g & 3], _mm_loadu_si128((const __m128i*)&K256[4 * g]));
            s1 = _mm_sha256rnds2_epu32(s1, s0, k);
            if (g >= 3 && g <= 14) /* W[4g+4..4g+7], before m[(g-1)&3] takes its msg1 below */
                m[(g + 1) & 3] = _mm_sha256msg2_epu32(
                    _mm_add_epi32(m[(g + 1) & 3], _mm_alignr_epi8(m[g & 3], m[(g - 1) & 3], 4)),
                    m[g & 3]);
            s0 = _mm_sha256rnds2_epu32(s0, s1, _mm_shuffle_epi32(k, 0x0E));
            if (g >= 1 && g <= 12) m[(g - 1) & 3] = _mm_sha256msg1_epu32(m[(g - 1) & 3], m[g & 3]);
        }
        s0 = _mm_add_epi32(s0, save0);
        s1 = _mm_add_epi32(s1, save1);
    }
    t = _mm_shuffle_epi32(s0, 0x1B);                         /* A B E F */
    s1 = _mm_shuffle_epi32(s1, 0xB1);                        /* C D G H */
    s0 = _mm_blend_epi16(t, s1, 0xF0);                       /* A B C D */
    s1 = _mm_alignr_epi8(s1, t, 8);                          /* E F G H */
    _mm_storeu_si128((__m128i*)&st[0], s0);
    _mm_storeu_si128((__m128i*)&st[4], s1);
}

static int host_has_sha_ni(void) {
    unsigned a, b, c, d;
    if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return 0;
    if (!(b & (1u << 29))) return 0;                      /* SHA */
    if (!__get_cpuid(1, &a, &b, &c, &d)) return 0;
    return (c & (1u << 19)) && (c & (1u << 9));           /* SSE4.1, SSSE3 */
}
#else
static void sha256_blocks_ni(uint32_t st[8], const uint8_t* p, size_t nblocks) {
    (void)st; (void)p; (void)nblocks;
}
static int host_has_sha_ni(void) { return 0; }
#endif

/* -1: not probed; 0: scalar; 1: SHA-NI. bso_sha256_use(0) forces scalar (tests). */
static volatile int g_sha_impl = -1;

int bso_sha256_use(int want_ni) {
    g_sha_impl = (want_ni && host_has_sha_ni()) ? 1 : 0;
    return g_sha_impl;
}

int bso_sha256_impl(void) {
    if (g_sha_impl < 0) g_sha_impl = host_has_sha_ni();
    return g_sha_impl;
}

static void sha256_blocks(uint32_t st[8], const uint8_t* p, size_t nblocks) {
    if (bso_sha256_impl() == 1) {
        sha256_blocks_ni(st, p, nblocks);
        return;
    }
    for (size_t i = 0; i < nblocks; i++) sha256_block(st, p + 64 * i);
}

void bso_sha256(const uint8_t* data, size_t n, uint8_t out[32]) {
    uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                      0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    size_t full = n / 64;
    sha256_blocks(st, data, full);
    uint8_t tail[128];
    size_t r = n - 64 * full;
    memset(tail, 0, sizeof tail);
    memcpy(tail, data + 64 * full, r);
    tail[r] = 0x80;
    size_t tl = (r + 9 <= 64) ? 64 : 128;
    uint64_t bits = (uint64_t)n * 8;
    for (int i = 0; i < 8; i++) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
    sha256_blocks(st, tail, tl / 64);
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)(st[i] >> 24);
        out[4 * i + 1] = (uint8_t)(st[i] >> 16);
        out[4 * i + 2] = (uint8_t)(st[i] >> 8);
        out[4 * i + 3] = (uint8_t)st[i];
    }
}

/* ------------------------------------------------------------------------------------------
 * hashsplit.Splitter restatement (one stream).
 * ---------------------------------------------------------------------------------------- */
static inline unsigned tz32(uint32_t h) { return h ? (unsigned)__builtin_ctz(h) : 32u; }

static void emit(bso_chunk* out, size_t cap, size_t k, const uint8_t* x, uint64_t start,
                 uint64_t len, unsigned level, int with_refs, uint32_t stream) {
    if (k >= cap) return;
    out[k].offset = start;
    out[k].len = len;
    out[k].level = level;
    out[k].stream = stream;
    if (with_refs) bso_sha256(x + start, (size_t)len, out[k].ref);
    else memset(out[k].ref, 0, 32);
}

static size_t split_one(const uint32_t table[256], const uint8_t* x, size_t n, unsigned split_bits,
                        unsigned min_size, int with_refs, bso_chunk* out, size_t cap,
                        uint32_t stream) {
    buzhash32 d;
    buzhash32_init_zero(&d, table);
    if (min_size == 0) min_size = 64; /* hashsplit defaultMinSize = windowSize */
    if (split_bits == 0) split_bits = 13; /* hashsplit defaultSplitBits */
    size_t k = 0;
    uint64_t start = 0;
    /* Buzhash32.Roll with the state in locals: the window is read back from the stream (the
     * byte leaving a 64-byte window is x[p-64], or a priming zero before the stream), which is
     * what the ring buffer holds; the sum stays in a register (a uint8_t ring store would alias
     * it and force a reload per byte). */
    uint32_t sum = d.sum;
    const uint32_t T0 = table[0];
    for (size_t p = 0; p < n; p++) {
        const uint32_t h0 = p >= 64 ? table[x[p - 64]] : T0;
        sum = rotl32(sum, 1) ^ h0 ^ table[x[p]];  /* rotl(h0, 64 % 32) = h0 */
        /* s.chunk = append(s.chunk, c); s.rs.Roll(c) */
        uint64_t len = (uint64_t)p + 1 - start;
        if (len < min_size) continue;          /* if len(s.chunk) < minSize { continue } */
        unsigned tz = tz32(sum);               /* checkSplit */
        if (tz >= split_bits) {
            emit(out, cap, k, x, start, len, tz - split_bits, with_refs, stream);
            k++;
            start = (uint64_t)p + 1;           /* s.chunk = nil; Reset=false: no re-prime */
        }
    }
    d.sum = sum;
    if (start < n) {                           /* Close(): flush the remainder */
        unsigned tz = tz32(d.sum);
        unsigned level = (tz >= split_bits) ? tz - split_bits : 0;
        emit(out, cap, k, x, start, (uint64_t)n - start, level, with_refs, stream);
        k++;
    }
    return k;
}

size_t bso_split(const uint32_t table[256], const uint8_t* x, size_t n, unsigned split_bits,
                 unsigned min_size, int with_refs, bso_chunk* out, size_t cap) {
    return split_one(table, x, n, split_bits, min_size, with_refs, out, cap, 0);
}

/* ---- multi-stream, multi-threaded (one stream per task; the reference is one goroutine per
 * stream, split/split.go:30-37 has no internal parallelism) ---- */
typedef struct {
    const uint32_t* table;
    const uint8_t* base;
    const uint64_t* off;
    const uint64_t* len;
    uint32_t nstreams;
    unsigned bits, min_size;
    bso_chunk** tmp;
    size_t* cnt;
    uint32_t next;
    pthread_mutex_t mu;
} mt_job;

static void* mt_worker(void* arg) {
    mt_job* j = (mt_job*)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        uint32_t s = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (s >= j->nstreams) break;
        const uint8_t* x = j->base + j->off[s];
        size_t n = (size_t)j->len[s];
        /* one pass: every non-final chunk has >= MinSize bytes */
        const size_t ms = j->min_size ? j->min_size : 64;
        const size_t bound = n / ms + 1;
        bso_chunk* buf = (bso_chunk*)malloc(bound * sizeof(bso_chunk));
        size_t c = split_one(j->table, x, n, j->bits, j->min_size, 1, buf, bound, s);
        j->tmp[s] = buf;
        j->cnt[s] = c;
    }
    return NULL;
}

size_t bso_split_streams(const uint32_t table[256], const uint8_t* base, const uint64_t* off,
                         const uint64_t* len, uint32_t nstreams, unsigned split_bits,
                         unsigned min_size, int threads, bso_chunk* out, size_t cap,
                         uint64_t* counts) {
    mt_job j;
    j.table = table; j.base = base; j.off = off; j.len = len; j.nstreams = nstreams;
    j.bits = split_bits; j.min_size = min_size; j.next = 0;
    j.tmp = (bso_chunk**)calloc(nstreams ? nstreams : 1, sizeof(bso_chunk*));
    j.cnt = (size_t*)calloc(nstreams ? nstreams : 1, sizeof(size_t));
    pthread_mutex_init(&j.mu, NULL);
    gorand_make_cooked(); /* not needed, but keeps first-call latency out of workers */
    if (threads < 1) threads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
    for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, mt_worker, &j);
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    size_t total = 0;
    for (uint32_t s = 0; s < nstreams; s++) {
        if (counts) counts[s] = j.cnt[s];
        for (size_t i = 0; i < j.cnt[s]; i++) {
            if (total < cap) out[total] = j.tmp[s][i];
            total++;
        }
        free(j.tmp[s]);
    }
    free(th); free(j.tmp); free(j.cnt);
    pthread_mutex_destroy(&j.mu);
    return total;
}

/* ------------------------------------------------------------------------------------------
 * split.Writer end to end (CPU restatement, test infrastructure and the "full Writer" CPU
 * baseline): the Splitter above, then hashsplit's TreeBuilder as wired by split.NewWriter
 * (split/split.go:51-90: Add(chunk, level / fanout); F PutProto's child nodes and Put's chunks
 * into Node{Offset, Size, Nodes, Leaves}), Writer.Close (split.go:104-126: TreeBuilder.Root,
 * PutProto(root)). The TreeBuilder rules are restated as in oracle.py's py_tree_root (recalled,
 * Go-unpinned: DESIGN.md §2). store/mem Puts are emulated by copying each blob (Go's Splitter
 * builds every chunk by appending its bytes; mem.go:71 keeps that slice).
 * ---------------------------------------------------------------------------------------- */
typedef struct wnode wnode;
typedef struct { uint8_t ref[32]; uint64_t off; wnode* node; } wchild; /* node: child Node */
struct wnode { wchild* nodes; size_t nn; wchild* leaves; size_t nl; uint64_t offset, size; };
typedef struct { wnode** nodes; size_t nn, cn; wchild* chunks; size_t nc, cc;
                 uint64_t offset, size; } tbnode;
typedef struct {
    tbnode* lv; size_t nlv, clv;
    wnode** all; size_t nall, call;        /* every wnode made, freed at the end */
    uint8_t** blobs; size_t nblobs, cblobs; /* emulated store/mem copies */
    int keep;
    unsigned fanout;
} wstate;

static void* grow(void* p, size_t* cap, size_t need, size_t elt) {
    if (need <= *cap) return p;
    size_t nc = *cap ? *cap * 2 : 8;
    while (nc < need) nc *= 2;
    *cap = nc;
    return realloc(p, nc * elt);
}

static void ws_put(wstate* w, const uint8_t* b, size_t n, uint8_t ref[32]) {
    bso_sha256(b, n, ref);
    if (!w->keep) return;
    w->blobs = (uint8_t**)grow(w->blobs, &w->cblobs, w->nblobs + 1, sizeof(uint8_t*));
    uint8_t* c = (uint8_t*)malloc(n ? n : 1);
    memcpy(c, b, n);
    w->blobs[w->nblobs++] = c;
}

static size_t put_varint(uint8_t* o, uint64_t v) {
    size_t k = 0;
    while (v >= 0x80) { o[k++] = (uint8_t)(v | 0x80); v >>= 7; }
    o[k++] = (uint8_t)v;
    return k;
}

/* split.proto Node, deterministic proto3 as Go's proto.Marshal (fields in order, zeros
 * omitted); returns the length written into o (o must hold 50 * (nn + nl) + 24 bytes). */
static size_t marshal_node(const wnode* n, uint8_t* o) {
    size_t k = 0;
    for (int pass = 0; pass < 2; pass++) {
        const wchild* cs = pass ? n->leaves : n->nodes;
        size_t cnt = pass ? n->nl : n->nn;
        for (size_t i = 0; i < cnt; i++) {
            uint8_t c[48];
            size_t m = 0;
            c[m++] = 0x0a; c[m++] = 32;
            memcpy(c + m, cs[i].ref, 32); m += 32;
            if (cs[i].off) { c[m++] = 0x10; m += put_varint(c + m, cs[i].off); }
            o[k++] = pass ? 0x12 : 0x0a;
            k += put_varint(o + k, m);
            memcpy(o + k, c, m); k += m;
        }
    }
    if (n->offset) { o[k++] = 0x18; k += put_varint(o + k, n->offset); }
    if (n->size) { o[k++] = 0x20; k += put_varint(o + k, n->size); }
    return k;
}

static void put_node(wstate* w, const wnode* n, uint8_t ref[32]) {
    uint8_t* buf = (uint8_t*)malloc(50 * (n->nn + n->nl) + 24);
    size_t len = marshal_node(n, buf);
    ws_put(w, buf, len, ref);
    free(buf);
}

static wnode* tb_F(wstate* w, tbnode* t) { /* split/split.go:52-81 */
    wnode* n = (wnode*)calloc(1, sizeof(wnode));
    w->all = (wnode**)grow(w->all, &w->call, w->nall + 1, sizeof(wnode*));
    w->all[w->nall++] = n;
    n->offset = t->offset;
    n->size = t->size;
    uint64_t off = t->offset;
    n->nodes = (wchild*)malloc((t->nn ? t->nn : 1) * sizeof(wchild));
    for (size_t i = 0; i < t->nn; i++) {
        put_node(w, t->nodes[i], n->nodes[i].ref);  /* bs.PutProto(child) */
        n->nodes[i].off = off;
        n->nodes[i].node = t->nodes[i];
        off += t->nodes[i]->size;
    }
    n->nn = t->nn;
    n->leaves = (wchild*)malloc((t->nc ? t->nc : 1) * sizeof(wchild));
    for (size_t i = 0; i < t->nc; i++) {  /* chunks were Put when added: refs in chunks[] */
        memcpy(n->leaves[i].ref, t->chunks[i].ref, 32);
        n->leaves[i].off = off;
        n->leaves[i].node = NULL;
        off += t->chunks[i].off;  /* chunks[].off holds the chunk length */
    }
    n->nl = t->nc;
    return n;
}

static void tb_reset(tbnode* t, uint64_t offset) {
    t->nn = 0; t->nc = 0; t->offset = offset; t->size = 0;
}

static void tb_add(wstate* w, const uint8_t ref[32], uint64_t len, unsigned level) {
    if (w->nlv == 0) {
        w->lv = (tbnode*)grow(w->lv, &w->clv, 1, sizeof(tbnode));
        memset(&w->lv[0], 0, sizeof(tbnode));
        w->nlv = 1;
    }
    tbnode* l0 = &w->lv[0];
    l0->chunks = (wchild*)grow(l0->chunks, &l0->cc, l0->nc + 1, sizeof(wchild));
    memcpy(l0->chunks[l0->nc].ref, ref, 32);
    l0->chunks[l0->nc].off = len;
    l0->nc++;
    for (size_t i = 0; i < w->nlv; i++) w->lv[i].size += len;
    for (unsigned i = 0; i < level; i++) {
        if (i == w->nlv - 1) {
            w->lv = (tbnode*)grow(w->lv, &w->clv, w->nlv + 1, sizeof(tbnode));
            memset(&w->lv[w->nlv], 0, sizeof(tbnode));
            w->lv[w->nlv].offset = w->lv[i].offset;
            w->lv[w->nlv].size = w->lv[i].size;
            w->nlv++;
        }
        wnode* f = tb_F(w, &w->lv[i]);
        tbnode* up = &w->lv[i + 1];
        up->nodes = (wnode**)grow(up->nodes, &up->cn, up->nn + 1, sizeof(wnode*));
        up->nodes[up->nn++] = f;
        tb_reset(&w->lv[i], up->offset + up->size);
    }
}

size_t bso_writer_root(const uint32_t table[256], const uint8_t* x, size_t n, unsigned split_bits,
                       unsigned min_size, unsigned fanout, int keep_copies, uint8_t root[32]) {
    return bso_writer_root_fold(table, x, n, split_bits, min_size, fanout, keep_copies, 0, root);
}

/* fold_mode selects the recalled TreeBuilder.Root detail: 0 folds every
 * non-empty level below the top (the library's choice); 1 folds only when the leaf level holds
 * chunks (not when the last chunk itself closed a level). */
size_t bso_writer_root_fold(const uint32_t table[256], const uint8_t* x, size_t n,
                            unsigned split_bits, unsigned min_size, unsigned fanout,
                            int keep_copies, int fold_mode, uint8_t root[32]) {
    wstate w;
    memset(&w, 0, sizeof w);
    w.keep = keep_copies;
    w.fanout = fanout ? fanout : 1;
    memset(root, 0, 32);                      /* no input: Root stays bs.Zero */
    const size_t ms = min_size ? min_size : 64;
    const size_t bound = n / ms + 1;
    bso_chunk* ch = (bso_chunk*)malloc(bound * sizeof(bso_chunk));
    size_t nch = split_one(table, x, n, split_bits, min_size, 1, ch, bound, 0);
    for (size_t i = 0; i < nch; i++) {
        if (keep_copies) {                    /* store/mem Put of the chunk (ref known) */
            w.blobs = (uint8_t**)grow(w.blobs, &w.cblobs, w.nblobs + 1, sizeof(uint8_t*));
            uint8_t* c = (uint8_t*)malloc(ch[i].len ? ch[i].len : 1);
            memcpy(c, x + ch[i].offset, ch[i].len);
            w.blobs[w.nblobs++] = c;
        }
        tb_add(&w, ch[i].ref, ch[i].len, ch[i].level / w.fanout);  /* split/split.go:86 */
    }
    free(ch);
    size_t puts = w.nblobs;
    if (w.nlv) {
        /* TreeBuilder.Root: fold every non-empty level below the top into its parent */
        const int fold = fold_mode == 0 || w.lv[0].nc > 0;
        for (size_t i = 0; fold && i + 1 < w.nlv; i++) {
            tbnode* t = &w.lv[i];
            if (!t->nc && !t->nn) continue;
            wnode* f = tb_F(&w, t);
            tbnode* up = &w.lv[i + 1];
            up->nodes = (wnode**)grow(up->nodes, &up->cn, up->nn + 1, sizeof(wnode*));
            up->nodes[up->nn++] = f;
        }
        wnode* r;
        if (w.nlv == 1) {
            r = tb_F(&w, &w.lv[0]);
        } else {
            tbnode* top = &w.lv[w.nlv - 1];
            if (top->nn > 1) {
                r = tb_F(&w, top);
            } else {                          /* prune single-child roots (their F already ran) */
                r = top->nodes[0];
                while (r->nn == 1) r = r->nodes[0].node;
            }
        }
        put_node(&w, r, root);                /* PutProto(root) -> Writer.Root */
        puts = w.nblobs;
    }
    for (size_t i = 0; i < w.nlv; i++) { free(w.lv[i].nodes); free(w.lv[i].chunks); }
    free(w.lv);
    for (size_t i = 0; i < w.nall; i++) { free(w.all[i]->nodes); free(w.all[i]->leaves); free(w.all[i]); }
    free(w.all);
    for (size_t i = 0; i < w.nblobs; i++) free(w.blobs[i]);
    free(w.blobs);
    return puts;
}

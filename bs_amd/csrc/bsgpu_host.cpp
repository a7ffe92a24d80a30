// bsgpu_host.cpp — libbsgpu host side: device workspaces, the run pipeline and the C ABI
// declared in include/bsgpu.h.
//
// A run = one launch sequence over a batch of stream segments (bsgpu_internal.h):
//   k_start (descriptors in, counters zeroed) → k_scan (+ its exact pass) → prefix(strip counts) →
//   k_compact → k_select → prefix(flags) → k_chunks → … → k_sha (→ k_early_fix), with the early
//   chains (k_pick → k_early) on a second stream from k_compact on
// Everything after k_scan sizes itself from device-side counters, so a run never waits on the
// host; bsg_engine_finish() is the only synchronisation (and the place where a too-small
// candidate buffer is grown and the run repeated).
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <emmintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/bsgpu.h"
#include "bsgpu_internal.h"
#include "bsgpu_launch.h"
#include "buzhash32_table.inc"
#include "host_pool.h"

using namespace bsg;

static int device_node(int device);  // NUMA node of a HIP device (below)

namespace {

const uint32_t kIV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                         0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (bytes <= cap) return hipSuccess;
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = bytes + bytes / 8;  // headroom against regrowth
    hipError_t e = hipMalloc(&p, want);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      e = hipMalloc(&p, bytes);
      if (e != hipSuccess) return e;
      want = bytes;
    }
    cap = want;
    return hipSuccess;
  }
  void release() {
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T> T* as() const { return static_cast<T*>(p); }
};

// Page-locked host memory. Two kinds:
//  * kernel-visible (default): hipHostMalloc, mapped for the device, so kernels can write
//    results straight into it (records, counters, snapshots);
//  * DMA staging (dma_only): an anonymous mapping with transparent huge pages requested, pinned
//    with hipHostRegister and only ever read by hipMemcpyAsync. On the MI355X box this takes
//    17 ms per 256 MiB (mostly zero-filling the pages) and 10 ms to free, against 50-65 ms and
//    29-43 ms for hipHostMalloc / hipHostFree (tools/ubench/pin_cost.cpp,
//    profiles/r03_pin_cost.log). Falls back to hipHostMalloc if registration fails.
// Host ThreadSanitizer builds (tools/tsan_host.sh): hipHostMalloc / hipHostFree recycle pinned
// buffers between threads under the HIP runtime's own (uninstrumented) locks, which TSan cannot
// see; a release before every free and an acquire after every allocation restore the
// happens-before a real allocator lock gives, so reuse of a freed buffer by another context is
// not reported as a race.
#if defined(__has_feature)
#if __has_feature(thread_sanitizer)
#define BSG_TSAN 1
#endif
#endif
#ifdef BSG_TSAN
extern "C" void __tsan_acquire(void* addr);
extern "C" void __tsan_release(void* addr);
static char g_tsan_pinned_sync;
static inline void tsan_after_alloc() { __tsan_acquire(&g_tsan_pinned_sync); }
static inline void tsan_before_free() { __tsan_release(&g_tsan_pinned_sync); }
#else
static inline void tsan_after_alloc() {}
static inline void tsan_before_free() {}
#endif

// DMA staging pages on the current device's NUMA node (preferred, not bound: a full node falls
// back to the other). The H2D of a stage on the far node ran at 49.4-49.7 GB/s against
// 56.2-56.3 from the GPU's own node, the same box and library (profiles/r06_c6_bench1.log /
// bench2.log, bsg_stream_stats), so the 1 GiB e2e took 31.0 ms a rep instead of 28.3: the pages
// were simply placed by first touch, on whichever node the registering thread ran.
void prefer_device_node(void* m, size_t n) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    (void)hipGetLastError();
    return;
  }
  const int node = device_node(dev);
  if (node < 0 || node >= 64) return;
  const unsigned long mask = 1ul << node;
  (void)syscall(SYS_mbind, m, n, 1 /* MPOL_PREFERRED */, &mask, 64UL, 0U);
}

struct PinBuf {
  void* p = nullptr;
  size_t cap = 0;
  bool dma_only = false;
  size_t map_len = 0;  // > 0: p is an mmap of map_len bytes registered with hipHostRegister
  // the device-side address of p (kernels write results straight into pinned host memory)
  void* dev() const {
    void* d = nullptr;
    if (p && hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
      (void)hipGetLastError();
      d = nullptr;
    }
    return d;
  }
  static constexpr size_t kHuge = 2ull << 20;
  // allocates into (*q, *len): *len > 0 for the registered mapping, 0 for hipHostMalloc
  hipError_t alloc(size_t bytes, void** q, size_t* len) const {
    *q = nullptr;
    *len = 0;
    if (dma_only && bytes >= kHuge) {
      const size_t n = (bytes + kHuge - 1) & ~(kHuge - 1);
      void* m = ::mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
      if (m != MAP_FAILED) {
        (void)::madvise(m, n, MADV_HUGEPAGE);
        prefer_device_node(m, n);  // before the registration faults the pages in
        if (hipHostRegister(m, n, hipHostRegisterDefault) == hipSuccess) {
          *q = m;
          *len = n;
          return hipSuccess;
        }
        (void)hipGetLastError();
        ::munmap(m, n);
      }
    }
    const hipError_t e = hipHostMalloc(q, bytes, hipHostMallocDefault);
    tsan_after_alloc();
    return e;
  }
  static void free_(void* q, size_t len) {
    if (!q) return;
    if (len) {
      (void)hipHostUnregister(q);
      ::munmap(q, len);
    } else {
      tsan_before_free();
      (void)hipHostFree(q);
    }
  }
  hipError_t ensure(size_t bytes) { return grow(bytes, 0); }
  // ensure() that keeps the first `keep` bytes
  hipError_t grow(size_t bytes, size_t keep) {
    if (bytes == 0) bytes = 16;
    if (bytes <= cap) return hipSuccess;
    void* q = nullptr;
    size_t len = 0;
    hipError_t e = alloc(bytes, &q, &len);
    if (e != hipSuccess) return e;
    if (keep) std::memcpy(q, p, keep);
    free_(p, map_len);
    p = q;
    map_len = len;
    cap = len ? len : bytes;
    return hipSuccess;
  }
  void release() {
    free_(p, map_len);
    p = nullptr;
    cap = 0;
    map_len = 0;
  }
  template <class T> T* as() const { return static_cast<T*>(p); }
};

int herr(hipError_t e) { return e == hipSuccess ? BSG_OK : BSG_EDEVICE; }

// HIP streams come from a process-wide pool per device: creating one costs 12-13 ms for each
// of the process's first four (each gets a hardware queue) and ~4 ms after, destroying one
// ~3 ms (tools/ubench/first_use.hip, profiles/r03_first_use.log), which a context per file and
// an engine per tile slot paid every time. Streams go back to the pool instead.
constexpr size_t kStreamPoolMax = 32;
std::mutex g_stream_mu;
std::vector<hipStream_t>& stream_pool(int device) {
  static auto* pools = new std::vector<std::vector<hipStream_t>>(64);  // never destroyed
  return (*pools)[(size_t)device & 63];
}
hipError_t stream_acquire(int device, hipStream_t* s) {
  {
    std::lock_guard<std::mutex> g(g_stream_mu);
    auto& v = stream_pool(device);
    if (!v.empty()) {
      *s = v.back();
      v.pop_back();
      return hipSuccess;
    }
  }
  return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}
// The stream must be idle (callers synchronise it first); the device must be current.
void stream_release(int device, hipStream_t s) {
  if (!s) return;
  {
    std::lock_guard<std::mutex> g(g_stream_mu);
    auto& v = stream_pool(device);
    if (v.size() < kStreamPoolMax) {
      v.push_back(s);
      return;
    }
  }
  (void)hipStreamDestroy(s);
}

// CUs of a device (one attribute query; the device-properties call fills the whole struct and
// costs milliseconds, which an engine per tile slot paid on every bsg_open)
int device_cus(int device) {
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
      n <= 0) {
    (void)hipGetLastError();
    n = 256;
  }
  return n;
}

// BSG_DEBUG_SYNC=1: synchronise and report after every launch (debugging hangs/faults)
bool debug_sync() {
  static const bool v = [] {
    const char* e = std::getenv("BSG_DEBUG_SYNC");
    return e && *e == '1';
  }();
  return v;
}
hipError_t dbg(const char* what, hipStream_t s, hipError_t e) {
  if (!debug_sync() || e != hipSuccess) return e;
  std::fprintf(stderr, "bsgpu: %s ...", what);
  std::fflush(stderr);
  e = hipStreamSynchronize(s);
  std::fprintf(stderr, " %s\n", hipGetErrorString(e));
  std::fflush(stderr);
  return e;
}

// Test and debug knobs (bsg_debug_set). Each starts from its environment variable, read once
// (a getenv racing a test's setenv on another thread is a data race in glibc), and tests change
// it through bsg_debug_set instead of the environment.
std::atomic<int64_t>& knob(int k) {
  static std::atomic<int64_t> seq_wait{[] {
    // polls of a k_sha helper-wave handshake before it gives up and flags a device error
    // (~1 s); 0 makes every handshake fail at once, which is how the tests drive the
    // device-error path (Counters::error -> BSG_EDEVICE)
    const char* e = std::getenv("BSG_DEBUG_SEQ_WAIT");
    return e ? (int64_t)std::strtoul(e, nullptr, 10) : (int64_t)(1u << 24);
  }()};
  static std::atomic<int64_t> long_mode{[] {  // BSG_LONG_MODE = off | all (experiments)
    const char* e = std::getenv("BSG_LONG_MODE");
    if (e && !std::strcmp(e, "off")) return (int64_t)1;
    if (e && !std::strcmp(e, "all")) return (int64_t)2;
    return (int64_t)0;
  }()};
  static std::atomic<int64_t> verify_window{[] {  // split::Reader window (0: 256 MiB)
    const char* e = std::getenv("BSG_VERIFY_WINDOW");
    return e ? (int64_t)std::strtoull(e, nullptr, 10) : (int64_t)0;
  }()};
  static std::atomic<int64_t> early{[] {  // early chains (Early): 1 on, 0 off
    const char* e = std::getenv("BSG_EARLY");
    return e ? (int64_t)std::strtoull(e, nullptr, 10) : (int64_t)1;
  }()};
  static std::atomic<int64_t> poll{[] {  // bsg_engine_finish: 1 polls the stream, 0 blocks
    const char* e = std::getenv("BSG_POLL");
    return e ? (int64_t)(std::strtoull(e, nullptr, 10) != 0) : (int64_t)1;
  }()};
  static std::atomic<int64_t> copy_nt{[] {  // Write copies: 1 non-temporal stores, 0 memcpy
    const char* e = std::getenv("BSG_COPY_NT");
    return e ? (int64_t)(std::strtoull(e, nullptr, 10) != 0) : (int64_t)1;
  }()};
  static std::atomic<int64_t> light_bytes{(int64_t)(4ull << 30)};  // engine runs: light schedule
  static std::atomic<int64_t> none{0};
  switch (k) {
    case BSG_KNOB_SEQ_WAIT: return seq_wait;
    case BSG_KNOB_LONG_MODE: return long_mode;
    case BSG_KNOB_VERIFY_WINDOW: return verify_window;
    case BSG_KNOB_EARLY: return early;
    case BSG_KNOB_POLL: return poll;
    case BSG_KNOB_COPY_NT: return copy_nt;
    case BSG_KNOB_LIGHT_BYTES: return light_bytes;
    default: return none;
  }
}
// bsg_engine_finish's wait. hipStreamSynchronize sleeps on an interrupt once its short active
// wait has passed and woke 7-43 us after the engine stream's last command ended (a configs[1]
// step is ~9 ms; tools/step_gaps.py, profiles/r05_step_gaps.txt). BSG_KNOB_POLL (default on)
// queries the stream instead, with a CPU pause between queries, for at most kPollMaxNs (a run
// longer than that pays the wake-up once, relatively nothing) and then blocks: no wake-up latency
// on a step-sized run, and no core spinning without bound.
constexpr int64_t kPollMaxNs = 100'000'000;
hipError_t stream_wait(hipStream_t s) {
  if (!knob(BSG_KNOB_POLL).load(std::memory_order_relaxed)) return hipStreamSynchronize(s);
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t e = hipStreamQuery(s);
    if (e != hipErrorNotReady) return e;
    (void)hipGetLastError();
    for (int i = 0; i < 32; ++i) _mm_pause();
    if (std::chrono::steady_clock::now() - t0 > std::chrono::nanoseconds(kPollMaxNs))
      return hipStreamSynchronize(s);
  }
}
uint32_t seq_wait_limit() { return (uint32_t)knob(BSG_KNOB_SEQ_WAIT).load(); }
int long_mode() { return (int)knob(BSG_KNOB_LONG_MODE).load(); }

#define HCHECK(x)                           \
  do {                                      \
    hipError_t e_ = (x);                    \
    if (e_ != hipSuccess) {                 \
      (void)hipGetLastError();              \
      return BSG_EDEVICE;                   \
    }                                       \
  } while (0)

int normalize(const bsg_params* in, Params* out, bsg_params* norm) {
  bsg_params p = in ? *in : bsg_params_default();
  // Every value split.Bits / split.MinSize accept (split/split.go:137-152 store them unchecked)
  // is valid: 0 takes hashsplit's default (SplitBits 13, MinSize 64 = the window); MinSize 1..63
  // lets a window span a boundary (the hash still depends only on the last 64 stream bytes, so
  // nothing changes but the greedy rule); Bits > 32 can never be met by TrailingZeros32 (<= 32),
  // so the stream is one final chunk. fanout 0 is our C default (Fanout(0) in Go would divide by
  // zero in split.go:86).
  if (p.split_bits == 0) p.split_bits = 13;  // hashsplit defaultSplitBits
  if (p.min_size == 0) p.min_size = 64;      // hashsplit defaultMinSize (window size)
  if (p.fanout == 0) p.fanout = 8;
  out->split_bits = p.split_bits;
  out->min_size = p.min_size;
  out->mask = p.split_bits >= 32 ? 0xffffffffu : ((1u << p.split_bits) - 1u);
  out->pad_ = 0;
  if (norm) *norm = p;
  return BSG_OK;
}

}  // namespace

struct bsg_engine {
  int dev = 0;
  int num_cus = 256;
  hipStream_t stream = nullptr;
  DevBuf table, streams, strip0, counts, refine, slots, strip_off, partials_a, partials_b, cand, flags,
      fidx, bnd_end, bnd_info, scount, last_end, out, carry, ctr, long_list, order, buckets, jinfo, jdesc,
      regions, oreg, rorder;
  PinBuf h_streams, h_strip0, h_ctr;
  uint32_t htable[256];  // the table in `table` (a pooled batch engine may get another one)
  // Optional snapshot right after selection (streaming pipeline): the counters and every
  // stream's last chunk end land in pinned memory and sel_ev fires, long before k_sha ends.
  bool snapshot = false;
  PinBuf h_snap;  // Counters, then nstreams x u64 last_end
  hipEvent_t sel_ev = nullptr;
  // current run
  const uint8_t* d_data = nullptr;
  std::vector<StreamDesc> descs;
  Params p{};
  uint64_t nstrips = 0, cand_cap = 0, chunk_cap = 0;
  uint64_t data_span = 1;  // bytes from d_data to the end of the last stream (k_sha regions)
  uint64_t retry_cap = 0;  // exact candidate capacity after an overflow (one re-run)
  uint32_t nstreams = 0;
  bool enqueued = false;
  bool hash_mode = false;  // bsg_engine_hash: every stream is one blob (enqueue_hash)
  int hash_long_mode = -1;  // >= 0: enqueue_hash's SHA path choice instead of the knob's
  Counters last{};
  // optional per-stage HIP events on the engine stream: [scan, compact..chunks, sha]
  int profile = 0;  // bsg_engine_profile mode
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  float stage_ms[3] = {0, 0, 0};
  // Early chains (bsgpu_internal.h, Early): the two longest sure chunks hashed on a second
  // stream from right after k_compact. The Early record lives after the Counters in `ctr`, so
  // the run's one memset clears both.
  hipStream_t estream = nullptr;
  hipEvent_t cand_ev = nullptr, pick_ev = nullptr, early_ev = nullptr;
  bool early_open = false;  // chains launched whose end the engine stream does not wait for yet
  static constexpr uint64_t kEarlyMinBytes = 256ull << 20;  // smaller runs: not worth a stream
  uint64_t early_min = kEarlyMinBytes;  // bsg_init's warm-up run lowers it to load the kernels
  bool early_ok() const {
    return !snapshot && !hash_mode && knob(BSG_KNOB_EARLY) != 0;
  }

  // Round 5: a lightly loaded run (at most BSG_KNOB_LIGHT_BYTES, default 4 GiB, where the
  // longest chunk's chain is the step: configs[1], [3], [4]) keeps its early chains on the
  // engine stream right after k_pick and moves selection and k_sha to the second stream, so the
  // chain pays no cross-stream wait (≈ 10-14 us between k_compact and k_pick,
  // profiles/r04_run_timelines_early.txt) and no dispatch gap; selection, which has slack there,
  // pays it instead. A loaded run (configs[2], where the hash work ends with the chain) keeps
  // selection on the engine stream. The knob lets the tests run one input both ways.

  // profile 1: every stage boundary; 2: the SHA-256 stage's two only (on the stream it runs on)
  void mark(int i, hipStream_t on = nullptr) {
    if (profile && ev[i] && (profile == 1 || i >= 2)) (void)hipEventRecord(ev[i], on ? on : stream);
  }

  int setdev() { return herr(hipSetDevice(dev)); }

  int enqueue() {
    const uint32_t ns = nstreams;
    if (early_open) {  // a failed run left second-stream work its engine stream never waited for
      HCHECK(hipStreamSynchronize(estream));
      early_open = false;
    }
    // strips
    std::vector<uint64_t> s0(ns + 1);
    uint64_t strips = 0, total_len = 0, chunk_bound = 0;
    data_span = 1;
    for (uint32_t s = 0; s < ns; ++s) {
      descs[s].strip0 = strips;
      s0[s] = strips;
      strips += (descs[s].len + kStrip - 1) / kStrip;
      total_len += descs[s].len;
      data_span = std::max<uint64_t>(data_span, descs[s].data_off + descs[s].len);
      chunk_bound += (descs[s].len + (descs[s].seg_base - descs[s].open_start)) / p.min_size + 2;
    }
    s0[ns] = strips;
    nstrips = strips;
    {
      // random input yields ~len/2^bits candidates; degenerate input (e.g. all zeros: one per
      // byte) overflows this estimate and is re-run once at its exact size by finish().
      const uint32_t b = std::min<uint32_t>(p.split_bits, 16);
      cand_cap = std::max<uint64_t>(1u << 16, ((total_len >> b) << 2) + 2ull * ns + 1024);
      if (retry_cap > cand_cap) cand_cap = retry_cap;
    }
    // Every chunk ends at a candidate (the forced final one included), and a run whose
    // candidates overflow cand_cap selects nothing, so cand_cap also bounds the chunk count; it
    // is the tighter bound for small MinSize (len / MinSize records would be ~len for MinSize 1).
    chunk_cap = std::min(chunk_bound, cand_cap);
    HCHECK(streams.ensure(sizeof(StreamDesc) * (ns ? ns : 1)));
    HCHECK(strip0.ensure(sizeof(uint64_t) * (ns + 1)));
    HCHECK(counts.ensure(sizeof(uint32_t) * (strips ? strips : 1)));
    // the refine lists (one per k_scan workgroup, scan_list_cap entries each), then their
    // lengths (u32 per list)
    const uint32_t lists = strips ? scan_lists(strips, num_cus) : 0;
    const uint64_t list_cap = scan_list_cap(strips, lists);
    HCHECK(refine.ensure(sizeof(uint64_t) * (lists * list_cap + 1) + sizeof(uint32_t) * (lists + 1)));
    HCHECK(slots.ensure(sizeof(uint32_t) * kSlotCap * (strips ? strips : 1)));
    HCHECK(strip_off.ensure(sizeof(uint64_t) * (strips ? strips : 1)));
    HCHECK(partials_a.ensure(sizeof(uint64_t) * prefix_partials_needed(strips)));
    HCHECK(partials_b.ensure(sizeof(uint64_t) * prefix_partials_needed(cand_cap)));
    HCHECK(cand.ensure(sizeof(uint64_t) * cand_cap));
    HCHECK(flags.ensure(sizeof(uint32_t) * cand_cap));
    HCHECK(fidx.ensure(sizeof(uint64_t) * cand_cap));
    HCHECK(bnd_end.ensure(sizeof(uint64_t) * chunk_cap));
    HCHECK(bnd_info.ensure(sizeof(uint64_t) * chunk_cap));
    HCHECK(out.ensure(sizeof(ChunkRec) * chunk_cap));
    HCHECK(scount.ensure(sizeof(uint64_t) * (ns ? ns : 1)));
    HCHECK(last_end.ensure(sizeof(uint64_t) * (ns ? ns : 1)));
    HCHECK(carry.ensure(sizeof(CarryOut) * (ns ? ns : 1)));
    HCHECK(ctr.ensure(sizeof(Counters) + sizeof(Early)));
    HCHECK(long_list.ensure(sizeof(uint64_t) * (chunk_cap + ns)));
    HCHECK(order.ensure(sizeof(uint64_t) * (chunk_cap + ns)));
    HCHECK(jinfo.ensure(sizeof(uint32_t) * (chunk_cap + ns)));
    HCHECK(jdesc.ensure(sizeof(LaneJob) * (chunk_cap + ns)));
    HCHECK(regions.ensure(sizeof(Regions)));
    HCHECK(oreg.ensure(chunk_cap + ns));
    HCHECK(rorder.ensure(sizeof(uint64_t) * (chunk_cap + ns)));
    HCHECK(buckets.ensure(sizeof(uint32_t) * 4 * kLptBuckets));
    HCHECK(h_streams.ensure(sizeof(StreamDesc) * (ns ? ns : 1)));
    HCHECK(h_strip0.ensure(sizeof(uint64_t) * (ns + 1)));
    HCHECK(h_ctr.ensure(sizeof(Counters)));

    // The pinned staging of the previous run may still be in flight: finish() synchronised.
    std::memcpy(h_streams.p, descs.data(), sizeof(StreamDesc) * ns);
    std::memcpy(h_strip0.p, s0.data(), sizeof(uint64_t) * (ns + 1));
    {  // descriptors in, counters and bucket counts zeroed, streams initialised: one dispatch
      const auto* hs = static_cast<const StreamDesc*>(h_streams.dev());
      const auto* h0 = static_cast<const uint64_t*>(h_strip0.dev());
      if (!hs || !h0) return BSG_EDEVICE;
      StartArgs st{hs, h0, streams.as<StreamDesc>(), strip0.as<uint64_t>(), ns,
                   last_end.as<uint64_t>(), scount.as<uint64_t>(), carry.as<CarryOut>(),
                   ctr.as<uint32_t>(), (uint32_t)((sizeof(Counters) + sizeof(Early)) / 4),
                   buckets.as<uint32_t>(), 2 * kLptBuckets,
                   partials_a.as<uint32_t>(), (uint32_t)(2 * prefix_partials_needed(strips)),
                   partials_b.as<uint32_t>(), (uint32_t)(2 * prefix_partials_needed(cand_cap))};
      HCHECK(dbg("launch_start", stream, launch_start(st, stream)));
    }
    Counters* dctr = ctr.as<Counters>();
    Early* dearly = reinterpret_cast<Early*>(ctr.as<uint8_t>() + sizeof(Counters));
    const bool early = early_ok() && total_len >= early_min && strips;
    if (early) {
      if (!estream) HCHECK(stream_acquire(dev, &estream));
      // device-side dependencies only: no system-scope release (an L2 write-back) at record
      const unsigned fl = hipEventDisableTiming | hipEventDisableSystemFence;
      if (!cand_ev) HCHECK(hipEventCreateWithFlags(&cand_ev, fl));
      if (!pick_ev) HCHECK(hipEventCreateWithFlags(&pick_ev, fl));
      if (!early_ev) HCHECK(hipEventCreateWithFlags(&early_ev, fl));
    }
    ShaArgs sh{d_data, streams.as<StreamDesc>(), ns, bnd_end.as<uint64_t>(),
               bnd_info.as<uint64_t>(), last_end.as<uint64_t>(), dctr, out.as<ChunkRec>(),
               carry.as<CarryOut>(), chunk_cap, long_list.as<uint64_t>(), order.as<uint64_t>(),
               buckets.as<uint32_t>(), buckets.as<uint32_t>() + kLptBuckets,
               buckets.as<uint32_t>() + 2 * kLptBuckets, buckets.as<uint32_t>() + 3 * kLptBuckets,
               jinfo.as<uint32_t>(), jdesc.as<LaneJob>(), regions.as<Regions>(), oreg.as<uint8_t>(),
               data_span > kRegionBytes ? rorder.as<uint64_t>() : order.as<uint64_t>(), data_span,
               long_mode(), 4u * (uint32_t)num_cus, seq_wait_limit(), cand.as<uint64_t>(),
               early ? dearly : nullptr};

    ScanArgs sa{};
    sa.data = d_data;
    sa.streams = streams.as<StreamDesc>();
    sa.strip0 = strip0.as<uint64_t>();
    sa.nstreams = ns;
    sa.nstrips = strips;
    sa.table = table.as<uint32_t>();
    sa.p = p;
    sa.counts = counts.as<uint32_t>();
    sa.refine = refine.as<uint64_t>();
    sa.slots = slots.as<uint32_t>();
    sa.cand_off = strip_off.as<uint64_t>();
    sa.cand = cand.as<uint64_t>();
    sa.cand_cap = cand_cap;
    sa.ctr = dctr;
    sa.lists = lists;
    sa.list_cap = list_cap;
    sa.list_cnt = reinterpret_cast<uint32_t*>(refine.as<uint64_t>() + lists * list_cap + 1);
    mark(0);
    // k_scan: the fast pass, then each workgroup's exact pass over its own refine list
    if (strips) HCHECK(dbg("launch_scan", stream, launch_scan(sa, stream, num_cus)));
    mark(1);

    PrefixArgs pa{};
    pa.in = counts.as<uint32_t>();
    pa.out = strip_off.as<uint64_t>();
    pa.partials = partials_a.as<uint64_t>();
    pa.n_bound = strips;
    pa.n_dev = nullptr;
    pa.total = &dctr->ncand;
    pa.overflow = &dctr->overflow;
    pa.cap = cand_cap;
    pa.skip_if = nullptr;
    pa.error = &dctr->error;
    HCHECK(dbg("launch_prefix", stream, launch_prefix(pa, stream)));

    if (strips) HCHECK(dbg("launch_compact", stream, launch_compact(sa, stream, num_cus)));
    // (exits at once unless a strip had more candidates than slots; k_pick needs them all)
    if (strips) HCHECK(dbg("launch_rescan", stream, launch_rescan(sa, stream, num_cus)));
    const bool light = early && total_len <= (uint64_t)knob(BSG_KNOB_LIGHT_BYTES).load();
    hipStream_t sel_stream = stream;  // where selection and k_sha run
    if (early && light) {  // chains on the engine stream, selection beside them
      HCHECK(dbg("launch_pick", stream,
                 launch_pick(cand.as<uint64_t>(), cand_cap, dctr, p.min_size, dearly, stream,
                             num_cus)));
      HCHECK(hipEventRecord(pick_ev, stream));
      HCHECK(dbg("launch_early", stream, launch_early(sh, p.split_bits, stream)));
      HCHECK(hipStreamWaitEvent(estream, pick_ev, 0));
      sel_stream = estream;
      early_open = true;  // until the engine stream waits for the selection stream's end
    } else if (early) {  // the sorted candidates are final: pick and start two chains beside selection
      HCHECK(hipEventRecord(cand_ev, stream));
      HCHECK(hipStreamWaitEvent(estream, cand_ev, 0));
      HCHECK(dbg("launch_pick", estream,
                 launch_pick(cand.as<uint64_t>(), cand_cap, dctr, p.min_size, dearly, estream,
                             num_cus)));
      HCHECK(hipEventRecord(pick_ev, estream));
      HCHECK(dbg("launch_early", estream, launch_early(sh, p.split_bits, estream)));
      HCHECK(hipEventRecord(early_ev, estream));
      early_open = true;
    }
    SelArgs sel{cand.as<uint64_t>(), streams.as<StreamDesc>(), flags.as<uint32_t>(), p, dctr};
    HCHECK(dbg("launch_select", sel_stream, launch_select(sel, cand_cap, sel_stream, num_cus)));

    PrefixArgs pf{};
    pf.in = flags.as<uint32_t>();
    pf.out = fidx.as<uint64_t>();
    pf.partials = partials_b.as<uint64_t>();
    pf.n_bound = cand_cap;
    pf.n_dev = &dctr->ncand;
    pf.total = &dctr->nchunks;
    pf.overflow = nullptr;
    pf.cap = 0;
    pf.skip_if = &dctr->overflow;
    pf.error = &dctr->error;
    HCHECK(dbg("launch_prefix", sel_stream, launch_prefix(pf, sel_stream)));

    ChunkArgs ca{cand.as<uint64_t>(), flags.as<uint32_t>(), fidx.as<uint64_t>(),
                 bnd_end.as<uint64_t>(), bnd_info.as<uint64_t>(), scount.as<uint64_t>(),
                 last_end.as<uint64_t>(), chunk_cap, p, dctr, streams.as<StreamDesc>()};
    HCHECK(dbg("launch_chunks", sel_stream, launch_chunks(ca, cand_cap, ns, sel_stream, num_cus)));
    if (snapshot) {  // by kernel, not by the copy engine (see launch_copy_out)
      HCHECK(h_snap.ensure(sizeof(Counters) + 8ull * (ns ? ns : 1)));
      if (!sel_ev) HCHECK(hipEventCreateWithFlags(&sel_ev, hipEventDisableTiming));
      uint8_t* hs = static_cast<uint8_t*>(h_snap.dev());
      if (!hs) return BSG_EDEVICE;
      HCHECK(launch_copy_out(ctr.p, hs, sizeof(Counters), stream));
      if (ns) HCHECK(launch_copy_out(last_end.p, hs + sizeof(Counters), 8ull * ns, stream));
      HCHECK(hipEventRecord(sel_ev, stream));
    }

    if (early && !light) HCHECK(hipStreamWaitEvent(stream, pick_ev, 0));  // k_lens reads the picks
    HCHECK(dbg("launch_longlist", sel_stream, launch_longlist(sh, chunk_cap + ns, sel_stream, num_cus)));
    mark(2, sel_stream);
    HCHECK(dbg("launch_sha", sel_stream, launch_sha(sh, chunk_cap + ns, sel_stream, num_cus)));
    if (early && light) HCHECK(hipEventRecord(early_ev, estream));  // selection + k_sha done
    if (early) {  // the early chains' records into place, once they (and k_sha) are done
      HCHECK(hipStreamWaitEvent(stream, early_ev, 0));
      early_open = false;  // the engine stream now orders everything after the chains
      HCHECK(dbg("launch_early_fix", stream, launch_early_fix(dearly, out.as<ChunkRec>(), dctr,
                                                              stream)));
    }
    mark(3);
    enqueued = true;
    return BSG_OK;
  }

  // bsg_engine_hash: every stream is one blob, hashed whole (Blob.Ref of many blobs): no scan or
  // selection, one final chunk per stream, then the same job ordering and k_sha as a split run.
  int enqueue_hash() {
    const uint32_t ns = nstreams;
    data_span = 1;
    for (uint32_t s = 0; s < ns; ++s)
      data_span = std::max<uint64_t>(data_span, descs[s].data_off + descs[s].len);
    nstrips = 0;
    cand_cap = 0;
    chunk_cap = ns;
    const uint64_t nn = ns ? ns : 1;
    HCHECK(streams.ensure(sizeof(StreamDesc) * nn));
    HCHECK(bnd_end.ensure(sizeof(uint64_t) * nn));
    HCHECK(bnd_info.ensure(sizeof(uint64_t) * nn));
    HCHECK(out.ensure(sizeof(ChunkRec) * nn));
    HCHECK(scount.ensure(sizeof(uint64_t) * nn));
    HCHECK(last_end.ensure(sizeof(uint64_t) * nn));
    HCHECK(carry.ensure(sizeof(CarryOut) * nn));
    HCHECK(ctr.ensure(sizeof(Counters)));
    HCHECK(long_list.ensure(sizeof(uint64_t) * 2 * nn));
    HCHECK(order.ensure(sizeof(uint64_t) * 2 * nn));
    HCHECK(jinfo.ensure(sizeof(uint32_t) * 2 * nn));
    HCHECK(jdesc.ensure(sizeof(LaneJob) * 2 * nn));
    HCHECK(regions.ensure(sizeof(Regions)));
    HCHECK(oreg.ensure(2 * nn));
    HCHECK(rorder.ensure(sizeof(uint64_t) * 2 * nn));
    HCHECK(buckets.ensure(sizeof(uint32_t) * 4 * kLptBuckets));
    HCHECK(h_streams.ensure(sizeof(StreamDesc) * nn));
    HCHECK(h_ctr.ensure(sizeof(Counters)));
    std::memcpy(h_streams.p, descs.data(), sizeof(StreamDesc) * ns);
    {
      const auto* hs = static_cast<const StreamDesc*>(h_streams.dev());
      if (!hs) return BSG_EDEVICE;
      StartArgs st{hs, nullptr, streams.as<StreamDesc>(), nullptr, ns, last_end.as<uint64_t>(),
                   scount.as<uint64_t>(), carry.as<CarryOut>(), ctr.as<uint32_t>(),
                   (uint32_t)(sizeof(Counters) / 4), buckets.as<uint32_t>(), 2 * kLptBuckets,
                   nullptr, 0, nullptr, 0};
      HCHECK(dbg("launch_start", stream, launch_start(st, stream)));
    }
    Counters* dctr = ctr.as<Counters>();
    mark(0);
    mark(1);  // no scan / selection stage
    ChunkArgs ca{nullptr, nullptr, nullptr, bnd_end.as<uint64_t>(), bnd_info.as<uint64_t>(),
                 scount.as<uint64_t>(), last_end.as<uint64_t>(), chunk_cap, p, dctr,
                 streams.as<StreamDesc>()};
    if (ns) HCHECK(dbg("launch_blob_jobs", stream,
                       launch_blob_jobs(ca, streams.as<StreamDesc>(), ns, stream, num_cus)));
    ShaArgs sh{d_data, streams.as<StreamDesc>(), ns, bnd_end.as<uint64_t>(),
               bnd_info.as<uint64_t>(), last_end.as<uint64_t>(), dctr, out.as<ChunkRec>(),
               carry.as<CarryOut>(), chunk_cap, long_list.as<uint64_t>(), order.as<uint64_t>(),
               buckets.as<uint32_t>(), buckets.as<uint32_t>() + kLptBuckets,
               buckets.as<uint32_t>() + 2 * kLptBuckets, buckets.as<uint32_t>() + 3 * kLptBuckets,
               jinfo.as<uint32_t>(), jdesc.as<LaneJob>(), regions.as<Regions>(), oreg.as<uint8_t>(),
               data_span > kRegionBytes ? rorder.as<uint64_t>() : order.as<uint64_t>(), data_span,
               hash_long_mode >= 0 ? hash_long_mode : long_mode(), 4u * (uint32_t)num_cus,
               seq_wait_limit()};
    HCHECK(dbg("launch_longlist", stream, launch_longlist(sh, chunk_cap + ns, stream, num_cus)));
    mark(2);
    HCHECK(dbg("launch_sha", stream, launch_sha(sh, chunk_cap + ns, stream, num_cus)));
    mark(3);
    enqueued = true;
    return BSG_OK;
  }

  int finish(uint64_t* nchunks) {
    if (!enqueued) return BSG_ESTATE;
    for (int attempt = 0; attempt < 3; ++attempt) {
      HCHECK(hipMemcpyAsync(h_ctr.p, ctr.p, sizeof(Counters), hipMemcpyDeviceToHost, stream));
      HCHECK(stream_wait(stream));
      last = *h_ctr.as<Counters>();
      if (!last.overflow) break;
      retry_cap = last.ncand + 1024;  // exact size for this input, then run again
      int rc = hash_mode ? enqueue_hash() : enqueue();
      if (rc) return rc;
    }
    retry_cap = 0;
    if (last.overflow) return BSG_ENOMEM;
    if (last.error) {
      std::fprintf(stderr, "bsgpu: device sanity check failed (code %llu)\n",
                   (unsigned long long)last.error);
      enqueued = false;
      return BSG_EDEVICE;
    }
    enqueued = false;
    if (profile) {
      for (int i = 0; i < 3; ++i)
        if ((profile == 2 && i < 2) ||
            hipEventElapsedTime(&stage_ms[i], ev[i], ev[i + 1]) != hipSuccess) {
          (void)hipGetLastError();
          stage_ms[i] = -1.f;
        }
    }
    if (nchunks) *nchunks = last.nchunks;
    return BSG_OK;
  }
};

// ------------------------------------------------------------------------------------------
// Streaming split.Writer (bsg_open / bsg_write / bsg_close / bsg_drain): a pipeline of tiles.
// Tile i's bytes go through a ring of pinned stages, by H2D on the context's copy stream, into
// data slot i mod ndata; its kernels run on engine slot i mod nslots (HIP stream + work buffers).
//
//   host:    copy Write()s into stage s ... flush s (H2D) ... stage s+1 ... submit tile i ...
//   data:    [carry area kCarryCap | tile bytes | read slack]
//   copies:  H2D(i, stage 0..3) -> copied_ev(i)      (waits for data slot i's previous tile)
//   engine:  wait copied_ev(i) -> scan/select(i) -> sel_ev(i) -> k_sha(i) -> records(i)
//
// Tile i+1 needs from tile i only where its open chunk starts, which is known at sel_ev(i), a
// fraction of a millisecond into tile i: the open chunk's bytes (at most kCarryCap; k_sha
// leaves such a chunk unhashed) are copied device-to-device in front of tile i+1's bytes and
// hashed there from the start. Tile i's k_sha — bound by its longest chunk's serial SHA-256
// chain — therefore runs concurrently with tiles i+1, i+2, ... instead of in front of them.
// A longer open chunk falls back to the midstate carry: tile i hashes its whole blocks, and
// tile i+1 waits for tile i's k_sha and continues from the exported midstate.
// Records complete in tile order; bsg_pending/bsg_drain hand them out in stream order.
// ------------------------------------------------------------------------------------------
namespace bsg {

// Host threads copying a large Write into pinned staging (BSG_COPY_THREADS, default 8).
int copy_threads() {
  static const int v = [] {
    const char* e = std::getenv("BSG_COPY_THREADS");
    const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    return std::max(1, std::min(hw, e ? std::min(64, std::atoi(e)) : 8));
  }();
  return v;
}

namespace {
// One parallel_for call: workers and the caller take indices from `next` until none are left.
struct PoolJob {
  const std::function<void(size_t)>* fn = nullptr;
  size_t n = 0;
  std::atomic<size_t> next{0}, done{0};
  std::mutex mu;
  std::condition_variable cv;
  void run() {
    for (size_t i; (i = next.fetch_add(1)) < n;) {
      (*fn)(i);
      if (done.fetch_add(1) + 1 == n) {
        std::lock_guard<std::mutex> g(mu);
        cv.notify_all();
      }
    }
  }
};

class CopyPool {
 public:
  explicit CopyPool(int workers) {
    for (int i = 0; i < workers; ++i) th_.emplace_back([this] { Work(); });
  }
  void Run(size_t n, const std::function<void(size_t)>& fn) {
    auto job = std::make_shared<PoolJob>();
    job->fn = &fn;
    job->n = n;
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(job);
    }
    cv_.notify_all();
    job->run();  // the caller works too
    {
      std::unique_lock<std::mutex> g(job->mu);
      job->cv.wait(g, [&] { return job->done.load() == job->n; });
    }
    std::lock_guard<std::mutex> g(mu_);
    for (auto it = q_.begin(); it != q_.end(); ++it)
      if (*it == job) {
        q_.erase(it);
        break;
      }
  }

 private:
  void Work() {
    for (;;) {
      std::shared_ptr<PoolJob> job;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return !q_.empty(); });
        job = q_.front();
        if (job->next.load() >= job->n) {  // every index taken: nothing left to help with
          q_.pop_front();
          continue;
        }
      }
      job->run();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::shared_ptr<PoolJob>> q_;
  std::vector<std::thread> th_;
};

CopyPool* copy_pool() {
  // never destroyed: its workers stay blocked on the queue until the process exits
  static CopyPool* pool = copy_threads() > 1 ? new CopyPool(copy_threads() - 1) : nullptr;
  return pool;
}
}  // namespace

void parallel_for(size_t n, const std::function<void(size_t)>& fn) {
  if (n == 0) return;
  if (n == 1 || copy_threads() <= 1) {
    for (size_t i = 0; i < n; ++i) fn(i);
    return;
  }
  copy_pool()->Run(n, fn);
}

bool copy_nt_enabled() { return knob(BSG_KNOB_COPY_NT).load(std::memory_order_relaxed) != 0; }

namespace {
// 64 bytes (one cache line) per iteration: four unaligned 16-byte loads, four streaming stores
// to a 16-byte aligned destination (SSE2, every x86-64 host)
inline void nt_lines(uint8_t* d, const uint8_t* s, size_t lines) {
  for (size_t i = 0; i < lines; ++i, d += 64, s += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + 32));
    const __m128i e = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + 48));
    _mm_stream_si128(reinterpret_cast<__m128i*>(d), a);
    _mm_stream_si128(reinterpret_cast<__m128i*>(d + 16), b);
    _mm_stream_si128(reinterpret_cast<__m128i*>(d + 32), c);
    _mm_stream_si128(reinterpret_cast<__m128i*>(d + 48), e);
  }
}
// the same into two destinations; d2 streams only if it has d1's alignment mod 16, else it
// takes ordinary stores
inline void nt_lines2(uint8_t* d1, uint8_t* d2, const uint8_t* s, size_t lines, bool d2nt) {
  for (size_t i = 0; i < lines; ++i, d1 += 64, d2 += 64, s += 64) {
    __m128i v[4];
    for (int j = 0; j < 4; ++j) v[j] = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + 16 * j));
    for (int j = 0; j < 4; ++j) _mm_stream_si128(reinterpret_cast<__m128i*>(d1 + 16 * j), v[j]);
    if (d2nt) {
      for (int j = 0; j < 4; ++j) _mm_stream_si128(reinterpret_cast<__m128i*>(d2 + 16 * j), v[j]);
    } else {
      for (int j = 0; j < 4; ++j) _mm_storeu_si128(reinterpret_cast<__m128i*>(d2 + 16 * j), v[j]);
    }
  }
}
}  // namespace

// The streaming stores are weakly ordered: each copy ends with an sfence, so the bytes are in
// memory before the caller publishes them (a parallel_for's completion, then an H2D copy).
void copy_nt(uint8_t* dst, const uint8_t* src, size_t n) {
  const size_t head = std::min(n, (size_t)(-(uintptr_t)dst & 63));
  std::memcpy(dst, src, head);
  const size_t lines = (n - head) / 64;
  nt_lines(dst + head, src + head, lines);
  const size_t done = head + lines * 64;
  std::memcpy(dst + done, src + done, n - done);
  _mm_sfence();
}

void copy_nt2(uint8_t* d1, uint8_t* d2, const uint8_t* src, size_t n) {
  const size_t head = std::min(n, (size_t)(-(uintptr_t)d1 & 63));
  std::memcpy(d1, src, head);
  std::memcpy(d2, src, head);
  const size_t lines = (n - head) / 64;
  const bool d2nt = (((uintptr_t)d1 ^ (uintptr_t)d2) & 15) == 0;
  nt_lines2(d1 + head, d2 + head, src + head, lines, d2nt);
  const size_t done = head + lines * 64;
  std::memcpy(d1 + done, src + done, n - done);
  std::memcpy(d2 + done, src + done, n - done);
  _mm_sfence();
}

int cpu_node() {
  unsigned cpu = 0, node = 0;
  if (syscall(SYS_getcpu, &cpu, &node, nullptr) != 0) return -1;
  return (int)node;
}

}  // namespace bsg

constexpr int kMaxSlots = 8;
constexpr uint64_t kDefaultCarryCap = 8ull << 20;
// Tiles in flight. Each has its own HIP stream, and streams beyond the process's hardware
// queues (GPU_MAX_HW_QUEUES, 4 by default) share a queue and serialise behind each other's
// k_sha, so the default stays below that.
static int default_slots() {
  const char* e = std::getenv("BSG_STREAM_SLOTS");
  const int v = e ? std::atoi(e) : 3;
  return std::max(2, std::min(kMaxSlots, v));
}

// Device copies of the tiles' bytes, decoupled from the engines: tile i's bytes go to data slot
// i mod ndata and its kernels run on engine slot i mod nslots. With one more data slot than
// engines, tile i's H2D does not wait for tile i - nslots' k_sha (which still reads that engine's
// previous tile), only for tile i - ndata's: the copies run back to back on their own stream
// while the chains of earlier tiles finish.
constexpr int kMaxData = 8;
static int default_data_slots(int nslots) {
  const char* e = std::getenv("BSG_DATA_SLOTS");
  const int v = e ? std::atoi(e) : nslots + 1;
  return std::max(std::max(2, nslots), std::min(kMaxData, v));
}

struct DataSlot {
  DevBuf dbuf;                  // carry area + tile + slack
  hipEvent_t free_ev = nullptr; // recorded on an engine stream after the last reader of dbuf
  bool free_pending = false;    // free_ev recorded, not yet waited for by the copy stream
};

struct TileSlot {
  bsg_engine* eng = nullptr;  // created at the slot's first tile (a small stream needs one)
  PinBuf recs;            // records, D2H'd after k_sha
  hipEvent_t h2d_ev = nullptr, done_ev = nullptr, copied_ev = nullptr;
  int dslot = 0;          // data slot of the tile using this engine
  // state of the tile currently using the slot
  bool busy = false;          // submitted, records not yet collected
  bool sel_read = false;      // selection snapshot consumed (open_next / nchunks known)
  bool recs_enq = false;      // D2H of records enqueued (done_ev recorded)
  bool final_seg = false;
  uint64_t seg_base = 0, len = 0, nchunks = 0, open_next = 0;
};

// Host staging of the streaming path: a ring of pinned buffers, independent of the device tiles.
// The host fills one stage; a full stage is copied (hipMemcpyAsync, on the engine stream of the
// tile it belongs to) into that tile's device slot right away, so a tile's H2D runs while the
// host is still filling the rest of it, and the pinned memory a context holds is the ring
// (4 x 64 MiB: as much host-side slack as one whole tile), not three whole tiles (3 x 256 MiB).
constexpr int kStages = 4;
constexpr size_t kStageMax = 64ull << 20;
// Full-size stages (kStageMax) are shared process-wide: a context takes them from this pool as
// its stream grows past a stage and gives them back at bsg_reset / bsg_free, so an idle pooled
// context holds no pinned staging, N concurrent contexts share what they use, and bsg_init can
// pin a ring's worth ahead of the first Writer. (Smaller stages — small tiles, a stream's first
// stage while it grows — stay with their context.)
class StagePool {
 public:
  static StagePool& get() {
    static auto* p = new StagePool();  // never destroyed (its buffers live until exit)
    return *p;
  }
  bool take(PinBuf* out) {  // out: empty
    std::lock_guard<std::mutex> g(mu_);
    if (free_.empty()) return false;
    *out = free_.back();
    free_.pop_back();
    return true;
  }
  void give(PinBuf* b) {  // takes b's buffer if it is a full-size one; b is empty afterwards
    if (!b->p) return;
    if (b->cap >= kStageMax && b->map_len) {
      std::lock_guard<std::mutex> g(mu_);
      if (free_.size() < kMaxFree) {
        free_.push_back(*b);
        *b = PinBuf{};
        b->dma_only = true;
        return;
      }
    }
    b->release();
  }
  int fill(int n) {  // bsg_init: make sure n full-size stages are pinned and waiting
    for (;;) {
      {
        std::lock_guard<std::mutex> g(mu_);
        if ((int)free_.size() >= n) return BSG_OK;
      }
      PinBuf b;
      b.dma_only = true;
      if (b.ensure(kStageMax) != hipSuccess) return BSG_ENOMEM;
      give(&b);
      if (b.p) {  // not taken (not a registered mapping): leave the pool as it is
        b.release();
        return BSG_OK;
      }
    }
  }

 private:
  static constexpr size_t kMaxFree = 16;  // at most 1 GiB of idle pinned staging
  std::mutex mu_;
  std::vector<PinBuf> free_;
};

struct Stage {
  PinBuf buf;                // DMA staging (PinBuf::dma_only)
  hipEvent_t ev = nullptr;   // recorded after the H2D that reads the stage
  bool inflight = false;     // an H2D from it may still be running
  hipEvent_t t0 = nullptr, t1 = nullptr;  // timing events around that H2D (bsg_stream_stats)
  bool timed = false;        // t0/t1 recorded and not yet read
};

// NUMA node of the page holding p (get_mempolicy MPOL_F_NODE | MPOL_F_ADDR; -1 unknown)
static int page_node(const void* p) {
  int node = -1;
  if (!p || syscall(SYS_get_mempolicy, &node, nullptr, 0UL, p, 3UL) != 0) return -1;
  return node;
}

// NUMA node of a HIP device, from its PCI function in sysfs (-1 unknown)
static int device_node(int device) {
  static std::mutex mu;
  static int cache[64];
  static bool have[64];
  std::lock_guard<std::mutex> g(mu);
  const int k = device & 63;
  if (have[k]) return cache[k];
  char bus[64] = {0};
  int node = -1;
  if (hipDeviceGetPCIBusId(bus, sizeof bus, device) == hipSuccess) {
    for (char* q = bus; *q; ++q) *q = (char)std::tolower((unsigned char)*q);
    char path[160];
    std::snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
    if (FILE* f = std::fopen(path, "r")) {
      if (std::fscanf(f, "%d", &node) != 1) node = -1;
      std::fclose(f);
    }
  } else {
    (void)hipGetLastError();
  }
  cache[k] = node;
  have[k] = true;
  return node;
}

static uint64_t ns_since(std::chrono::steady_clock::time_point t0) {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now() - t0).count();
}

struct bsg_ctx {
  bsg_params params{};
  Params p{};
  int dev = 0;
  uint32_t table[256];
  size_t tile = 256ull << 20;
  uint64_t carry_cap = kDefaultCarryCap;
  int nslots = default_slots();
  TileSlot slots[kMaxSlots];
  int ndata = default_data_slots(nslots);
  DataSlot data[kMaxData];
  int dcur = 0;             // data slot of the tile the host is filling
  bool dready = false;      // the copy stream waits for data[dcur]'s previous readers already
  hipStream_t cstream = nullptr;  // H2D copies of every tile (from the process's stream pool)
  Stage stages[kStages];
  int cur = 0;              // slot of the tile the host is filling
  size_t fill = 0;          // bytes of the current tile (copied to the device or staged)
  int scur = 0;             // stage the host is filling
  size_t sfill = 0;         // bytes in stages[scur] (the current tile's last sfill bytes)
  int prev = -1;            // last submitted slot (its open chunk continues into `cur`)
  std::deque<int> inflight; // submitted slots in stream order
  uint64_t pos = 0;         // stream offset of slots[cur]'s first byte
  uint64_t stream0 = 0;     // stream offset of the stream's first byte (0; bsg_set_stream_base)
  uint8_t hist[64];         // the 64 stream bytes before pos
  uint8_t tail[64];         // the last 64 stream bytes copied to the device so far
  std::deque<bsg_chunk> ready;
  bool closed = false, started = false;
  int sticky = BSG_OK;
  // bsg_stream_stats: counters since open / reset
  bsg_stream_stats stats{};
  std::atomic<uint64_t> node_bytes[4] = {};
  hipEvent_t span0 = nullptr;  // recorded before the first H2D of the stream
  bool span_set = false;
  hipEvent_t tail0 = nullptr, tail1 = nullptr;  // the final tile's kernels: start, records out
  bool tail_set = false;
  int slast = -1;              // stage of the latest H2D
  bool sent = false;           // the stream's first H2D is issued (first_flush())

  size_t stage_size() const { return std::min(tile, kStageMax); }

  int init(int device, const uint32_t* tab) {
    dev = device;
    std::memcpy(table, tab ? tab : kBuzhash32Seed1, sizeof table);
    for (Stage& st : stages) {
      st.buf.dma_only = true;
      HCHECK(hipEventCreateWithFlags(&st.ev, hipEventDisableTiming));
      HCHECK(hipEventCreate(&st.t0));
      HCHECK(hipEventCreate(&st.t1));
    }
    HCHECK(hipEventCreate(&span0));
    HCHECK(hipEventCreate(&tail0));
    HCHECK(hipEventCreate(&tail1));
    std::memset(hist, 0, 64);
    std::memset(tail, 0, 64);
    return ensure_slot(0);  // the first tile's engine: errors surface at bsg_open
  }

  int ensure_slot(int i) {
    TileSlot& t = slots[i];
    if (t.eng) return BSG_OK;
    int err = BSG_OK;
    t.eng = bsg_engine_create(dev, table, &err);
    if (!t.eng) return err;
    t.eng->snapshot = true;
    HCHECK(hipEventCreateWithFlags(&t.h2d_ev, hipEventDisableTiming));
    HCHECK(hipEventCreateWithFlags(&t.done_ev, hipEventDisableTiming));
    HCHECK(hipEventCreateWithFlags(&t.copied_ev, hipEventDisableTiming));
    return BSG_OK;
  }

  // data[dcur] ready to receive the current tile's bytes on the copy stream: allocated, and
  // ordered after the kernels of the tile that used it last.
  int copy_prepare() {
    if (!cstream) HCHECK(stream_acquire(dev, &cstream));
    DataSlot& ds = data[dcur];
    HCHECK(ds.dbuf.ensure(carry_cap + tile + kReadSlack));
    if (!ds.free_ev) HCHECK(hipEventCreateWithFlags(&ds.free_ev, hipEventDisableTiming));
    if (!dready) {
      if (ds.free_pending) HCHECK(hipStreamWaitEvent(cstream, ds.free_ev, 0));
      ds.free_pending = false;
      dready = true;
    }
    return BSG_OK;
  }

  void release() {
    (void)hipSetDevice(dev);
    if (cstream) (void)hipStreamSynchronize(cstream);
    for (TileSlot& t : slots) {
      if (t.eng) (void)hipStreamSynchronize(t.eng->stream);
      t.recs.release();
      if (t.h2d_ev) (void)hipEventDestroy(t.h2d_ev);
      if (t.done_ev) (void)hipEventDestroy(t.done_ev);
      if (t.copied_ev) (void)hipEventDestroy(t.copied_ev);
      bsg_engine_destroy(t.eng);
      t.eng = nullptr;
    }
    for (DataSlot& ds : data) {
      ds.dbuf.release();
      if (ds.free_ev) (void)hipEventDestroy(ds.free_ev);
      ds.free_ev = nullptr;
    }
    if (cstream) stream_release(dev, cstream);
    cstream = nullptr;
    for (Stage& st : stages) {
      if (st.ev) (void)hipEventSynchronize(st.ev);
      StagePool::get().give(&st.buf);
      for (hipEvent_t* e : {&st.ev, &st.t0, &st.t1}) {
        if (*e) (void)hipEventDestroy(*e);
        *e = nullptr;
      }
    }
    for (hipEvent_t* e : {&span0, &tail0, &tail1}) {
      if (*e) (void)hipEventDestroy(*e);
      *e = nullptr;
    }
  }

  // the finished H2D of stage st into the busy time
  void harvest(Stage& st) {
    if (!st.timed) return;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, st.t0, st.t1) == hipSuccess)
      stats.h2d_busy_ns += (uint64_t)((double)ms * 1e6);
    else
      (void)hipGetLastError();
    st.timed = false;
  }

  int get_stats(bsg_stream_stats* out) {
    if (cstream) HCHECK(hipStreamSynchronize(cstream));
    for (Stage& st : stages) harvest(st);
    bsg_stream_stats s = stats;
    if (span_set && slast >= 0) {
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, span0, stages[slast].t1) == hipSuccess)
        s.h2d_span_ns = (uint64_t)((double)ms * 1e6);
      else
        (void)hipGetLastError();
    }
    if (tail_set) {
      float ms = 0.f;
      if (hipEventSynchronize(tail1) == hipSuccess &&
          hipEventElapsedTime(&ms, tail0, tail1) == hipSuccess)
        s.last_tile_ns = (uint64_t)((double)ms * 1e6);
      else
        (void)hipGetLastError();
      if (slast >= 0 && hipEventElapsedTime(&ms, stages[slast].t1, tail1) == hipSuccess)
        s.tail_ns = ms > 0.f ? (uint64_t)((double)ms * 1e6) : 0;
      else
        (void)hipGetLastError();
    }
    for (int k = 0; k < 4; ++k) s.copy_bytes_node[k] = node_bytes[k].load();
    s.gpu_node = device_node(dev);
    for (const Stage& st : stages) {
      if (!st.buf.p) continue;
      for (size_t at : {(size_t)0, st.buf.cap / 2}) {
        const int nd = page_node(st.buf.as<uint8_t>() + at);
        if (nd >= 0 && nd < 32) s.stage_nodes |= 1u << nd;
      }
    }
    s.copy_nt = bsg::copy_nt_enabled() ? 1u : 0u;
    *out = s;
    return BSG_OK;
  }

  // Selection of slot i is done: learn its chunk count and where its open chunk starts. A
  // candidate-buffer overflow (degenerate input) is re-run synchronously at exact capacity.
  int read_sel(int i) {
    TileSlot& t = slots[i];
    if (t.sel_read) return BSG_OK;
    HCHECK(hipEventSynchronize(t.eng->sel_ev));
    Counters c = *t.eng->h_snap.as<Counters>();
    uint64_t last_end =
        *reinterpret_cast<const uint64_t*>(t.eng->h_snap.as<uint8_t>() + sizeof(Counters));
    if (c.overflow || c.error) {
      uint64_t n = 0;
      int rc = t.eng->finish(&n);  // synchronous; re-runs after an overflow
      if (rc) return rc;
      c = t.eng->last;
      HCHECK(hipMemcpy(&last_end, t.eng->last_end.p, 8, hipMemcpyDeviceToHost));
    }
    t.nchunks = c.nchunks;
    t.open_next = last_end;
    t.sel_read = true;
    return BSG_OK;
  }

  // Enqueue the D2H of slot i's records behind its k_sha.
  int enqueue_recs(int i) {
    TileSlot& t = slots[i];
    if (t.recs_enq) return BSG_OK;
    int rc = read_sel(i);
    if (rc) return rc;
    // by kernel behind k_sha: a hipMemcpyAsync D2H queued here would wait for k_sha inside the
    // shared copy-engine queue and hold up the next tiles' H2D copies behind it
    HCHECK(t.recs.ensure(sizeof(bsg_chunk) * (t.nchunks ? t.nchunks : 1)));
    void* rd = t.recs.dev();
    void* cd = t.eng->h_ctr.dev();
    if (!rd || !cd) return BSG_EDEVICE;
    if (t.nchunks)
      HCHECK(launch_copy_out(t.eng->out.p, rd, sizeof(bsg_chunk) * t.nchunks, t.eng->stream));
    HCHECK(launch_copy_out(t.eng->ctr.p, cd, sizeof(Counters), t.eng->stream));
    HCHECK(hipEventRecord(t.done_ev, t.eng->stream));
    if (t.final_seg) {
      HCHECK(hipEventRecord(tail1, t.eng->stream));
      tail_set = true;
    }
    t.recs_enq = true;
    return BSG_OK;
  }

  // Wait for the oldest in-flight tile (if `wait`) and move its records to `ready`.
  int collect_front(bool wait, bool* got) {
    *got = false;
    if (inflight.empty()) return BSG_OK;
    const int i = inflight.front();
    TileSlot& t = slots[i];
    if (!t.recs_enq) {
      if (!wait) return BSG_OK;
      int rc = enqueue_recs(i);
      if (rc) return rc;
    }
    if (!wait) {
      hipError_t q = hipEventQuery(t.done_ev);
      if (q == hipErrorNotReady) {
        (void)hipGetLastError();
        return BSG_OK;
      }
      HCHECK(q);
    }
    HCHECK(hipEventSynchronize(t.done_ev));
    const Counters& c = *t.eng->h_ctr.as<Counters>();
    if (c.error) {
      std::fprintf(stderr, "bsgpu: device sanity check failed (code %llu)\n",
                   (unsigned long long)c.error);
      return BSG_EDEVICE;
    }
    const bsg_chunk* r = t.recs.as<bsg_chunk>();
    for (uint64_t k = 0; k < t.nchunks; ++k) ready.push_back(r[k]);
    t.busy = false;
    t.eng->enqueued = false;
    inflight.pop_front();
    *got = true;
    return BSG_OK;
  }

  int poll() {
    bool got = true;
    while (got) {
      int rc = collect_front(false, &got);
      if (rc) return rc;
    }
    return BSG_OK;
  }

  // Make slots[i] free for a new tile: its previous tile's records are collected.
  int reclaim(int i) {
    while (slots[i].busy) {
      bool got = false;
      int rc = collect_front(true, &got);
      if (rc) return rc;
    }
    return BSG_OK;
  }

  // Copy the staged bytes of the current tile to its data slot (on the copy stream) and move to
  // the next stage.
  int flush_stage() {
    if (sfill == 0) return BSG_OK;
    int rc = copy_prepare();
    if (rc) return rc;
    Stage& st = stages[scur];
    tail_append(st.buf.as<uint8_t>(), sfill);  // history for the next tile
    if (!span_set) {
      HCHECK(hipEventRecord(span0, cstream));
      span_set = true;
    }
    HCHECK(hipEventRecord(st.t0, cstream));
    HCHECK(hipMemcpyAsync(data[dcur].dbuf.as<uint8_t>() + carry_cap + (fill - sfill), st.buf.p,
                          sfill, hipMemcpyHostToDevice, cstream));
    HCHECK(hipEventRecord(st.t1, cstream));
    HCHECK(hipEventRecord(st.ev, cstream));
    st.inflight = true;
    st.timed = true;
    sent = true;
    stats.h2d_bytes += sfill;
    stats.h2d_copies++;
    slast = scur;
    scur = (scur + 1) % kStages;
    sfill = 0;
    return BSG_OK;
  }

  // stages[scur] ready to take bytes: its previous H2D has run, and it can hold `need` bytes.
  // A stream's first stage grows (doubling from 4 MiB) so a small stream pins a few MiB; once
  // the stream has passed a stage's worth of bytes, stages are allocated whole.
  static constexpr size_t kMinStaging = 4ull << 20;
  int stage_ready(size_t need) {
    Stage& st = stages[scur];
    if (st.inflight) {
      const auto t0 = std::chrono::steady_clock::now();
      HCHECK(hipEventSynchronize(st.ev));
      stats.stage_wait_ns += ns_since(t0);
      st.inflight = false;
      harvest(st);
    }
    const size_t full = stage_size();
    const bool big = pos - stream0 + fill >= full;  // past a stage's worth: whole stages
    const size_t want = big ? full : std::min(full, std::max(need, kMinStaging));
    const size_t have = std::min(st.buf.cap, full);
    if (have >= want) return BSG_OK;
    const size_t nc = big ? full : std::min(full, std::max(want, 2 * have));
    PinBuf pooled;
    // a full-size stage already pinned in the pool beats pinning a new one of any size
    if (full == kStageMax && StagePool::get().take(&pooled)) {
      if (sfill) std::memcpy(pooled.p, st.buf.p, sfill);
      st.buf.release();
      st.buf = pooled;
      return BSG_OK;
    }
    HCHECK(st.buf.grow(nc, sfill));
    return BSG_OK;
  }
  size_t stage_room() const {
    return std::min(stages[scur].buf.cap, stage_size()) - sfill;
  }
  // The stream's first kFirstFlush staged bytes go to the device at once instead of when the
  // first stage is full, so the H2D pipeline starts a 32 MiB Write earlier (with a full 64 MiB
  // first stage the copy stream idled until the second Write was copied). Later stages flush
  // full, as before; not the tile's last bytes (a final segment keeps them, see write()).
  static constexpr size_t kFirstFlush = 8ull << 20;
  int first_flush() {
    if (sent || sfill < kFirstFlush || fill >= tile) return BSG_OK;
    return flush_stage();
  }

  int submit(bool final_seg) {
    int rc0 = flush_stage();  // every byte of the tile is on its way to the device slot
    if (rc0) return rc0;
    const int i = cur;
    if ((rc0 = ensure_slot(i))) return rc0;
    TileSlot& t = slots[i];
    bsg_engine* e = t.eng;
    // Two invariants keep a tile's buffers safe. reclaim(i) protects the ENGINE's work buffers:
    // the records of the tile kSlots back on this engine are collected before its buffers are
    // reused. The DATA slot is protected by copy_prepare() and its free_ev: the H2D copies run
    // on the context's copy stream (cstream), which waits for the event recorded after the last
    // kernels (and the carry copy) that read the slot, before refilling it.
    rc0 = reclaim(i);
    if (rc0) return rc0;
    if ((rc0 = copy_prepare())) return rc0;
    // the tile's kernels (and the carry copy into its data slot) run after its H2D copies
    HCHECK(hipEventRecord(t.copied_ev, cstream));
    HCHECK(hipStreamWaitEvent(e->stream, t.copied_ev, 0));
    if (final_seg) HCHECK(hipEventRecord(tail0, e->stream));
    uint8_t* base = data[dcur].dbuf.as<uint8_t>();
    StreamDesc d{};
    d.data_off = carry_cap;
    d.len = fill;
    d.seg_base = pos;
    d.open_start = stream0;  // the first tile; later tiles take the previous tile's open chunk
    d.finalize = final_seg ? 1u : 0u;
    d.carry_cap = final_seg ? 0u : (uint32_t)std::min<uint64_t>(carry_cap, 0xffffffffu);
    std::memcpy(d.hist, hist, 64);
    std::memcpy(d.mid, kIV, sizeof kIV);
    if (prev >= 0) {
      TileSlot& pt = slots[prev];
      int rc = read_sel(prev);
      if (rc) return rc;
      const uint64_t open = pt.open_next;
      const uint64_t carry = pos - open;
      d.open_start = open;
      if (carry <= pt.eng->descs[0].carry_cap) {  // bytes carried on the device
        if (carry) {
          // the open chunk may itself have started in front of pt's tile (carried into it)
          const uint8_t* src = data[pt.dslot].dbuf.as<uint8_t>() + (int64_t)carry_cap +
                               ((int64_t)open - (int64_t)pt.seg_base);
          HCHECK(hipMemcpyAsync(base + carry_cap - carry, src, carry, hipMemcpyDeviceToDevice,
                                e->stream));
          // the previous slot must not be overwritten before this copy has read it
          HCHECK(hipEventRecord(t.h2d_ev, e->stream));
          HCHECK(hipStreamWaitEvent(pt.eng->stream, t.h2d_ev, 0));
          d.flags = kDescOpenInDevice;
        }
      } else {  // midstate carry: wait for the previous tile's k_sha
        rc = enqueue_recs(prev);
        if (rc) return rc;
        HCHECK(hipEventSynchronize(pt.done_ev));
        CarryOut co;
        HCHECK(hipMemcpy(&co, pt.eng->carry.p, sizeof co, hipMemcpyDeviceToHost));
        if (!co.valid || co.open_start != open) return BSG_EDEVICE;
        d.consumed = co.consumed;
        d.prefix_len = co.prefix_len;
        std::memcpy(d.mid, co.mid, sizeof co.mid);
      }
      // the previous tile's records can be fetched as soon as its k_sha is done
      rc = enqueue_recs(prev);
      if (rc) return rc;
      // the previous tile's data slot is free once its kernels (and the carry copy above, which
      // its stream now waits for) are done: the copy stream waits for this before refilling it
      DataSlot& pd = data[pt.dslot];
      HCHECK(hipEventRecord(pd.free_ev, pt.eng->stream));
      pd.free_pending = true;
    }
    e->d_data = base;
    e->descs.assign(1, d);
    e->nstreams = 1;
    e->p = p;
    int rc = e->enqueue();
    if (rc) return rc;
    t.busy = true;
    t.sel_read = false;
    t.recs_enq = false;
    t.final_seg = final_seg;
    t.seg_base = pos;
    t.len = fill;
    t.dslot = dcur;
    dcur = (dcur + 1) % ndata;
    dready = false;
    inflight.push_back(i);
    std::memcpy(hist, tail, 64);  // window history for the next tile
    pos += fill;
    fill = 0;
    prev = i;
    cur = (cur + 1) % nslots;
    if (final_seg) return enqueue_recs(i);
    return BSG_OK;
  }

  // Host side of Write: bytes into the staging ring (large pieces on several threads), each full
  // stage on its way to the device at once, full tiles submitted as more data arrives. A stream
  // has no length limit (split.Writer.Write has none, split/split.go:99-101): stream offsets are
  // u64 everywhere; only candidate positions inside one tile travel in 40-bit fields.
  int write(const uint8_t* p, size_t n) {
    if (n >= (1u << 20)) {
      const int nd = page_node(p);
      if (nd >= 0 && nd < 32) stats.src_nodes |= 1u << nd;
    }
    while (n) {
      if (fill == tile) {  // full tile and more data coming: submit it (never the last one)
        int rc = submit(false);
        if (rc) return rc;
      }
      int rc = stage_ready(sfill + std::min(n, tile - fill));
      if (rc) return rc;
      const size_t k = std::min({n, tile - fill, stage_room()});
      const auto t0 = std::chrono::steady_clock::now();
      par_copy(stages[scur].buf.as<uint8_t>() + sfill, p, k);
      stats.host_copy_ns += ns_since(t0);
      stats.host_bytes += k;
      sfill += k;
      fill += k;
      p += k;
      n -= k;
      // a full stage goes to the device now, except the tile's last one: if the stream ends
      // here, it is submitted as the final segment
      if (stage_room() == 0 && fill < tile && (rc = flush_stage())) return rc;
    }
    if (int rc = first_flush()) return rc;
    return poll();
  }

  // Appends bytes that already went to the device (or are on their way) to the running tail.
  void tail_append(const uint8_t* q, size_t k) {
    if (k >= 64) {
      std::memcpy(tail, q + k - 64, 64);
    } else {
      std::memmove(tail, tail + k, 64 - k);
      std::memcpy(tail + 64 - k, q, k);
    }
  }

  // write() from host memory the caller registered (bsg_host_register): no staging copy, the
  // H2D reads the caller's bytes directly, on the engine stream of the tile they belong to. The
  // last bytes (up to 4 KiB) of a segment that completes a tile are staged instead, so that a
  // full tile always keeps unflushed bytes that window() can hold back for the next tile (a
  // final segment needs at least one byte).
  int write_pinned(const uint8_t* q, size_t n) {
    while (n) {
      if (fill == tile) {
        int rc = submit(false);
        if (rc) return rc;
      }
      int rc = flush_stage();  // staged bytes of this tile go first (offsets stay in order)
      if (rc) return rc;
      if ((rc = copy_prepare())) return rc;
      const size_t k = std::min(n, tile - fill);
      const size_t staged = fill + k == tile ? std::min<size_t>(k, 4096) : 0;
      const size_t direct = k - staged;
      if (direct) {
        HCHECK(hipMemcpyAsync(data[dcur].dbuf.as<uint8_t>() + carry_cap + fill, q, direct,
                              hipMemcpyHostToDevice, cstream));
        tail_append(q, direct);
        fill += direct;
      }
      if (staged) {
        if ((rc = stage_ready(staged))) return rc;
        std::memcpy(stages[scur].buf.as<uint8_t>(), q + direct, staged);
        sfill = staged;
        fill += staged;
      }
      q += k;
      n -= k;
    }
    return poll();
  }

  // Zero-copy form of write(): the caller fills pinned staging directly (an io.Reader reads
  // into it), then commits. The window is the rest of the current stage (within the tile).
  int window(uint8_t** p, size_t* cap) {
    if (fill == tile) {
      // The caller may be at EOF, so this tile cannot be the last one submitted as non-final:
      // hold its last bytes (still in the current stage) back for the next tile. (A final
      // segment must hold at least one byte: the flush of the open chunk is emitted by the scan
      // of the final segment's last strip, and an empty segment has none.)
      constexpr size_t kHold = 4096;
      uint8_t held[kHold];
      const size_t hold = std::min({kHold, tile / 2, sfill});
      std::memcpy(held, stages[scur].buf.as<uint8_t>() + sfill - hold, hold);
      sfill -= hold;
      fill -= hold;
      int rc = submit(false);
      if (rc) return rc;
      if ((rc = stage_ready(hold))) return rc;
      std::memcpy(stages[scur].buf.p, held, hold);
      sfill = fill = hold;
    }
    // the window is the stage's free part (within the tile); a full stage grows or is flushed
    int rc = stage_ready(sfill + 1);
    if (rc) return rc;
    if (stage_room() == 0) {  // a full stage below the tile's end: move on to the next one
      if ((rc = flush_stage()) || (rc = stage_ready(1))) return rc;
    }
    *p = stages[scur].buf.as<uint8_t>() + sfill;
    *cap = std::min(stage_room(), tile - fill);
    return BSG_OK;
  }
  int commit(size_t n) {
    if (n > std::min(stage_room(), tile - fill)) return BSG_EINVAL;
    sfill += n;
    fill += n;
    if (stage_room() == 0 && fill < tile) {
      int rc = flush_stage();
      if (rc) return rc;
    }
    if (int rc = first_flush()) return rc;
    return poll();
  }

  // Bytes into pinned staging on the copy pool; the bytes each thread copied are counted by the
  // NUMA node it ran on (bsg_stream_stats)
  void par_copy(uint8_t* dst, const uint8_t* src, size_t n) {
    constexpr size_t kPiece = 2ull << 20;  // per thread, at least
    const bool nt_ok = bsg::copy_nt_enabled() && n >= kPiece;
    auto one = [this, nt_ok](uint8_t* d, const uint8_t* s, size_t m) {
      if (nt_ok)
        bsg::copy_nt(d, s, m);
      else
        std::memcpy(d, s, m);
      const int nd = bsg::cpu_node();
      if (nd >= 0 && nd < 4) node_bytes[nd].fetch_add(m, std::memory_order_relaxed);
    };
    const size_t nt = std::min<size_t>((size_t)copy_threads(), n / kPiece);
    if (nt <= 1) {
      one(dst, src, n);
      return;
    }
    // 1 MiB slices taken dynamically, so a thread that wakes late or runs slow takes fewer
    // (one slice per thread left the others waiting for it)
    const size_t ns = (n + kCopySlice - 1) / kCopySlice;
    parallel_for(ns, [=](size_t k) {
      const size_t o = k * kCopySlice;
      one(dst + o, src + o, std::min(kCopySlice, n - o));
    });
  }

  // Start a new stream on the same buffers (bsg_reset): everything in flight is waited for and
  // discarded, also after a device error (Counters::error is per run: the buffers stay valid).
  // Only a failing HIP call (a real fault) leaves the context unusable: bsg_free it.
  int reset() {
    if (cstream) HCHECK(hipStreamSynchronize(cstream));
    for (DataSlot& ds : data) ds.free_pending = false;
    dcur = 0;
    dready = false;
    for (int k = 0; k < nslots; ++k) {
      TileSlot& t = slots[k];
      if (t.eng) HCHECK(hipStreamSynchronize(t.eng->stream));
      t.busy = false;
      t.sel_read = t.recs_enq = false;
      if (t.eng) t.eng->enqueued = false;
    }
    // Full-size stages go back to the process-wide pool, last stage first: the pool is a stack
    // and the next stream takes stage 0's buffer first, so every stream of the context gets the
    // same buffer in the same stage. In the given order, the buffers came back reversed at every
    // reset, and every other 1 GiB rep ran ~3.5 ms (12 %) longer (profiles/r05_bench_final.log,
    // end_to_end.reps_ms: 28.1 / 32.3 / 28.4 ms).
    for (int k = kStages - 1; k >= 0; --k) {
      Stage& st = stages[k];
      if (st.inflight) HCHECK(hipEventSynchronize(st.ev));
      st.inflight = false;
      st.timed = false;
      StagePool::get().give(&st.buf);
    }
    stats = bsg_stream_stats{};
    for (auto& b : node_bytes) b.store(0);
    span_set = false;
    tail_set = false;
    slast = -1;
    sent = false;
    inflight.clear();
    ready.clear();
    cur = 0;
    fill = 0;
    scur = 0;
    sfill = 0;
    prev = -1;
    stream0 = 0;
    pos = 0;
    std::memset(hist, 0, 64);
    std::memset(tail, 0, 64);
    closed = false;
    started = false;
    sticky = BSG_OK;
    return BSG_OK;
  }

  int close_begin() {
    if (fill == 0 && pos == stream0) return BSG_OK;  // empty stream: no chunks
    // The final segment must hold at least one byte: the open chunk's flush is emitted by the
    // scan of its last strip. write() and window() never submit a tile without leaving bytes
    // behind, so this cannot happen; fail loudly rather than drop the last chunk.
    if (fill == 0) return BSG_ESTATE;
    return submit(true);
  }
  int close_step(size_t* left) {  // the oldest tile on the device: wait, collect its records
    bool got = false;
    int rc = collect_front(true, &got);
    *left = inflight.size();
    return rc;
  }
  int close() {
    int rc = close_begin();
    for (size_t left = inflight.size(); rc == BSG_OK && left;) rc = close_step(&left);
    return rc;
  }
};

// ------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------
extern "C" {

int64_t bsg_debug_get(int k) {
  if (k < BSG_KNOB_SEQ_WAIT || k > BSG_KNOB_LAST) return -1;
  return knob(k).load();
}

int bsg_debug_set(int k, int64_t value) {
  if (k < BSG_KNOB_SEQ_WAIT || k > BSG_KNOB_LAST || value < 0) return BSG_EINVAL;
  if (k == BSG_KNOB_LONG_MODE && value > 2) return BSG_EINVAL;
  if ((k == BSG_KNOB_EARLY || k == BSG_KNOB_POLL || k == BSG_KNOB_COPY_NT) && value > 1)
    return BSG_EINVAL;
  if (k == BSG_KNOB_SEQ_WAIT && value > (int64_t)UINT32_MAX) return BSG_EINVAL;  // a u32 poll count
  knob(k).store(value);
  return BSG_OK;
}

const char* bsg_errstr(int err) {
  switch (err) {
    case BSG_OK: return "ok";
    case BSG_EINVAL: return "invalid argument";
    case BSG_ENOMEM: return "out of memory";
    case BSG_EDEVICE: return "HIP device error";
    case BSG_ESTATE: return "invalid state (write after close?)";
    case BSG_ENODEV: return "no such HIP device";
    case BSG_ENOTFOUND: return "not found";
    case BSG_ECORRUPT: return "blob does not match its ref";
    case BSG_EIO: return "filesystem error";
    default: return "unknown error";
  }
}

bsg_params bsg_params_default(void) {
  bsg_params p;
  p.split_bits = 16;  // split/split.go:89
  p.min_size = 1024;  // split/split.go:88
  p.fanout = 8;       // split/split.go:48
  p.reserved = 0;
  return p;
}

void bsg_default_table(uint32_t out[256]) { std::memcpy(out, kBuzhash32Seed1, 1024); }

int bsg_init(int device) {
  if (device < 0 || device >= bsg_device_count()) return BSG_ENODEV;
  HCHECK(hipSetDevice(device));
  // streams for the pool. The first four get the process's hardware queues (GPU_MAX_HW_QUEUES,
  // 4); every further one still costs ~2.4 ms to create, and each live split::Writer holds
  // three (its hasher's, its first engine's, its copy stream): a Writer opened while others are
  // alive spent 7.5 of its 13 ms creating them (profiles/r03_fresh_ctx_api_trace.txt). So the
  // pool starts with BSG_INIT_STREAMS of them (default 16: five live Writers' worth).
  static const int kWarmStreams = [] {
    const char* v = std::getenv("BSG_INIT_STREAMS");
    const int n = v ? std::atoi(v) : 16;
    return std::max(1, std::min<int>(n, (int)kStreamPoolMax));
  }();
  hipStream_t s[kStreamPoolMax] = {};
  int got = 0;
  hipError_t e = hipSuccess;
  for (; got < kWarmStreams && e == hipSuccess; ++got) e = stream_acquire(device, &s[got]);
  if (e != hipSuccess) --got;
  // the device context, the copy engines and libbsgpu's code object: one small H2D, kernel and
  // D2H on each warm stream (the process's first DMA copy alone costs tens of ms)
  void* d = nullptr;
  PinBuf h;
  if (e == hipSuccess) e = hipMalloc(&d, 4096);
  if (e == hipSuccess) e = h.ensure(4096);
  for (int i = 0; i < got && e == hipSuccess; ++i) {
    e = hipMemcpyAsync(d, h.p, 2048, hipMemcpyHostToDevice, s[i]);
    if (e == hipSuccess) e = launch_copy_out(d, static_cast<uint8_t*>(d) + 2048, 64, s[i]);
    if (e == hipSuccess) e = hipMemcpyAsync(h.p, d, 64, hipMemcpyDeviceToHost, s[i]);
    if (e == hipSuccess) e = hipStreamSynchronize(s[i]);
  }
  if (d) (void)hipFree(d);
  h.release();
  for (int i = 0; i < got; ++i) stream_release(device, s[i]);
  HCHECK(e);
  // every kernel of the split and hash paths once (HIP loads a kernel at its first launch,
  // ~0.5 ms each, ~20 of them): a 64 KiB split, the same bytes as one blob, one blob per lane
  int rc = BSG_OK;
  bsg_engine* eng = bsg_engine_create(device, nullptr, &rc);
  if (!eng) return rc;
  constexpr uint64_t kWarm = 64 << 10;
  uint8_t* buf = static_cast<uint8_t*>(bsg_device_malloc(device, kWarm + kReadSlack));
  const uint64_t off = 0, len = kWarm;
  uint64_t n = 0;
  if (!buf) rc = BSG_ENOMEM;
  eng->early_min = 0;  // the early-chain kernels too (they pick nothing in 64 KiB)
  if (rc == BSG_OK) rc = bsg_fill_splitmix(device, buf, kWarm, 1, eng->stream);
  if (rc == BSG_OK) rc = bsg_engine_run(eng, buf, &off, &len, 1, nullptr);
  if (rc == BSG_OK) rc = bsg_engine_finish(eng, &n);
  if (rc == BSG_OK) rc = bsg_engine_hash(eng, buf, &off, &len, 1);
  if (rc == BSG_OK) rc = bsg_engine_finish(eng, &n);
  if (rc == BSG_OK) {
    uint8_t ref[32];
    uint8_t blob[64] = {0};
    const uint64_t boff = 0, blen = sizeof blob;
    bsg_hasher* hs = bsg_hasher_new(device);
    rc = hs ? bsg_hasher_sum(hs, blob, &boff, &blen, 1, ref) : BSG_EDEVICE;
    bsg_hasher_free(hs);
  }
  bsg_device_free(device, buf);
  bsg_engine_destroy(eng);
  if (rc) return rc;
  bsg::parallel_for(bsg::copy_threads(), [](size_t) {});  // the host copy pool's threads
  // a ring's worth of full-size pinned stages for the first large stream
  if ((rc = StagePool::get().fill(kStages))) return rc;
  // the streaming path once (registered staging, H2D from it, kernels writing into mapped
  // host memory, events): first uses the process would otherwise pay in its first Writer
  bsg_ctx* c = bsg_open(device, nullptr, nullptr, &rc);
  if (!c) return rc;
  std::vector<uint8_t> bytes(kWarm);
  for (size_t i = 0; i < bytes.size(); ++i) bytes[i] = (uint8_t)(i * 2654435761u >> 24);
  rc = bsg_write(c, bytes.data(), bytes.size());
  if (rc == BSG_OK) rc = bsg_close(c);
  bsg_free(c);
  return rc;
}

int bsg_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

bsg_engine* bsg_engine_create(int device, const uint32_t* table, int* err) {
  int dummy;
  if (!err) err = &dummy;
  int n = bsg_device_count();
  if (device < 0 || device >= n) {
    *err = BSG_ENODEV;
    return nullptr;
  }
  bsg_engine* e = new (std::nothrow) bsg_engine();
  if (!e) {
    *err = BSG_ENOMEM;
    return nullptr;
  }
  e->dev = device;
  if (hipSetDevice(device) != hipSuccess ||
      stream_acquire(device, &e->stream) != hipSuccess) {
    delete e;
    *err = BSG_EDEVICE;
    return nullptr;
  }
  e->num_cus = device_cus(device);
  std::memcpy(e->htable, table ? table : kBuzhash32Seed1, sizeof e->htable);
  if (e->table.ensure(1024) != hipSuccess ||
      hipMemcpy(e->table.p, e->htable, 1024, hipMemcpyHostToDevice) != hipSuccess) {
    bsg_engine_destroy(e);
    *err = BSG_EDEVICE;
    return nullptr;
  }
  *err = BSG_OK;
  return e;
}

void bsg_engine_destroy(bsg_engine* e) {
  if (!e) return;
  hipSetDevice(e->dev);
  if (e->stream) hipStreamSynchronize(e->stream);
  // a failed run may have left early chains (k_pick / k_early on estream) that the engine
  // stream never waited for: they read cand, ctr and the data, so they end before any release
  if (e->estream) hipStreamSynchronize(e->estream);
  DevBuf* bufs[] = {&e->table, &e->streams, &e->strip0, &e->counts, &e->refine, &e->slots,
                    &e->strip_off, &e->partials_a, &e->partials_b, &e->cand, &e->flags,
                    &e->fidx, &e->bnd_end, &e->bnd_info, &e->scount, &e->last_end,
                    &e->out, &e->carry, &e->ctr, &e->long_list, &e->order, &e->buckets, &e->jinfo, &e->jdesc,
                    &e->regions, &e->oreg, &e->rorder};
  for (DevBuf* b : bufs) b->release();
  for (int i = 0; i < 4; ++i)
    if (e->ev[i]) hipEventDestroy(e->ev[i]);
  e->h_streams.release();
  e->h_strip0.release();
  e->h_ctr.release();
  e->h_snap.release();
  if (e->sel_ev) hipEventDestroy(e->sel_ev);
  if (e->cand_ev) hipEventDestroy(e->cand_ev);
  if (e->pick_ev) hipEventDestroy(e->pick_ev);
  if (e->early_ev) hipEventDestroy(e->early_ev);
  if (e->estream) stream_release(e->dev, e->estream);  // (synchronised above)
  if (e->stream) stream_release(e->dev, e->stream);
  delete e;
}

// Checks a device-resident batch (16-byte aligned offsets, streams under 2^40 bytes, the read
// slack inside the allocation) and fills the engine's descriptors: fresh, final streams.
static int engine_batch(bsg_engine* e, const uint8_t* d_data, const uint64_t* off,
                        const uint64_t* len, uint32_t nstreams) {
  if (!e || (nstreams && (!d_data || !off || !len)) || nstreams > 65535) return BSG_EINVAL;
  int rc;
  if ((rc = e->setdev())) return rc;
  // the SHA-256 loader reads up to kReadSlack bytes past a stream's end (masked): that memory
  // must belong to the same allocation
  uint64_t hi = 0;
  for (uint32_t s = 0; s < nstreams; ++s) hi = std::max<uint64_t>(hi, off[s] + len[s]);
  if (nstreams) {
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)d_data) != hipSuccess) {
      (void)hipGetLastError();
      return BSG_EINVAL;  // not a HIP device allocation
    }
    const uint64_t avail = (uint64_t)((const uint8_t*)base + size - d_data);
    if (hi + kReadSlack > avail) {
      std::fprintf(stderr, "bsgpu: device buffer needs %llu readable bytes after the last "
                           "stream (has %llu)\n", (unsigned long long)kReadSlack,
                   (unsigned long long)(avail > hi ? avail - hi : 0));
      return BSG_EINVAL;
    }
  }
  e->descs.assign(nstreams, StreamDesc{});
  for (uint32_t s = 0; s < nstreams; ++s) {
    if (off[s] % 16 != 0 || len[s] >= (1ull << 40)) return BSG_EINVAL;
    StreamDesc& d = e->descs[s];
    d.data_off = off[s];
    d.len = len[s];
    d.seg_base = 0;
    d.open_start = 0;
    d.consumed = 0;
    d.finalize = 1;
    d.prefix_len = 0;
    std::memcpy(d.mid, kIV, sizeof kIV);
  }
  e->d_data = d_data;
  e->nstreams = nstreams;
  return BSG_OK;
}

int bsg_engine_run(bsg_engine* e, const uint8_t* d_data, const uint64_t* off, const uint64_t* len,
                   uint32_t nstreams, const bsg_params* params) {
  Params p;
  int rc = normalize(params, &p, nullptr);
  if (rc) return rc;
  if ((rc = engine_batch(e, d_data, off, len, nstreams))) return rc;
  e->p = p;
  e->hash_mode = false;
  return e->enqueue();
}

int bsg_engine_hash(bsg_engine* e, const uint8_t* d_data, const uint64_t* off, const uint64_t* len,
                    uint32_t nblobs) {
  int rc = engine_batch(e, d_data, off, len, nblobs);
  if (rc) return rc;
  normalize(nullptr, &e->p, nullptr);
  e->hash_mode = true;
  return e->enqueue_hash();
}

int bsg_engine_finish(bsg_engine* e, uint64_t* nchunks) {
  if (!e) return BSG_EINVAL;
  int rc = e->setdev();
  if (rc) return rc;
  return e->finish(nchunks);
}

const bsg_chunk* bsg_engine_chunks_device(const bsg_engine* e) {
  return e ? static_cast<const bsg_chunk*>(e->out.p) : nullptr;
}

int bsg_engine_copy_chunks(bsg_engine* e, bsg_chunk* out, uint64_t cap) {
  if (!e || (!out && cap)) return BSG_EINVAL;
  int rc = e->setdev();
  if (rc) return rc;
  const uint64_t n = std::min<uint64_t>(cap, e->last.nchunks);
  if (n) HCHECK(hipMemcpy(out, e->out.p, sizeof(bsg_chunk) * n, hipMemcpyDeviceToHost));
  return BSG_OK;
}

int bsg_engine_copy_counts(bsg_engine* e, uint64_t* counts, uint32_t nstreams) {
  if (!e || !counts || nstreams > e->nstreams) return BSG_EINVAL;
  int rc = e->setdev();
  if (rc) return rc;
  if (nstreams)
    HCHECK(hipMemcpy(counts, e->scount.p, sizeof(uint64_t) * nstreams, hipMemcpyDeviceToHost));
  return BSG_OK;
}

void* bsg_engine_stream(bsg_engine* e) { return e ? (void*)e->stream : nullptr; }

int bsg_engine_profile(bsg_engine* e, int enable) {
  if (!e || enable < 0 || enable > 2) return BSG_EINVAL;
  int rc = e->setdev();
  if (rc) return rc;
  if (enable && !e->ev[0])
    for (int i = 0; i < 4; ++i) HCHECK(hipEventCreate(&e->ev[i]));
  e->profile = enable;
  return BSG_OK;
}

int bsg_engine_stage_ms(const bsg_engine* e, float out[3]) {
  if (!e || !out || !e->profile) return BSG_EINVAL;
  for (int i = 0; i < 3; ++i) out[i] = e->stage_ms[i];
  return BSG_OK;
}

uint64_t bsg_engine_candidates(const bsg_engine* e) { return e ? e->last.ncand : 0; }

int bsg_engine_diag(const bsg_engine* e, uint64_t out[16]) {
  if (!e || !out) return BSG_EINVAL;
  out[0] = e->last.nlong;
  out[1] = e->last.long_thresh;
  out[2] = e->last.max_nblocks;
  for (int i = 0; i < 5; ++i) out[3 + i] = e->last.diag[i];
  for (int i = 0; i < 5; ++i) out[8 + i] = e->last.diag2[i];
  out[13] = e->last.nshort;
  out[14] = e->last.ntickets;
  out[15] = e->last.total_blocks;
  return BSG_OK;
}

// Experiment tooling (not in include/bsgpu.h): copies the region queues' state after the last
// run (tools/stress_regions.py).
extern "C" int bsg_engine_regions_debug(bsg_engine* e, void* out, uint64_t nbytes) {
  if (!e || !out || !e->regions.p) return BSG_EINVAL;
  if (e->setdev()) return BSG_EDEVICE;
  const uint64_t n = std::min<uint64_t>(nbytes, sizeof(Regions));
  if (hipStreamSynchronize(e->stream) != hipSuccess) return BSG_EDEVICE;
  return hipMemcpy(out, e->regions.p, n, hipMemcpyDeviceToHost) == hipSuccess ? BSG_OK : BSG_EDEVICE;
}

int bsg_engine_timeline(const bsg_engine* e, uint64_t out[4]) {
  if (!e || !out) return BSG_EINVAL;
  out[0] = e->last.sha_start_rt;
  out[1] = e->last.diag[2];  // longest wave-mode job: start, end
  out[2] = e->last.diag[3];
  out[3] = e->last.lane_end_rt;
  return BSG_OK;
}

bsg_ctx* bsg_open(int device, const bsg_params* params, const uint32_t* table, int* err) {
  int dummy;
  if (!err) err = &dummy;
  Params p;
  bsg_params norm;
  int rc = normalize(params, &p, &norm);
  if (rc) {
    *err = rc;
    return nullptr;
  }
  if (device < 0 || device >= bsg_device_count()) {
    *err = BSG_ENODEV;
    return nullptr;
  }
  bsg_ctx* c = new (std::nothrow) bsg_ctx();
  if (!c) {
    *err = BSG_ENOMEM;
    return nullptr;
  }
  c->params = norm;
  c->p = p;
  if (hipSetDevice(device) != hipSuccess || (rc = c->init(device, table)) != BSG_OK) {
    c->release();
    delete c;
    *err = rc ? rc : BSG_EDEVICE;
    return nullptr;
  }
  *err = BSG_OK;
  return c;
}

int bsg_set_tile(bsg_ctx* c, size_t tile) {
  if (!c || tile < 4096 || c->fill || c->pos != c->stream0 || c->started) return BSG_EINVAL;
  c->tile = tile;
  return BSG_OK;
}

int bsg_set_carry_cap(bsg_ctx* c, size_t bytes) {
  if (!c || c->fill || c->pos != c->stream0 || c->started || bytes > 0xffffffffull)
    return BSG_EINVAL;
  c->carry_cap = bytes;
  return BSG_OK;
}

int bsg_set_stream_base(bsg_ctx* c, uint64_t base) {
  if (!c || c->fill || c->pos != c->stream0 || c->started || c->closed) return BSG_EINVAL;
  c->stream0 = c->pos = base;
  return BSG_OK;
}

int bsg_write(bsg_ctx* c, const uint8_t* p, size_t n) {
  if (!c) return BSG_EINVAL;
  if (c->closed) return BSG_ESTATE;
  if (c->sticky) return c->sticky;
  if (n && !p) return BSG_EINVAL;
  if (hipSetDevice(c->dev) != hipSuccess) return BSG_EDEVICE;
  c->started = true;
  int rc = c->write(p, n);
  if (rc) c->sticky = rc;
  return rc;
}

int bsg_host_register(void* p, size_t n) {
  if (!p || !n) return BSG_EINVAL;
  HCHECK(hipHostRegister(p, n, hipHostRegisterDefault));
  return BSG_OK;
}

int bsg_host_unregister(void* p) {
  if (!p) return BSG_EINVAL;
  HCHECK(hipHostUnregister(p));
  return BSG_OK;
}

int bsg_write_pinned(bsg_ctx* c, const uint8_t* p, size_t n) {
  if (!c) return BSG_EINVAL;
  if (c->closed) return BSG_ESTATE;
  if (c->sticky) return c->sticky;
  if (n && !p) return BSG_EINVAL;
  if (hipSetDevice(c->dev) != hipSuccess) return BSG_EDEVICE;
  c->started = true;
  int rc = c->write_pinned(p, n);
  if (rc) c->sticky = rc;
  return rc;
}

int bsg_write_window(bsg_ctx* c, uint8_t** p, size_t* cap) {
  if (!c || !p || !cap) return BSG_EINVAL;
  if (c->closed) return BSG_ESTATE;
  if (c->sticky) return c->sticky;
  if (hipSetDevice(c->dev) != hipSuccess) return BSG_EDEVICE;
  c->started = true;
  int rc = c->window(p, cap);
  if (rc) c->sticky = rc;
  return rc;
}

int bsg_write_commit(bsg_ctx* c, size_t n) {
  if (!c) return BSG_EINVAL;
  if (c->closed) return BSG_ESTATE;
  if (c->sticky) return c->sticky;
  if (hipSetDevice(c->dev) != hipSuccess) return BSG_EDEVICE;
  int rc = c->commit(n);
  if (rc) c->sticky = rc;
  return rc;
}

int bsg_close(bsg_ctx* c) {
  if (!c) return BSG_EINVAL;
  if (c->closed) return c->sticky;
  c->closed = true;
  if (c->sticky) return c->sticky;
  if (hipSetDevice(c->dev) != hipSuccess) return c->sticky = BSG_EDEVICE;
  int rc = c->close();
  if (rc) c->sticky = rc;
  return rc;
}

int bsg_close_begin(bsg_ctx* c) {
  if (!c) return BSG_EINVAL;
  if (c->closed) return c->sticky;
  c->closed = true;
  if (c->sticky) return c->sticky;
  if (hipSetDevice(c->dev) != hipSuccess) return c->sticky = BSG_EDEVICE;
  int rc = c->close_begin();
  if (rc) c->sticky = rc;
  return rc;
}

int bsg_close_step(bsg_ctx* c, size_t* left) {
  if (!c || !left) return BSG_EINVAL;
  *left = 0;
  if (!c->closed) return BSG_ESTATE;
  if (c->sticky) return c->sticky;
  if (c->inflight.empty()) return BSG_OK;
  if (hipSetDevice(c->dev) != hipSuccess) return c->sticky = BSG_EDEVICE;
  int rc = c->close_step(left);
  if (rc) c->sticky = rc;
  return rc;
}

size_t bsg_pending(const bsg_ctx* c) {
  if (!c) return 0;
  bsg_ctx* m = const_cast<bsg_ctx*>(c);  // polling completed tiles is not a visible change
  if (!m->sticky && hipSetDevice(m->dev) == hipSuccess) {
    int rc = m->poll();
    if (rc) m->sticky = rc;
  }
  return m->ready.size();
}

size_t bsg_drain(bsg_ctx* c, bsg_chunk* out, size_t cap) {
  if (!c || !out) return 0;
  if (!c->sticky && hipSetDevice(c->dev) == hipSuccess) {
    int rc = c->poll();
    if (rc) c->sticky = rc;
  }
  size_t k = 0;
  while (k < cap && !c->ready.empty()) {
    out[k++] = c->ready.front();
    c->ready.pop_front();
  }
  return k;
}

int bsg_reset(bsg_ctx* c) {
  if (!c) return BSG_EINVAL;
  if (hipSetDevice(c->dev) != hipSuccess) return BSG_EDEVICE;
  return c->reset();
}

void bsg_free(bsg_ctx* c) {
  if (!c) return;
  c->release();
  delete c;
}

int bsg_stream_stats_get(bsg_ctx* c, bsg_stream_stats* out) {
  if (!c || !out) return BSG_EINVAL;
  if (hipSetDevice(c->dev) != hipSuccess) return BSG_EDEVICE;
  return c->get_stats(out);
}

// bsg_split_hash_batch keeps a few engines (work buffers, pinned counters) for the next call:
// creating and freeing one per call cost ~1 ms of allocations (profiles/r03_split_hash_batch_*).
static std::mutex g_batch_eng_mu;
static std::vector<bsg_engine*>& batch_engines() {
  static auto* v = new std::vector<bsg_engine*>();  // never destroyed (see ctx_pool)
  return *v;
}
static bsg_engine* batch_engine_take(int device, const uint32_t* table, int* rc) {
  bsg_engine* e = nullptr;
  {
    std::lock_guard<std::mutex> g(g_batch_eng_mu);
    auto& v = batch_engines();
    for (size_t i = 0; i < v.size(); ++i)
      if (v[i]->dev == device) {
        e = v[i];
        v.erase(v.begin() + (long)i);
        break;
      }
  }
  if (!e) return bsg_engine_create(device, table, rc);
  *rc = BSG_OK;
  const uint32_t* t = table ? table : kBuzhash32Seed1;
  if (std::memcmp(e->htable, t, sizeof e->htable) != 0) {
    std::memcpy(e->htable, t, sizeof e->htable);
    if (hipSetDevice(device) != hipSuccess ||
        hipMemcpy(e->table.p, e->htable, 1024, hipMemcpyHostToDevice) != hipSuccess) {
      bsg_engine_destroy(e);
      *rc = BSG_EDEVICE;
      return nullptr;
    }
  }
  return e;
}
static void batch_engine_give(bsg_engine* e, bool ok) {
  if (ok && hipSetDevice(e->dev) == hipSuccess && hipStreamSynchronize(e->stream) == hipSuccess) {
    e->retry_cap = 0;
    std::lock_guard<std::mutex> g(g_batch_eng_mu);
    if (batch_engines().size() < 2) {
      batch_engines().push_back(e);
      return;
    }
  }
  (void)hipGetLastError();
  bsg_engine_destroy(e);
}

int bsg_split_hash_batch(int device, const uint8_t* host_data, const uint64_t* off,
                         const uint64_t* len, uint32_t nstreams, const bsg_params* params,
                         const uint32_t* table, bsg_chunk* out, uint64_t cap, uint64_t* counts,
                         uint64_t* nchunks) {
  if (nstreams && (!host_data || !off || !len)) return BSG_EINVAL;
  if (!out && cap) return BSG_EINVAL;
  int rc;
  bsg_engine* e = batch_engine_take(device, table, &rc);
  if (!e) return rc;
  // Runs of at most 65,535 streams (the engine's limit) and about 8 GiB of device bytes (a
  // larger stream goes alone); each run's streams are packed 16-byte aligned into one buffer.
  constexpr uint32_t kRunStreams = 65535;
  constexpr uint64_t kRunBytes = 8ull << 30;
  constexpr uint64_t kPackWindow = 64ull << 20;
  DevBuf d;
  PinBuf pack;  // the packing window: a full-size stage from the process's pool when one is free
  pack.dma_only = true;
  std::vector<uint64_t> doff;
  uint64_t n = 0;  // records of all runs so far (written to out while they fit in cap)
  for (uint32_t s0 = 0; s0 < nstreams && rc == BSG_OK;) {
    uint32_t s1 = s0;
    uint64_t total = 0;
    doff.clear();
    while (s1 < nstreams && s1 - s0 < kRunStreams &&
           (s1 == s0 || total + len[s1] <= kRunBytes)) {
      doff.push_back(total);
      total += (len[s1] + 15) & ~15ull;
      ++s1;
    }
    if (d.ensure(total + kReadSlack) != hipSuccess) {
      rc = BSG_ENOMEM;
      break;
    }
    // Streams shorter than the pinned window are packed at their device offsets into it and
    // copied a window at a time (one H2D for many small streams); longer ones directly.
    const uint64_t win = std::min<uint64_t>(total, kPackWindow);
    static_assert(kPackWindow <= kStageMax, "a pooled stage holds the packing window");
    if (win && !pack.p) (void)StagePool::get().take(&pack);
    if (win && pack.ensure(win) != hipSuccess) {
      rc = BSG_ENOMEM;
      break;
    }
    uint64_t wlo = 0, whi = 0;  // device span [wlo, whi) staged in pack
    auto flush = [&]() {
      if (whi > wlo && hipMemcpy(static_cast<uint8_t*>(d.p) + wlo, pack.p, whi - wlo,
                                 hipMemcpyHostToDevice) != hipSuccess)
        rc = BSG_EDEVICE;
      wlo = whi;
    };
    for (uint32_t s = s0; s < s1 && rc == BSG_OK; ++s) {
      const uint64_t at = doff[s - s0];
      if (!len[s]) continue;
      if (len[s] > win / 2) {
        flush();
        if (rc == BSG_OK &&
            hipMemcpy(static_cast<uint8_t*>(d.p) + at, host_data + off[s], len[s],
                      hipMemcpyHostToDevice) != hipSuccess)
          rc = BSG_EDEVICE;
        wlo = whi = at + len[s];
        continue;
      }
      if (at + len[s] - wlo > win) flush();
      if (whi == wlo) wlo = whi = at;
      std::memcpy(pack.as<uint8_t>() + (at - wlo), host_data + off[s], len[s]);
      whi = at + len[s];
    }
    if (rc == BSG_OK) flush();
    uint64_t rn = 0;
    if (rc == BSG_OK) rc = bsg_engine_run(e, d.as<uint8_t>(), doff.data(), len + s0, s1 - s0, params);
    if (rc == BSG_OK) rc = bsg_engine_finish(e, &rn);
    if (rc == BSG_OK && n < cap) {
      rc = bsg_engine_copy_chunks(e, out + n, cap - n);
      // records name their stream within the run: make them batch indices
      for (uint64_t k = n; rc == BSG_OK && s0 && k < std::min(cap, n + rn); ++k) out[k].stream += s0;
    }
    if (rc == BSG_OK && counts) rc = bsg_engine_copy_counts(e, counts + s0, s1 - s0);
    n += rn;
    s0 = s1;
  }
  if (nchunks) *nchunks = n;
  d.release();
  StagePool::get().give(&pack);  // keeps a full-size registered stage, frees anything else
  batch_engine_give(e, rc == BSG_OK);
  return rc;
}

void* bsg_device_malloc(int device, size_t bytes) {
  if (device < 0 || device >= bsg_device_count() || hipSetDevice(device) != hipSuccess)
    return nullptr;
  void* p = nullptr;
  if (hipMalloc(&p, bytes ? bytes : 16) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return p;
}

int bsg_device_free(int device, void* p) {
  if (!p) return BSG_OK;
  HCHECK(hipSetDevice(device));
  HCHECK(hipFree(p));
  return BSG_OK;
}

int bsg_memcpy(int device, void* dst, const void* src, size_t n, int kind) {
  if (n && (!dst || !src)) return BSG_EINVAL;
  HCHECK(hipSetDevice(device));
  hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice
                  : kind == 1 ? hipMemcpyDeviceToHost
                              : hipMemcpyDeviceToDevice;
  if (n) HCHECK(hipMemcpy(dst, src, n, k));
  return BSG_OK;
}

int bsg_device_synchronize(int device) {
  HCHECK(hipSetDevice(device));
  HCHECK(hipDeviceSynchronize());
  return BSG_OK;
}

int bsg_fill_splitmix(int device, uint8_t* d_ptr, uint64_t nbytes, uint64_t seed, void* stream) {
  if (!d_ptr && nbytes) return BSG_EINVAL;
  if (device < 0 || device >= bsg_device_count()) return BSG_ENODEV;
  HCHECK(hipSetDevice(device));
  const int cus = device_cus(device);
  if (nbytes) HCHECK(launch_fill_splitmix(d_ptr, nbytes, seed, (hipStream_t)stream, cus));
  return BSG_OK;
}

}  // extern "C"

// Batched Blob.Ref() with persistent device buffers and stream (bsg_hasher_*): a Writer hashes
// every tree node through one, so a call costs one H2D, one launch and one D2H, not four
// allocations.
// Copies n blobs src[so[k] .. +sl[k]) to dst + dofs[k], on up to copy_threads() threads, each
// taking a run of whole blobs of about total / threads bytes.
static void par_gather(uint8_t* dst, const uint8_t* src, const uint64_t* so,
                       const uint8_t* const* sp, const uint64_t* sl, const uint64_t* dofs,
                       uint32_t n, uint64_t total) {
  constexpr uint64_t kPiece = 2ull << 20;  // per thread, at least
  const uint64_t nt = std::min<uint64_t>((uint64_t)copy_threads(), total / kPiece);
  auto run = [=](uint32_t a, uint32_t b) {
    for (uint32_t k = a; k < b; ++k)
      if (sl[k]) std::memcpy(dst + dofs[k], sp ? sp[k] : src + so[k], sl[k]);
  };
  if (nt <= 1) {
    run(0, n);
    return;
  }
  std::vector<std::pair<uint32_t, uint32_t>> runs;
  const uint64_t per = (total + nt - 1) / nt;
  uint32_t a = 0;
  uint64_t acc = 0;
  for (uint32_t k = 0; k < n; ++k) {
    acc += sl[k];
    if (acc >= per || k + 1 == n) {
      runs.emplace_back(a, k + 1);
      a = k + 1;
      acc = 0;
    }
  }
  parallel_for(runs.size(), [&](size_t i) { run(runs[i].first, runs[i].second); });
}

struct bsg_hasher {
  int dev = 0;
  int num_cus = 256;
  hipStream_t stream = nullptr;
  DevBuf data, off, len, refs;
  PinBuf h_meta;  // off[n] | len[n] staged for one H2D
  PinBuf h_small; // a small batch's host bytes, then its refs: pinned, so both copies are DMA
  // Large batches (the verifying split.Reader, bsg_sha256_batch of many blobs): the blobs are
  // packed at 16-byte offsets into pinned staging and hashed by an engine in bsg_engine_hash
  // mode, whose wave-mode chains take the longest blobs (k_sha_blobs hashes one blob per lane,
  // so a batch waits for its longest blob at per-lane speed, ~2.5x slower per block).
  static constexpr uint32_t kEngineMinBlobs = 16;
  static constexpr uint64_t kEngineMinBytes = 4ull << 20;
  static constexpr uint64_t kEngineLongBlob = 16ull << 10;  // (small batches, see sum())
  static constexpr uint64_t kEngineBatch = 256ull << 20;  // bytes per engine run (one blob may exceed)
  static constexpr uint64_t kGatherPiece = 32ull << 20;   // packed and copied to the device at once
  bsg_engine* eng = nullptr;
  PinBuf stage;
  PinBuf h_recs;  // an engine run's records, D2H
  DevBuf dstage;
  std::vector<uint64_t> aoff;

  // blob k is base + o[k], or ptrs[k] when ptrs is given (scattered blobs, e.g. a store's)
  int sum_engine(const uint8_t* base, const uint64_t* o, const uint8_t* const* ptrs,
                 const uint64_t* l, uint32_t n, uint8_t* out) {
    int err = 0;
    if (!eng && !(eng = bsg_engine_create(dev, nullptr, &err))) return err ? err : BSG_EDEVICE;
    hipStream_t es = static_cast<hipStream_t>(bsg_engine_stream(eng));
    stage.dma_only = true;  // read only by the H2D: a registered huge-page mapping pins faster
    uint64_t left = 0;      // bytes of the blobs not yet in a run
    for (uint32_t k = 0; k < n; ++k) left += l[k];
    // a small batch (see sum()) puts every blob on wave tickets: the engine's own choice keeps
    // blobs under kLongMinBlocks (64 KiB) per-lane
    eng->hash_long_mode = left < kEngineMinBytes ? 2 : -1;
    for (uint32_t i = 0; i < n;) {
      // A run is up to kEngineBatch bytes, or everything left if that is at most a quarter more:
      // every run waits for its longest blob's chain (~10 ms for a 256 MiB run), so a small
      // remainder run (a verifying Reader's window just over 256 MiB) doubled the wait.
      const uint64_t cap = left <= kEngineBatch + kEngineBatch / 4 ? UINT64_MAX : kEngineBatch;
      uint64_t bytes = 0;
      uint32_t j = i;
      aoff.clear();
      while (j < n && j - i < 65535u) {
        const uint64_t a = (bytes + 15) & ~15ull;
        if (j > i && a + l[j] > cap) break;
        aoff.push_back(a);
        bytes = a + l[j];
        left -= l[j];
        ++j;
      }
      // sized once for the largest run (a growth re-pins: ~35 ms per 256 MiB)
      const uint64_t want =
          bytes >= kEngineBatch / 2 ? std::max(bytes, kEngineBatch + kEngineBatch / 4) : bytes;
      HCHECK(stage.ensure(want + kReadSlack));
      HCHECK(dstage.ensure(want + kReadSlack));
      // gathered a piece at a time, each piece's H2D queued as soon as it is packed, so the copy
      // engine moves piece k while the host threads pack piece k+1
      for (uint32_t a = 0; a < j - i;) {
        uint32_t b = a;
        uint64_t pbytes = 0;
        while (b < j - i && (b == a || pbytes < kGatherPiece)) pbytes += l[i + b++];
        const uint64_t lo = aoff[a];
        const uint64_t hi = (b < j - i) ? aoff[b] : bytes;
        par_gather(stage.as<uint8_t>(), base, o ? o + i + a : nullptr,
                   ptrs ? ptrs + i + a : nullptr, l + i + a, aoff.data() + a, b - a, pbytes);
        if (hi > lo)
          HCHECK(hipMemcpyAsync(dstage.as<uint8_t>() + lo, stage.as<uint8_t>() + lo, hi - lo,
                                hipMemcpyHostToDevice, es));
        a = b;
      }
      int rc = bsg_engine_hash(eng, dstage.as<uint8_t>(), aoff.data(), l + i, j - i);
      uint64_t nch = 0;
      if (!rc) rc = bsg_engine_finish(eng, &nch);
      if (!rc && nch != j - i) rc = BSG_EDEVICE;
      if (rc) return rc;
      // the records through pinned memory (a D2H into a fresh pageable vector cost ~12 ms the
      // first time: the runtime pins its pages)
      HCHECK(h_recs.ensure(sizeof(bsg_chunk) * (j - i)));
      HCHECK(hipMemcpyAsync(h_recs.p, eng->out.p, sizeof(bsg_chunk) * (j - i),
                            hipMemcpyDeviceToHost, es));
      HCHECK(hipStreamSynchronize(es));
      const bsg_chunk* rec = h_recs.as<bsg_chunk>();
      for (uint32_t k = 0; k < j - i; ++k) std::memcpy(out + 32ull * (i + k), rec[k].ref, 32);
      i = j;
    }
    return BSG_OK;
  }

  int sum(const uint8_t* base, const uint64_t* o, const uint64_t* l, uint32_t n, uint8_t* out) {
    static const bool dbg_times = std::getenv("BSG_DEBUG_HASHER") != nullptr;
    const auto t_in = std::chrono::steady_clock::now();
    struct Report {  // BSG_DEBUG_HASHER: where one call's time went (stderr)
      bool on;
      std::chrono::steady_clock::time_point t0;
      uint32_t n;
      uint64_t marks[4] = {};
      ~Report() {
        if (on)
          std::fprintf(stderr, "bsgpu hasher: %u blobs, %.3f ms (ensure %.3f, copies %.3f, launch %.3f)\n",
                       n, ns_since(t0) / 1e6, marks[0] / 1e6, (marks[1] - marks[0]) / 1e6,
                       (marks[2] - marks[1]) / 1e6);
      }
    } rep{dbg_times, t_in, n};
    hipPointerAttribute_t attr;
    bool on_device = false;
    if (hipPointerGetAttributes(&attr, base) == hipSuccess)
      on_device = (attr.type == hipMemoryTypeDevice);
    else
      (void)hipGetLastError();
    uint64_t hi = 0, total = 0, longest = 0;
    for (uint32_t i = 0; i < n; ++i) {
      hi = std::max<uint64_t>(hi, o[i] + l[i]);
      total += l[i];
      longest = std::max<uint64_t>(longest, l[i]);
    }
    if (!on_device && n >= kEngineMinBlobs && total >= kEngineMinBytes)
      return sum_engine(base, o, nullptr, l, n, out);
    // A small batch with a long blob goes to the engine too, every blob on a wave ticket: one
    // blob per lane hashes a block per ~6,000-8,000 cycles and the batch waits for its longest
    // blob, where a solo wave chain takes ~2,300 (plus ~0.1 ms of launches). A split::Writer's tree nodes are such a batch:
    // their leaf counts are geometric, so 1 GiB's 63 nodes of ~11 KB include one of ~50 KB, and
    // k_sha_blobs took 2.7-3.1 ms for them (profiles/r06_writer_trace_kernel_stats.csv). Its
    // staging stays the batch's size (< kEngineMinBytes), so a pooled hasher pins nothing big.
    if (!on_device && n >= 2 && total < kEngineMinBytes && longest >= kEngineLongBlob)
      return sum_engine(base, o, nullptr, l, n, out);
    // always hash from a private copy with kReadSlack bytes of tail padding
    HCHECK(data.ensure(hi + kReadSlack));
    HCHECK(off.ensure(8ull * n));
    HCHECK(len.ensure(8ull * n));
    HCHECK(refs.ensure(32ull * n));
    HCHECK(h_meta.ensure(16ull * n));
    std::memcpy(h_meta.p, o, 8ull * n);
    std::memcpy(h_meta.as<uint8_t>() + 8ull * n, l, 8ull * n);
    // Small host batches (tree nodes: pageable std::string) go through pinned memory, whose
    // H2D / D2H are single DMAs instead of the runtime's chunked staging of pageable memory.
    // The path is chosen by blob count, so one large blob can land here too: above
    // kEngineMinBytes its bytes are copied straight from pageable memory instead, so that a
    // pooled hasher never keeps a blob-sized pinned buffer (pinning costs ~50-65 ms per 256 MiB
    // and would stay held for the life of the process).
    const bool via_pinned = !on_device && hi <= kEngineMinBytes;
    HCHECK(h_small.ensure(std::max<uint64_t>(via_pinned ? hi : 0, 32ull * n)));
    rep.marks[0] = ns_since(t_in);
    if (hi) {
      if (on_device) {
        HCHECK(hipMemcpyAsync(data.p, base, hi, hipMemcpyDeviceToDevice, stream));
      } else if (!via_pinned) {
        HCHECK(hipMemcpyAsync(data.p, base, hi, hipMemcpyHostToDevice, stream));
      } else {
        std::memcpy(h_small.p, base, hi);
        HCHECK(hipMemcpyAsync(data.p, h_small.p, hi, hipMemcpyHostToDevice, stream));
      }
    }
    HCHECK(hipMemcpyAsync(off.p, h_meta.p, 8ull * n, hipMemcpyHostToDevice, stream));
    HCHECK(hipMemcpyAsync(len.p, h_meta.as<uint8_t>() + 8ull * n, 8ull * n,
                          hipMemcpyHostToDevice, stream));
    rep.marks[1] = ns_since(t_in);
    BlobShaArgs a{data.as<uint8_t>(), off.as<uint64_t>(), len.as<uint64_t>(), n,
                  refs.as<uint8_t>()};
    HCHECK(launch_sha_blobs(a, stream, num_cus));
    rep.marks[2] = ns_since(t_in);
    HCHECK(hipMemcpyAsync(h_small.p, refs.p, 32ull * n, hipMemcpyDeviceToHost, stream));
    HCHECK(hipStreamSynchronize(stream));
    std::memcpy(out, h_small.p, 32ull * n);
    return BSG_OK;
  }
};

extern "C" {

bsg_hasher* bsg_hasher_new(int device) {
  if (device < 0 || device >= bsg_device_count() || hipSetDevice(device) != hipSuccess)
    return nullptr;
  bsg_hasher* h = new (std::nothrow) bsg_hasher();
  if (!h) return nullptr;
  h->dev = device;
  h->num_cus = device_cus(device);
  if (stream_acquire(device, &h->stream) != hipSuccess) {
    delete h;
    return nullptr;
  }
  return h;
}

int bsg_hasher_sum(bsg_hasher* h, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                   uint32_t n, uint8_t* refs) {
  if (!h || (n && (!base || !off || !len || !refs))) return BSG_EINVAL;
  if (n == 0) return BSG_OK;
  HCHECK(hipSetDevice(h->dev));
  return h->sum(base, off, len, n, refs);
}

int bsg_hasher_sum_ptrs(bsg_hasher* h, const uint8_t* const* ptrs, const uint64_t* len,
                        uint32_t n, uint8_t* refs) {
  if (!h || (n && (!ptrs || !len || !refs))) return BSG_EINVAL;
  if (n == 0) return BSG_OK;
  HCHECK(hipSetDevice(h->dev));
  uint64_t total = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (len[i] && !ptrs[i]) return BSG_EINVAL;
    total += len[i];
  }
  if (n >= bsg_hasher::kEngineMinBlobs && total >= bsg_hasher::kEngineMinBytes)
    return h->sum_engine(nullptr, nullptr, ptrs, len, n, refs);
  // small batches: packed, then the one-blob-per-lane kernel
  std::vector<uint8_t> packed(total ? total : 1);
  std::vector<uint64_t> off(n);
  uint64_t o = 0;
  for (uint32_t i = 0; i < n; ++i) {
    off[i] = o;
    if (len[i]) std::memcpy(packed.data() + o, ptrs[i], len[i]);
    o += len[i];
  }
  return h->sum(packed.data(), off.data(), len, n, refs);
}

size_t bsg_hasher_pinned_bytes(const bsg_hasher* h) {
  if (!h) return 0;
  return h->h_meta.cap + h->h_small.cap + h->stage.cap + h->h_recs.cap;
}

void bsg_hasher_free(bsg_hasher* h) {
  if (!h) return;
  hipSetDevice(h->dev);
  if (h->stream) hipStreamSynchronize(h->stream);
  h->data.release();
  h->off.release();
  h->len.release();
  h->refs.release();
  h->h_meta.release();
  h->h_small.release();
  h->stage.release();
  h->h_recs.release();
  h->dstage.release();
  if (h->eng) bsg_engine_destroy(h->eng);
  if (h->stream) stream_release(h->dev, h->stream);
  delete h;
}

// bsg_sha256_batch keeps a few hashers (device buffers, pinned staging, an engine) for the next
// call instead of creating and freeing them every time.
static std::mutex g_hasher_pool_mu;
static std::vector<bsg_hasher*>& hasher_pool() {
  static auto* v = new std::vector<bsg_hasher*>();  // never destroyed (see ctx_pool)
  return *v;
}

int bsg_sha256_batch(int device, const uint8_t* base, const uint64_t* off, const uint64_t* len,
                     uint32_t n, uint8_t* refs) {
  if (n && (!base || !off || !len || !refs)) return BSG_EINVAL;
  if (n == 0) return BSG_OK;
  if (device < 0 || device >= bsg_device_count()) return BSG_ENODEV;
  bsg_hasher* h = nullptr;
  {
    std::lock_guard<std::mutex> g(g_hasher_pool_mu);
    auto& v = hasher_pool();
    for (size_t i = 0; i < v.size(); ++i)
      if (v[i]->dev == device) {
        h = v[i];
        v.erase(v.begin() + (long)i);
        break;
      }
  }
  if (!h && !(h = bsg_hasher_new(device))) return BSG_EDEVICE;
  if (hipSetDevice(device) != hipSuccess) {
    bsg_hasher_free(h);
    return BSG_EDEVICE;
  }
  const int rc = h->sum(base, off, len, n, refs);
  {
    std::lock_guard<std::mutex> g(g_hasher_pool_mu);
    if (rc == BSG_OK && hasher_pool().size() < 2) {
      hasher_pool().push_back(h);
      h = nullptr;
    }
  }
  if (h) bsg_hasher_free(h);
  return rc;
}

}  // extern "C"

// host_pool.h — the process-wide pool of host threads that copy bytes for libbsgpu (Write
// pieces into pinned staging, blob gathers, a Reader's chunk fetches).
//
// Every caller shares the same workers: N split.Writers running at once (fs.Dir.AddDir's
// per-file writers, fs/dir.go:157-174) use at most copy_threads() pool threads between them plus
// their own calling threads, instead of N × 8 fresh threads per Write call.
#pragma once

#include <cstddef>
#include <cstdint>
#include <functional>

namespace bsg {

// Threads a large copy is split over (BSG_COPY_THREADS, default 8, at most the host's cores).
int copy_threads();
// A large copy's unit of work: slices are taken dynamically by the pool's threads.
constexpr size_t kCopySlice = 1ull << 20;

// Runs fn(i) for every i in [0, n) on the pool and on the calling thread, and returns when all
// have run. fn must not call parallel_for itself.
void parallel_for(size_t n, const std::function<void(size_t)>& fn);

// Copies of Write bytes into buffers nobody reads soon from the CPU (pinned stages the DMA engine
// reads, Write pieces a store keeps): non-temporal stores (BSG_KNOB_COPY_NT, default on), so the
// destination lines are written without first being read into the cache. A plain memcpy reads
// every destination line before writing it: on the staging path that is 4 passes over host
// memory per byte (source read, stage read + written back, DMA read), this is 3.
void copy_nt(uint8_t* dst, const uint8_t* src, size_t n);
// One read of src feeding two destinations (the Writer's piece and the pinned stage): 3 passes
// over host memory per byte instead of 5 for two memcpys (piece read+written, stage read+written,
// and the DMA read aside).
void copy_nt2(uint8_t* d1, uint8_t* d2, const uint8_t* src, size_t n);
bool copy_nt_enabled();
// NUMA node of the CPU the calling thread runs on (-1 unknown)
int cpu_node();

}  // namespace bsg

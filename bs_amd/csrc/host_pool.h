// host_pool.h — the process-wide pool of host threads that copy bytes for libbsgpu (Write
// pieces into pinned staging, blob gathers, a Reader's chunk fetches).
//
// Every caller shares the same workers: N split.Writers running at once (fs.Dir.AddDir's
// per-file writers, fs/dir.go:157-174) use at most copy_threads() pool threads between them plus
// their own calling threads, instead of N × 8 fresh threads per Write call.
#pragma once

#include <cstddef>
#include <functional>

namespace bsg {

// Threads a large copy is split over (BSG_COPY_THREADS, default 8, at most the host's cores).
int copy_threads();

// Runs fn(i) for every i in [0, n) on the pool and on the calling thread, and returns when all
// have run. fn must not call parallel_for itself.
void parallel_for(size_t n, const std::function<void(size_t)>& fn);

}  // namespace bsg

// Cost of getting pinned (page-locked, device-mapped) host staging on this box: hipHostMalloc
// vs an anonymous mapping (transparent huge pages requested, pre-faulted) + hipHostRegister, for
// 4 / 64 / 256 MiB; and the H2D rate from each. Host-side only (no kernels).
//   hipcc -O2 -o /tmp/pin_cost tools/ubench/pin_cost.cpp && /tmp/pin_cost
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstring>

static double now_ms() {
  return std::chrono::duration<double, std::milli>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  if (hipSetDevice(0) != hipSuccess) return 1;
  void* d = nullptr;
  if (hipMalloc(&d, 256ull << 20) != hipSuccess) return 1;
  hipStream_t s;
  (void)hipStreamCreate(&s);
  for (size_t mib : {4, 64, 256, 256}) {
    const size_t n = mib << 20;
    double t0 = now_ms();
    void* p = nullptr;
    if (hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess) return 2;
    double t1 = now_ms();
    std::memset(p, 1, n);
    double t2 = now_ms();
    (void)hipMemcpyAsync(d, p, n, hipMemcpyHostToDevice, s);
    (void)hipStreamSynchronize(s);
    double t3 = now_ms();
    (void)hipHostFree(p);
    double t4 = now_ms();
    std::printf("hipHostMalloc %4zu MiB: alloc %7.2f ms  first touch %7.2f ms  H2D %6.2f ms (%5.1f GB/s)  free %6.2f ms\n",
                mib, t1 - t0, t2 - t1, t3 - t2, n / (t3 - t2) / 1e6, t4 - t3);
    t0 = now_ms();
    void* m = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    (void)madvise(m, n, MADV_HUGEPAGE);
    std::memset(m, 0, n);
    t1 = now_ms();
    if (hipHostRegister(m, n, hipHostRegisterDefault) != hipSuccess) return 3;
    t2 = now_ms();
    (void)hipMemcpyAsync(d, m, n, hipMemcpyHostToDevice, s);
    (void)hipStreamSynchronize(s);
    t3 = now_ms();
    (void)hipHostUnregister(m);
    munmap(m, n);
    t4 = now_ms();
    std::printf("mmap+THP+register %4zu MiB: map+touch %7.2f ms  register %7.2f ms  H2D %6.2f ms (%5.1f GB/s)  free %6.2f ms\n",
                mib, t1 - t0, t2 - t1, t3 - t2, n / (t3 - t2) / 1e6, t4 - t3);
  }
  return 0;
}

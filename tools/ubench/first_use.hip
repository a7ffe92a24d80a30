// One-time HIP costs on this box, in the order a process meets them: the device context, HIP
// streams (the first ones get hardware queues of their own), events, small device and pinned
// allocations, the first kernel launch (code object load). Host-side timing only.
//   hipcc --offload-arch=gfx950 -O2 -o tools/ubench/first_use tools/ubench/first_use.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void k_touch(int* p) { p[threadIdx.x] += 1; }

static double now_ms() {
  return std::chrono::duration<double, std::milli>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  double t = now_ms();
  auto lap = [&](const char* what, int n) {
    const double u = now_ms();
    std::printf("%-34s %8.3f ms total, %7.3f ms each\n", what, u - t, (u - t) / n);
    t = u;
  };
  (void)hipSetDevice(0);
  (void)hipFree(nullptr);
  lap("hipSetDevice + hipFree(0)", 1);
  hipStream_t s[12];
  for (int i = 0; i < 4; ++i) (void)hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking);
  lap("hipStreamCreate x4 (first)", 4);
  for (int i = 4; i < 12; ++i) (void)hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking);
  lap("hipStreamCreate x8 (more)", 8);
  hipEvent_t e[16];
  for (int i = 0; i < 16; ++i) (void)hipEventCreateWithFlags(&e[i], hipEventDisableTiming);
  lap("hipEventCreate x16", 16);
  void* d[32];
  for (int i = 0; i < 32; ++i) (void)hipMalloc(&d[i], 4096 << (i % 8));
  lap("hipMalloc x32 (4 KiB..512 KiB)", 32);
  void* h[8];
  for (int i = 0; i < 8; ++i) (void)hipHostMalloc(&h[i], 4096, hipHostMallocDefault);
  lap("hipHostMalloc x8 (4 KiB)", 8);
  hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, s[0], (int*)d[0]);
  (void)hipStreamSynchronize(s[0]);
  lap("first kernel launch + sync", 1);
  for (int i = 0; i < 12; ++i) {
    hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, s[i], (int*)d[0]);
    (void)hipStreamSynchronize(s[i]);
  }
  lap("kernel + sync on each of 12 streams", 12);
  for (int i = 0; i < 12; ++i) {
    hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, s[i], (int*)d[0]);
    (void)hipStreamSynchronize(s[i]);
  }
  lap("again", 12);
  void* big[3];
  for (int i = 0; i < 3; ++i) (void)hipMalloc(&big[i], (264ull << 20) + 256);
  lap("hipMalloc x3 (264 MiB)", 3);
  for (int i = 0; i < 3; ++i) (void)hipMemsetAsync(big[i], 0, 4096, s[i]);
  for (int i = 0; i < 3; ++i) (void)hipStreamSynchronize(s[i]);
  lap("first touch x3 (memset 4 KiB)", 3);
  for (int i = 0; i < 3; ++i) (void)hipFree(big[i]);
  lap("hipFree x3 (264 MiB)", 3);
  for (int i = 0; i < 32; ++i) (void)hipFree(d[i]);
  lap("hipFree x32", 32);
  for (int i = 0; i < 8; ++i) (void)hipHostFree(h[i]);
  lap("hipHostFree x8", 8);
  for (int i = 0; i < 12; ++i) (void)hipStreamDestroy(s[i]);
  lap("hipStreamDestroy x12", 12);
  return 0;
}

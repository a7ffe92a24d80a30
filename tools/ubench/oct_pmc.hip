// The skewed octet chain of oct.hip (one lone wave, K+W rows in LDS, 544 VALU per block) run
// once for 4,000 blocks, for a rocprofv3 --pmc pass beside k_early's: the
// same counters on the bare loop say what the real kernel's counts mean.
#define main oct_main
#include "oct.hip"
#undef main
int main() {
  uint64_t* d; uint32_t* io;
  (void)hipMalloc(&d, 16); (void)hipMalloc(&io, 8192 * 4);
  (void)hipMemset(io, 3, 8192 * 4);
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(kb<2>, dim3(1), dim3(64), 0, 0, d, io, 4000);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  uint64_t h; (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  printf("octet chain, 4000 blocks: %.1f cycles/block\n", (double)h / 4000);
  // round 6: the solo loop (sha256_blocks_oct_solo), same launches
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(kb<3>, dim3(1), dim3(64), 0, 0, d, io, 4000);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  printf("octet solo chain, 4000 blocks: %.1f cycles/block\n", (double)h / 4000);
  return 0;
}

// EXPERIMENT (tools/gen_oct_variants.py): the octet chain loop with other K+W load / wait
// schedules, one lone wave as oct.hip; each variant's final state checked against the
// single-lane rounds (nowait: timing only), cycles per block from s_memtime.
#define main oct_main
#include "oct.hip"
#undef main
#include "oct_variants.inc"

#define OCTV_KERNEL(NAME, ASM, CLOB)                                                             \
  __global__ __launch_bounds__(64) void kv_##NAME(uint64_t* out, uint32_t* io, int blocks) {     \
    __shared__ __attribute__((aligned(16))) uint32_t rows[2][68];                                \
    for (int i = threadIdx.x; i < 68; i += blockDim.x) {                                        \
      rows[0][i] = io[i] * 2654435761u + i;                                                      \
      rows[1][i] = 1u;                                                                           \
    }                                                                                            \
    __syncthreads();                                                                             \
    const uint32_t H0[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,                      \
                            0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};                     \
    const int emap[4] = {6, 7, 4, 5};                                                            \
    const OctLane ol = oct_lane();                                                               \
    uint32_t hs[4];                                                                              \
    for (int k = 0; k < 4; ++k) hs[k] = ol.a_side ? H0[k] : H0[emap[k]];                         \
    const uint32_t addr = (uint32_t)reinterpret_cast<uintptr_t>(                                 \
        (__attribute__((address_space(3))) const uint32_t*)rows[ol.a_side ? 1 : 0]);             \
    const uint64_t amask = 0xF0F0F0F0F0F0F0F0ull;                                                \
    uint32_t cnt, stride = 0, nblk = (uint32_t)blocks;                                           \
    int32_t lim = blocks;                                                                        \
    uint64_t sexec, t0, t1;                                                                      \
    STAMP(t0);                                                                                   \
    asm volatile(ASM                                                                             \
                 : [h0] "+v"(hs[0]), [h1] "+v"(hs[1]), [h2] "+v"(hs[2]), [h3] "+v"(hs[3]),      \
                   [cnt] "=&s"(cnt), [sexec] "=&s"(sexec)                                        \
                 : [addr] "v"(addr), [stride] "v"(stride), [nblk] "s"(nblk), [lim] "v"(lim),     \
                   [xm] "v"(ol.xm), [s1] "v"(ol.rot), [amask] "s"(amask)                         \
                 : "memory", CLOB);                                                              \
    STAMP(t1);                                                                                   \
    if (threadIdx.x == 0 || threadIdx.x == 4)                                                    \
      for (int k = 0; k < 4; ++k) io[2000 + (threadIdx.x == 4 ? k : emap[k])] = hs[k];            \
    if (threadIdx.x == 0) out[0] = t1 - t0;                                                      \
  }
OCTV_KERNEL(base, OCTV_BASE, OCTV_BASE_CLOB)
OCTV_KERNEL(base_a, OCTV_BASE_A, OCTV_BASE_A_CLOB)
OCTV_KERNEL(base_a32, OCTV_BASE_A32, OCTV_BASE_A32_CLOB)
OCTV_KERNEL(base_m, OCTV_BASE_M, OCTV_BASE_M_CLOB)
OCTV_KERNEL(pair, OCTV_PAIR, OCTV_PAIR_CLOB)
OCTV_KERNEL(pair_a, OCTV_PAIR_A, OCTV_PAIR_A_CLOB)
OCTV_KERNEL(pair_a32, OCTV_PAIR_A32, OCTV_PAIR_A32_CLOB)
OCTV_KERNEL(pair_m, OCTV_PAIR_M, OCTV_PAIR_M_CLOB)
OCTV_KERNEL(far, OCTV_FAR, OCTV_FAR_CLOB)
OCTV_KERNEL(far_a, OCTV_FAR_A, OCTV_FAR_A_CLOB)
OCTV_KERNEL(far_a32, OCTV_FAR_A32, OCTV_FAR_A32_CLOB)
OCTV_KERNEL(far_m, OCTV_FAR_M, OCTV_FAR_M_CLOB)
OCTV_KERNEL(quad4, OCTV_QUAD4, OCTV_QUAD4_CLOB)
OCTV_KERNEL(quad4_a, OCTV_QUAD4_A, OCTV_QUAD4_A_CLOB)
OCTV_KERNEL(quad4_a32, OCTV_QUAD4_A32, OCTV_QUAD4_A32_CLOB)
OCTV_KERNEL(quad4_m, OCTV_QUAD4_M, OCTV_QUAD4_M_CLOB)
OCTV_KERNEL(nowait, OCTV_NOWAIT, OCTV_NOWAIT_CLOB)
OCTV_KERNEL(nowait_a, OCTV_NOWAIT_A, OCTV_NOWAIT_A_CLOB)
OCTV_KERNEL(nowait_a32, OCTV_NOWAIT_A32, OCTV_NOWAIT_A32_CLOB)
OCTV_KERNEL(nowait_m, OCTV_NOWAIT_M, OCTV_NOWAIT_M_CLOB)

typedef void (*kfn)(uint64_t*, uint32_t*, int);
static void run_v(const char* name, kfn k, const uint32_t* ref, int blocks) {
  uint64_t* d; uint32_t* io;
  (void)hipMalloc(&d, 16); (void)hipMalloc(&io, 8192 * 4);
  (void)hipMemset(io, 3, 8192 * 4);
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, io, blocks);
  (void)hipDeviceSynchronize();
  uint64_t h; (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  uint32_t fin[8]; (void)hipMemcpy(fin, io + 2000, 32, hipMemcpyDeviceToHost);
  bool ok = true;
  for (int i = 0; i < 8; ++i) ok &= ref[i] == fin[i];
  printf("%-8s blocks %5d %8.1f cycles/block  %s\n", name, blocks, (double)h / blocks,
         ok ? "MATCH" : "MISMATCH");
  (void)hipFree(d); (void)hipFree(io);
}

int main() {
  for (int blocks : {400, 4000}) {
    uint32_t ref[8];
    run<0>("single lane reference", ref, blocks);
    for (int r = 0; r < 2; ++r) {
      run_v("base", kv_base, ref, blocks);
      run_v("base_a", kv_base_a, ref, blocks);
      run_v("base_a32", kv_base_a32, ref, blocks);
      run_v("base_m", kv_base_m, ref, blocks);
      run_v("pair", kv_pair, ref, blocks);
      run_v("pair_a", kv_pair_a, ref, blocks);
      run_v("pair_a32", kv_pair_a32, ref, blocks);
      run_v("pair_m", kv_pair_m, ref, blocks);
      run_v("far", kv_far, ref, blocks);
      run_v("far_a", kv_far_a, ref, blocks);
      run_v("far_a32", kv_far_a32, ref, blocks);
      run_v("far_m", kv_far_m, ref, blocks);
      run_v("quad4", kv_quad4, ref, blocks);
      run_v("quad4_a", kv_quad4_a, ref, blocks);
      run_v("quad4_a32", kv_quad4_a32, ref, blocks);
      run_v("quad4_m", kv_quad4_m, ref, blocks);
      run_v("nowait", kv_nowait, ref, blocks);
      run_v("nowait_a", kv_nowait_a, ref, blocks);
      run_v("nowait_a32", kv_nowait_a32, ref, blocks);
      run_v("nowait_m", kv_nowait_m, ref, blocks);
    }
  }
  return 0;
}

// Micro-benchmark: per-CU LDS-DMA rate when the source is L2 / Infinity-Cache resident.
// 256 workgroups x 1024 threads; workgroup b reads "symbols" of 256 KB (8 rows of 32 KB) from a
// small pool of buffers (POOL symbols, shared by the 8 workgroups b, b+8, .., b+56 of an XCD
// group, as a residue-class decode would), antenna row by antenna row into a double-buffered
// 2 x 32 KB LDS ring (one row in flight while the previous row is read), every wave issuing
// its share of the row's 32 x 1 KB DMA pieces. Reports the per-CU rate.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/micro/l2dma tools/micro/l2dma.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
constexpr int T = 1024, ROWB = 32768, ROWS = 8;

__device__ inline void dma16(uint32_t voff, const void *sbase, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds) : "memory");
}

template <int PER_WAVE>   // DMA pieces per wave per row (32 pieces per row over 32/PER_WAVE waves)
__global__ __launch_bounds__(T) void kern(const char *pool, uint32_t npool, uint32_t nsym, float *sink) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t grp = (blockIdx.x & 7u) + 8u * (blockIdx.x >> 6);   // one XCD's group
  const uint32_t base = (uint32_t)(uintptr_t)lds;
  float acc = 0.0f;
  constexpr int NW = 32 / PER_WAVE;                    // issuing waves per row
  auto issue = [&](uint32_t sym, int row, int buf) {
    const char *src = pool + ((uint64_t)(sym % npool) * ROWS + row) * ROWB;
    if (wv < (uint32_t)NW)
      for (int j = 0; j < PER_WAVE; j++) {
        const uint32_t b = wv * PER_WAVE + j;
        dma16(b * 1024u + lane * 16u, src, __builtin_amdgcn_readfirstlane(base + buf * ROWB + b * 1024u));
      }
  };
  uint32_t k = 0;
  issue(grp * 7, 0, 0);
  for (uint32_t s = 0; s < nsym; s++) {
    for (int row = 0; row < ROWS; row++, k++) {
      // next row in flight, this one waited for
      const bool last = s + 1 == nsym && row + 1 == ROWS;
      if (!last) issue(grp * 7 + s + (row + 1) / ROWS, (row + 1) % ROWS, (k + 1) & 1);
      if (wv < (uint32_t)NW) {
        if (!last) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(PER_WAVE) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
      const float *r = lds + (k & 1) * (ROWB / 4);
      for (int i = tid; i < ROWB / 4; i += T) acc += r[i];
      __syncthreads();
    }
  }
  if (acc == 1.2345f) sink[0] = acc;
}

template <int PW>
void run(const char *pool, uint32_t npool, int ncu, float *sink) {
  const uint32_t nsym = 200;
  auto k = kern<PW>;
  CHK(hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * ROWB));
  for (int w = 0; w < 2; w++) k<<<ncu, T, 2 * ROWB>>>(pool, npool, nsym, sink);
  hipEvent_t a, b;
  CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
  CHK(hipEventRecord(a));
  for (int w = 0; w < 5; w++) k<<<ncu, T, 2 * ROWB>>>(pool, npool, nsym, sink);
  CHK(hipEventRecord(b)); CHK(hipEventSynchronize(b));
  float ms; CHK(hipEventElapsedTime(&ms, a, b)); ms /= 5;
  const double bytes = (double)ncu * nsym * ROWS * ROWB;
  printf("pool %5u symbols (%7.1f MB)  %2d pieces/wave: %.3f ms  %.2f TB/s chip, %.1f GB/s per CU\n",
         npool, npool * ROWS * ROWB / 1e6, PW, ms, bytes / ms * 1e-9, bytes / ms * 1e-6 / ncu);
}

int main() {
  int ncu = 0;
  CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const uint32_t maxpool = 8192;   // 2 GB: beyond the Infinity Cache
  char *pool; float *sink;
  CHK(hipMalloc(&pool, (size_t)maxpool * ROWS * ROWB));
  CHK(hipMemset(pool, 0, (size_t)maxpool * ROWS * ROWB));
  CHK(hipMalloc(&sink, 64));
  for (uint32_t np : {8u, 64u, 512u, 8192u}) {
    run<1>(pool, np, ncu, sink);
    run<4>(pool, np, ncu, sink);
  }
  return 0;
}

// Micro-benchmark: the memory pattern of decode_stream_kernel<11, 4> (C3) without its math.
// 256 persistent 1024-thread workgroups walk 51000 "symbols"; per symbol 4 antenna rows of 2050
// complex64 samples (rows a capture length apart, as the batch lays them out) are staged into
// LDS by LDS-DMA (17 x 1 KB per row, one row per wave 0..3) plus 8 KB of reference indices
// (waves 4..11), and every thread stores 4 x 16 B (symbols) + 4 x 2 B (indices) to output rows
// laid out [frame][stream][symbol][2048]. Variants:
//   mode 0: the kernel's schedule -- counted vmcnt wait + barrier at the top, staging reads,
//           barrier, next symbol's DMA, VALU/LDS filler, stores
//   mode 1: two staging buffers, the next symbol's DMA issued at the top of this one
//   mode 2: mode 0 without stores;  mode 3: mode 0 without the DMA (stores only)
//   mode 4: neither (the filler alone)
// FILL = VALU filler iterations per thread and symbol, LDSX = LDS exchange rounds.
// Build: hipcc -O3 --offload-arch=gfx950 -o /tmp/sc tools/micro/stream_ceiling.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int M = 2048, NA = 4, T = 1024, SL = 2200, RS = M + 2;
constexpr int NBLK = 17, LASTC = RS / 2 - 16 * 64;   // 1 KB DMA blocks per row, last block's chunks
constexpr int NSTORE = 8;
typedef float v4f __attribute__((ext_vector_type(4)));

template <bool NT = true>
__device__ inline void dma16(uint32_t voff, const void *sbase, uint32_t lds) {
  uint32_t keep;
  if constexpr (NT)
    asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, %2 nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds) : "memory");
  else
    asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds) : "memory");
}
// OPT bits: 1 plain (not nt) stores, 2 plain DMA loads, 4 no index stores, 8 symbol-major
// outputs ([frame][symbol][stream][M]: a symbol's streams contiguous, instead of [frame][stream][symbol][M])
template <bool NT, typename V, typename P>
__device__ inline void st(V v, P p) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <int MODE, int FILL, int LDSX, int OPT = 0>
__global__ __launch_bounds__(T) void kern(const float2 *iq, uint64_t L, const uint8_t *ref, float2 *osym,
                                          uint8_t *oidx, uint32_t nsym, uint32_t spf, float *sink) {
  extern __shared__ __attribute__((aligned(16))) float2 lds[];
  constexpr bool DB = MODE == 1;
  float2 *stg0 = lds;                                  // [NA][RS]
  float2 *stg1 = lds + NA * RS;                        // (second buffer)
  uint8_t *rstg = reinterpret_cast<uint8_t *>(lds + (DB ? 2 : 1) * NA * RS);   // [NA][M]
  float2 *xch = reinterpret_cast<float2 *>(rstg + NA * M);                       // exchange
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t chunk = (nsym + gridDim.x - 1) / gridDim.x;
  // OPT 16: symbols interleaved over the grid (workgroup b takes b, b + G, ..: every
  // workgroup's writes adjacent to the others'), else a contiguous chunk per workgroup
  constexpr bool ILV = (OPT & 16) != 0;
  const uint32_t i0 = ILV ? blockIdx.x : blockIdx.x * chunk;
  const uint32_t i1 = ILV ? nsym : min(i0 + chunk, nsym);
  const uint32_t ST = ILV ? gridDim.x : 1u;
  if (i0 >= i1) return;
  const uint32_t rowwave0 = 0;
  auto fetch = [&](uint32_t i, float2 *stg) {
    const uint32_t f = i / spf, s = i % spf;
    if (MODE != 3 && MODE != 4 && wv >= rowwave0 && wv < rowwave0 + NA) {
      const uint32_t g = wv - rowwave0;
      const uint64_t e = (uint64_t)(f * NA + g) * L + 1000 + (uint64_t)s * SL;   // even: aligned
      const char *xa = reinterpret_cast<const char *>(iq + e);
      const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(stg + g * RS));
      for (int b = 0; b < NBLK; b++)
        if (b + 1 < NBLK || lane < LASTC) dma16<!(OPT & 2)>(b * 1024u + lane * 16u, xa, dst + b * 1024u);
    }
    if (MODE != 3 && MODE != 4 && wv >= 4 && wv < 12) {             // reference indices: 8 x 1 KB
      const uint32_t w = wv - 4, t = w / 2, h = w % 2;
      const uint8_t *rb = ref + ((uint64_t)(f * NA + t) * spf + s) * M + h * 1024;
      dma16<!(OPT & 2)>(lane * 16u, rb, __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(rstg + t * M + h * 1024)));
    }
  };
  fetch(i0, stg0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  float acc = 0.0f;
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  uint32_t nsym_wg = 0;
  for (uint32_t i = i0; i < i1; i += ST) {
    nsym_wg++;
    float2 *cur = (DB && ((i - i0) / ST) % 2) ? stg1 : stg0;
    float2 *nxt = (DB && ((i - i0) / ST) % 2) ? stg0 : stg1;
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(MODE == 2 || MODE == 4 ? 0 : ((OPT & 4) ? NSTORE / 2 : NSTORE)) : "memory");
    __syncthreads();
    if (DB && i + ST < i1) fetch(i + ST, nxt);
    const uint32_t f = i / spf, s = i % spf;
    float2 v[8];
    const int g = tid / 256, n = tid % 256;
    for (int r = 0; r < 8; r++) v[r] = cur[g * RS + n + 256 * r];
    const uint32_t refw = *reinterpret_cast<const uint16_t *>(rstg + (tid & 3) * M + 2 * (tid >> 2));
    __syncthreads();
    if (!DB && i + ST < i1) fetch(i + ST, stg0);
    // filler: VALU and LDS exchanges (the transform's work stands in here)
    for (int k = 0; k < FILL; k++)
      for (int r = 0; r < 8; r++) v[r] = make_float2(v[r].x * 0.999f + v[(r + 1) & 7].y, v[r].y * 1.001f - v[r].x);
    for (int x = 0; x < LDSX; x++) {
      float2 *rg = xch;   // (shared by the waves: traffic, not results)
      for (int r = 0; r < 8; r++) rg[lane * 9 + r] = v[r];
      __builtin_amdgcn_wave_barrier();
      for (int r = 0; r < 8; r++) v[r] = rg[((lane + 5 * r) & 63) * 9 + r];
      __builtin_amdgcn_wave_barrier();
    }
    acc += v[0].x + (float)(refw & 1);
    if (MODE != 2 && MODE != 4) {
      const uint32_t kb = 2 * (uint32_t)tid;
      for (int t = 0; t < NA; t++) {
        const uint64_t ob = (OPT & 8) ? ((uint64_t)(f * spf + s) * NA + t) * M
                                      : ((uint64_t)(f * NA + t) * spf + s) * M;
        st<!(OPT & 1)>(v4f{v[2 * t].x, v[2 * t].y, v[2 * t + 1].x, v[2 * t + 1].y},
                       reinterpret_cast<v4f *>(osym + ob + kb));
        if constexpr (!(OPT & 4))
          st<!(OPT & 1)>((uint16_t)(refw + t), reinterpret_cast<uint16_t *>(oidx + ob + kb));
      }
    }
  }
  if (acc == 12345.0f) sink[0] = acc;
  if (tid == 0) {   // shader cycles per symbol of this workgroup, summed over the grid
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    atomicAdd(reinterpret_cast<unsigned long long *>(sink) + 1, (c1 - c0) / (nsym_wg ? nsym_wg : 1));
  }
}

// pure write rate: n16 16-byte non-temporal stores (ILV 0: a contiguous chunk per workgroup,
// 1: grid-stride, every workgroup's wave stores adjacent)
template <int ILV>
__global__ __launch_bounds__(T) void wkern(v4f *out, uint64_t n16) {
  const uint64_t G = (uint64_t)gridDim.x * T;
  if (ILV) {
    for (uint64_t i = (uint64_t)blockIdx.x * T + threadIdx.x; i < n16; i += G)
      __builtin_nontemporal_store(v4f{1.0f, 2.0f, 3.0f, (float)i}, out + i);
  } else {
    const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x, b = blockIdx.x * per;
    const uint64_t e = b + per < n16 ? b + per : n16;
    for (uint64_t i = b + threadIdx.x; i < e; i += T)
      __builtin_nontemporal_store(v4f{1.0f, 2.0f, 3.0f, (float)i}, out + i);
  }
}
template <int ILV>
float wrun(v4f *out, uint64_t n16, int ncu) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
  for (int w = 0; w < 3; w++) wkern<ILV><<<ncu, T>>>(out, n16);
  CHK(hipEventRecord(a));
  for (int w = 0; w < 10; w++) wkern<ILV><<<ncu, T>>>(out, n16);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms;
  CHK(hipEventElapsedTime(&ms, a, b));
  return ms / 10;
}

template <int MODE, int FILL, int LDSX, int OPT = 0>
float run(const float2 *iq, uint64_t L, const uint8_t *ref, float2 *osym, uint8_t *oidx, uint32_t nsym,
          uint32_t spf, float *sink, int ncu) {
  const size_t lds = sizeof(float2) * NA * RS * (MODE == 1 ? 2 : 1) + NA * M + sizeof(float2) * 64 * 9;
  auto k = kern<MODE, FILL, LDSX, OPT>;
  CHK(hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
  for (int w = 0; w < 3; w++) k<<<ncu, T, lds>>>(iq, L, ref, osym, oidx, nsym, spf, sink);
  CHK(hipMemset(sink, 0, 64));
  CHK(hipEventRecord(a));
  const int reps = 10;
  for (int w = 0; w < reps; w++) k<<<ncu, T, lds>>>(iq, L, ref, osym, oidx, nsym, spf, sink);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms;
  CHK(hipEventElapsedTime(&ms, a, b));
  unsigned long long cyc[2];
  CHK(hipMemcpy(cyc, sink, 16, hipMemcpyDeviceToHost));
  printf("  [%llu cycles/symbol, %.2f GHz]", cyc[1] / (reps * (unsigned long long)ncu),
         (double)(cyc[1] / (reps * (unsigned long long)ncu)) * (nsym / (double)ncu) / (ms / reps * 1e6));
  return ms / reps;
}

int main() {
  int ncu = 0;
  CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const uint32_t spf = 1000, nf = 51, nsym = spf * nf;
  const uint64_t L = 2563688;
  float2 *iq; uint8_t *ref, *oidx; float2 *osym; float *sink;
  CHK(hipMalloc(&iq, sizeof(float2) * nf * NA * L));
  CHK(hipMalloc(&ref, (size_t)nf * NA * spf * M));
  CHK(hipMalloc(&osym, sizeof(float2) * nf * NA * spf * M));
  CHK(hipMalloc(&oidx, (size_t)nf * NA * spf * M));
  CHK(hipMalloc(&sink, 64));
  CHK(hipMemset(iq, 0, sizeof(float2) * nf * NA * L));
  CHK(hipMemset(ref, 1, (size_t)nf * NA * spf * M));
  const double bytes = (double)nsym * (NA * M * 8 + NA * M * 9 + NA * M);
  auto rep = [&](const char *name, float ms, double b) {
    printf("%-34s %.4f ms  %.2f TB/s\n", name, ms, b / ms * 1e-9);
  };
  const double bytes_ld = (double)nsym * NA * M * 9, bytes_noidx = (double)nsym * NA * M * 17;
  rep("mode0 (kernel schedule)", run<0, 0, 0>(iq, L, ref, osym, oidx, nsym, spf, sink, ncu), bytes);
  rep("mode0 symbol-major", run<0, 0, 0, 8>(iq, L, ref, osym, oidx, nsym, spf, sink, ncu), bytes);
  rep("mode0 symbol-major interleaved", run<0, 0, 0, 24>(iq, L, ref, osym, oidx, nsym, spf, sink, ncu), bytes);
  rep("mode3 symbol-major", run<3, 0, 0, 8>(iq, L, ref, osym, oidx, nsym, spf, sink, ncu), bytes_ld);
  rep("mode3 symbol-major interleaved", run<3, 0, 0, 24>(iq, L, ref, osym, oidx, nsym, spf, sink, ncu), bytes_ld);
  rep("mode2 (loads only)", run<2, 0, 0>(iq, L, ref, osym, oidx, nsym, spf, sink, ncu), bytes_ld);
  rep("mode2 (loads only) interleaved", run<2, 0, 0, 16>(iq, L, ref, osym, oidx, nsym, spf, sink, ncu), bytes_ld);
  {
    // the symbol buffer's bytes exactly (osym holds nsym NA M complex64)
    const size_t osym_bytes = sizeof(float2) * (size_t)nf * NA * spf * M;
    const uint64_t n16 = osym_bytes / 16;
    rep("pure 16 B nt stores, chunk per WG", wrun<0>(reinterpret_cast<v4f *>(osym), n16, ncu), (double)osym_bytes);
    rep("pure 16 B nt stores, grid-stride", wrun<1>(reinterpret_cast<v4f *>(osym), n16, ncu), (double)osym_bytes);
  }
  rep("mode0 symbol-major again", run<0, 0, 0, 8>(iq, L, ref, osym, oidx, nsym, spf, sink, ncu), bytes);
  return 0;
}

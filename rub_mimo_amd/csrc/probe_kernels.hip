// rub_mimo_amd/csrc/probe_kernels.hip -- roofline probe: the streaming decode's memory pattern
// without its arithmetic (diagnostic; bench.py times it on the same box, in the same process,
// right after the timed region, so the decode's time can be stated against the rate this box's
// HBM gives that exact pattern).
//
// decode_stream_kernel<LOG2M, NA> (decode_stream.hip) moves, per decoded symbol, N antenna rows
// of M + 2 complex64 samples (the body from its 16-byte-aligned start) into LDS by LDS-DMA, the
// N x M_occ uint8 transmitted indices likewise (ref_mode 1), and writes N x M_occ complex64
// symbols (16-byte non-temporal stores) and N x M_occ uint8 indices (2-byte stores,
// non-temporal from M = 2048 up), symbol-major. pattern_kernel does exactly that -- the same
// persistent grid of one NA x M / 8-thread workgroup per CU walking a contiguous range of the
// symbols, the same staging DMA pieces and counted vmcnt wait at the top of a symbol, the next
// symbol's DMA issued after the staging reads, the same store instructions -- with no transform,
// no apply and no demap: the stored values are the staged samples. Its time is the floor the
// decode's own instruction stream sits on (tools/micro/stream_ceiling.hip is the standalone
// form of the same pattern, with its variants).
#include "common.hpp"
#include "fft.hpp"

namespace mimo {
namespace {

MIMO_DEV void probe_dma16(uint32_t voff, __attribute__((address_space(1))) const void *sbase,
                          uint32_t lds) {
  uint32_t keep;
  asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, %2 nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds) : "memory");
}

struct PatternArgs {
  const float2 *iq;           // [n_caps][N][stride]
  uint64_t stride;            // samples between antenna rows
  const uint8_t *ref;         // [F][spf][N][M] reference indices (symbol-major)
  float2 *out_sym;            // [F][spf][N][M]
  uint8_t *out_idx;
  uint32_t n_frames, spf, SL, body0;   // body of symbol s of frame f at (f N + r) stride + body0 + s SL
};

template <int LOG2M, int NA>
__global__ __launch_bounds__(NA * (1 << LOG2M) / 8) void pattern_kernel(PatternArgs a) {
  constexpr int M = 1 << LOG2M, T = NA * M / 8;
  constexpr int RS = M + 2;                              // staged samples per row
  constexpr int NPC = (RS * 8 + 1023) / 1024;            // 1 KB DMA pieces per row
  constexpr int LASTC = (RS * 8 - (NPC - 1) * 1024) / 16;   // 16-byte chunks of the last piece
  constexpr int CPT = (M / 2) / T;                       // 16-byte symbol chunks per stream and thread
  constexpr int NREF = NA * M / 1024;                    // reference pieces per symbol
  constexpr int NSTORE = 2 * NA * CPT;                   // store instructions per thread and symbol
  static_assert(CPT >= 1 && T / 64 >= NA + 1, "row waves and reference waves");
  extern __shared__ __attribute__((aligned(16))) float2 stg[];          // [NA][RS] then [NA][M] bytes
  uint8_t *rstg = reinterpret_cast<uint8_t *>(stg + NA * RS);
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane((uint32_t)tid >> 6);
  const uint32_t nsym = a.n_frames * a.spf;
  const uint32_t chunk = (nsym + gridDim.x - 1) / gridDim.x;
  const uint32_t i0 = blockIdx.x * chunk, i1 = min(i0 + chunk, nsym);
  if (i0 >= i1) return;
  auto fetch = [&](uint32_t i) {
    const uint32_t f = i / a.spf, s = i % a.spf;
    if (wv < (uint32_t)NA) {                             // wave g stages antenna row g
      // (from the 16-byte-aligned sample at or before the body, as the decode stages a row)
      const uint64_t e = (((uint64_t)f * NA + wv) * a.stride + a.body0 + (uint64_t)s * a.SL) & ~1ull;
      const auto xa = sgpr_ptr(reinterpret_cast<const char *>(a.iq + e));
      const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(stg + wv * RS));
#pragma unroll
      for (int b = 0; b < NPC; b++)
        if (b + 1 < NPC || lane < LASTC) probe_dma16(b * 1024u + lane * 16u, xa, dst + b * 1024u);
    } else {                                             // the next waves the reference pieces
      for (uint32_t p = wv - NA; p < (uint32_t)NREF; p += T / 64 - NA) {
        const auto rb = sgpr_ptr(a.ref + ((uint64_t)f * a.spf + s) * NA * M + p * 1024u);
        probe_dma16(lane * 16u, rb,
                    __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(rstg + p * 1024u)));
      }
    }
  };
  fetch(i0);
  for (uint32_t i = i0; i < i1; i++) {
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NSTORE) : "memory");
    __syncthreads();
    const uint32_t f = i / a.spf, s = i % a.spf;
    // the thread's staged values: stream t's chunk c (subcarriers 2 (tid + T c), + 1)
    v4f v[NA][CPT];
    uint16_t rw[NA][CPT];
#pragma unroll
    for (int t = 0; t < NA; t++)
#pragma unroll
      for (int c = 0; c < CPT; c++) {
        const int k = 2 * (tid + T * c);
        v[t][c] = *reinterpret_cast<const v4f *>(stg + t * RS + k);
        rw[t][c] = *reinterpret_cast<const uint16_t *>(rstg + t * M + k);
      }
    __syncthreads();
    if (i + 1 < i1) fetch(i + 1);
    const uint64_t ob = ((uint64_t)f * a.spf + s) * NA * M;
#pragma unroll
    for (int t = 0; t < NA; t++)
#pragma unroll
      for (int c = 0; c < CPT; c++) {
        const uint32_t k = 2u * (uint32_t)(tid + T * c);
        __builtin_nontemporal_store(v[t][c], reinterpret_cast<v4f *>(a.out_sym + ob + (uint64_t)t * M + k));
        if constexpr (LOG2M >= 11)
          __builtin_nontemporal_store(rw[t][c], reinterpret_cast<uint16_t *>(a.out_idx + ob + (uint64_t)t * M + k));
        else
          *reinterpret_cast<uint16_t *>(a.out_idx + ob + (uint64_t)t * M + k) = rw[t][c];
      }
  }
}

template <int LOG2M, int NA>
int pattern_launch(const PatternArgs &a, int n_cu, hipStream_t s) {
  constexpr int M = 1 << LOG2M, T = NA * M / 8;
  const size_t shm = sizeof(float2) * NA * (M + 2) + (size_t)NA * M;
  auto k = pattern_kernel<LOG2M, NA>;
  if (hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm) !=
      hipSuccess)
    return -1;
  hipLaunchKernelGGL(k, dim3(n_cu), dim3(T), shm, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace
}  // namespace mimo

extern "C" int mimo_probe_decode_pattern(const void *d_iq, uint64_t stride, uint32_t n_caps,
                                         uint32_t N, uint32_t M, uint32_t cp, uint32_t n_frames,
                                         uint32_t spf, const void *d_ref, void *d_out_sym,
                                         void *d_out_idx, int reps, void *hip_stream,
                                         float *ms_per_launch) {
  using namespace mimo;
  if (!d_iq || !d_ref || !d_out_sym || !d_out_idx || !ms_per_launch || reps < 1 || !n_frames ||
      !spf || n_frames > n_caps)
    return 1;
  const uint32_t SL = M + cp;
  // the bodies of spf symbols from sample 2 SL on (16-byte aligned, as the decode stages them)
  const uint64_t body0 = 2ull * SL & ~1ull;
  if (body0 + (uint64_t)spf * SL + 2 > stride) return 1;
  PatternArgs a{};
  a.iq = reinterpret_cast<const float2 *>(d_iq);
  a.stride = stride;
  a.ref = reinterpret_cast<const uint8_t *>(d_ref);
  a.out_sym = reinterpret_cast<float2 *>(d_out_sym);
  a.out_idx = reinterpret_cast<uint8_t *>(d_out_idx);
  a.n_frames = n_frames;
  a.spf = spf;
  a.SL = SL;
  a.body0 = (uint32_t)body0;
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 1)
    return 2;
  hipStream_t s = reinterpret_cast<hipStream_t>(hip_stream);
  auto launch = [&]() -> int {
    if (N == 4 && M == 2048) return pattern_launch<11, 4>(a, ncu, s);
    if (N == 4 && M == 1024) return pattern_launch<10, 4>(a, ncu, s);
    if (N == 2 && M == 4096) return pattern_launch<12, 2>(a, ncu, s);
    if (N == 2 && M == 2048) return pattern_launch<11, 2>(a, ncu, s);
    if (N == 2 && M == 1024) return pattern_launch<10, 2>(a, ncu, s);
    return 3;
  };
  int rc = launch();                                     // warm-up
  if (rc) return rc;
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return 2;
  (void)hipEventRecord(e0, s);
  for (int r = 0; r < reps && !rc; r++) rc = launch();
  (void)hipEventRecord(e1, s);
  float ms = 0.0f;
  if (!rc && (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess))
    rc = 2;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  *ms_per_launch = rc ? 0.0f : ms / (float)reps;
  return rc;
}

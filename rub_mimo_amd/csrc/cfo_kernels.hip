// cfo_kernels.hip -- carrier-frequency-offset estimate from the Schmidl-Cox correlation and
// derotation (the reference leaves it as a FIXME, mimo/framing.cc:486).
//
// The S0 preamble has period M/2 in time (mimo/framing.cc:1054-1111), so over its body
//   P = sum_{n=start}^{start+M/2-1} conj(x[n]) x[n + M/2]
// has angle 2 pi nu M/2 for a frequency offset of nu cycles/sample; in subcarrier spacings
// eps = nu M = arg(P) / pi (|eps| < 1). Derotation multiplies x[n] by exp(-j 2 pi nu (n - n0)).
// Both are opt-in building blocks beside the parity path: the reference never derotates.
//
// Estimate: one workgroup per antenna row, fp64 accumulation, LDS tree reduction.
// Derotate: elementwise, phase in fp64 reduced mod 1 before sincospi, so long captures keep
// their phase accuracy.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>

#include "kernels.hpp"

namespace mimo {

namespace {

constexpr int kCfoThreads = 256;

__global__ __launch_bounds__(kCfoThreads) void cfo_corr_kernel(const float2 *__restrict__ x,
                                                               uint64_t stride, uint64_t start,
                                                               uint32_t half,
                                                               double *__restrict__ out) {
  const float2 *row = x + blockIdx.x * stride + start;
  double re = 0.0, im = 0.0;
  for (uint32_t n = threadIdx.x; n < half; n += kCfoThreads) {
    const float2 a = row[n], b = row[n + half];
    // conj(a) * b
    re += (double)a.x * b.x + (double)a.y * b.y;
    im += (double)a.x * b.y - (double)a.y * b.x;
  }
  __shared__ double sre[kCfoThreads], sim[kCfoThreads];
  sre[threadIdx.x] = re;
  sim[threadIdx.x] = im;
  __syncthreads();
  for (int w = kCfoThreads / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      sre[threadIdx.x] += sre[threadIdx.x + w];
      sim[threadIdx.x] += sim[threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = sre[0];
    out[2 * blockIdx.x + 1] = sim[0];
  }
}

__global__ __launch_bounds__(kCfoThreads) void cfo_derotate_kernel(float2 *__restrict__ x,
                                                                   uint64_t stride, uint64_t n,
                                                                   int64_t n0, double nu) {
  const uint64_t i = uint64_t(blockIdx.x) * kCfoThreads + threadIdx.x;
  if (i >= n) return;
  float2 *p = x + blockIdx.y * stride + i;
  double ph = -2.0 * nu * (double)((int64_t)i - n0);   // in units of pi
  ph -= 2.0 * rint(ph * 0.5);                           // reduce to [-1, 1]
  double s, c;
  sincospi(ph, &s, &c);
  const float2 v = *p;
  *p = make_float2((float)(v.x * c - v.y * s), (float)(v.x * s + v.y * c));
}

// Batched path (mimo_rx_config.cfo_correct), two stages per synced frame, sums over the
// antennas in fp64:
//  1. coarse, |eps| < 1, before the search: the S0 half-period correlation over the S&C window
//     ending at the trigger (x[t-M+1 .. t] lies in the M/2-periodic S0, cyclic prefix included,
//     since y[t] > thr on every antenna): eps0 = arg(P) / pi; the frame's window is derotated by
//     eps0 into a scratch capture that search, LS, weights and decode read.
//  2. fine, after the search: one S0 leaves a residual of ~1e-4 subcarrier spacings at 30 dB,
//     ~0.3-1 rad of drift over 1000 symbols (and a phase spread across the access codes that
//     the MMSE noise estimate would read as noise). The cyclic prefixes of the data symbols --
//     their positions known from the search (base + i0 + s SL, framing.cc:857) -- correlate
//     conj(x[k]) x[k + M] over each prefix's interior: delta = arg(P) / (2 pi) on the coarse-
//     corrected samples. The LS terms are rotated by delta at their code windows
//     (ls_combine_q_kernel) and the data region is derotated by delta, both about base.
// Blocks sum fixed symbol subsets into partials, combined in fixed order by the rotation
// kernels (bitwise reproducible).
constexpr uint32_t kCfoMargin = 4;   // prefix samples skipped at each end

MIMO_DEV bool cfo_live(const FrameInfo &I) { return I.status == 0 || I.status == 2; }

// replay start from the search's last access-code key (framing.cc:857), as weights_kernel
MIMO_DEV int64_t cfo_i0(const CfoBatchArgs &a, uint32_t f) {
  const unsigned long long key =
      a.keys[((uint64_t)f * a.N + (a.N - 1)) * a.n_slots + a.n_slots - 1];
  const uint32_t ci = key ? (0xFFFFFFFFu - (uint32_t)(key & 0xFFFFFFFFull)) : 0u;
  return (int64_t)ci + a.M;
}

template <int STAGE>
__global__ __launch_bounds__(kCfoThreads) void cfo_batch_est_kernel(CfoBatchArgs a) {
  const uint32_t f = blockIdx.y, b = blockIdx.x;
  const FrameInfo &I = a.info[f];
  __shared__ double sre[kCfoThreads], sim[kCfoThreads];
  const bool live = STAGE == 1 ? cfo_live(I) : I.status == 0;
  double re = 0.0, im = 0.0;
  const int64_t L = (int64_t)a.frame_len;
  // folded path: no scratch, stage 2 reads the raw samples (below)
  const float2 *src = (STAGE == 1 || a.fold) ? a.iq : a.out;
  if (live && STAGE == 1) {
    for (uint32_t r = 0; r < a.N; r++) {
      const float2 *row = src + ((uint64_t)I.cap * a.N + r) * a.stride;
      const uint32_t half = a.M / 2;
      const int64_t start = (int64_t)I.trigger - (int64_t)a.M + 1;
      for (uint32_t n = b * kCfoThreads + threadIdx.x; n < half; n += kCfoBlocks * kCfoThreads) {
        const int64_t k = start + n;
        if (k < 0 || k + half >= L) continue;
        const float2 u = row[k], v = row[k + half];
        re += (double)u.x * v.x + (double)u.y * v.y;
        im += (double)u.x * v.y - (double)u.y * v.x;
      }
    }
  } else if (live) {
    // the block's symbols sym = b + kCfoBlocks j, every antenna, the prefix interiors: the
    // block's (run, sample) pairs -- run p = (symbol j, antenna r), sample n < inner --
    // flattened over the threads (a thread per sample of one run left 256 - inner lanes idle),
    // U pairs per thread with all 2U loads issued before the sums
    const uint32_t inner = a.cp > 2 * kCfoMargin ? a.cp - 2 * kCfoMargin : 0;
    const int64_t d0 = I.base + cfo_i0(a, f);               // data symbol 0's prefix
    // (the reads stay inside the framesync's window, as the reference's ring holds it: the
    // capture may hold more, the window does not)
    const int64_t wend = std::min<int64_t>(L, I.base + (int64_t)a.win);
    const uint32_t nsym = a.n_data > b ? (a.n_data - b + kCfoBlocks - 1) / kCfoBlocks : 0u;
    const uint32_t items = nsym * a.N * inner;
    const float inv_inner = inner ? 1.0f / (float)inner : 0.0f;
    const float2 *cap = src + (uint64_t)I.cap * a.N * a.stride;
    constexpr int U = 8;
    for (uint32_t g0 = 0; g0 < items; g0 += U * kCfoThreads) {
      float2 u[U], v[U];
      bool ok[U];
#pragma unroll
      for (int e = 0; e < U; e++) {
        const uint32_t g = g0 + (uint32_t)e * kCfoThreads + threadIdx.x;
        // p = g / inner, n = g % inner (the fp32 quotient is within one of it: corrected)
        int32_t p = (int32_t)((float)g * inv_inner);
        int32_t n = (int32_t)g - p * (int32_t)inner;
        if (n >= (int32_t)inner) { p++; n -= (int32_t)inner; }
        if (n < 0) { p--; n += (int32_t)inner; }
        const uint32_t js = (uint32_t)p / a.N, r = (uint32_t)p % a.N;
        const int64_t k = d0 + (int64_t)(b + js * kCfoBlocks) * a.SL + kCfoMargin + n;
        ok[e] = g < items && k >= 0 && k + a.M < wend;
        const float2 *row = cap + (uint64_t)(g < items ? r : 0u) * a.stride;
        const int64_t kk = ok[e] ? k : 0;
        u[e] = row[kk];
        v[e] = row[kk + (ok[e] ? a.M : 0)];
      }
#pragma unroll
      for (int e = 0; e < U; e++) {
        if (!ok[e]) continue;
        re += (double)u[e].x * v[e].x + (double)u[e].y * v[e].y;
        im += (double)u[e].x * v[e].y - (double)u[e].y * v[e].x;
      }
    }
  }
  sre[threadIdx.x] = re;
  sim[threadIdx.x] = im;
  __syncthreads();
  for (int w = kCfoThreads / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      sre[threadIdx.x] += sre[threadIdx.x + w];
      sim[threadIdx.x] += sim[threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    double re0 = sre[0], im0 = sim[0];
    if (STAGE == 2 && a.fold && live) {
      // on the raw samples conj(x[k]) x[k + M] lacks the stage-1 derotation's constant factor
      // exp(-j 2 pi eps0): applied to the block's partial (the sum is linear in it)
      double ph = -2.0 * cfo_stage_eps(a.part, f, 1);   // units of pi
      ph -= 2.0 * rint(ph * 0.5);
      double sn, cs;
      sincospi(ph, &sn, &cs);
      const double r2 = re0 * cs - im0 * sn, i2 = re0 * sn + im0 * cs;
      re0 = r2;
      im0 = i2;
    }
    double *p = a.part + (((uint64_t)f * 2 + (STAGE - 1)) * kCfoBlocks + b) * 2;
    p[0] = re0;
    p[1] = im0;
  }
}

// x[n] exp(-j 2 pi (eps / M)(n - base)) over [n0, n0 + len) of every antenna: stage 1 from the
// input into the scratch capture over the frame's window (n0 = base); stage 2 in place, over
// the data region (n0 = base + i0; the LS terms were corrected to the same reference in
// ls_combine_q_kernel) or, before a separate LS pass, over the whole window
template <int STAGE>
__global__ __launch_bounds__(kCfoThreads) void cfo_batch_rot_kernel(CfoBatchArgs a) {
  FrameInfo &I = a.info[blockIdx.z];
  if (STAGE == 1 ? !cfo_live(I) : I.status != 0) return;
  const double eps = cfo_stage_eps(a.part, blockIdx.z, STAGE);
  const double eps0 = STAGE == 2 ? cfo_stage_eps(a.part, blockIdx.z, 1) : 0.0;
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    I.cfo_eps = (float)(eps + eps0);
    I.cfo_E = cfo_fixed_freq(eps + eps0, a.M);
  }
  const double nu = eps / (double)a.M;
  const uint64_t off = ((uint64_t)I.cap * a.N + blockIdx.y) * a.stride;
  const bool whole = STAGE == 1 || a.rot_window;
  const int64_t n0 = whole ? I.base : I.base + cfo_i0(a, blockIdx.z);
  const int64_t nref = I.base;
  const uint64_t len = whole ? a.len : (uint64_t)a.n_data * a.SL + 64;
  const float2 *src = STAGE == 1 ? a.iq : a.out;
  for (uint64_t i = (uint64_t)blockIdx.x * kCfoThreads + threadIdx.x; i < len;
       i += (uint64_t)gridDim.x * kCfoThreads) {
    const int64_t n = n0 + (int64_t)i;
    if (n < 0 || n >= (int64_t)a.frame_len) continue;
    double ph = -2.0 * nu * (double)(n - nref);                // in units of pi, fp64
    ph -= 2.0 * rint(ph * 0.5);                                // [-1, 1]: fp32 from here on
    float s, c;
    sincospif((float)ph, &s, &c);
    const float2 v = src[off + n];
    a.out[off + n] = make_float2(v.x * c - v.y * s, v.x * s + v.y * c);
  }
}

}  // namespace

size_t cfo_batch_part_doubles(uint32_t n_frames) { return (size_t)n_frames * 2 * kCfoBlocks * 2; }

void launch_cfo_batch(const CfoBatchArgs &a, uint32_t n_frames, int stage, hipStream_t s) {
  if (n_frames == 0) return;
  const uint32_t blocks =
      (uint32_t)std::min<uint64_t>((a.len + kCfoThreads - 1) / kCfoThreads, 2048);
  if (stage == 1) {
    cfo_batch_est_kernel<1><<<dim3(kCfoBlocks, n_frames), kCfoThreads, 0, s>>>(a);
    if (!a.fold) cfo_batch_rot_kernel<1><<<dim3(blocks, a.N, n_frames), kCfoThreads, 0, s>>>(a);
  } else {
    cfo_batch_est_kernel<2><<<dim3(kCfoBlocks, n_frames), kCfoThreads, 0, s>>>(a);
    if (a.rot_window)
      cfo_batch_rot_kernel<2><<<dim3(blocks, a.N, n_frames), kCfoThreads, 0, s>>>(a);
  }
}

void launch_cfo_batch_rot2(const CfoBatchArgs &a, uint32_t n_frames, hipStream_t s) {
  if (n_frames == 0) return;
  const uint64_t span = (uint64_t)a.n_data * a.SL + 64;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((span + kCfoThreads - 1) / kCfoThreads, 2048);
  cfo_batch_rot_kernel<2><<<dim3(blocks, a.N, n_frames), kCfoThreads, 0, s>>>(a);
}

bool launch_cfo_corr(const void *x, uint64_t stride, uint32_t rows, uint64_t start,
                     uint32_t half, double *d_out, hipStream_t s) {
  if (rows == 0 || rows > 65535) return false;
  cfo_corr_kernel<<<rows, kCfoThreads, 0, s>>>(static_cast<const float2 *>(x), stride, start,
                                               half, d_out);
  return true;
}

bool launch_cfo_derotate(void *x, uint64_t stride, uint32_t rows, uint64_t n, int64_t n0,
                         double nu, hipStream_t s) {
  if (n == 0 || rows == 0) return true;
  const uint64_t blocks = (n + kCfoThreads - 1) / kCfoThreads;
  if (blocks > 0x7fffffffull || rows > 65535) return false;
  cfo_derotate_kernel<<<dim3(uint32_t(blocks), rows), kCfoThreads, 0, s>>>(
      static_cast<float2 *>(x), stride, n, n0, nu);
  return true;
}

}  // namespace mimo

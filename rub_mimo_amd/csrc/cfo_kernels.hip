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

}  // namespace

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

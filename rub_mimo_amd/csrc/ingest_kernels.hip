// ingest_kernels.hip -- capture ingest at the wire format.
//
// The reference's rx worker asks UHD for fc32 on the host (mimo/config.h:51-52: CPU format
// fc32, wire sc16) and so moves 8 B per sample over PCIe and into framesync's window
// (mimo/main.cc:837-848, 872-898). Here the capture can stay sc16 (interleaved int16 I/Q,
// 4 B per sample) up to HBM; this kernel widens it into the planar complex64 batch layout of
// mimo_batch (include/mimo_rx.h) on the device: 4 B read + 8 B written per sample, HBM-bound.
//
// One thread converts 4 samples: one 16-byte load, two 16-byte stores. Rows (antenna arrays)
// are independent; the grid is (chunks of 4 * 256 samples, rows). Arithmetic: float(i16) *
// scale, one rounding, bit-identical to numpy's astype(float32) * float32(scale) and to the
// kernels that read sc16 in place (Iq<true>, common.hpp).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"

namespace mimo {

namespace {

constexpr int kThreads = 256;

// One thread converts 4 samples from the row's first 16-byte-aligned source sample h (rows of
// any stride: h = (-row * src_stride) mod 4 when the bases are aligned); the h head samples and
// the ragged tail go one per thread. The destination is 16-byte aligned at h whenever
// row * dst_stride + h is even, which the launcher checks for every row (equal strides, or an
// even dst_stride with a src_stride that is a multiple of 4).
__device__ __forceinline__ float wide(int16_t v, float scale) { return float(v) * scale; }

__global__ __launch_bounds__(kThreads) void sc16_to_fc32_vec_kernel(
    const int16_t *__restrict__ src, uint64_t src_stride, float *__restrict__ dst,
    uint64_t dst_stride, uint64_t n, float scale) {
  const uint64_t row = blockIdx.y;
  const uint64_t h = (4 - (row * src_stride) % 4) % 4;
  const int16_t *s = src + 2 * row * src_stride;
  float *d = dst + 2 * row * dst_stride;
  const uint64_t t = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  if (t < h && t < n) {
    d[2 * t] = wide(s[2 * t], scale);
    d[2 * t + 1] = wide(s[2 * t + 1], scale);
  }
  const uint64_t i = h + t * 4;                  // first sample of this thread's group
  if (i >= n) return;
  if (i + 4 <= n) {
    const int4 v = *reinterpret_cast<const int4 *>(s + 2 * i);      // 4 samples = 8 int16
    const int w[4] = {v.x, v.y, v.z, v.w};
    float o[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      o[2 * k] = wide(int16_t(w[k] & 0xffff), scale);
      o[2 * k + 1] = wide(int16_t(uint32_t(w[k]) >> 16), scale);
    }
    reinterpret_cast<float4 *>(d + 2 * i)[0] = make_float4(o[0], o[1], o[2], o[3]);
    reinterpret_cast<float4 *>(d + 2 * i)[1] = make_float4(o[4], o[5], o[6], o[7]);
  } else {
    for (uint64_t k = i; k < n; ++k) {
      d[2 * k] = wide(s[2 * k], scale);
      d[2 * k + 1] = wide(s[2 * k + 1], scale);
    }
  }
}

// misaligned bases: one sample per thread
__global__ __launch_bounds__(kThreads) void sc16_to_fc32_kernel(
    const int16_t *__restrict__ src, uint64_t src_stride, float *__restrict__ dst,
    uint64_t dst_stride, uint64_t n, float scale) {
  const uint64_t row = blockIdx.y;
  const uint64_t i = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  if (i >= n) return;
  const int16_t *s = src + 2 * (row * src_stride + i);
  float *d = dst + 2 * (row * dst_stride + i);
  d[0] = wide(s[0], scale);
  d[1] = wide(s[1], scale);
}

}  // namespace

bool launch_sc16_to_fc32(const void *src, uint64_t src_stride, void *dst, uint64_t dst_stride,
                         uint32_t rows, uint64_t n, float scale, hipStream_t s) {
  if (n == 0 || rows == 0) return true;
  const bool vec = (reinterpret_cast<uintptr_t>(src) % 16 == 0) &&
                   (reinterpret_cast<uintptr_t>(dst) % 16 == 0) &&
                   (src_stride == dst_stride || (src_stride % 4 == 0 && dst_stride % 2 == 0));
  const uint64_t per_block = vec ? uint64_t(kThreads) * 4 : uint64_t(kThreads);
  const uint64_t blocks = (n + per_block - 1) / per_block;
  if (blocks > 0x7fffffffull || rows > 65535) return false;
  const dim3 grid(uint32_t(blocks), rows);
  if (vec)
    sc16_to_fc32_vec_kernel<<<grid, kThreads, 0, s>>>(
        static_cast<const int16_t *>(src), src_stride, static_cast<float *>(dst), dst_stride, n,
        scale);
  else
    sc16_to_fc32_kernel<<<grid, kThreads, 0, s>>>(static_cast<const int16_t *>(src),
                                                  src_stride, static_cast<float *>(dst),
                                                  dst_stride, n, scale);
  return true;
}

}  // namespace mimo

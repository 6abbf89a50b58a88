// rub_mimo_amd/csrc/common.hpp -- shared device helpers for the gfx950 receive pipeline.
//
// Complex values are float2 (x = re, y = im), the interleaved std::complex<float> layout of
// gr_complex. Arithmetic helpers spell out every product and sum: the translation units that
// must agree bit-for-bit with the CPU oracle compile with -ffp-contract=off.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define MIMO_DEV __device__ __forceinline__

namespace mimo {

constexpr int kMaxStreams = 8;
constexpr int kTwLog2 = 14;             // twiddle table covers transforms up to 16384 points
constexpr int kTwN = 1 << kTwLog2;

MIMO_DEV float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
MIMO_DEV float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
MIMO_DEV float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
MIMO_DEV float2 cmulc(float2 a, float2 b) {  // a * conj(b)
  return make_float2(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y);
}
MIMO_DEV float2 cconj(float2 a) { return make_float2(a.x, -a.y); }
MIMO_DEV float2 cneg(float2 a) { return make_float2(-a.x, -a.y); }
MIMO_DEV float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
MIMO_DEV float cabs2(float2 a) { return a.x * a.x + a.y * a.y; }
MIMO_DEV float2 cdiv(float2 a, float2 b) {  // (a conj b)/|b|^2, exact for b = +-1
  float d = b.x * b.x + b.y * b.y;
  return make_float2((a.x * b.x + a.y * b.y) / d, (a.y * b.x - a.x * b.y) / d);
}

// ---------------- capture samples: complex64, or UHD sc16 on the wire ----------------
// A capture row is either interleaved fp32 (re, im) -- the fc32 samples the reference's rx
// worker hands framesync (mimo/main.cc:837-848) -- or the sc16 wire format (interleaved int16
// I/Q, mimo/config.h:52), read as float(i16) * scale: the same product as UHD's sc16 -> fc32
// converter and as mimo_ingest_sc16, so both give bit-identical samples to every kernel.
template <bool SC16>
struct Iq;

template <>
struct Iq<false> {
  const float2 *p;
  MIMO_DEV float2 at(int64_t i) const { return p[i]; }
  // samples i, i + 1 (i even, the row 16-byte aligned)
  MIMO_DEV float4 pair(int64_t i) const { return *reinterpret_cast<const float4 *>(p + i); }
  MIMO_DEV bool pair_ok() const { return ((uintptr_t)p & 15u) == 0; }
  MIMO_DEV Iq row(uint64_t off) const { return Iq{p + off}; }
};

template <>
struct Iq<true> {
  const short2 *p;
  float scale;
  MIMO_DEV float2 cvt(short2 s) const { return make_float2(wide16(s.x), wide16(s.y)); }
  // one rounded product, never contracted into a following add (hipcc's default
  // -ffp-contract=fast-honor-pragmas would otherwise fuse it into the FFT's first butterfly),
  // so the sample is the same fp32 value in every kernel and in mimo_ingest_sc16
  MIMO_DEV float wide16(short v) const {
#pragma clang fp contract(off)
    return (float)v * scale;
  }
  MIMO_DEV float2 at(int64_t i) const { return cvt(p[i]); }
  MIMO_DEV float4 pair(int64_t i) const {
    const uint2 w = *reinterpret_cast<const uint2 *>(p + i);
    const short2 a = make_short2((short)(w.x & 0xFFFFu), (short)(w.x >> 16));
    const short2 b = make_short2((short)(w.y & 0xFFFFu), (short)(w.y >> 16));
    const float2 fa = cvt(a), fb = cvt(b);
    return make_float4(fa.x, fa.y, fb.x, fb.y);
  }
  MIMO_DEV bool pair_ok() const { return ((uintptr_t)p & 7u) == 0; }
  MIMO_DEV Iq row(uint64_t off) const { return Iq{p + off, scale}; }
};

// row `off` (in samples) of a capture held as fc32 (S = false) or sc16 (S = true)
template <bool S>
MIMO_DEV Iq<S> iq_row(const float2 *iq, float scale, uint64_t off) {
  if constexpr (S) {
    return Iq<true>{reinterpret_cast<const short2 *>(iq) + off, scale};
  } else {
    (void)scale;
    return Iq<false>{iq + off};
  }
}

// ---------------- counter-based PRNG, bit-identical to oracle ref_hash5 ----------------
MIMO_DEV uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
MIMO_DEV uint64_t hash5(uint64_t seed, uint64_t dom, uint64_t a, uint64_t b, uint64_t c) {
  uint64_t h = mix64(seed ^ (dom * 0xD6E8FEB86659FD93ull));
  h = mix64(h ^ a);
  h = mix64(h ^ b);
  h = mix64(h ^ c);
  return h;
}
enum { DOM_DATA = 1, DOM_CHAN = 2, DOM_NOISE = 3, DOM_OFFSET = 4 };

MIMO_DEV float2 hash_cnormal(uint64_t h) {  // CN(0,1), Box-Muller
  float u1 = (float)((h >> 40) + 1ull) * 5.9604644775390625e-08f;
  float u2 = (float)((h >> 16) & 0xFFFFFFull) * 5.9604644775390625e-08f;
  float r = sqrtf(-2.0f * logf(u1));
  float th = 6.283185307179586f * u2;
  float s, c;
  sincosf(th, &s, &c);
  return make_float2(r * c * 0.70710678118654752f, r * s * 0.70710678118654752f);
}

// ---------------- square Gray QAM (same definition as oracle ref_qam_*) ----------------
struct Qam {
  uint32_t b;      // bits per dimension
  uint32_t L;      // levels per dimension
  float scale;     // 1/sqrt(2(L^2-1)/3)
  float inv_scale; // sqrt(2(L^2-1)/3)
};

MIMO_DEV uint32_t gray_enc(uint32_t m) { return m ^ (m >> 1); }
MIMO_DEV uint32_t gray_dec(uint32_t g) {
  uint32_t m = g;
  m ^= m >> 1; m ^= m >> 2; m ^= m >> 4; m ^= m >> 8;
  return m;
}
MIMO_DEV float2 qam_point(uint32_t idx, const Qam &q) {
  uint32_t mI = gray_dec(idx >> q.b), mQ = gray_dec(idx & (q.L - 1));
  return make_float2((float)(int32_t)(2 * mI - (q.L - 1)) * q.scale,
                     (float)(int32_t)(2 * mQ - (q.L - 1)) * q.scale);
}
MIMO_DEV uint32_t qam_level(float v, uint32_t L) {
  float t = (v + (float)L) * 0.5f;
  if (t != t) return 0;
  float f = floorf(t);
  int32_t m = (f < 0.0f) ? 0 : ((f > (float)(L - 1)) ? (int32_t)(L - 1) : (int32_t)f);
  return (uint32_t)m;
}
MIMO_DEV uint32_t qam_demap(float2 y, const Qam &q) {
  uint32_t mI = qam_level(y.x * q.inv_scale, q.L), mQ = qam_level(y.y * q.inv_scale, q.L);
  return (gray_enc(mI) << q.b) | gray_enc(mQ);
}

// ---------------- per-frame bookkeeping shared by the stages ----------------
// opt-in CFO partial correlations: [F][2 stages][kCfoBlocks][2] doubles (cfo_kernels.hip);
// stage 1 -> eps0 = arg / pi, stage 2 -> delta = arg / (2 pi), summed in fixed block order
constexpr int kCfoBlocks = 32;
MIMO_DEV double cfo_stage_eps(const double *part, uint32_t f, int stage) {
  const double *p = part + ((uint64_t)f * 2 + (uint64_t)(stage - 1)) * kCfoBlocks * 2;
  double re = 0.0, im = 0.0;
  for (int b = 0; b < kCfoBlocks; b++) {
    re += p[2 * b];
    im += p[2 * b + 1];
  }
  if (re == 0.0 && im == 0.0) return 0.0;
  return atan2(im, re) / (stage == 1 ? M_PI : 2.0 * M_PI);
}

struct FrameInfo {
  int32_t status;          // MIMO_FRAME_*
  uint32_t n_sym;          // decode callbacks available in the window
  uint64_t trigger;
  uint64_t sync_index;
  uint64_t nsp;            // num_samples_processed after one execute over the frame
  int64_t base;            // window start = sync_index - SL (absolute sample index)
  uint64_t plateau_start[kMaxStreams];
  uint64_t plateau_end[kMaxStreams];
  float noise_var;
  uint32_t i0;             // replay start, window index corr[N-1][last] + M
  uint64_t origin;         // capture sample where this frame's framesync started (0, or the
                           // re-arm point of a back-to-back stream); positions are absolute
  uint32_t cap;            // capture holding the frame (f when each capture is one frame)
  uint32_t ref;            // reference frame (ref_mode 1 index row, ref_mode 2 frame id - id0)
  float cfo_eps;           // opt-in CFO estimate (subcarrier spacings), 0 when off
  uint32_t pad_;
  int64_t cfo_E;           // the same as nu = eps / M cycles per sample in 64-bit fixed point
                           // (nu 2^64; the decode's per-symbol phasors, cfo_fixed_freq)
};
// the 64-bit fixed-point frequency of an offset of eps subcarrier spacings (|eps| < 2): the
// phase of sample j in turns is the wrapped product E j / 2^64, exact for every j
MIMO_DEV int64_t cfo_fixed_freq(double eps, uint32_t M) {
  return (int64_t)rint(ldexp(eps / (double)M, 64));
}

}  // namespace mimo

// rub_mimo_amd/csrc/fft.hpp -- LDS-resident Stockham FFT for one workgroup (gfx950).
//
// B transforms of N = 2^LOG2N points sit contiguously in LDS (buf[b*N + i]); T threads run
// radix-8 passes (a radix-4/2 tail when log2 N is not a multiple of 3). Each pass: every
// thread pulls its butterflies' inputs into registers, barrier, in-register radix-R DFT with
// table twiddles, writes in Stockham autosort order, barrier. Natural order in and out,
// unnormalised, FFTW sign convention (forward e^{-i}), replacing fftwf_plan_dft_1d /
// fftwf_execute of framing.cc:135-139, 368-372, 1066-1070, 1229-1233.
//
// The LDS image is padded: logical index i lives at i + (i >> 5) so the radix-8 stride-8
// writes of the first pass spread over the 32 banks instead of landing on two.
#pragma once

#include "common.hpp"

namespace mimo {

MIMO_DEV int lds_pad(int i) { return i + (i >> 5); }
constexpr int lds_padded_len(int n) { return n + (n >> 5); }

template <bool INV>
MIMO_DEV float2 twiddle(const float2 *__restrict__ tw, int idx) {
  float2 w = tw[idx];
  return INV ? make_float2(w.x, -w.y) : w;
}

// (x + iy) * (-i) forward, * (+i) inverse
template <bool INV>
MIMO_DEV float2 rot_mi(float2 a) {
  return INV ? make_float2(-a.y, a.x) : make_float2(a.y, -a.x);
}

template <int R, bool INV>
MIMO_DEV void dft_small(float2 *a) {
  if constexpr (R == 2) {
    float2 t0 = cadd(a[0], a[1]), t1 = csub(a[0], a[1]);
    a[0] = t0; a[1] = t1;
  } else if constexpr (R == 4) {
    float2 b0 = cadd(a[0], a[2]), b1 = csub(a[0], a[2]);
    float2 b2 = cadd(a[1], a[3]), b3 = rot_mi<INV>(csub(a[1], a[3]));
    a[0] = cadd(b0, b2); a[2] = csub(b0, b2);
    a[1] = cadd(b1, b3); a[3] = csub(b1, b3);
  } else {
    static_assert(R == 8, "radix");
    const float c = 0.70710678118654752f;
    float2 b0 = cadd(a[0], a[4]), b4 = csub(a[0], a[4]);
    float2 b1 = cadd(a[1], a[5]), b5 = csub(a[1], a[5]);
    float2 b2 = cadd(a[2], a[6]), b6 = csub(a[2], a[6]);
    float2 b3 = cadd(a[3], a[7]), b7 = csub(a[3], a[7]);
    if (!INV) {
      b5 = make_float2(c * (b5.x + b5.y), c * (b5.y - b5.x));   // * W8^1
      b6 = make_float2(b6.y, -b6.x);                            // * W8^2 = -i
      b7 = make_float2(c * (b7.y - b7.x), -c * (b7.x + b7.y));  // * W8^3
    } else {
      b5 = make_float2(c * (b5.x - b5.y), c * (b5.x + b5.y));
      b6 = make_float2(-b6.y, b6.x);
      b7 = make_float2(-c * (b7.x + b7.y), c * (b7.x - b7.y));
    }
    float2 c0 = cadd(b0, b2), c2 = csub(b0, b2);
    float2 c1 = cadd(b1, b3), c3 = rot_mi<INV>(csub(b1, b3));
    float2 c4 = cadd(b4, b6), c6 = csub(b4, b6);
    float2 c5 = cadd(b5, b7), c7 = rot_mi<INV>(csub(b5, b7));
    a[0] = cadd(c0, c1); a[4] = csub(c0, c1);
    a[2] = cadd(c2, c3); a[6] = csub(c2, c3);
    a[1] = cadd(c4, c5); a[5] = csub(c4, c5);
    a[3] = cadd(c6, c7); a[7] = csub(c6, c7);
  }
}

// one Stockham pass: sub-transform size NS -> NS*R
template <int N, int R, int NS, int T, int B, bool INV>
MIMO_DEV void fft_pass(float2 *buf, const float2 *__restrict__ tw) {
  constexpr int NB = N / R;
  constexpr int TOT = NB * B;
  constexpr int PER = (TOT + T - 1) / T;
  constexpr int PB = lds_padded_len(N);
  float2 a[PER][R];
#pragma unroll
  for (int q = 0; q < PER; q++) {
    const int g = threadIdx.x + q * T;
    if ((TOT % T == 0) || g < TOT) {
      const int b = g / NB, j = g % NB;
      const float2 *base = buf + b * PB;
#pragma unroll
      for (int r = 0; r < R; r++) a[q][r] = base[lds_pad(j + r * NB)];
      if constexpr (NS > 1) {
        // one table read per butterfly; the other R-2 twiddles are products of it
        // (<= 3 roundings deep, well inside the fp32 FFT error budget)
        const int k = j % NS;
        constexpr int STEP = kTwN / (NS * R);
        float2 w[R];
        w[1] = twiddle<INV>(tw, k * STEP);
        if constexpr (R >= 4) {
          w[2] = cmul(w[1], w[1]);
          w[3] = cmul(w[2], w[1]);
        }
        if constexpr (R == 8) {
          w[4] = cmul(w[2], w[2]);
          w[5] = cmul(w[4], w[1]);
          w[6] = cmul(w[3], w[3]);
          w[7] = cmul(w[4], w[3]);
        }
#pragma unroll
        for (int r = 1; r < R; r++) a[q][r] = cmul(a[q][r], w[r]);
      }
      dft_small<R, INV>(a[q]);
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < PER; q++) {
    const int g = threadIdx.x + q * T;
    if ((TOT % T == 0) || g < TOT) {
      const int b = g / NB, j = g % NB;
      const int k = j % NS;
      const int o = (j / NS) * NS * R + k;
      float2 *base = buf + b * PB;
#pragma unroll
      for (int r = 0; r < R; r++) base[lds_pad(o + r * NS)] = a[q][r];
    }
  }
  __syncthreads();
}

template <int N, int NS, int REM, int T, int B, bool INV>
MIMO_DEV void fft_passes(float2 *buf, const float2 *__restrict__ tw) {
  if constexpr (REM > 0) {
    constexpr int LR = (REM == 4) ? 2 : ((REM >= 3) ? 3 : REM);
    constexpr int R = 1 << LR;
    fft_pass<N, R, NS, T, B, INV>(buf, tw);
    fft_passes<N, NS * R, REM - LR, T, B, INV>(buf, tw);
  }
}

// B transforms of 2^LOG2N points at buf[b * lds_padded_len(N) + lds_pad(i)]. Caller must
// __syncthreads() after filling buf; on return buf holds the result (barrier included).
template <int LOG2N, int T, int B, bool INV>
MIMO_DEV void fft_lds(float2 *buf, const float2 *__restrict__ tw) {
  fft_passes<(1 << LOG2N), 1, LOG2N, T, B, INV>(buf, tw);
}

}  // namespace mimo

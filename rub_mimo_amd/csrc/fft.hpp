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

// complex values as 2-wide fp32 vectors: adds, multiplies and FMAs on them lower to the
// packed v_pk_add/mul/fma_f32 instructions (two lanes of work per VALU op), with swizzles and
// negations folded into op_sel / neg modifiers
typedef float v2f __attribute__((ext_vector_type(2)));


// The same operations as single VOP3P instructions with the swizzle and the sign folded into
// op_sel / neg modifiers (the compiler materialises {-b.y, b.x} with a v_xor and a v_mov
// first). Results are bitwise those of vmul / rot_mi forms above.
// a wave-uniform global pointer held in SGPRs (address arithmetic feeding it may sit in
// VGPRs); global address space, so accesses through it are global_* with an SGPR base and a
// 32-bit lane offset, not flat_* (flat stores also count on lgkmcnt: every LDS wait would
// drain them)
MIMO_DEV uint64_t rfl64(uint64_t v) {   // a uniform 64-bit value, held in SGPRs
  // (the builtin returns int: each half goes through uint32_t, or a low half with bit 31 set
  // would sign-extend over the high half)
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

template <typename P>
using gptr = __attribute__((address_space(1))) P *;
typedef float v4f __attribute__((ext_vector_type(4)));
template <typename P>
MIMO_DEV gptr<P> sgpr_ptr(P *p) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (gptr<P>)(((uint64_t)hi << 32) | lo);
}


MIMO_DEV v2f cmul_pk(v2f a, v2f b) {     // a * b: (a.x b.x - a.y b.y, a.x b.y + a.y b.x)
  v2f r;
  // one asm block: the compiler pads between separate inline-asm VALU blocks with s_nop
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]\n\t"
      "v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
      : "=&v"(r) : "v"(a), "v"(b));
  return r;
}
MIMO_DEV v2f cmac_pk(v2f y, v2f w, v2f x) {   // y + w * x, as fma(w.xx, x, y) then fma(w.yy, ix, .)
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]\n\t"
      "v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
      : "+v"(y) : "v"(w), "v"(x));
  return y;
}
MIMO_DEV v2f add_mi(v2f a, v2f b) {      // a + b * (-i) = (a.x + b.y, a.y - b.x)
  v2f r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
MIMO_DEV v2f sub_mi(v2f a, v2f b) {      // a - b * (-i) = (a.x - b.y, a.y + b.x)
  v2f r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
MIMO_DEV v2f rot_m_b(v2f b) {            // b * (-i) - b = (b.y - b.x, -b.x - b.y)
  v2f r;
  asm("v_pk_add_f32 %0, %1, %1 op_sel:[1,0] op_sel_hi:[0,1] neg_lo:[0,1] neg_hi:[1,1]" : "=v"(r) : "v"(b));
  return r;
}

MIMO_DEV v2f rot_p_b(v2f b) {            // b * (+i) - b = (-b.y - b.x, b.x - b.y)
  v2f r;
  asm("v_pk_add_f32 %0, %1, %1 op_sel:[1,0] op_sel_hi:[0,1] neg_lo:[1,1] neg_hi:[0,1]" : "=v"(r) : "v"(b));
  return r;
}

// a * b = fma(a.yy, {-b.y, b.x}, a.xx * b) and a * conj(b) = fma(b.yy, {a.y, -a.x}, b.xx * a),
// each as two VOP3P instructions
MIMO_DEV v2f vmul(v2f a, v2f b) { return cmul_pk(a, b); }
MIMO_DEV v2f vmulc(v2f a, v2f b) {
  v2f r;
  asm("v_pk_mul_f32 %0, %2, %1 op_sel_hi:[0,1]\n\t"
      "v_pk_fma_f32 %0, %2, %1, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_hi:[0,1,0]"
      : "=&v"(r) : "v"(a), "v"(b));
  return r;
}

// w[q] = w1^q for q < R (w[0] unused), at most three roundings deep (as reg_compute)
template <int R>
MIMO_DEV void twiddle_powers(v2f *w, v2f w1) {
  w[1] = w1;
  if constexpr (R >= 4) {
    w[2] = vmul(w[1], w[1]);
    w[3] = vmul(w[2], w[1]);
  }
  if constexpr (R >= 8) {
    w[4] = vmul(w[2], w[2]);
    w[5] = vmul(w[4], w[1]);
    w[6] = vmul(w[3], w[3]);
    w[7] = vmul(w[4], w[3]);
  }
  if constexpr (R == 16) {
    w[8] = vmul(w[4], w[4]);
    w[9] = vmul(w[8], w[1]);
    w[10] = vmul(w[5], w[5]);
    w[11] = vmul(w[8], w[3]);
    w[12] = vmul(w[6], w[6]);
    w[13] = vmul(w[8], w[5]);
    w[14] = vmul(w[7], w[7]);
    w[15] = vmul(w[8], w[7]);
  }
}

// forward radix-2/4/8 DFTs on the packed forms (same arithmetic as dft_small<R, false>)
template <int R>
MIMO_DEV void dft_fwd_pk(v2f *a) {
  if constexpr (R == 2) {
    const v2f t0 = a[0] + a[1], t1 = a[0] - a[1];
    a[0] = t0; a[1] = t1;
  } else if constexpr (R == 4) {
    const v2f b0 = a[0] + a[2], b1 = a[0] - a[2];
    const v2f b2 = a[1] + a[3], d3 = a[1] - a[3];
    a[0] = b0 + b2; a[2] = b0 - b2;
    a[1] = add_mi(b1, d3); a[3] = sub_mi(b1, d3);
  } else {
    static_assert(R == 8, "radix");
    const float c = 0.70710678118654752f;
    const v2f b0 = a[0] + a[4], b4 = a[0] - a[4];
    const v2f b1 = a[1] + a[5], b5r = a[1] - a[5];
    const v2f b2 = a[2] + a[6], b6 = a[2] - a[6];
    const v2f b3 = a[3] + a[7], b7r = a[3] - a[7];
    const v2f b5 = c * add_mi(b5r, b5r);                 // * W8^1
    const v2f b7 = c * rot_m_b(b7r);                     // * W8^3
    const v2f c0 = b0 + b2, c2 = b0 - b2;
    const v2f c1 = b1 + b3, d3 = b1 - b3;
    const v2f c4 = add_mi(b4, b6), c6 = sub_mi(b4, b6);  // b6 * W8^2 = -i
    const v2f c5 = b5 + b7, d7 = b5 - b7;
    a[0] = c0 + c1; a[4] = c0 - c1;
    a[2] = add_mi(c2, d3); a[6] = sub_mi(c2, d3);
    a[1] = c4 + c5; a[5] = c4 - c5;
    a[3] = add_mi(c6, d7); a[7] = sub_mi(c6, d7);
  }
}

// inverse radix-2/4/8 DFTs on the packed forms (same arithmetic as the rot_mi<true> forms)
template <int R>
MIMO_DEV void dft_inv_pk(v2f *a) {
  if constexpr (R == 2) {
    const v2f t0 = a[0] + a[1], t1 = a[0] - a[1];
    a[0] = t0; a[1] = t1;
  } else if constexpr (R == 4) {
    const v2f b0 = a[0] + a[2], b1 = a[0] - a[2];
    const v2f b2 = a[1] + a[3], d3 = a[1] - a[3];
    a[0] = b0 + b2; a[2] = b0 - b2;
    a[1] = sub_mi(b1, d3); a[3] = add_mi(b1, d3);
  } else {
    static_assert(R == 8, "radix");
    const float c = 0.70710678118654752f;
    const v2f b0 = a[0] + a[4], b4 = a[0] - a[4];
    const v2f b1 = a[1] + a[5], b5r = a[1] - a[5];
    const v2f b2 = a[2] + a[6], b6 = a[2] - a[6];
    const v2f b3 = a[3] + a[7], b7r = a[3] - a[7];
    const v2f b5 = c * sub_mi(b5r, b5r);                 // * conj(W8^1)
    const v2f b7 = c * rot_p_b(b7r);                     // * conj(W8^3)
    const v2f c0 = b0 + b2, c2 = b0 - b2;
    const v2f c1 = b1 + b3, d3 = b1 - b3;
    const v2f c4 = sub_mi(b4, b6), c6 = add_mi(b4, b6);  // b6 * (+i)
    const v2f c5 = b5 + b7, d7 = b5 - b7;
    a[0] = c0 + c1; a[4] = c0 - c1;
    a[2] = sub_mi(c2, d3); a[6] = add_mi(c2, d3);
    a[1] = c4 + c5; a[5] = c4 - c5;
    a[3] = sub_mi(c6, d7); a[7] = add_mi(c6, d7);
  }
}

// radix-16 DFT (natural order in and out) as 4 x 4: DFT4 over n1 of x[4 n1 + n2] for each n2,
// the twiddles W16^(n2 k1), then DFT4 over n2 for each k1 -> X[k1 + 4 k2]
template <bool INV>
MIMO_DEV void dft16_pk(v2f *a) {
  constexpr float C1 = 0.92387953251128674f, S1 = 0.38268343236508978f;
  constexpr float R2 = 0.70710678118654752f;
  v2f y[16];                                           // y[4 n2 + k1]
#pragma unroll
  for (int n2 = 0; n2 < 4; n2++) {
    v2f t[4] = {a[n2], a[n2 + 4], a[n2 + 8], a[n2 + 12]};
    if constexpr (INV) dft_inv_pk<4>(t); else dft_fwd_pk<4>(t);
#pragma unroll
    for (int k1 = 0; k1 < 4; k1++) y[4 * n2 + k1] = t[k1];
  }
  // W16^e (e = n2 k1): 1, 2, 3 | 2, 4, 6 | 3, 6, 9; conjugated for the inverse
  const v2f w1 = INV ? v2f{C1, S1} : v2f{C1, -S1};
  const v2f w3 = INV ? v2f{S1, C1} : v2f{S1, -C1};
  const v2f w9 = INV ? v2f{-C1, -S1} : v2f{-C1, S1};
  auto w2 = [&](v2f x) { return R2 * (INV ? sub_mi(x, x) : add_mi(x, x)); };
  auto w6 = [&](v2f x) { return R2 * (INV ? rot_p_b(x) : rot_m_b(x)); };
  auto w4 = [&](v2f x) { return INV ? v2f{-x.y, x.x} : v2f{x.y, -x.x}; };
  y[5] = cmul_pk(y[5], w1);
  y[6] = w2(y[6]);
  y[7] = cmul_pk(y[7], w3);
  y[9] = w2(y[9]);
  y[10] = w4(y[10]);
  y[11] = w6(y[11]);
  y[13] = cmul_pk(y[13], w3);
  y[14] = w6(y[14]);
  y[15] = cmul_pk(y[15], w9);
#pragma unroll
  for (int k1 = 0; k1 < 4; k1++) {
    v2f t[4] = {y[k1], y[4 + k1], y[8 + k1], y[12 + k1]};
    if constexpr (INV) dft_inv_pk<4>(t); else dft_fwd_pk<4>(t);
#pragma unroll
    for (int k2 = 0; k2 < 4; k2++) a[k1 + 4 * k2] = t[k2];
  }
}

template <bool INV>
MIMO_DEV v2f twiddle(const float2 *__restrict__ tw, int idx) {
  const float2 w = tw[idx];
  return INV ? v2f{w.x, -w.y} : v2f{w.x, w.y};
}

// (x + iy) * (-i) forward, * (+i) inverse
template <bool INV>
MIMO_DEV v2f rot_mi(v2f a) {
  return INV ? v2f{-a.y, a.x} : v2f{a.y, -a.x};
}

template <int R, bool INV>
MIMO_DEV void dft_small(v2f *a) {
  if constexpr (R == 16) {
    dft16_pk<INV>(a);
  } else if constexpr (true) {              // single-instruction packed forms, same arithmetic
    if constexpr (INV) dft_inv_pk<R>(a); else dft_fwd_pk<R>(a);
  } else if constexpr (R == 2) {
    const v2f t0 = a[0] + a[1], t1 = a[0] - a[1];
    a[0] = t0; a[1] = t1;
  } else if constexpr (R == 4) {
    const v2f b0 = a[0] + a[2], b1 = a[0] - a[2];
    const v2f b2 = a[1] + a[3], b3 = rot_mi<INV>(a[1] - a[3]);
    a[0] = b0 + b2; a[2] = b0 - b2;
    a[1] = b1 + b3; a[3] = b1 - b3;
  } else {
    static_assert(R == 8, "radix");
    const float c = 0.70710678118654752f;
    const v2f b0 = a[0] + a[4], b4 = a[0] - a[4];
    const v2f b1 = a[1] + a[5];
    v2f b5 = a[1] - a[5];
    const v2f b2 = a[2] + a[6];
    v2f b6 = a[2] - a[6];
    const v2f b3 = a[3] + a[7];
    v2f b7 = a[3] - a[7];
    b6 = rot_mi<INV>(b6);                                    // * W8^2 = -i (fwd)
    if (!INV) {
      b5 = c * (b5 + v2f{b5.y, -b5.x});                      // * W8^1
      b7 = c * (v2f{b7.y, -b7.x} - b7);                      // * W8^3
    } else {
      b5 = c * (b5 + v2f{-b5.y, b5.x});
      b7 = c * (v2f{-b7.y, b7.x} - b7);
    }
    const v2f c0 = b0 + b2, c2 = b0 - b2;
    const v2f c1 = b1 + b3, c3 = rot_mi<INV>(b1 - b3);
    const v2f c4 = b4 + b6, c6 = b4 - b6;
    const v2f c5 = b5 + b7, c7 = rot_mi<INV>(b5 - b7);
    a[0] = c0 + c1; a[4] = c0 - c1;
    a[2] = c2 + c3; a[6] = c2 - c3;
    a[1] = c4 + c5; a[5] = c4 - c5;
    a[3] = c6 + c7; a[7] = c6 - c7;
  }
}

// one Stockham pass: sub-transform size NS -> NS*R
template <int N, int R, int NS, int T, int B, bool INV, int TWN>
MIMO_DEV void fft_pass(float2 *buf, const float2 *__restrict__ tw, int tid) {
  constexpr int NB = N / R;
  constexpr int TOT = NB * B;
  constexpr int PER = (TOT + T - 1) / T;
  constexpr int PB = lds_padded_len(N);
  v2f *vb = reinterpret_cast<v2f *>(buf);
  v2f a[PER][R];
#pragma unroll
  for (int q = 0; q < PER; q++) {
    const int g = tid + q * T;
    if ((TOT % T == 0) || g < TOT) {
      const int b = g / NB, j = g % NB;
      const v2f *base = vb + b * PB;
      if constexpr (NB % 32 == 0) {          // one padded base + compile-time offsets
        const v2f *bp = base + lds_pad(j);
#pragma unroll
        for (int r = 0; r < R; r++) a[q][r] = bp[r * NB + (r * NB) / 32];
      } else {
#pragma unroll
        for (int r = 0; r < R; r++) a[q][r] = base[lds_pad(j + r * NB)];
      }
      if constexpr (NS > 1) {
        // one table read per butterfly; the other R-2 twiddles are products of it
        // (<= 3 roundings deep, well inside the fp32 FFT error budget)
        const int k = j % NS;
        constexpr int STEP = TWN / (NS * R);
        v2f w[R];
        w[1] = twiddle<INV>(tw, k * STEP);
        if constexpr (R >= 4) {
          w[2] = vmul(w[1], w[1]);
          w[3] = vmul(w[2], w[1]);
        }
        if constexpr (R == 8) {
          w[4] = vmul(w[2], w[2]);
          w[5] = vmul(w[4], w[1]);
          w[6] = vmul(w[3], w[3]);
          w[7] = vmul(w[4], w[3]);
        }
#pragma unroll
        for (int r = 1; r < R; r++) a[q][r] = vmul(a[q][r], w[r]);
      }
      dft_small<R, INV>(a[q]);
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < PER; q++) {
    const int g = tid + q * T;
    if ((TOT % T == 0) || g < TOT) {
      const int b = g / NB, j = g % NB;
      const int k = j % NS;
      const int o = (j / NS) * NS * R + k;
      v2f *bp = vb + b * PB + lds_pad(o);     // lds_pad(o + r NS) = lds_pad(o) + r NS + r NS / 32
#pragma unroll
      for (int r = 0; r < R; r++) bp[r * NS + (r * NS) / 32] = a[q][r];
    }
  }
  __syncthreads();
}

template <int N, int NS, int REM, int T, int B, bool INV, int TWN>
MIMO_DEV void fft_passes(float2 *buf, const float2 *__restrict__ tw, int tid) {
  if constexpr (REM > 0) {
    constexpr int LR = (REM == 4) ? 2 : ((REM >= 3) ? 3 : REM);
    constexpr int R = 1 << LR;
    fft_pass<N, R, NS, T, B, INV, TWN>(buf, tw, tid);
    fft_passes<N, NS * R, REM - LR, T, B, INV, TWN>(buf, tw, tid);
  }
}

// B transforms of 2^LOG2N points at buf[b * lds_padded_len(N) + lds_pad(i)]. Caller must
// __syncthreads() after filling buf; on return buf holds the result (barrier included).
// tw is the process-wide kTwN-entry table (global memory) ...
template <int LOG2N, int T, int B, bool INV>
MIMO_DEV void fft_lds(float2 *buf, const float2 *__restrict__ tw) {
  fft_passes<(1 << LOG2N), 1, LOG2N, T, B, INV, kTwN>(buf, tw, (int)threadIdx.x);
}

// ... or an N/2-entry table in LDS (tw[m] = e^{-2 pi i m / N}, see fill_twiddles_lds): no
// vector-memory wait inside the passes, so loads in flight (a prefetched next item) are not
// drained by the first twiddle read. tid is threadIdx.x, passed in so a persistent caller
// can keep the per-pass address arithmetic inside its loop (no hoisted, spilled invariants).
template <int LOG2N, int T, int B, bool INV>
MIMO_DEV void fft_lds_twl(float2 *buf, const float2 *tw_lds, int tid) {
  fft_passes<(1 << LOG2N), 1, LOG2N, T, B, INV, (1 << LOG2N)>(buf, tw_lds, tid);
}

template <int LOG2N, int T>
MIMO_DEV void fill_twiddles_lds(float2 *tw_lds, const float2 *__restrict__ tw) {
  constexpr int N = 1 << LOG2N;
  for (int m = threadIdx.x; m < N / 2; m += T) tw_lds[m] = tw[m * (kTwN / N)];
}

}  // namespace mimo

// rub_mimo_amd/csrc/est_kernels.hip -- channel estimation stages on gfx950:
//   codes_kernel   : S0/S1 time-domain codes and their zero-padded F-point spectra
//   search_kernel  : access-code timing search (framing.cc:702-744)
//   ls_kernel      : LS channel estimate + training-residual noise variance (framing.cc:797-824)
//   weights_kernel : per-subcarrier detector weights (framing.cc:826-831 -> 1344-1367)
//
// Search. The reference takes, for every lag i in [0, SL) and every (rx, slot), an M-point
// FFT of the window at i and the metric |sum_k X_k conj(S_k)|^2 / M^2: SL*N*(N*nac+1) FFTs
// (712,800 at C3). By Parseval, sum_k X_k conj(S_k) = sqrt(M) * sum_n w[i+n] conj(s[n])
// with s the time-domain code (sqrt(M_S0) for S0), i.e. a sliding cross-correlation. One
// workgroup computes all SL lags of one (frame, rx, slot) with overlap-save: FFT_F of the
// F-sample window segment, multiply by conj(FFT_F(zero-padded code)), IFFT_F; lags
// [0, F-M] are exact linear correlations. First-maximum semantics (strict '>', initial 0,
// framing.cc:718, 735) are kept by packing (value bits, ~index) into one 64-bit atomicMax.
#include <cstring>

#include "fft.hpp"
#include "fft_reg.hpp"
#include "kernels.hpp"

namespace mimo {

constexpr int kEstT = 256;

// ------------------------------------------------------------------------------------
template <int LOG2M, int LOG2F>
__global__ __launch_bounds__(kEstT) void codes_kernel(CodesArgs a) {
  constexpr int M = 1 << LOG2M, F = 1 << LOG2F;
  extern __shared__ __attribute__((aligned(16))) float2 lds[];
  float2 *buf = lds;
  const int slot = blockIdx.x, tid = threadIdx.x;
  // frequency-domain code on the first M entries
  for (int i = tid; i < M; i += kEstT) {
    float v = 0.0f;
    if (a.p[i] != 0) {
      if (slot == 0) {
        if ((i & 1) == 0) v = (a.s0_bits[i] & 1) ? 1.0f : -1.0f;  // framing.cc:1077-1089
      } else {
        const int ac = slot - 1, c = ac / a.N, t = ac % a.N;
        v = (a.s1_bits[((size_t)t * a.nac + c) * M + i] & 1) ? 1.0f : -1.0f;  // :1243-1248
      }
    }
    buf[lds_pad(i)] = make_float2(v, 0.0f);
  }
  __syncthreads();
  fft_lds<LOG2M, kEstT, 1, true>(buf, a.tw);
  const float dn = (slot == 0) ? a.dn_s0 : a.dn_s1;
  for (int i = tid; i < M; i += kEstT) {
    float2 v = buf[lds_pad(i)];
    v = make_float2(v.x * dn, v.y * dn);
    a.code_time[(size_t)slot * M + i] = v;
    buf[lds_pad(i)] = v;
  }
  if (a.codespec == nullptr) return;
  __syncthreads();
  // zero-pad to F (in place: move is safe because M <= F/2 and we only clear [M, F))
  for (int i = M + tid; i < F; i += kEstT) buf[lds_pad(i)] = make_float2(0.0f, 0.0f);
  __syncthreads();
  fft_lds<LOG2F, kEstT, 1, false>(buf, a.tw);
  for (int i = tid; i < F; i += kEstT) a.codespec[(size_t)slot * F + i] = buf[lds_pad(i)];
  if constexpr (F >= 1024) {
    // the wave-local search's order: bin B k + q at q * 1024 + k (B = F / 1024)
    constexpr int B = F / 1024;
    if (a.codespec_w)
      for (int i = tid; i < F; i += kEstT)
        a.codespec_w[(size_t)slot * F + (i % B) * 1024 + i / B] = buf[lds_pad(i)];
  }
}

// DEBUG_LOG trace (framing.cc:675-696, 873-883, opt-in): every lag's metric of (frame, rx, slot)
MIMO_DEV void corr_trace_put(const SearchArgs &a, uint32_t f, uint32_t r, uint32_t slot,
                             int64_t lag, float v) {
  if (a.corr_trace && lag >= 0 && lag < (int64_t)a.SL)
    a.corr_trace[(((uint64_t)f * a.N + r) * a.n_slots + slot) * a.SL + lag] = v;
}

// ------------------------------------------------------------------------------------
template <int LOG2F>
__global__ __launch_bounds__(kEstT) void search_kernel(SearchArgs a) {
  constexpr int F = 1 << LOG2F;
  extern __shared__ __attribute__((aligned(16))) float2 lds[];
  __shared__ unsigned long long s_key;
  const uint32_t f = blockIdx.y;
  const FrameInfo &I = a.info[f];
  if (I.status != 0) return;
  const int tid = threadIdx.x;
  const uint32_t lc = blockIdx.x % a.n_lagc;
  const uint32_t r = (blockIdx.x / a.n_lagc) % a.N;
  const uint32_t slot = blockIdx.x / (a.n_lagc * a.N);
  const int64_t lag0 = (int64_t)lc * a.lagc;
  const int64_t nl = min((int64_t)a.lagc, (int64_t)a.SL - lag0);
  const int64_t ws = (int64_t)a.SL * slot + lag0;   // window index of lag 0 of this segment
  const int64_t abs0 = I.base + ws;
  const float2 *__restrict__ x = a.iq + ((uint64_t)I.cap * a.N + r) * a.stride;
  const int64_t L = (int64_t)a.frame_len;
  for (int i = tid; i < F; i += kEstT) {
    const int64_t n = abs0 + i;
    lds[lds_pad(i)] = (n >= 0 && n < L) ? x[n] : make_float2(0.0f, 0.0f);
  }
  if (tid == 0) s_key = 0ull;
  __syncthreads();
  fft_lds<LOG2F, kEstT, 1, false>(lds, a.tw);
  const float2 *__restrict__ cs = a.codespec + (size_t)slot * F;
  for (int i = tid; i < F; i += kEstT) lds[lds_pad(i)] = cmulc(lds[lds_pad(i)], cs[i]);
  __syncthreads();
  fft_lds<LOG2F, kEstT, 1, true>(lds, a.tw);
  const float vs = a.vscale[slot];
  unsigned long long best = 0ull;
  for (int i = tid; i < nl; i += kEstT) {
    const float v = cabs2(lds[lds_pad(i)]) * vs;
    corr_trace_put(a, f, r, slot, lag0 + i, v);
    if (v > 0.0f) {
      const unsigned long long key =
          ((unsigned long long)__float_as_uint(v) << 32) |
          (unsigned long long)(0xFFFFFFFFu - (uint32_t)(ws + i));
      best = key > best ? key : best;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long o = __shfl_xor(best, off);
    best = o > best ? o : best;
  }
  if ((tid & 63) == 0 && best) atomicMax(&s_key, best);
  __syncthreads();
  if (tid == 0 && s_key)
    atomicMax(&a.keys[((uint64_t)f * a.N + r) * a.n_slots + slot], s_key);
}

// Register-resident form (F >= 1024): T = F/16 threads, 16 points each. The forward FFT_F
// reads the window segment straight from HBM in its first pass, its last pass leaves
// elements j + r*F/8 in the thread, which are multiplied by conj(code spectrum) in place and
// are exactly the inputs of the inverse's first pass; the inverse's last pass leaves lags
// j + r*F/8, scored in registers. 2*(NP-1) LDS exchanges per (frame, rx, slot, lag chunk),
// twiddles loaded once per thread.
template <int LOG2F>
__global__ __launch_bounds__((1 << LOG2F) / 16) __attribute__((amdgpu_waves_per_eu(4)))
void search_reg_kernel(SearchArgs a) {
  constexpr int PTS = 16;
  using PL = RegPlan<LOG2F, PTS>;
  constexpr int F = PL::N;
  extern __shared__ __attribute__((aligned(16))) float2 lds_raw[];
  v2f *buf = reinterpret_cast<v2f *>(lds_raw);
  __shared__ unsigned long long s_key;
  const uint32_t f = blockIdx.y;
  const FrameInfo &I = a.info[f];
  if (I.status != 0) return;
  const int tid = threadIdx.x;
  const uint32_t lc = blockIdx.x % a.n_lagc;
  const uint32_t r = (blockIdx.x / a.n_lagc) % a.N;
  const uint32_t slot = blockIdx.x / (a.n_lagc * a.N);
  const int64_t lag0 = (int64_t)lc * a.lagc;
  const int64_t nl = min((int64_t)a.lagc, (int64_t)a.SL - lag0);
  const int64_t ws = (int64_t)a.SL * slot + lag0;   // window index of lag 0 of this segment
  const int64_t abs0 = I.base + ws;
  const int64_t L = (int64_t)a.frame_len;
  const v2f *__restrict__ x = reinterpret_cast<const v2f *>(a.iq + ((uint64_t)I.cap * a.N + r) * a.stride);
  const bool inb = abs0 >= 0 && abs0 + F <= L;
  v2f v[PTS], cs[PTS];
  // unconditional loads from clamped indices, masked afterwards: a per-element "load or zero"
  // select makes hipcc branch around each load and wait for it (one latency per element)
#pragma unroll
  for (int e = 0; e < PTS; e++) {
    const int64_t n = abs0 + reg_index<LOG2F, PTS>(tid, e);
    v[e] = x[inb ? n : (n < 0 ? 0 : (n >= L ? L - 1 : n))];
  }
  if (!inb) {
#pragma unroll
    for (int e = 0; e < PTS; e++) {
      const int64_t n = abs0 + reg_index<LOG2F, PTS>(tid, e);
      if (n < 0 || n >= L) v[e] = v2f{0.0f, 0.0f};
    }
  }
  v2f w1[PL::NTW > 0 ? PL::NTW : 1];
  reg_twiddles<LOG2F, PTS>(w1, a.tw, tid);
  if (tid == 0) s_key = 0ull;
  reg_compute<LOG2F, PTS, 0, false>(v, w1);
  reg_rest<LOG2F, PTS, 1, false>(buf, v, w1, tid);
  const v2f *__restrict__ csp = reinterpret_cast<const v2f *>(a.codespec + (size_t)slot * F);
#pragma unroll
  for (int e = 0; e < PTS; e++) cs[e] = csp[reg_index<LOG2F, PTS>(tid, e)];   // L2-resident
#pragma unroll
  for (int e = 0; e < PTS; e++) v[e] = vmulc(v[e], cs[e]);   // X * conj(S_F)
  reg_compute<LOG2F, PTS, 0, true>(v, w1);
  reg_rest<LOG2F, PTS, 1, true>(buf, v, w1, tid);
  const float vs = a.vscale[slot];
  unsigned long long best = 0ull;
#pragma unroll
  for (int e = 0; e < PTS; e++) {
    const int i = reg_index<LOG2F, PTS>(tid, e);
    const float val = (v[e].x * v[e].x + v[e].y * v[e].y) * vs;
    if (i < nl) corr_trace_put(a, f, r, slot, lag0 + i, val);
    if (i < nl && val > 0.0f) {
      const unsigned long long key = ((unsigned long long)__float_as_uint(val) << 32) |
                                     (unsigned long long)(0xFFFFFFFFu - (uint32_t)(ws + i));
      best = key > best ? key : best;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long o = __shfl_xor(best, off);
    best = o > best ? o : best;
  }
  if ((tid & 63) == 0 && best) atomicMax(&s_key, best);
  __syncthreads();
  if (tid == 0 && s_key)
    atomicMax(&a.keys[((uint64_t)f * a.N + r) * a.n_slots + slot], s_key);
}

// exp(-j 2 pi cyc) for a phase in cycles given in fp64 (reduced to [-1/2, 1/2] first, so
// long offsets keep their accuracy), as an fp32 phasor
MIMO_DEV v2f phasor_cycles(double cyc) {
  double ph = -2.0 * cyc;                             // units of pi
  ph -= 2.0 * rint(ph * 0.5);
  double sn, cs;
  sincospi(ph, &sn, &cs);
  return v2f{(float)cs, (float)sn};
}

// the same from an exactly reduced phase with the fp32 sincos (per-thread start phasors of the
// folded CFO; the per-workgroup values below keep the fp64 one)
MIMO_DEV v2f phasor_cycles32(double cyc) {
  double ph = -2.0 * cyc;                             // units of pi
  ph -= 2.0 * rint(ph * 0.5);
  float sn, cs;
  sincospif((float)ph, &sn, &cs);
  return v2f{cs, sn};
}

// folded CFO of a search workgroup: the frame's stage-1 frequency nu (cycles per sample) and the
// workgroup-uniform step phasors exp(-j 2 pi nu d), formed once by thread 0 (the stage partials'
// sum, its atan2 and the fp64 sincospi were per thread) and read by every thread from LDS
struct CfoSearchLds {
  double nu;
  v2f step[3];
};
MIMO_DEV double cfo_search_setup(CfoSearchLds &c, const double *part, uint32_t f, uint32_t M,
                                 double d0, double d1, double d2) {
  if (threadIdx.x == 0) {
    const double nu = cfo_stage_eps(part, f, 1) / (double)M;
    c.nu = nu;
    c.step[0] = phasor_cycles(nu * d0);
    c.step[1] = phasor_cycles(nu * d1);
    c.step[2] = phasor_cycles(nu * d2);
  }
  __syncthreads();
  return c.nu;
}

// the wave's largest 64-bit key in every lane, over DPP and permlane swaps (quad xor 1 and 2,
// the row's half-mirror and mirror, then the 16- and 32-lane swaps) instead of six rounds of
// ds_bpermute through the LDS unit (__shfl_xor): the same maximum, a few cycles per step
template <int CTRL>
MIMO_DEV unsigned long long dpp_u64(unsigned long long x) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)x, CTRL, 0xf, 0xf, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(x >> 32), CTRL, 0xf, 0xf, false);
  return ((unsigned long long)hi << 32) | lo;
}
MIMO_DEV unsigned long long max_u64(unsigned long long a, unsigned long long b) { return a > b ? a : b; }
MIMO_DEV unsigned long long wave_max_u64(unsigned long long x) {
  x = max_u64(x, dpp_u64<0xB1>(x));    // quad_perm [1, 0, 3, 2]: lane ^ 1
  x = max_u64(x, dpp_u64<0x4E>(x));    // quad_perm [2, 3, 0, 1]: lane ^ 2
  x = max_u64(x, dpp_u64<0x141>(x));   // row_half_mirror: the other quad of the 8
  x = max_u64(x, dpp_u64<0x140>(x));   // row_mirror: the other 8 of the row
  {
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    x = max_u64(((unsigned long long)h[0] << 32) | l[0], ((unsigned long long)h[1] << 32) | l[1]);
  }
  {
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    x = max_u64(((unsigned long long)h[0] << 32) | l[0], ((unsigned long long)h[1] << 32) | l[1]);
  }
  return x;
}

MIMO_DEV uint32_t key_index(unsigned long long k) {
  return k ? (0xFFFFFFFFu - (uint32_t)(k & 0xFFFFFFFFull)) : 0u;
}

// Search of two consecutive slots with the LS term of each fused in (one lag chunk per slot,
// 2 SL + M - 1 <= F). Slot s0 + u's window at lag i is segment offset u SL + i of the F-point
// segment starting at window index SL s0, so one forward FFT_F serves both slots: per slot a
// product with conj(its code spectrum), the inverse and the first-maximum score over its SL
// lags (3 FFT_F per two slots instead of 4). The workgroup is then the only writer of the
// slot's key, so the argmax is final and the LS term of access code ac = slot - 1 follows at
// once: the M-point FFT of the window at the argmax (framing.cc:801-806), times the S1 sign
// (X / S1, S1 = +-1, framing.cc:811), stored per code in lsq[f][rx][tx][code][M] for
// ls_combine_q_kernel's fixed-order sum. The separate LS pass re-read and re-transformed the
// same windows; here the window is still in L2 from the segment load.
template <int LOG2F, int LOG2M, bool SC16 = false, bool CFO = false>
__global__ __launch_bounds__((1 << LOG2F) / 16) __attribute__((amdgpu_waves_per_eu(4)))
void search_ls_kernel(SearchArgs a) {
  constexpr int PTS = 16;
  using PL = RegPlan<LOG2F, PTS>;
  constexpr int F = PL::N, T = PL::T, M = 1 << LOG2M;
  extern __shared__ __attribute__((aligned(16))) float2 lds_raw[];
  v2f *buf = reinterpret_cast<v2f *>(lds_raw);
  __shared__ unsigned long long s_key[2];
  __shared__ CfoSearchLds cfo_lds;                    // (folded CFO only)
  // (frame, rx, pair) of this workgroup. xcd_order: workgroups are dispatched round-robin over
  // the 8 XCDs (hardware id b -> XCD b mod 8); each XCD is given a contiguous range of the
  // order (pair, frame, rx), so the workgroups resident on one XCD at a time share the two
  // 64 KB code spectra of one slot pair in that XCD's L2 (all 81 slots' spectra, 5.2 MB at
  // C3, exceed one XCD's 4 MB L2 when every XCD sees every pair)
  uint32_t f = blockIdx.y, bx = blockIdx.x;
  if (a.xcd_order) {
    const uint32_t G = gridDim.x * gridDim.y, b = blockIdx.y * gridDim.x + blockIdx.x;
    const uint32_t x = b % 8, q = G / 8, rem = G % 8;
    const uint32_t lid = x * q + min(x, rem) + b / 8;
    const uint32_t nf = gridDim.y, nrx = a.N;
    bx = (lid / (nrx * nf)) * nrx + lid % nrx;
    f = (lid / nrx) % nf;
  }
  const FrameInfo &I = a.info[f];
  if (I.status != 0) return;
  const int tid = threadIdx.x;
  const uint32_t r = bx % a.N;
  const uint32_t s0 = 2 * (bx / a.N);
  const uint32_t ns = min(2u, a.n_slots - s0);
  const int64_t abs0 = I.base + (int64_t)a.SL * s0;
  const int64_t L = (int64_t)a.frame_len;
  const auto xs = iq_row<SC16>(a.iq, a.iq_scale, ((uint64_t)I.cap * a.N + r) * a.stride);
  const bool inb = abs0 >= 0 && abs0 + F <= L;
  v2f v[PTS], X[PTS];
#ifdef SL_ABL_NOLOAD   // timing ablation: no segment loads
#pragma unroll
  for (int e = 0; e < PTS; e++) v[e] = v2f{(float)e, (float)(tid + (int)abs0)};
  if (false) {
#else
#pragma unroll
  for (int e = 0; e < PTS; e++) {
    const int64_t n = abs0 + reg_index<LOG2F, PTS>(tid, e);
    const float2 t = xs.at(inb ? n : (n < 0 ? 0 : (n >= L ? L - 1 : n)));
    v[e] = v2f{t.x, t.y};
  }
  if (!inb) {
#endif
#pragma unroll
    for (int e = 0; e < PTS; e++) {
      const int64_t n = abs0 + reg_index<LOG2F, PTS>(tid, e);
      if (n < 0 || n >= L) v[e] = v2f{0.0f, 0.0f};
    }
  }
  double nu = 0.0;                                    // folded CFO: eps0 / M cycles per sample
  if constexpr (CFO) {
    // sample tid + e F/16 of the segment, relative to base: SL s0 + tid + e F/16
    static_assert(PTS == 16 && PL::RM == 16, "reg_index = tid + e F/16");
    nu = cfo_search_setup(cfo_lds, a.cfo_part, f, M, (double)(F / 16), (double)(M / 8), 0.0);
    v2f rb = phasor_cycles32(nu * (double)((int64_t)a.SL * s0 + tid));
    const v2f st = cfo_lds.step[0];
#pragma unroll
    for (int e = 0; e < PTS; e++) {
      v[e] = vmul(v[e], rb);
      rb = vmul(rb, st);
    }
  }
  v2f w1[PL::NTW > 0 ? PL::NTW : 1];
  reg_twiddles<LOG2F, PTS>(w1, a.tw, tid);
  // LS transform: register-resident (M/8 threads and 8 points per window, one window per half
  // of the workgroup) when T = 2 M/8, else batched in LDS with its twiddles in LDS
#ifdef SL_ABL_LSLDS   // A/B build: the LDS-batched LS transform everywhere
  constexpr bool LSREG = false;
#else
  // (M >= 512: the register plan's last pass is radix 8 and each window fills whole waves)
  constexpr bool LSREG = 2 * (M / 8) == T && LOG2M >= 9;
#endif
  float2 *twm = reinterpret_cast<float2 *>(lds_raw) + lds_padded_len(F);
  if constexpr (!LSREG) fill_twiddles_lds<LOG2M, T>(twm, a.tw);
  if (tid == 0) { s_key[0] = 0ull; s_key[1] = 0ull; }
#ifndef SL_ABL_NOFWD   // timing ablation: no forward transform
  reg_compute<LOG2F, PTS, 0, false>(v, w1);
  reg_rest<LOG2F, PTS, 1, false>(buf, v, w1, tid);
#endif
#pragma unroll
  for (int e = 0; e < PTS; e++) X[e] = v[e];
  for (uint32_t u = 0; u < ns; u++) {                 // uniform
    const uint32_t slot = s0 + u;
    const v2f *__restrict__ csp = reinterpret_cast<const v2f *>(a.codespec + (size_t)slot * F);
#pragma unroll
    for (int e = 0; e < PTS; e++) v[e] = vmulc(X[e], csp[reg_index<LOG2F, PTS>(tid, e)]);
#ifndef SL_ABL_NOINV   // timing ablation: no inverse transforms
    reg_compute<LOG2F, PTS, 0, true>(v, w1);
    reg_rest<LOG2F, PTS, 1, true>(buf, v, w1, tid);
#endif
    const float vs = a.vscale[slot];
    const int off = (int)(u * a.SL);
    const uint32_t ws = a.SL * slot;                  // window index of lag 0
    unsigned long long best = 0ull;
#pragma unroll
    for (int e = 0; e < PTS; e++) {
      const int i = reg_index<LOG2F, PTS>(tid, e) - off;
      const float val = (v[e].x * v[e].x + v[e].y * v[e].y) * vs;
      corr_trace_put(a, f, r, slot, i, val);
      if (i >= 0 && i < (int)a.SL && val > 0.0f) {
        const unsigned long long key = ((unsigned long long)__float_as_uint(val) << 32) |
                                       (unsigned long long)(0xFFFFFFFFu - (ws + (uint32_t)i));
        best = key > best ? key : best;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long q = __shfl_xor(best, o);
      best = q > best ? q : best;
    }
    if ((tid & 63) == 0 && best) atomicMax(&s_key[u], best);
    __syncthreads();                                  // key final; every reader of buf is done
    if (tid == 0) a.keys[((uint64_t)f * a.N + r) * a.n_slots + slot] = s_key[u];
  }
#ifdef SL_ABL_NOLS   // timing ablation (tools/abl_search.sh): no LS term
  return;
#endif
  // LS terms of the pair's access codes (slot 0 = S0 has none): both windows (at their final
  // argmax) gathered with every load in flight, then one batched M-point transform
  constexpr int PBM = lds_padded_len(M), NL = 2 * M / T;
  static_assert(2 * M % T == 0, "whole windows per thread");
  const bool valid0 = s0 != 0, valid1 = ns > 1;
  if ((!valid0 && !valid1) || !a.lsq) return;         // uniform (no lsq: ls_window_kernel)
  const int64_t w0 = I.base + (int64_t)key_index(s_key[0]);
  const int64_t w1v = I.base + (int64_t)key_index(s_key[1]);
  if constexpr (LSREG) {
    // window u = tid / (M/8) on its half: 8 loads per thread straight into the first radix-8
    // pass, two LDS exchanges, and X[k] of the last pass stored from registers
    using PM = RegPlan<LOG2M, 8>;
    const uint32_t u = (uint32_t)tid / PM::T, lt = (uint32_t)tid % PM::T;   // u uniform per wave
    const bool valid = u ? valid1 : valid0;
    const int64_t wb = u ? w1v : w0;
    v2f xw[8];
#pragma unroll
    for (int e = 0; e < 8; e++) {
      const int64_t n = wb + reg_index<LOG2M, 8>((int)lt, e);
      const bool ok = valid && n >= 0 && n < L;
      const float2 t = xs.at(n < 0 ? 0 : (n >= L ? L - 1 : n));   // clamped, masked below
      xw[e] = ok ? v2f{t.x, t.y} : v2f{0.0f, 0.0f};
    }
    if constexpr (CFO) {   // window sample lt + e M/8, relative to base
      v2f rb = phasor_cycles32(nu * (double)(wb - I.base + (int64_t)lt));
      const v2f st = cfo_lds.step[1];
#pragma unroll
      for (int e = 0; e < 8; e++) {
        xw[e] = vmul(xw[e], rb);
        rb = vmul(rb, st);
      }
    }
    v2f wm[PM::NTW > 0 ? PM::NTW : 1];
    reg_twiddles<LOG2M, 8>(wm, a.tw, (int)lt);
    reg_compute<LOG2M, 8, 0, false>(xw, wm);
    reg_rest<LOG2M, 8, 1, false>(buf + u * PBM, xw, wm, (int)lt);
    if (!valid) return;                               // uniform per wave
    const uint32_t ac = s0 + u - 1, code = ac / a.N, tx = ac % a.N;
    const int8_t *sg = a.s1sign + ((size_t)tx * a.nac + code) * M;
    float2 *q = a.lsq + ((((uint64_t)f * a.N + r) * a.N + tx) * a.nac + code) * M;
#pragma unroll
    for (int e = 0; e < 8; e++) {
      const int k = reg_index<LOG2M, 8>((int)lt, e);
      const int sgn = sg[k];
      const float2 Xk = make_float2(xw[e].x, xw[e].y);
      q[k] = sgn > 0 ? Xk : (sgn < 0 ? cneg(Xk) : make_float2(0.0f, 0.0f));
    }
    return;
  }
  float2 win[NL];
#pragma unroll
  for (int e = 0; e < NL; e++) {
    const int i = tid + e * T, u = i / M, j = i % M;
    const int64_t n = (u ? w1v : w0) + j;
    const bool ok = (u ? valid1 : valid0) && n >= 0 && n < L;
    win[e] = ok ? xs.at(n) : make_float2(0.0f, 0.0f);
    if constexpr (CFO) {
      const v2f w = vmul(v2f{win[e].x, win[e].y}, phasor_cycles(nu * (double)(n - I.base)));
      win[e] = make_float2(w.x, w.y);
    }
  }
  float2 *lb = reinterpret_cast<float2 *>(buf);
#pragma unroll
  for (int e = 0; e < NL; e++) {
    const int i = tid + e * T, u = i / M, j = i % M;
    lb[u * PBM + lds_pad(j)] = win[e];
  }
  __syncthreads();
  fft_lds_twl<LOG2M, T, 2, false>(lb, twm, tid);
#pragma unroll
  for (int e = 0; e < NL; e++) {
    const int i = tid + e * T, u = i / M, k = i % M;
    if (!(u ? valid1 : valid0)) continue;
    const uint32_t ac = s0 + u - 1, code = ac / a.N, tx = ac % a.N;
    const int8_t *sg = a.s1sign + ((size_t)tx * a.nac + code) * M;
    float2 *q = a.lsq + ((((uint64_t)f * a.N + r) * a.N + tx) * a.nac + code) * M;
    const float2 Xk = lb[u * PBM + lds_pad(k)];
    const int s = sg[k];
    q[k] = s > 0 ? Xk : (s < 0 ? cneg(Xk) : make_float2(0.0f, 0.0f));
  }
}

// LS term store: non-temporal, read once by ls_combine_q_kernel
template <typename PT>   // v2f * or gptr<v2f>
__device__ __forceinline__ void ls_term_store(PT p, v2f t) {
  __builtin_nontemporal_store(t, p);
}

// The same search + LS with the FFT_F split into one workgroup-wide radix-B pass and B
// wave-local 1024-point transforms (F = 1024 B, one wave per sub-transform, T = 64 B):
//   forward  X[B k + q] = DFT_1024( c_q )[k],   c_q[n] = W_F^{nq} sum_r x[n + 1024 r] W_B^{rq}
//   inverse  y[m' + 1024 p] = sum_q W_B^{-pq} W_F^{-m'q} Y_q[m'],  Y_q = IDFT_1024( Z[B k + q] )
// The radix-B pass runs on 16/B butterflies per thread straight from the segment loads; one
// workgroup exchange hands c_q to wave q, whose 1024-point transform (RegPlan<10, 16>: radix
// 16, 4, 16) exchanges only through its own LDS region (wave-local order, no barrier) and
// leaves X[B (l + 64 s) + q] in lane l, slot s -- the inverse's first-pass input order, so the
// product with conj(code spectrum) (stored permuted, codespec_w[slot][q][k]) and the inverse
// run on in registers. One exchange back gathers Y_q[m'] over q for the final radix-B pass.
// Three workgroup exchanges per slot pair instead of nine.
// CFO (opt-in, folded): every loaded sample n is derotated by the frame's coarse estimate,
// x[n] exp(-j 2 pi eps0 (n - base) / M) -- what the scratch pass of the unfolded path wrote --
// as a per-thread phasor (fp64 phase) times per-frame step phasors.
template <int LOG2F, int LOG2M, bool SC16 = false, bool CFO = false>
__global__ __launch_bounds__((1 << LOG2F) / 16) __attribute__((amdgpu_waves_per_eu(4)))
void search_ls_wave_kernel(SearchArgs a) {
  constexpr int F = 1 << LOG2F, T = F / 16, M = 1 << LOG2M;
  constexpr int B = F / 1024;                          // waves = sub-transforms = block radix
  constexpr int NB = 16 / B;                           // block butterflies per thread
  constexpr int RB = lds_padded_len(1024);             // region stride (entries)
  using PW = RegPlan<10, 16>;
  static_assert(B >= 1 && B <= 16 && T == 64 * B, "F = 1024 B, one wave per sub-transform");
  extern __shared__ __attribute__((aligned(16))) float2 lds_raw[];
  v2f *buf = reinterpret_cast<v2f *>(lds_raw);
  __shared__ unsigned long long s_key[2];
  __shared__ CfoSearchLds cfo_lds;                    // (folded CFO only)
  uint32_t f = blockIdx.y, bx = blockIdx.x;
  if (a.xcd_order) {   // as search_ls_kernel: slot pair slowest within each XCD's range
    const uint32_t G = gridDim.x * gridDim.y, b = blockIdx.y * gridDim.x + blockIdx.x;
    const uint32_t x = b % 8, q = G / 8, rem = G % 8;
    const uint32_t lid = x * q + min(x, rem) + b / 8;
    const uint32_t nf = gridDim.y, nrx = a.N;
    bx = (lid / (nrx * nf)) * nrx + lid % nrx;
    f = (lid / nrx) % nf;
  }
  const FrameInfo &I = a.info[f];
  if (I.status != 0) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t wq = __builtin_amdgcn_readfirstlane((uint32_t)tid >> 6);   // this wave's q
  const uint32_t r = bx % a.N;
  const uint32_t s0 = 2 * (bx / a.N);
  const uint32_t ns = min(2u, a.n_slots - s0);
  const int64_t abs0 = I.base + (int64_t)a.SL * s0;
  const int64_t L = (int64_t)a.frame_len;
  const auto xs = iq_row<SC16>(a.iq, a.iq_scale, ((uint64_t)I.cap * a.N + r) * a.stride);
  const bool inb = abs0 >= 0 && abs0 + F <= L;
  v2f v[16], X[16];
  // segment loads in the block pass's order: v[i B + rr] = x[n_i + 1024 rr], n_i = tid + T i
  // (a uniform branch: inside the capture plain loads off one base, else clamped indices)
#ifdef SL_ABL_NOLOAD   // timing ablation (tools/abl_search.sh): no segment loads
#pragma unroll
  for (int e = 0; e < 16; e++) v[e] = v2f{(float)e, (float)(tid + (int)abs0)};
  if (false) {
#else
  if (inb) {
#endif
    const auto xb = xs.row((uint64_t)abs0);
#pragma unroll
    for (int i = 0; i < NB; i++)
#pragma unroll
      for (int rr = 0; rr < B; rr++) {
        const float2 t = xb.at(tid + T * i + 1024 * rr);
        v[i * B + rr] = v2f{t.x, t.y};
      }
  } else {
#pragma unroll
    for (int i = 0; i < NB; i++)
#pragma unroll
      for (int rr = 0; rr < B; rr++) {
        const int64_t n = abs0 + tid + T * i + 1024 * rr;
        const float2 t = xs.at(n < 0 ? 0 : (n >= L ? L - 1 : n));
        v[i * B + rr] = v2f{t.x, t.y};
      }
  }
  if (!inb) {
#pragma unroll
    for (int i = 0; i < NB; i++)
#pragma unroll
      for (int rr = 0; rr < B; rr++) {
        const int64_t n = abs0 + tid + T * i + 1024 * rr;
        if (n < 0 || n >= L) v[i * B + rr] = v2f{0.0f, 0.0f};
      }
  }
  if constexpr (CFO) {   // eps0 / M, cycles per sample (kept in cfo_lds.nu)
    const double nu = cfo_search_setup(cfo_lds, a.cfo_part, f, M, (double)T, 1024.0, (double)(M / 8));
    // sample n_i + 1024 rr, n_i = tid + T i, relative to base: SL s0 + n_i + 1024 rr
    v2f ri = phasor_cycles32(nu * (double)((int64_t)a.SL * s0 + tid));
    const v2f sa = cfo_lds.step[0], sb = cfo_lds.step[1];
#pragma unroll
    for (int i = 0; i < NB; i++) {
      v2f rb = ri;
#pragma unroll
      for (int rr = 0; rr < B; rr++) {
        v[i * B + rr] = vmul(v[i * B + rr], rb);
        rb = vmul(rb, sb);
      }
      ri = vmul(ri, sa);
    }
  }
  v2f w1[PW::NTW > 0 ? PW::NTW : 1];
  reg_twiddles<10, 16>(w1, a.tw, lane);
  if (tid == 0) { s_key[0] = 0ull; s_key[1] = 0ull; }
  // radix-B block pass (forward): DFT_B over rr, twiddle W_F^{nq}, c_q[n] -> region q
  // (W_F^{n_i} of the thread's n_i read once: the inverse block passes use its conjugate --
  // the same table entry twiddle<true> reads -- instead of reading it again per slot, one L2
  // round trip exposed before each slot's recombination)
  // (held at F = 8192, two per thread; at F = 2048, eight per thread, they would spill)
  v2f *rg = buf + wq * RB;                             // this wave's region
  constexpr bool TW_ONCE = LOG2F == 13;             // (B = 8: two per thread)
  v2f wfb[TW_ONCE ? NB : 1];
  if constexpr (TW_ONCE) {
#pragma unroll
    for (int i = 0; i < NB; i++) wfb[i] = twiddle<false>(a.tw, (tid + T * i) * (kTwN / F));
  }
  if constexpr (B > 1) {
#pragma unroll
    for (int i = 0; i < NB; i++) {
      dft_small<B, false>(v + i * B);
      const int n = tid + T * i;
      v2f w[B > 1 ? B : 2];
      twiddle_powers<B>(w, TW_ONCE ? wfb[TW_ONCE ? i : 0] : twiddle<false>(a.tw, n * (kTwN / F)));
#pragma unroll
      for (int q = 1; q < B; q++) v[i * B + q] = vmul(v[i * B + q], w[q]);
#pragma unroll
      for (int q = 0; q < B; q++) buf[q * RB + lds_pad(n)] = v[i * B + q];
    }
    __syncthreads();                                   // every c_q complete
#pragma unroll
    for (int e = 0; e < 16; e++) v[e] = rg[lds_pad(reg_index<10, 16>(lane, e))];
  }
  // wave-local 1024-point forward transform of c_q: X[B k + q], k = lane + 64 e, in v[e]
#ifndef SL_ABL_NOFWD   // timing ablation: no forward sub-transforms
  reg_compute<10, 16, 0, false>(v, w1);
  wave1024_rest<false>(rg, v, w1, lane);
#endif
  // both slots' code spectra in one round of loads: slot s0's product into v, slot s0 + 1's
  // into X (the forward spectrum is not needed after), instead of one L2 round trip per slot
  // (at F = 8192 only: the CFO variant, with its derotation state live, and the other
  // transform sizes would spill -- one round per slot there)
  constexpr bool CSP_PAIR = !CFO && LOG2F == 13;
  if constexpr (!CSP_PAIR) {
#pragma unroll
    for (int e = 0; e < 16; e++) X[e] = v[e];
  } else {
    const v2f *__restrict__ csp0 =
        reinterpret_cast<const v2f *>(a.codespec_w + (size_t)s0 * F) + wq * 1024 + lane;
    const v2f *__restrict__ csp1 =
        reinterpret_cast<const v2f *>(a.codespec_w + (size_t)(s0 + ns - 1) * F) + wq * 1024 + lane;
    v2f c1[16];
#pragma unroll
    for (int e = 0; e < 16; e++) {
      X[e] = v[e];
      c1[e] = csp1[64 * e];
      v[e] = csp0[64 * e];
    }
#pragma unroll
    for (int e = 0; e < 16; e++) {
      v[e] = vmulc(X[e], v[e]);
      X[e] = vmulc(X[e], c1[e]);
    }
  }
  for (uint32_t u = 0; u < ns; u++) {                 // uniform
    const uint32_t slot = s0 + u;
    if constexpr (!CSP_PAIR) {
      const v2f *__restrict__ csp =
          reinterpret_cast<const v2f *>(a.codespec_w + (size_t)slot * F) + wq * 1024 + lane;
#pragma unroll
      for (int e = 0; e < 16; e++) v[e] = vmulc(X[e], csp[64 * e]);
    } else if (u) {
#pragma unroll
      for (int e = 0; e < 16; e++) v[e] = X[e];
    }
#ifndef SL_ABL_NOINV   // timing ablation: no inverse sub-transforms
    reg_compute<10, 16, 0, true>(v, w1);
    wave1024_rest<true>(rg, v, w1, lane);
#endif
    // Y_q[m'] (m' = lane + 64 e) -> region q; then the radix-B pass over q per m'
    if constexpr (B > 1) {
#pragma unroll
      for (int e = 0; e < 16; e++) rg[lds_pad(reg_index<10, 16>(lane, e))] = v[e];
      __syncthreads();
#pragma unroll
      for (int i = 0; i < NB; i++) {
        // (no held twiddle: an opaque copy per use, so the reads are issued here and not
        // hoisted out of the slot loop into registers held across it)
        int n = tid + T * i;
        if constexpr (!TW_ONCE) asm volatile("" : "+v"(n));
#pragma unroll
        for (int q = 0; q < B; q++) v[i * B + q] = buf[q * RB + lds_pad(n)];
        v2f w[B > 1 ? B : 2];
        twiddle_powers<B>(w, TW_ONCE ? v2f{wfb[TW_ONCE ? i : 0].x, -wfb[TW_ONCE ? i : 0].y}
                                     : twiddle<true>(a.tw, n * (kTwN / F)));
#pragma unroll
        for (int q = 1; q < B; q++) v[i * B + q] = vmul(v[i * B + q], w[q]);
        dft_small<B, true>(v + i * B);
      }
    }
    // lag index of v[i B + p]: m = n_i + 1024 p (B > 1), or lane + 64 e (B = 1)
    const float vs = a.vscale[slot];
    const int off = (int)(u * a.SL);
    const uint32_t ws = a.SL * slot;                  // window index of lag 0
    unsigned long long best = 0ull;
    if (a.corr_trace) {                               // uniform: DEBUG_LOG trace only
#pragma unroll
      for (int e = 0; e < 16; e++) {
        const int m = (B > 1) ? tid + T * (e / B) + 1024 * (e % B) : reg_index<10, 16>(lane, e);
        corr_trace_put(a, f, r, slot, m - off, (v[e].x * v[e].x + v[e].y * v[e].y) * vs);
      }
    }
    // first maximum over the thread's lags, branch-free (selects, no per-lag exec masks): a
    // lag outside [0, SL) or with a zero metric scores key 0, as the strict '>' from 0 of
    // framing.cc:718, 735 ignores it
    const uint32_t sl = a.SL;
    // (B > 1: the thread's lags m lie in 1024-blocks p = e mod B; only the blocks that meet
    // [off, off + SL) -- three of B at C3 -- can score, so the others are skipped on a uniform
    // test instead of being masked lane by lane)
    const int p_lo = off / 1024, p_hi = (off + (int)sl - 1) / 1024;
#pragma unroll
    for (int e = 0; e < 16; e++) {
      if constexpr (B > 1)
        if (e % B < p_lo || e % B > p_hi) continue;   // uniform
      const int m = (B > 1) ? tid + T * (e / B) + 1024 * (e % B) : reg_index<10, 16>(lane, e);
      const uint32_t i = (uint32_t)(m - off);         // wraps for m < off: out of range
      const float val = (v[e].x * v[e].x + v[e].y * v[e].y) * vs;
      const uint32_t hi = (i < sl && val > 0.0f) ? __float_as_uint(val) : 0u;
      const unsigned long long key = ((unsigned long long)hi << 32) |
                                     (unsigned long long)(0xFFFFFFFFu - (ws + i));
      best = (hi != 0u && key > best) ? key : best;
    }
    best = wave_max_u64(best);
    if (lane == 0 && best) atomicMax(&s_key[u], best);
    __syncthreads();                                  // key final; every reader of buf is done
    if (tid == 0) a.keys[((uint64_t)f * a.N + r) * a.n_slots + slot] = s_key[u];
  }
  // LS terms of the pair's access codes, as search_ls_kernel (register-resident form where
  // the workgroup holds two M-point windows of M/8 threads, else batched through LDS)
#ifdef SL_ABL_NOLS   // timing ablation: no LS terms
  return;
#endif
  constexpr int PBM = lds_padded_len(M), NL = 2 * M / T;
  static_assert(2 * M % T == 0, "whole windows per thread");
  const bool valid0 = s0 != 0, valid1 = ns > 1;
  if ((!valid0 && !valid1) || !a.lsq) return;         // uniform (no lsq: ls_window_kernel)
  const int64_t w0 = I.base + (int64_t)key_index(s_key[0]);
  const int64_t w1v = I.base + (int64_t)key_index(s_key[1]);
  constexpr bool LSREG = 2 * (M / 8) == T && LOG2M >= 9;
  if constexpr (LSREG) {
    using PM = RegPlan<LOG2M, 8>;
    constexpr int PBX = reg_image_len<LOG2M, 8>();     // conflict-free exchange layouts
    static_assert(2 * PBX <= lds_padded_len(F), "both LS images in the search's buffer");
    const uint32_t u = (uint32_t)tid / PM::T, lt = (uint32_t)tid % PM::T;   // u uniform per wave
    const bool valid = u ? valid1 : valid0;
    const int64_t wb = u ? w1v : w0;
    v2f xw[8];
    if (valid && wb >= 0 && wb + M <= L) {            // uniform per wave: one row base
      const auto xr = xs.row((uint64_t)wb);
#pragma unroll
      for (int e = 0; e < 8; e++) {
        const float2 t = xr.at(reg_index<LOG2M, 8>((int)lt, e));
        xw[e] = v2f{t.x, t.y};
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; e++) {
        const int64_t n = wb + reg_index<LOG2M, 8>((int)lt, e);
        const bool ok = valid && n >= 0 && n < L;
        const float2 t = xs.at(n < 0 ? 0 : (n >= L ? L - 1 : n));
        xw[e] = ok ? v2f{t.x, t.y} : v2f{0.0f, 0.0f};
      }
    }
    if constexpr (CFO) {   // window sample lt + e M/8, relative to base: wb - base + ...
      // (nu from LDS, not a register held across the search: fewer spills at F = 2048)
      v2f rb = phasor_cycles32(cfo_lds.nu * (double)(wb - I.base + (int64_t)lt));
      const v2f st = cfo_lds.step[2];
#pragma unroll
      for (int e = 0; e < 8; e++) {
        xw[e] = vmul(xw[e], rb);
        rb = vmul(rb, st);
      }
    }
    v2f wm[PM::NTW > 0 ? PM::NTW : 1];
    reg_twiddles<LOG2M, 8>(wm, a.tw, (int)lt);
    reg_compute<LOG2M, 8, 0, false>(xw, wm);
    reg_rest_lay<LOG2M, 8, 1, false>(buf + u * PBX, xw, wm, (int)lt);
    if (valid) {                                      // uniform per wave
      const uint32_t ac = s0 + u - 1, code = ac / a.N, tx = ac % a.N;
      // (code row bases uniform per wave: SGPR pointers, 32-bit lane offsets; X S1 as a product
      // with the sign, exact for +-1; a null subcarrier's term is an exact +0, as the unfused
      // ls_kernel writes it, whatever X holds)
      const auto sg = sgpr_ptr(a.s1sign + ((size_t)tx * a.nac + code) * M);
      const auto q = sgpr_ptr(reinterpret_cast<v2f *>(a.lsq) +
                              ((((uint64_t)f * a.N + r) * a.N + tx) * a.nac + code) * M);
#pragma unroll
      for (int e = 0; e < 8; e++) {
        const uint32_t k = (uint32_t)reg_index<LOG2M, 8>((int)lt, e);
        const int8_t sv = sg[k];
        const float sgn = (float)sv;
        const v2f term = sv ? xw[e] * v2f{sgn, sgn} : v2f{0.0f, 0.0f};
        ls_term_store(&q[k], term);   // read once, by the combine
      }
    }
  } else {
    float2 *twm = reinterpret_cast<float2 *>(lds_raw) + lds_padded_len(F);
    fill_twiddles_lds<LOG2M, T>(twm, a.tw);
    float2 win[NL];
#pragma unroll
    for (int e = 0; e < NL; e++) {
      const int i = tid + e * T, uu = i / M, j = i % M;
      const int64_t n = (uu ? w1v : w0) + j;
      const bool ok = (uu ? valid1 : valid0) && n >= 0 && n < L;
      win[e] = ok ? xs.at(n) : make_float2(0.0f, 0.0f);
      if constexpr (CFO) {
        const v2f ph = phasor_cycles(cfo_lds.nu * (double)(n - I.base));
        const v2f w = vmul(v2f{win[e].x, win[e].y}, ph);
        win[e] = make_float2(w.x, w.y);
      }
    }
    float2 *lb = reinterpret_cast<float2 *>(buf);
#pragma unroll
    for (int e = 0; e < NL; e++) {
      const int i = tid + e * T, uu = i / M, j = i % M;
      lb[uu * PBM + lds_pad(j)] = win[e];
    }
    __syncthreads();
    fft_lds_twl<LOG2M, T, 2, false>(lb, twm, tid);
#pragma unroll
    for (int e = 0; e < NL; e++) {
      const int i = tid + e * T, uu = i / M, k = i % M;
      if (!(uu ? valid1 : valid0)) continue;
      const uint32_t ac = s0 + uu - 1, code = ac / a.N, tx = ac % a.N;
      const int8_t *sg = a.s1sign + ((size_t)tx * a.nac + code) * M;
      float2 *q = a.lsq + ((((uint64_t)f * a.N + r) * a.N + tx) * a.nac + code) * M;
      const float2 Xk = lb[uu * PBM + lds_pad(k)];
      const int sgn = sg[k];
      const float2 t = sgn > 0 ? Xk : (sgn < 0 ? cneg(Xk) : make_float2(0.0f, 0.0f));
      q[k] = t;
    }
  }
}

// one thread per (frame, subcarrier, rx-tx pair): the codes' X/S1 of lsq in code order, G and
// this block's share of the residual variance (as ls_combine_kernel)
constexpr int kLsRotCodes = 256;   // CFO code rotations tabled in LDS
__global__ __launch_bounds__(256) void ls_combine_q_kernel(LsArgs a) {
  __shared__ double red[4];
  __shared__ double s_nu;
  __shared__ double2 s_rot[kLsRotCodes];
  const uint32_t rt = blockIdx.y, f = blockIdx.z;
  const FrameInfo &I = a.info[f];
  if (I.status != 0) return;
  const uint32_t M = a.M, N = a.N;
  const uint32_t k = blockIdx.x * 256 + threadIdx.x;
  const uint32_t r_ = rt / N, t_ = rt % N;
  // opt-in CFO: the residual's phase at each code's window (window-relative, about the frame's
  // base), as the data region is derotated (cfo_kernels.hip stage 2) -- uniform over the
  // workgroup, so tabled once per code instead of per subcarrier
  const bool rot_tab = a.cfo_part && a.nac <= (uint32_t)kLsRotCodes;
  if (a.cfo_part) {
    if (threadIdx.x == 0) {
      s_nu = cfo_stage_eps(a.cfo_part, f, 2) / (double)M;
      if (blockIdx.x == 0 && rt == 0)   // the frame's total estimate (stage 1 + stage 2)
      {
        const double eps = cfo_stage_eps(a.cfo_part, f, 1) + s_nu * M;
        const_cast<FrameInfo &>(I).cfo_eps = (float)eps;
        const_cast<FrameInfo &>(I).cfo_E = cfo_fixed_freq(eps, M);
      }
    }
    __syncthreads();
    if (rot_tab) {
      for (uint32_t c = threadIdx.x; c < a.nac; c += 256) {
        const unsigned long long key = a.keys[((uint64_t)f * N + r_) * a.n_slots + 1 + c * N + t_];
        const double w = (double)key_index(key) + 0.5 * (double)M;
        double ph = -2.0 * s_nu * w;
        ph -= 2.0 * rint(ph * 0.5);
        double sn, cs;
        sincospi(ph, &sn, &cs);
        s_rot[c] = make_double2(cs, sn);
      }
      __syncthreads();
    }
  }
  double nv = 0.0;
  if (k < M) {
    const bool occ = a.occ_index[k] >= 0;
    const float2 *q = a.lsq + ((uint64_t)f * N * N + rt) * a.nac * M + k;
    double sr = 0.0, si = 0.0, s2 = 0.0;
    const double nu = a.cfo_part ? s_nu : 0.0;
    // the codes' terms in batches of CB loads in flight (one latency per batch instead of per
    // code), summed in code order as before
    constexpr uint32_t CB = 8;
    for (uint32_t c0 = 0; c0 < a.nac; c0 += CB) {
      float2 vb[CB];
#pragma unroll
      for (uint32_t j = 0; j < CB; j++) {   // clamped: every load unconditional; read once
        const v2f t = __builtin_nontemporal_load(reinterpret_cast<const v2f *>(q) + (uint64_t)min(c0 + j, a.nac - 1) * M);
        vb[j] = make_float2(t.x, t.y);
      }
#pragma unroll
      for (uint32_t j = 0; j < CB; j++) {
        const uint32_t c = c0 + j;
        if (c >= a.nac) break;
        float2 v = vb[j];
        if (a.cfo_part) {
          double sn, cs;
          if (rot_tab) {
            cs = s_rot[c].x;
            sn = s_rot[c].y;
          } else {   // (more codes than the table holds)
            const unsigned long long key =
                a.keys[((uint64_t)f * N + r_) * a.n_slots + 1 + c * N + t_];
            const double w = (double)key_index(key) + 0.5 * (double)M;
            double ph = -2.0 * nu * w;
            ph -= 2.0 * rint(ph * 0.5);
            sincospi(ph, &sn, &cs);
          }
          v = make_float2((float)(v.x * cs - v.y * sn), (float)(v.x * sn + v.y * cs));
        }
        sr += (double)v.x;
        si += (double)v.y;
        s2 += (double)v.x * v.x + (double)v.y * v.y;
      }
    }
    const uint32_t r = rt / N, t = rt % N;
    const double bias = (a.keep_bias && r == t) ? 1.0 : 0.0;
    a.G[(((uint64_t)f * M + k) * N + r) * N + t] =
        occ ? make_float2((float)((bias + sr) * a.scale), (float)(si * a.scale))
            : make_float2(0.0f, 0.0f);
    if (occ) nv = s2 - (sr * sr + si * si) / (double)a.nac;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) nv += __shfl_xor(nv, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = nv;
  __syncthreads();
  if (threadIdx.x == 0)
    a.nv_part[(uint64_t)f * a.n_nvp + (uint64_t)rt * gridDim.x + blockIdx.x] =
        red[0] + red[1] + red[2] + red[3];
}

// ------------------------------------------------------------------------------------
// LS estimate, two stages. ls_kernel: one workgroup per (frame, rx, tx, code group) FFTs the
// group's CB access codes as received on rx (the window at the search's corr index) and
// writes the group's per-subcarrier sums of X/S1 (S1 = +-1, framing.cc:811) and |X/S1|^2 in
// fp64. ls_combine_kernel: per (frame, subcarrier) the groups are summed in fixed order into
// G = (I + sum) * dft_normalizer / nac (framing.cc:809-824, identity bias from :309-311) and
// the training-residual variance sum |v - mean|^2 for the MMSE noise estimate.
template <int LOG2M, int T, int CB>
__global__ __launch_bounds__(T) void ls_kernel(LsArgs a) {
  constexpr int M = 1 << LOG2M, PB = lds_padded_len(M), PER = M / T;
  extern __shared__ __attribute__((aligned(16))) float2 lds[];
  const uint32_t f = blockIdx.y;
  const FrameInfo &I = a.info[f];
  if (I.status != 0) return;
  const uint32_t P = a.n_groups;
  const uint32_t rt = blockIdx.x / P, grp = blockIdx.x % P;
  const uint32_t r = rt / a.N, t = rt % a.N;
  const int tid = threadIdx.x;
  const float2 *__restrict__ x = a.iq + ((uint64_t)I.cap * a.N + r) * a.stride;
  const int64_t L = (int64_t)a.frame_len;
  const uint32_t c0 = grp * CB;
  const uint32_t nb = min((uint32_t)CB, a.nac - c0);
  // every code's window start first, then all 16-byte loads in flight together, then the LDS
  // writes (a load -> ds_write loop waits out one memory latency per iteration)
  constexpr int P2 = (M / 2 + T - 1) / T;        // 16-byte pairs per thread per code
  int64_t abs0[CB];
  bool fast[CB];
#pragma unroll
  for (int b = 0; b < CB; b++) {
    abs0[b] = 0;
    if (b < (int)nb) {
      const uint32_t ac = (c0 + b) * a.N + t;
      abs0[b] = I.base + key_index(a.keys[((uint64_t)f * a.N + r) * a.n_slots + 1 + ac]);
    }
    fast[b] = b < (int)nb && abs0[b] >= 0 && abs0[b] + M <= L && (abs0[b] & 1) == 0;
  }
  float4 stg[CB][P2];
#pragma unroll
  for (int b = 0; b < CB; b++) {
    const float4 *x4 = reinterpret_cast<const float4 *>(x + (fast[b] ? abs0[b] : 0));
#pragma unroll
    for (int u = 0; u < P2; u++) {
      const int i = tid + u * T;
      stg[b][u] = (fast[b] && i < M / 2) ? x4[i] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
  }
#pragma unroll
  for (int b = 0; b < CB; b++) {
    if (fast[b]) {                   // 16-byte loads of two samples
#pragma unroll
      for (int u = 0; u < P2; u++) {
        const int i = tid + u * T;
        if (i < M / 2) *reinterpret_cast<float4 *>(lds + b * PB + lds_pad(2 * i)) = stg[b][u];
      }
    } else {
      for (int i = tid; i < M; i += T) {
        const int64_t n = abs0[b] + i;
        lds[b * PB + lds_pad(i)] =
            (b < (int)nb && n >= 0 && n < L) ? x[n] : make_float2(0.0f, 0.0f);
      }
    }
  }
  __syncthreads();
  fft_lds<LOG2M, T, CB, false>(lds, a.tw);
  double *pp = a.part + (((uint64_t)f * a.N * a.N + rt) * P + grp) * 3 * M;
#pragma unroll
  for (int q = 0; q < PER; q++) {
    const int k = tid + q * T;
    double sr = 0.0, si = 0.0, s2 = 0.0;
    for (int b = 0; b < (int)nb; b++) {
      const int sg = a.s1sign[((size_t)t * a.nac + c0 + b) * M + k];
      if (sg == 0) continue;                     // null subcarrier
      const float2 X = lds[b * PB + lds_pad(k)];
      const float2 v = (sg > 0) ? X : cneg(X);   // X / S1
      sr += (double)v.x;
      si += (double)v.y;
      s2 += (double)v.x * v.x + (double)v.y * v.y;
    }
    pp[k] = sr;
    pp[M + k] = si;
    pp[2 * M + k] = s2;
  }
}

// one thread per (frame, subcarrier, rx-tx pair): the code groups in fixed order, G, and this
// block's share of the residual variance (nv_part[f][rt][block], summed in order by weights)
__global__ __launch_bounds__(256) void ls_combine_kernel(LsArgs a) {
  __shared__ double red[4];
  const uint32_t rt = blockIdx.y, f = blockIdx.z;
  const FrameInfo &I = a.info[f];
  if (I.status != 0) return;
  const uint32_t M = a.M, N = a.N, P = a.n_groups;
  const uint32_t k = blockIdx.x * 256 + threadIdx.x;
  double nv = 0.0;
  if (k < M) {
    const bool occ = a.occ_index[k] >= 0;
    const double *pp = a.part + ((uint64_t)f * N * N + rt) * P * 3 * M;
    double sr = 0.0, si = 0.0, s2 = 0.0;
    for (uint32_t g = 0; g < P; g++) {
      sr += pp[(uint64_t)g * 3 * M + k];
      si += pp[(uint64_t)g * 3 * M + M + k];
      s2 += pp[(uint64_t)g * 3 * M + 2 * M + k];
    }
    const uint32_t r = rt / N, t = rt % N;
    const double bias = (a.keep_bias && r == t) ? 1.0 : 0.0;
    a.G[(((uint64_t)f * M + k) * N + r) * N + t] =
        occ ? make_float2((float)((bias + sr) * a.scale), (float)(si * a.scale))
            : make_float2(0.0f, 0.0f);
    if (occ) nv = s2 - (sr * sr + si * si) / (double)a.nac;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) nv += __shfl_xor(nv, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = nv;
  __syncthreads();
  if (threadIdx.x == 0)
    a.nv_part[(uint64_t)f * a.n_nvp + (uint64_t)rt * gridDim.x + blockIdx.x] =
        red[0] + red[1] + red[2] + red[3];
}

// ------------------------------------------------------------------------------------
// complex double Gauss-Jordan with partial pivoting (same algorithm as the oracle)
struct cd { double re, im; };

template <int N>
MIMO_DEV bool cd_solve(cd (&A)[N][N], cd (&B)[N][N]) {
#pragma unroll
  for (int c = 0; c < N; c++) {
    int piv = c;
    double best = A[c][c].re * A[c][c].re + A[c][c].im * A[c][c].im;
#pragma unroll
    for (int rr = c + 1; rr < N; rr++) {
      const double m = A[rr][c].re * A[rr][c].re + A[rr][c].im * A[rr][c].im;
      if (m > best) { best = m; piv = rr; }
    }
    // swap rows c and piv with static indexing
#pragma unroll
    for (int rr = c + 1; rr < N; rr++) {
      if (rr == piv) {
#pragma unroll
        for (int k = 0; k < N; k++) {
          cd t1 = A[c][k]; A[c][k] = A[rr][k]; A[rr][k] = t1;
          cd t2 = B[c][k]; B[c][k] = B[rr][k]; B[rr][k] = t2;
        }
      }
    }
    const cd d = A[c][c];
    const double dd = d.re * d.re + d.im * d.im;
    if (dd == 0.0) return false;
    const cd inv = {d.re / dd, -d.im / dd};
#pragma unroll
    for (int k = 0; k < N; k++) {
      const cd x = A[c][k], y = B[c][k];
      A[c][k] = {x.re * inv.re - x.im * inv.im, x.re * inv.im + x.im * inv.re};
      B[c][k] = {y.re * inv.re - y.im * inv.im, y.re * inv.im + y.im * inv.re};
    }
#pragma unroll
    for (int rr = 0; rr < N; rr++) {
      if (rr == c) continue;
      const cd fct = A[rr][c];
      if (fct.re == 0.0 && fct.im == 0.0) continue;
#pragma unroll
      for (int k = 0; k < N; k++) {
        const cd x = A[c][k], y = B[c][k];
        A[rr][k].re -= fct.re * x.re - fct.im * x.im;
        A[rr][k].im -= fct.re * x.im + fct.im * x.re;
        B[rr][k].re -= fct.re * y.re - fct.im * y.im;
        B[rr][k].im -= fct.re * y.im + fct.im * y.re;
      }
    }
  }
  return true;
}

template <int N>
__global__ __launch_bounds__(256) void weights_kernel(WeightArgs a) {
  const uint32_t f = blockIdx.y;
  FrameInfo &I = a.info[f];
  if (I.status != 0) return;
  const uint32_t k = blockIdx.x * 256 + threadIdx.x;
  // noise variance (same double expression as the oracle) and replay bookkeeping
  double s2 = (double)a.noise_var;
  if (a.noise_var < 0.0f) {
    // the residual-variance partials, summed by wave 0 in a fixed order (lane-strided, then a
    // fixed shuffle tree) and broadcast through LDS
    __shared__ double s_acc;
    if (threadIdx.x < 64) {
      double acc = 0.0;
      for (uint32_t e = threadIdx.x; e < a.n_nvp; e += 64)
        acc += a.nv_part[(uint64_t)f * a.n_nvp + e];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
      if (threadIdx.x == 0) s_acc = acc;
    }
    __syncthreads();
    s2 = (double)(float)(s_acc * a.nv_norm);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    I.noise_var = (float)s2;
    // replay from corr_indices[N-1][N*nac-1] + M (framing.cc:857, generalised from [1])
    const unsigned long long key =
        a.keys[((uint64_t)f * N + (N - 1)) * a.n_slots + a.n_slots - 1];
    const uint32_t ci = key ? (0xFFFFFFFFu - (uint32_t)(key & 0xFFFFFFFFull)) : 0u;
    const uint64_t i0 = (uint64_t)ci + a.M;
    I.i0 = (uint32_t)i0;
    I.n_sym = (i0 < a.win_len) ? (uint32_t)((a.win_len - i0) / a.SL) : 0u;
  }
  if (k >= a.M) return;
  const float2 *g = a.G + ((uint64_t)f * a.M + k) * N * N;
  float2 W[N][N];
  float gain = 1.0f;
  if (a.occ_index[k] < 0) {
#pragma unroll
    for (int i = 0; i < N; i++)
#pragma unroll
      for (int j = 0; j < N; j++) W[i][j] = make_float2(0.0f, 0.0f);
  } else if (a.detector == 0 || a.detector == 3) {  // reference 2x2 invert (framing.cc:1344)
    if constexpr (N == 2) {
      const float2 det = csub(cmul(g[0], g[3]), cmul(g[1], g[2]));
      const float2 di = cconj(det);
      W[0][0] = cmul(di, g[3]);
      W[1][1] = cmul(di, g[0]);
      W[1][0] = cmul(cneg(di), g[2]);
      W[0][1] = cmul(cneg(di), g[1]);
      gain = 1.0f / (det.x * det.x + det.y * det.y);
    } else {
#pragma unroll
      for (int i = 0; i < N; i++)
#pragma unroll
        for (int j = 0; j < N; j++) W[i][j] = make_float2(i == j ? 1.0f : 0.0f, 0.0f);
    }
  } else {
    cd A[N][N], B[N][N];
    if (a.detector == 1) {  // ZF: W = G^-1
#pragma unroll
      for (int i = 0; i < N; i++)
#pragma unroll
        for (int j = 0; j < N; j++) {
          A[i][j] = {(double)g[i * N + j].x, (double)g[i * N + j].y};
          B[i][j] = {i == j ? 1.0 : 0.0, 0.0};
        }
    } else {                // MMSE: W = (G^H G + s2 I)^-1 G^H
#pragma unroll
      for (int i = 0; i < N; i++)
#pragma unroll
        for (int j = 0; j < N; j++) {
          double sr = 0.0, si = 0.0;
#pragma unroll
          for (int rr = 0; rr < N; rr++) {
            const double gar = g[rr * N + i].x, gai = g[rr * N + i].y;
            const double gbr = g[rr * N + j].x, gbi = g[rr * N + j].y;
            sr += gar * gbr + gai * gbi;
            si += gar * gbi - gai * gbr;
          }
          A[i][j] = {sr + ((i == j) ? s2 : 0.0), si};
          B[i][j] = {(double)g[j * N + i].x, -(double)g[j * N + i].y};
        }
    }
    const bool ok = cd_solve<N>(A, B);
#pragma unroll
    for (int i = 0; i < N; i++)
#pragma unroll
      for (int j = 0; j < N; j++)
        W[i][j] = ok ? make_float2((float)B[i][j].re, (float)B[i][j].im) : make_float2(0.f, 0.f);
  }
#pragma unroll
  for (int t = 0; t < N; t++)
#pragma unroll
    for (int rr = 0; rr < N; rr++)
      a.W[(((uint64_t)f * N + t) * N + rr) * a.M + k] = W[t][rr];
  a.gain[(uint64_t)f * a.M + k] = gain;
}

// ------------------------------------------------------------------------------------
// N = 8: the per-thread form above needs 2 N^2 complex doubles in registers (512 VGPRs at
// 8x8) and spills to scratch. Here one subcarrier is solved by a group of 8 lanes, lane j
// holding row j of [A | B] (4 N doubles). The same Gauss-Jordan with partial pivoting as
// cd_solve / the oracle: a lane's `pos` is its row's current index in the oracle's row
// array, so the pivot search (largest |a|^2 among rows >= c, the smallest index winning
// ties = the oracle's strict '>' scan from c) and the row swap (two lanes exchange pos) follow
// the oracle exactly. The normalised pivot row is broadcast through LDS.
constexpr int kWRowT = 256;
constexpr int kWRowG = kWRowT / 8;   // subcarriers per workgroup

template <int N>
__global__ __launch_bounds__(kWRowT) void weights_row_kernel(WeightArgs a) {
  static_assert(N >= 2 && N <= 8, "row solve handles 2..8 streams");
  const uint32_t f = blockIdx.y;
  FrameInfo &I = a.info[f];
  if (I.status != 0) return;
  __shared__ float2 s_g[kWRowG][N * N];
  __shared__ cd s_piv[kWRowG][2 * N];
  __shared__ int s_sing[kWRowG];
  __shared__ double s_acc;
  const int tid = threadIdx.x, grp = tid >> 3, j = tid & 7;
  const uint32_t k = blockIdx.x * kWRowG + grp;
  double s2 = (double)a.noise_var;
  if (a.noise_var < 0.0f) {   // fixed-order partial sum, as weights_kernel
    if (tid < 64) {
      double acc = 0.0;
      for (uint32_t e = tid; e < a.n_nvp; e += 64) acc += a.nv_part[(uint64_t)f * a.n_nvp + e];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
      if (tid == 0) s_acc = acc;
    }
    __syncthreads();
    s2 = (double)(float)(s_acc * a.nv_norm);
  }
  if (blockIdx.x == 0 && tid == 0) {
    I.noise_var = (float)s2;
    const unsigned long long key =
        a.keys[((uint64_t)f * N + (N - 1)) * a.n_slots + a.n_slots - 1];
    const uint32_t ci = key ? (0xFFFFFFFFu - (uint32_t)(key & 0xFFFFFFFFull)) : 0u;
    const uint64_t i0 = (uint64_t)ci + a.M;
    I.i0 = (uint32_t)i0;
    I.n_sym = (i0 < a.win_len) ? (uint32_t)((a.win_len - i0) / a.SL) : 0u;
  }
  const bool live = k < a.M;
  const bool occ = live && a.occ_index[k] >= 0;
  if (live)
    for (int e = j; e < N * N; e += 8) s_g[grp][e] = a.G[((uint64_t)f * a.M + k) * N * N + e];
  __syncthreads();
  const bool row = j < N;
  cd A[N], B[N];
  const float2 *g = s_g[grp];
#pragma unroll
  for (int c = 0; c < N; c++) {
    A[c] = {0.0, 0.0};
    B[c] = {0.0, 0.0};
  }
  if (row) {
    if (a.detector == 1) {   // ZF: A = G, B = I
#pragma unroll
      for (int c = 0; c < N; c++) {
        A[c] = {(double)g[j * N + c].x, (double)g[j * N + c].y};
        B[c] = {c == j ? 1.0 : 0.0, 0.0};
      }
    } else {                 // MMSE: A = G^H G + s2 I, B = G^H
#pragma unroll
      for (int c = 0; c < N; c++) {
        double sr = 0.0, si = 0.0;
#pragma unroll
        for (int rr = 0; rr < N; rr++) {
          const double gar = g[rr * N + j].x, gai = g[rr * N + j].y;
          const double gbr = g[rr * N + c].x, gbi = g[rr * N + c].y;
          sr += gar * gbr + gai * gbi;
          si += gar * gbi - gai * gbr;
        }
        A[c] = {sr + ((c == j) ? s2 : 0.0), si};
        B[c] = {(double)g[c * N + j].x, -(double)g[c * N + j].y};
      }
    }
  }
  int pos = row ? j : 64;
  bool ok = true;
#pragma unroll
  for (int c = 0; c < N; c++) {
    // pivot: max |A[.][c]|^2 over rows with pos >= c, smallest pos on ties
    double m = (row && pos >= c) ? A[c].re * A[c].re + A[c].im * A[c].im : -1.0;
    int mp = (row && pos >= c) ? pos : 64;
#pragma unroll
    for (int off = 1; off < 8; off <<= 1) {
      const double om = __shfl_xor(m, off);
      const int op = __shfl_xor(mp, off);
      if (om > m || (om == m && op < mp)) { m = om; mp = op; }
    }
    // swap: the row at pos c takes the pivot's place
    if (pos == c) pos = mp;
    else if (pos == mp) pos = c;
    if (pos == c && row) {              // the pivot lane normalises and publishes its row
      const cd d = A[c];
      const double dd = d.re * d.re + d.im * d.im;
      s_sing[grp] = dd == 0.0 ? 1 : 0;
      if (dd != 0.0) {
        const cd inv = {d.re / dd, -d.im / dd};
#pragma unroll
        for (int q = 0; q < N; q++) {
          const cd x = A[q], y = B[q];
          A[q] = {x.re * inv.re - x.im * inv.im, x.re * inv.im + x.im * inv.re};
          B[q] = {y.re * inv.re - y.im * inv.im, y.re * inv.im + y.im * inv.re};
          s_piv[grp][q] = A[q];
          s_piv[grp][N + q] = B[q];
        }
      }
    }
    __syncthreads();
    const bool sing = s_sing[grp] != 0;
    ok = ok && !sing;
    if (!sing && row && pos != c) {
      const cd fct = A[c];
      if (!(fct.re == 0.0 && fct.im == 0.0)) {
#pragma unroll
        for (int q = 0; q < N; q++) {
          const cd x = s_piv[grp][q], y = s_piv[grp][N + q];
          A[q].re -= fct.re * x.re - fct.im * x.im;
          A[q].im -= fct.re * x.im + fct.im * x.re;
          B[q].re -= fct.re * y.re - fct.im * y.im;
          B[q].im -= fct.re * y.im + fct.im * y.re;
        }
      }
    }
    __syncthreads();
  }
  if (!live || !row) return;
  // row `pos` of B is row `pos` of W (output stream pos); zero on a null carrier or a singular
  // system (as weights_kernel); detectors other than ZF/MMSE keep the identity (weights_kernel)
  const bool solve = a.detector == 1 || a.detector == 2;
#pragma unroll
  for (int rr = 0; rr < N; rr++) {
    float2 w = make_float2(0.0f, 0.0f);
    if (occ && solve && ok) w = make_float2((float)B[rr].re, (float)B[rr].im);
    else if (occ && !solve && rr == pos) w = make_float2(1.0f, 0.0f);
    a.W[(((uint64_t)f * N + pos) * N + rr) * a.M + k] = w;
  }
  if (j == 0) a.gain[(uint64_t)f * a.M + k] = 1.0f;
}

// ------------------------------------------------------------------------------------
template <int LOG2M, int LOG2F>
static void codes_dispatch_f(const CodesArgs &a, int log2F, hipStream_t s) {
  if constexpr (LOG2F <= 14) {
    if (log2F == LOG2F) {
      constexpr int F = 1 << LOG2F;
      const size_t shm = sizeof(float2) * lds_padded_len(F);
      (void)hipFuncSetAttribute((const void *)codes_kernel<LOG2M, LOG2F>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
      hipLaunchKernelGGL((codes_kernel<LOG2M, LOG2F>), dim3(a.n_slots), dim3(kEstT), shm, s, a);
      return;
    }
    codes_dispatch_f<LOG2M, LOG2F + 1>(a, log2F, s);
  }
}

template <int LOG2M>
static void codes_dispatch(const CodesArgs &a, int log2M, int log2F, hipStream_t s) {
  if constexpr (LOG2M <= 12) {
    if (log2M == LOG2M) { codes_dispatch_f<LOG2M, LOG2M>(a, log2F, s); return; }
    codes_dispatch<LOG2M + 1>(a, log2M, log2F, s);
  }
}

void launch_codes(const CodesArgs &a, int log2M, int log2F, hipStream_t s) {
  codes_dispatch<6>(a, log2M, log2F, s);
}

template <int LOG2F>
static void search_dispatch(const SearchArgs &a, int log2F, uint32_t nf, hipStream_t s) {
  if constexpr (LOG2F <= 13) {
    if (log2F == LOG2F) {
      const size_t shm = sizeof(float2) * lds_padded_len(1 << LOG2F);
      dim3 grid(a.n_slots * a.N * a.n_lagc, nf);
      if constexpr (LOG2F >= 10) {
        (void)hipFuncSetAttribute((const void *)search_reg_kernel<LOG2F>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
        hipLaunchKernelGGL(search_reg_kernel<LOG2F>, grid, dim3((1 << LOG2F) / 16), shm, s, a);
      } else {
        (void)hipFuncSetAttribute((const void *)search_kernel<LOG2F>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
        hipLaunchKernelGGL(search_kernel<LOG2F>, grid, dim3(kEstT), shm, s, a);
      }
      return;
    }
    search_dispatch<LOG2F + 1>(a, log2F, nf, s);
  }
}

void launch_search(const SearchArgs &a, int log2F, uint32_t n_frames, hipStream_t s) {
  search_dispatch<7>(a, log2F, n_frames, s);
}

// search_ls_kernel instances: F = 2^10 .. 2^14 with F/M = 2, 4 or 8 (F is the smallest power
// of two >= max(2 SL + M - 1, 2M), so F/M <= 8 for cp <= M)
template <int LOG2F, int D>
static bool search_ls_try(const SearchArgs &a, int log2F, int log2M, uint32_t nf, hipStream_t s) {
  if constexpr (LOG2F <= 14) {
    if constexpr (D <= 3) {
      constexpr int LOG2M = LOG2F - D;
      if (log2F == LOG2F && log2M == LOG2M) {
        if (nf) {
          // the segment image, then the LS transform's M/2 twiddles
          const size_t shm = sizeof(float2) * (lds_padded_len(1 << LOG2F) + (1 << LOG2M) / 2);
          // wave-local sub-transforms (F = 1024 B) unless RMIMO_SEARCH_WAVE=0 (A/B)
          void (*kern)(SearchArgs) = nullptr;
          if constexpr (LOG2F >= 10) {
            if (search_ls_wave_enabled() && a.codespec_w)
              kern = a.cfo_part ? (a.sc16 ? search_ls_wave_kernel<LOG2F, LOG2M, true, true>
                                          : search_ls_wave_kernel<LOG2F, LOG2M, false, true>)
                                : (a.sc16 ? search_ls_wave_kernel<LOG2F, LOG2M, true>
                                          : search_ls_wave_kernel<LOG2F, LOG2M, false>);
          }
          if (!kern)
            kern = a.cfo_part ? (a.sc16 ? search_ls_kernel<LOG2F, LOG2M, true, true>
                                        : search_ls_kernel<LOG2F, LOG2M, false, true>)
                              : (a.sc16 ? search_ls_kernel<LOG2F, LOG2M, true>
                                        : search_ls_kernel<LOG2F, LOG2M, false>);
          (void)hipFuncSetAttribute((const void *)kern,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
          dim3 grid(((a.n_slots + 1) / 2) * a.N, nf);
          hipLaunchKernelGGL(kern, grid, dim3((1 << LOG2F) / 16), shm, s, a);
        }
        return true;
      }
      return search_ls_try<LOG2F, D + 1>(a, log2F, log2M, nf, s);
    } else {
      return search_ls_try<LOG2F + 1, 1>(a, log2F, log2M, nf, s);
    }
  }
  return false;
}

// the search form, a parity-test switch: the wave-local search_ls_wave_kernel (F >= 1024), or
// RMIMO_SEARCH_FORM=block: search_ls_kernel, the same two slots per transform with
// workgroup-wide exchanges
bool search_ls_wave_enabled() {
  static const bool block = [] { const char *e = getenv("RMIMO_SEARCH_FORM"); return e && strcmp(e, "block") == 0; }();
  return !block;
}

bool search_ls_supported(int log2F, int log2M) {
  return search_ls_try<10, 1>(SearchArgs{}, log2F, log2M, 0, nullptr);
}

bool launch_search_ls(const SearchArgs &a, int log2F, int log2M, uint32_t n_frames, hipStream_t s) {
  return search_ls_try<10, 1>(a, log2F, log2M, n_frames, s);
}

// ------------------------------------------------------------------------------------
// LS estimate of one (frame, rx, tx) straight from its nac access-code windows (framing.cc:
// 797-824): workgroup (rx tx, frame), M/8 threads with 8 subcarriers each (k = lt + T e); per
// code c the window at the search's key of slot 1 + c N + tx is loaded one code ahead (the
// barriers of the transform order LDS only, so the prefetch stays in flight), transformed in
// registers (the fused search's LS transform: RegPlan<LOG2M, 8> with the conflict-free
// exchange layouts), multiplied by the S1 sign and summed in fp64 in code order. G and the
// residual-variance partials are then ls_combine_q_kernel's bit for bit -- the same fp32 terms,
// summed in the same order, and the same reduction tree (64-lane butterfly, the four 64-runs of
// each 256-subcarrier block left to right) -- without the terms' round trip through HBM
// (268 MB each way per C3 x 64 batch).
//   With the opt-in CFO (CFO: a.cfo_part) the fused form's two corrections are one phasor
// sequence on the window's samples: the folded form's stage-1 derotation (the search's
// exp(-j 2 pi nu1 n) at window sample n - base) and the stage-2 residual's rotation of the code's
// term (exp(-j 2 pi nu2 (key + M/2)), ls_combine_q_kernel's) -- a constant per window, so it can
// multiply the samples instead of the transform's output. Per code a start phasor tabled in LDS
// (fp64 phase, both parts), per thread its lane's step exp(-j 2 pi nu1 lt): one complex product
// per code and thread, then the 8-point recurrence. G agrees with the fused form to fp32
// rounding (test_ls_window_with_cfo_equals_fused_terms). Workgroup (rx 0, tx 0) records the
// frame's total estimate.
template <int LOG2M, bool SC16, bool CFO>
__global__ __launch_bounds__((1 << LOG2M) / 8) __attribute__((amdgpu_waves_per_eu(4)))
void ls_window_kernel(LsArgs a) {
  using PM = RegPlan<LOG2M, 8>;
  constexpr int M = 1 << LOG2M, T = PM::T, NW = T / 64;
  static_assert(T % 64 == 0, "whole waves");
  extern __shared__ __attribute__((aligned(16))) float2 lds_raw[];
  v2f *buf = reinterpret_cast<v2f *>(lds_raw);
  // the |X/S1|^2 sums in registers up to M = 2048 (124 VGPRs; an LDS read-modify-write per
  // term cost 7 us of the kernel's 100); at M = 4096 they would spill and live in LDS after
  // the image (thread lt's at e T + lt: lane-contiguous, conflict-free 8-byte accesses)
  constexpr bool S2REG = LOG2M <= 11;
  double *s2l = reinterpret_cast<double *>(lds_raw + reg_image_len<LOG2M, 8>()) + threadIdx.x;
  // (up to M = 2048 the LDS the sums left holds a second transform image instead)
  v2f *pa = buf, *pb = buf + reg_image_len<LOG2M, 8>();
  __shared__ double red[M / 64];
  const uint32_t rt = blockIdx.x, f = blockIdx.y;
  const FrameInfo &I = a.info[f];
  if (I.status != 0) return;
  const uint32_t N = a.N, r = rt / N, t = rt % N, nac = a.nac;
  const int lt = threadIdx.x, lane = lt & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane((uint32_t)lt >> 6);
  const int64_t L = (int64_t)a.frame_len;
  const auto xs = iq_row<SC16>(a.iq, a.iq_scale, ((uint64_t)I.cap * N + r) * a.stride);
  const unsigned long long *kp = a.keys + ((uint64_t)f * N + r) * a.n_slots + 1 + t;
  __shared__ v2f s_rot[CFO ? kLsRotCodes : 1];       // CFO: code c's start phasor
  __shared__ double s_nu1, s_nu2;
  __shared__ v2f s_step;
  v2f q_lt = v2f{1.0f, 0.0f};                         // CFO: exp(-j 2 pi nu1 lt)
  if constexpr (CFO) {
    if (lt == 0) {
      const double nu2 = cfo_stage_eps(a.cfo_part, f, 2) / (double)M;
      s_nu2 = nu2;
      if (rt == 0) {   // the frame's total estimate (stage 1 + stage 2), as ls_combine_q_kernel
        const double eps = cfo_stage_eps(a.cfo_part, f, 1) + nu2 * M;
        const_cast<FrameInfo &>(I).cfo_eps = (float)eps;
        const_cast<FrameInfo &>(I).cfo_E = cfo_fixed_freq(eps, M);
      }
      s_nu1 = a.cfo_fold ? cfo_stage_eps(a.cfo_part, f, 1) / (double)M : 0.0;
      s_step = phasor_cycles(s_nu1 * (double)(M / 8));
    }
    __syncthreads();
    const double nu1 = s_nu1, nu2 = s_nu2;
    for (uint32_t c = lt; c < nac; c += T) {
      const double k = (double)key_index(kp[(uint64_t)c * N]);
      s_rot[c] = phasor_cycles(nu1 * k + nu2 * (k + 0.5 * (double)M));
    }
    q_lt = phasor_cycles(nu1 * (double)lt);
    __syncthreads();
  }
  auto load_win = [&](uint32_t c, v2f *xw) {
#ifdef LSW_ABL_NOLOAD   // timing ablation (tools/build_var.sh): no window loads
#pragma unroll
    for (int e = 0; e < 8; e++) xw[e] = v2f{(float)(e + c), (float)lt};
    return;
#endif
    const int64_t wb = I.base + (int64_t)key_index(kp[(uint64_t)c * N]);
    if (wb >= 0 && wb + M <= L) {                      // uniform: one row base
      const auto xr = xs.row((uint64_t)wb);
#pragma unroll
      for (int e = 0; e < 8; e++) {
        const float2 v = xr.at(reg_index<LOG2M, 8>(lt, e));
        xw[e] = v2f{v.x, v.y};
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; e++) {
        const int64_t n = wb + reg_index<LOG2M, 8>(lt, e);
        const float2 v = xs.at(n < 0 ? 0 : (n >= L ? L - 1 : n));
        xw[e] = (n >= 0 && n < L) ? v2f{v.x, v.y} : v2f{0.0f, 0.0f};
      }
    }
  };
  // CFO: window sample lt + e M/8 of code c times s_rot[c] q_lt step^e (when the code's
  // transform starts, so the prefetch is not waited for at its issue)
  auto derotate = [&](uint32_t c, v2f *xw) {
    v2f rb = vmul(s_rot[c], q_lt);
    const v2f st = s_step;
#pragma unroll
    for (int e = 0; e < 8; e++) {
      xw[e] = vmul(xw[e], rb);
      rb = vmul(rb, st);
    }
  };
  // the code's 8 signs of this thread, one 8-byte load (s1sign_w: [t][c][lt][e])
  auto load_sign = [&](uint32_t c) {
    return *reinterpret_cast<const uint2 *>(a.s1sign_w + ((size_t)t * nac + c) * M + 8 * lt);
  };
  v2f wm[PM::NTW > 0 ? PM::NTW : 1];
  reg_twiddles<LOG2M, 8>(wm, a.tw, lt);
  double sr[8], si[8], s2r[S2REG ? 8 : 1];
#pragma unroll
  for (int e = 0; e < 8; e++) {
    sr[e] = si[e] = 0.0;
    if constexpr (S2REG) s2r[e] = 0.0;
    else s2l[e * T] = 0.0;
  }
  v2f xn[8];
  load_win(0, xn);
  uint2 sn = load_sign(0);
  for (uint32_t c = 0; c < nac; c++) {
    v2f xw[8];
#pragma unroll
    for (int e = 0; e < 8; e++) xw[e] = xn[e];
    const uint2 sv = sn;
    if (c + 1 < nac) {                                 // uniform: the next code in flight
      load_win(c + 1, xn);
      sn = load_sign(c + 1);
    }
#ifdef LSW_ABL_NOPF   // timing ablation: the next code's loads complete before this transform
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    if constexpr (CFO) derotate(c, xw);
#ifndef LSW_ABL_NOFFT   // timing ablation: no transform
    reg_compute<LOG2M, 8, 0, false>(xw, wm);
    if constexpr (S2REG) {   // two images in turn, one barrier per exchange
      reg_rest_pp<LOG2M, 8, 1, false>(pa, pb, xw, wm, lt);
      if constexpr ((PM::NP - 1) & 1) {   // the next code starts on the image not used last
        v2f *tmp = pa;
        pa = pb;
        pb = tmp;
      }
    } else {
      reg_rest_lay<LOG2M, 8, 1, false, true>(buf, xw, wm, lt);
    }
#endif
#pragma unroll
    for (int e = 0; e < 8; e++) {
      // X / S1 (S1 = +-1: a product with the sign, exact; a null subcarrier's term is +0)
      const int8_t s8 = (int8_t)(((e < 4 ? sv.x : sv.y) >> (8 * (e & 3))) & 0xFFu);
      const float sgn = (float)s8;
      const v2f term = s8 ? xw[e] * v2f{sgn, sgn} : v2f{0.0f, 0.0f};
      sr[e] += (double)term.x;
      si[e] += (double)term.y;
      if constexpr (S2REG) s2r[e] += (double)term.x * term.x + (double)term.y * term.y;
      else s2l[e * T] += (double)term.x * term.x + (double)term.y * term.y;
    }
  }
  const double bias = (a.keep_bias && r == t) ? 1.0 : 0.0;
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const uint32_t k = (uint32_t)reg_index<LOG2M, 8>(lt, e);
    const bool occ = a.occ_index[k] >= 0;
    a.G[(((uint64_t)f * M + k) * N + r) * N + t] =
        occ ? make_float2((float)((bias + sr[e]) * a.scale), (float)(si[e] * a.scale))
            : make_float2(0.0f, 0.0f);
    const double s2 = S2REG ? s2r[S2REG ? e : 0] : s2l[e * T];
    double nv = occ ? s2 - (sr[e] * sr[e] + si[e] * si[e]) / (double)nac : 0.0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) nv += __shfl_xor(nv, off);
    // the wave's 64 subcarriers 64 wv + T e + lane: run (64 wv + T e) / 64 of the frame
    if (lane == 0) red[(64 * wv + T * e) / 64] = nv;
  }
  __syncthreads();
  for (int b = lt; b < M / 256; b += T)
    a.nv_part[(uint64_t)f * a.n_nvp + (uint64_t)rt * (M / 256) + b] =
        red[4 * b] + red[4 * b + 1] + red[4 * b + 2] + red[4 * b + 3];
  (void)NW;
}

bool launch_ls_window(const LsArgs &a, int log2M, uint32_t n_frames, hipStream_t s) {
  if (!a.s1sign_w || log2M < 9 || log2M > 12 || (a.cfo_part && a.nac > (uint32_t)kLsRotCodes))
    return false;
  if (!n_frames) return true;
  void (*kern)(LsArgs) = nullptr;
  size_t shm = 0;
  int T = 0;
  const bool cfo = a.cfo_part != nullptr;
  switch (log2M) {
#define LSW(L2)                                                                             \
  case L2:                                                                                  \
    kern = cfo ? (a.sc16 ? ls_window_kernel<L2, true, true> : ls_window_kernel<L2, false, true>) \
               : (a.sc16 ? ls_window_kernel<L2, true, false> : ls_window_kernel<L2, false, false>); \
    shm = sizeof(float2) * reg_image_len<L2, 8>() *                                          \
              (L2 > 11 ? 1 : 2) + (L2 > 11 ? sizeof(double) * (1 << L2) : 0);              \
    T = (1 << L2) / 8;                                                                      \
    break;
    LSW(9) LSW(10) LSW(11) LSW(12)
#undef LSW
  }
  (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  hipLaunchKernelGGL(kern, dim3(a.N * a.N, n_frames), dim3(T), shm, s, a);
  return true;
}

void launch_ls_combine_q(const LsArgs &a, uint32_t n_frames, hipStream_t s) {
  hipLaunchKernelGGL(ls_combine_q_kernel, dim3((a.M + 255) / 256, a.N * a.N, n_frames), dim3(256),
                     0, s, a);
}

template <int LOG2M>
static void ls_dispatch(const LsArgs &a, int log2M, uint32_t nf, hipStream_t s) {
  if constexpr (LOG2M <= 12) {
    if (log2M == LOG2M) {
      constexpr int M = 1 << LOG2M;
      constexpr int T = M < 256 ? M : 256;
      constexpr int CB = kLsCodesPerGroup;
      const size_t shm = sizeof(float2) * lds_padded_len(M) * CB;
      (void)hipFuncSetAttribute((const void *)ls_kernel<LOG2M, T, CB>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
      hipLaunchKernelGGL((ls_kernel<LOG2M, T, CB>), dim3(a.N * a.N * a.n_groups, nf), dim3(T),
                         shm, s, a);
      hipLaunchKernelGGL(ls_combine_kernel, dim3((a.M + 255) / 256, a.N * a.N, nf), dim3(256),
                         0, s, a);
      return;
    }
    ls_dispatch<LOG2M + 1>(a, log2M, nf, s);
  }
}

void launch_ls(const LsArgs &a, int log2M, uint32_t n_frames, hipStream_t s) {
  ls_dispatch<6>(a, log2M, n_frames, s);
}

void launch_weights(const WeightArgs &a, uint32_t n_frames, hipStream_t s) {
  dim3 grid((a.M + 255) / 256, n_frames);
  switch (a.N) {
    case 1: hipLaunchKernelGGL(weights_kernel<1>, grid, dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL(weights_kernel<2>, grid, dim3(256), 0, s, a); break;
    case 3: hipLaunchKernelGGL(weights_kernel<3>, grid, dim3(256), 0, s, a); break;
    case 4: hipLaunchKernelGGL(weights_kernel<4>, grid, dim3(256), 0, s, a); break;
    default: {   // 8 streams (mimo_rx_create admits 1, 2, 4, 8): the 8-lane row solve
      dim3 rgrid((a.M + kWRowG - 1) / kWRowG, n_frames);
      hipLaunchKernelGGL(weights_row_kernel<8>, rgrid, dim3(kWRowT), 0, s, a);
      break;
    }
  }
}

}  // namespace mimo

// rub_mimo_amd/csrc/decode_kernels.hip -- replay decode of the data symbols on gfx950, the
// HBM-bound hot kernel of the pipeline.
//
// Reference: estimate_channel's replay loop (framing.cc:853-868) calls execute_mimo_decode
// (framing.cc:535-589) every SL samples from window index corr_indices[N-1][last] + M:
// drop the CP, FFT each rx antenna, x dft_normalizer, x_t = sum_r W[sc][t][r] X_r[sc] on
// occupied carriers, x normalize_gain[j], callback; main.cc then demaps and counts symbol
// errors (main.cc:1394-1411). SISO (framing.cc:508-533): X[rx]/G[sc][rx][tx] on one stream.
//
// One workgroup per (frame, symbol): the N antenna bodies (M complex each) are read once,
// coalesced, straight into padded LDS; antennas are transformed in LDS-sized groups and the
// NxN apply accumulates in registers (thread owns subcarriers k = tid + q*T for all streams);
// W is stored [t][r][k] so every weight read is coalesced and L2-resident per frame; the
// demap, EVM partials and the equalised symbol + uint8 index stores are fused into the same
// pass. Algorithmic HBM traffic per symbol: N*M*8 read + N*M_occ*9 written.
#include <algorithm>
#include <type_traits>
#include <cstdlib>

#include "fft.hpp"
#include "kernels.hpp"

// per-phase cycle counters (build with -DMIMO_DEC_PROFILE, run with RMIMO_DEC_PROF=1)
#ifdef MIMO_DEC_PROFILE
#define DEC_PROF(...) __VA_ARGS__
#else
#define DEC_PROF(...)
#endif

namespace mimo {

constexpr uint32_t kDecMaxFrames = 256;   // frames per launch for the persistent decode

template <int LOG2M, int NA, int GA, int T>
__global__ __launch_bounds__(T) void decode_kernel(DecodeArgs a) {
  constexpr int M = 1 << LOG2M, PB = lds_padded_len(M), PER = M / T;
  extern __shared__ __attribute__((aligned(16))) float2 lds[];
  __shared__ double red[3][NA][T / 64];
  const uint32_t f = blockIdx.y, s = blockIdx.x;
  const FrameInfo &I = a.info[f];
  const int tid = threadIdx.x;
  const uint32_t n_out = (I.status == 0) ? min(I.n_sym, a.max_out) : 0u;
  double *ep = a.evm_part + (((uint64_t)f * a.max_out + s) * NA) * 3;
  if (s >= n_out) {
    if (tid < NA * 3) ep[tid] = 0.0;
    return;
  }
  const int64_t abs0 = I.base + (int64_t)I.i0 + (int64_t)s * a.SL + a.cp;
  const int64_t L = (int64_t)a.frame_len;

  float2 acc[PER][NA];
#pragma unroll
  for (int q = 0; q < PER; q++)
#pragma unroll
    for (int t = 0; t < NA; t++) acc[q][t] = make_float2(0.0f, 0.0f);

  const bool siso = (a.detector == 3);
  const float2 *__restrict__ Wf = a.W + (uint64_t)f * NA * NA * M;
#pragma unroll
  for (int g0 = 0; g0 < NA; g0 += GA) {
    if (g0 > 0) __syncthreads();
#pragma unroll
    for (int rr = 0; rr < GA; rr++) {
      const float2 *__restrict__ x = a.iq + ((uint64_t)I.cap * NA + g0 + rr) * a.stride;
      const bool inb = (abs0 >= 0) && (abs0 + M <= L);
      if (inb) {
        // 16-byte loads: two complex samples per lane per instruction
        const float4 *x4 = reinterpret_cast<const float4 *>(x + abs0);
        const bool al = ((abs0 & 1) == 0);
        if (al) {
          for (int i = tid; i < M / 2; i += T) {
            const float4 v = x4[i];
            lds[rr * PB + lds_pad(2 * i)] = make_float2(v.x, v.y);
            lds[rr * PB + lds_pad(2 * i + 1)] = make_float2(v.z, v.w);
          }
        } else {
          for (int i = tid; i < M; i += T) lds[rr * PB + lds_pad(i)] = x[abs0 + i];
        }
      } else {
        for (int i = tid; i < M; i += T) {
          const int64_t n = abs0 + i;
          lds[rr * PB + lds_pad(i)] = (n >= 0 && n < L) ? x[n] : make_float2(0.0f, 0.0f);
        }
      }
    }
    __syncthreads();
    fft_lds<LOG2M, T, GA, false>(lds, a.tw);
#pragma unroll
    for (int q = 0; q < PER; q++) {
      const int k = tid + q * T;
#pragma unroll
      for (int rr = 0; rr < GA; rr++) {
        const int r = g0 + rr;
        float2 X = lds[rr * PB + lds_pad(k)];
        X = make_float2(X.x * a.dn, X.y * a.dn);   // volk_32fc_s32fc_multiply_32fc (:561)
        if (siso) {
          if (r == (int)a.siso_rx) {
            const float2 gg = a.G[(((uint64_t)f * M + k) * NA + a.siso_rx) * NA + a.siso_tx];
#pragma unroll
            for (int t = 0; t < NA; t++)
              if (t == (int)a.siso_rx) acc[q][t] = cdiv(X, gg);
          }
        } else {
#pragma unroll
          for (int t = 0; t < NA; t++) {
            const float2 w = Wf[((uint64_t)t * NA + r) * M + k];
            acc[q][t] = (r == 0) ? cmul(w, X) : cadd(acc[q][t], cmul(w, X));
          }
        }
      }
    }
  }

  double e_num[NA], e_den[NA], e_err[NA];
#pragma unroll
  for (int t = 0; t < NA; t++) e_num[t] = e_den[t] = e_err[t] = 0.0;
  const uint64_t frame_id = a.frame_id0 + I.ref;
#pragma unroll
  for (int q = 0; q < PER; q++) {
    const int k = tid + q * T;
    const int j = a.occ_index[k];
    if (j < 0) continue;
    const float gn = siso ? 1.0f : a.gain[(uint64_t)f * M + k];
#pragma unroll
    for (int t = 0; t < NA; t++) {
      const float2 y = siso ? acc[q][t] : make_float2(acc[q][t].x * gn, acc[q][t].y * gn);
      const uint32_t d = qam_demap(y, a.qam);
      uint32_t ref = d;
      if (a.ref_mode == 1)
        ref = a.ref_idx[(uint64_t)I.ref * NA * a.max_out * a.M_occ + t * a.o_ts + s * a.o_ss + j];
      else if (a.ref_mode == 2)
        ref = (uint32_t)(hash5(a.ref_seed, DOM_DATA, frame_id, t,
                               (uint64_t)s * a.M_occ + j) & (uint64_t)(a.qam.L * a.qam.L - 1));
      const float2 sp = qam_point(ref, a.qam);
      const double er = (double)y.x - sp.x, ei = (double)y.y - sp.y;
      e_num[t] += er * er + ei * ei;
      e_den[t] += (double)sp.x * sp.x + (double)sp.y * sp.y;
      e_err[t] += (d != ref) ? 1.0 : 0.0;
      const uint64_t o = (uint64_t)f * NA * a.max_out * a.M_occ + t * a.o_ts + s * a.o_ss + j;
      if (a.out_sym) a.out_sym[o] = y;
      if (a.out_idx) a.out_idx[o] = (uint8_t)d;
    }
  }
#pragma unroll
  for (int t = 0; t < NA; t++) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      e_num[t] += __shfl_xor(e_num[t], off);
      e_den[t] += __shfl_xor(e_den[t], off);
      e_err[t] += __shfl_xor(e_err[t], off);
    }
    if ((tid & 63) == 0) {
      red[0][t][tid >> 6] = e_num[t];
      red[1][t][tid >> 6] = e_den[t];
      red[2][t][tid >> 6] = e_err[t];
    }
  }
  __syncthreads();
  if (tid < NA * 3) {
    const int t = tid / 3, c = tid % 3;
    double v = 0.0;
    for (int w = 0; w < T / 64; w++) v += red[c][t][w];
    ep[t * 3 + c] = v;
  }
}

// Persistent form for configurations whose N antennas fit one LDS batch (C1-C3): a grid of
// ~2 workgroups per CU walks the (frame, symbol) items; the next item's N x M input is
// loaded into registers (16-byte loads) while the current item is transformed, so HBM
// reads overlap the FFT and the NxN apply. Each thread owns 4 consecutive subcarriers per
// group, so weights, gains, equalised symbols and indices move as 16-byte / 4-byte vectors.
template <int LOG2M, int NA, int T, bool SB, bool PF, int REF>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(PF ? 1 : 2 * T / 256)))
void decode_persistent_kernel(DecodeArgs a) {
  constexpr int M = 1 << LOG2M, PB = lds_padded_len(M);
  constexpr int NPAIR = M / 2;                 // complex pairs per antenna body
  constexpr int NIN = NPAIR / T;               // 16-byte loads per thread per antenna
  constexpr int G4 = M / (4 * T);              // 4-subcarrier groups per thread
  static_assert(NIN >= 1 && G4 >= 1, "decode_persistent_kernel needs M >= 4T");
  extern __shared__ __attribute__((aligned(16))) float2 lds[];
  float2 *tw_lds = lds + NA * PB;              // N/2 twiddles after the antenna bodies
  const int tid = threadIdx.x;
  const bool siso = (a.detector == 3);
  fill_twiddles_lds<LOG2M, T>(tw_lds, a.tw);   // visible after the first item's barrier
  // the grid walks decodable symbols only: pfx[f] = symbols of frames < f
  __shared__ uint32_t pfx[kDecMaxFrames + 1];
  if (tid == 0) {
    uint32_t acc = 0;
    for (uint32_t f = 0; f < a.n_frames; f++) {
      pfx[f] = acc;
      const FrameInfo &I = a.info[f];
      acc += (I.status == 0) ? min(I.n_sym, a.max_out) : 0u;
    }
    pfx[a.n_frames] = acc;
  }
  __syncthreads();
  const uint32_t total = pfx[a.n_frames];
  auto locate = [&](uint32_t q, uint32_t &fo, uint32_t &so) {   // q < total
    uint32_t lo = 0, hi = a.n_frames;       // largest f with pfx[f] <= q
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (pfx[mid] <= q) lo = mid; else hi = mid;
    }
    fo = lo;
    so = q - pfx[lo];
  };

  float4 pre[NA][NIN];
  // issue the loads of one item into pre[] (zeros for items without a decodable symbol)
  auto fetch = [&](uint32_t item) {
    bool ok = false;
    int64_t abs0 = 0;
    uint32_t cap = 0;
    if (item < total) {
      uint32_t f, s;
      locate(item, f, s);
      const FrameInfo &I = a.info[f];
      abs0 = I.base + (int64_t)I.i0 + (int64_t)s * a.SL + a.cp;
      ok = abs0 >= 0 && abs0 + M <= (int64_t)a.frame_len;
      cap = I.cap;
    }
#pragma unroll
    for (int r = 0; r < NA; r++) {
      const float2 *__restrict__ x = a.iq + ((uint64_t)cap * NA + r) * a.stride + abs0;
#pragma unroll
      for (int u = 0; u < NIN; u++) {
        const int i2 = tid + u * T;
        if (!ok) {
          pre[r][u] = make_float4(0.f, 0.f, 0.f, 0.f);
        } else if ((abs0 & 1) == 0) {
          pre[r][u] = reinterpret_cast<const float4 *>(x)[i2];
        } else {
          const float2 v0 = x[2 * i2], v1 = x[2 * i2 + 1];
          pre[r][u] = make_float4(v0.x, v0.y, v1.x, v1.y);
        }
      }
    }
  };

  uint32_t item = blockIdx.x;
  if constexpr (PF) fetch(item);
  for (; item < total; item += gridDim.x) {
    // an opaque copy of the thread index: LDS/global address arithmetic is recomputed per
    // item instead of being hoisted out of the loop into (spilled) registers
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    uint32_t f, s;
    locate(item, f, s);
    DEC_PROF(const long long t0 = clock64();)
    if constexpr (!PF) fetch(item);   // two resident workgroups hide each other's loads
    __syncthreads();   // the previous item's LDS reads are done
#pragma unroll
    for (int r = 0; r < NA; r++)
#pragma unroll
      for (int u = 0; u < NIN; u++)   // samples 2i, 2i+1 are adjacent in the padded image
        *reinterpret_cast<float4 *>(lds + r * PB + lds_pad(2 * (tid + u * T))) = pre[r][u];
    if constexpr (PF) fetch(item + gridDim.x);   // next item's input in flight meanwhile
    __syncthreads();
    DEC_PROF(const long long t1 = clock64();)
    fft_lds_twl<LOG2M, T, NA, false>(lds, tw_lds, tid);
    DEC_PROF(const long long t2 = clock64();)

    // per-thread partials over <= 4*G4 subcarriers stay fp32; each wave writes its own
    // partial set (no block barrier), the EVM kernel sums them in fp64
    float e_num[NA], e_den[NA], e_err[NA];
#pragma unroll
    for (int t = 0; t < NA; t++) e_num[t] = e_den[t] = e_err[t] = 0.0f;
    const uint32_t fref = a.info[f].ref;
    const uint64_t frame_id = a.frame_id0 + fref;
    const float2 *__restrict__ Wf = a.W + (uint64_t)f * NA * NA * M;
    const float *__restrict__ gf = a.gain + (uint64_t)f * M;
    const v2f *vl = reinterpret_cast<const v2f *>(lds);
#pragma unroll
    for (int g = 0; g < G4; g++) {
      const int k0 = 4 * (tid + g * T);
      v2f X[NA][4];                      // 2 packed FMAs per complex MAC below
#pragma unroll
      for (int r = 0; r < NA; r++)
#pragma unroll
        for (int e = 0; e < 4; e++)
          X[r][e] = vl[r * PB + lds_pad(k0 + e)] * a.dn;   // (:561) x dft_normalizer
      float gn[4] = {1.0f, 1.0f, 1.0f, 1.0f};
      float4 wnext[NA][2];
      if (!siso) {
        const float4 g4 = *reinterpret_cast<const float4 *>(gf + k0);
        gn[0] = g4.x; gn[1] = g4.y; gn[2] = g4.z; gn[3] = g4.w;
#pragma unroll
        for (int r = 0; r < NA; r++) {   // stream 0's weight row
          const float4 *wp = reinterpret_cast<const float4 *>(Wf + (uint64_t)r * M + k0);
          wnext[r][0] = wp[0];
          wnext[r][1] = wp[1];
        }
      }
#pragma unroll
      for (int t = 0; t < NA; t++) {
        v2f y[4];
        if (siso) {
#pragma unroll
          for (int e = 0; e < 4; e++) {
            y[e] = v2f{0.0f, 0.0f};
            if (t == (int)a.siso_rx) {
              const float2 gg =
                  a.G[(((uint64_t)f * M + k0 + e) * NA + a.siso_rx) * NA + a.siso_tx];
              const float2 q = cdiv(make_float2(X[t][e].x, X[t][e].y), gg);
              y[e] = v2f{q.x, q.y};
            }
          }
        } else {
          // this stream's weight row is in registers; issue the next row's loads now
          float4 wcur[NA][2];
#pragma unroll
          for (int r = 0; r < NA; r++) { wcur[r][0] = wnext[r][0]; wcur[r][1] = wnext[r][1]; }
          if (t + 1 < NA) {
#pragma unroll
            for (int r = 0; r < NA; r++) {
              const float4 *wp =
                  reinterpret_cast<const float4 *>(Wf + ((uint64_t)(t + 1) * NA + r) * M + k0);
              wnext[r][0] = wp[0];
              wnext[r][1] = wp[1];
            }
          }
#pragma unroll
          for (int e = 0; e < 4; e++) y[e] = v2f{0.0f, 0.0f};
#pragma unroll
          for (int r = 0; r < NA; r++) {
            const float4 w01 = wcur[r][0], w23 = wcur[r][1];
            const v2f w[4] = {v2f{w01.x, w01.y}, v2f{w01.z, w01.w}, v2f{w23.x, w23.y},
                              v2f{w23.z, w23.w}};
#pragma unroll
            for (int e = 0; e < 4; e++) {
              y[e] = __builtin_elementwise_fma(w[e].xx, X[r][e], y[e]);
              y[e] = __builtin_elementwise_fma(w[e].yy, v2f{-X[r][e].y, X[r][e].x}, y[e]);
            }
          }
#pragma unroll
          for (int e = 0; e < 4; e++) y[e] = y[e] * gn[e];
        }
        uint32_t packed = 0;
        uint32_t refs = 0;
        if constexpr (REF == 1)
          refs = *reinterpret_cast<const uint32_t *>(
              a.ref_idx + (uint64_t)fref * NA * a.max_out * a.M_occ + t * a.o_ts + s * a.o_ss + k0);
#pragma unroll
        for (int e = 0; e < 4; e++) {
          const int k = k0 + e;
          const float2 ye = make_float2(y[e].x, y[e].y);
          const uint32_t d = qam_demap(ye, a.qam);
          uint32_t refi = d;
          if constexpr (REF == 1)
            refi = (refs >> (8 * e)) & 0xFFu;
          else if constexpr (REF == 2)
            refi = (uint32_t)(hash5(a.ref_seed, DOM_DATA, frame_id, t,
                                    (uint64_t)s * a.M_occ + k) &
                              (uint64_t)(a.qam.L * a.qam.L - 1));
          const float2 sp = qam_point(refi, a.qam);
          const float er = ye.x - sp.x, ei = ye.y - sp.y;
          e_num[t] += er * er + ei * ei;
          e_den[t] += sp.x * sp.x + sp.y * sp.y;
          e_err[t] += (d != refi) ? 1.0f : 0.0f;
          packed |= d << (8 * e);
        }
        const uint64_t o = (uint64_t)f * NA * a.max_out * a.M_occ + t * a.o_ts + s * a.o_ss + k0;
        if (a.out_sym) {
          float4 *op = reinterpret_cast<float4 *>(a.out_sym + o);
          op[0] = make_float4(y[0].x, y[0].y, y[1].x, y[1].y);
          op[1] = make_float4(y[2].x, y[2].y, y[3].x, y[3].y);
        }
        if (a.out_idx) *reinterpret_cast<uint32_t *>(a.out_idx + o) = packed;
        if constexpr (SB) __builtin_amdgcn_sched_barrier(0);   // stream t+1's W loads after t
      }
    }
    DEC_PROF(const long long t3 = clock64();)
    {
      const int lane = tid & 63, wv = tid >> 6;
      double *epw = a.evm_part + ((((uint64_t)f * a.max_out + s) * (T / 64) + wv) * NA) * 3;
#pragma unroll
      for (int t = 0; t < NA; t++) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
          e_num[t] += __shfl_xor(e_num[t], off);
          e_den[t] += __shfl_xor(e_den[t], off);
          e_err[t] += __shfl_xor(e_err[t], off);
        }
      }
      if (lane < NA * 3) {
        const int t = lane / 3, c = lane % 3;
        float v = 0.0f;
#pragma unroll
        for (int u = 0; u < NA; u++)
          if (u == t) v = c == 0 ? e_num[u] : (c == 1 ? e_den[u] : e_err[u]);
        epw[lane] = (double)v;
      }
    }
    DEC_PROF(if (a.prof && tid == 0) {
      const long long t4 = clock64();
      atomicAdd(&a.prof[0], 1ull);
      atomicAdd(&a.prof[1], (unsigned long long)(t1 - t0));
      atomicAdd(&a.prof[2], (unsigned long long)(t2 - t1));
      atomicAdd(&a.prof[3], (unsigned long long)(t3 - t2));
      atomicAdd(&a.prof[4], (unsigned long long)(t4 - t3));
    })
  }
}

// ------------------------------------------------------------------------------------
// Register-resident form (512 <= M <= 4096): one workgroup of T = M/4 threads per (frame,
// symbol). Antennas go through the FFT in pairs; in every pass each thread holds 8 points of
// the pair. Pass 0 is a radix-8 butterfly read straight from HBM (samples j + r*M/8 of one
// antenna: 512 B contiguous per wave instruction); the middle passes exchange through one
// LDS image per antenna of the pair; the last pass is radix-4 with the thread taking
// butterfly tid of BOTH antennas, so it ends holding subcarriers tid + T*q (q < 4) of the
// pair. After all pairs a thread owns 4 subcarriers of every antenna and runs the NxN apply,
// gain, demap and EVM in registers; every load of the item is issued before its first store
// (stores count on the same vmcnt as loads on gfx950, so a load behind stores waits for them).
// 34 KB of LDS and ~100 VGPRs per 512-thread workgroup let several share a CU: one's HBM
// wait overlaps another's FFT and apply.
template <int LOG2M>
struct RegFftPlan {
  static constexpr int M = 1 << LOG2M;
  static constexpr int T = M / 4;
  static constexpr int P8 = (LOG2M - 2) / 3;            // radix-8 passes (pass 0 included)
  static constexpr int TAIL = (LOG2M - 2) % 3;          // then one radix-2/-4 pass if nonzero
  static constexpr int NP = P8 + (TAIL ? 1 : 0) + 1;    // ... and a final radix-4 pass
  static constexpr int radix(int p) { return p < P8 ? 8 : (p == NP - 1 ? 4 : (1 << TAIL)); }
  static constexpr int ns(int p) {                      // sub-transform size before pass p
    int n = 1;
    for (int q = 0; q < p; q++) n *= radix(q);
    return n;
  }
  // butterflies per thread (over the antenna pair) and distinct base twiddles per thread
  static constexpr int bt(int p) { return 8 / radix(p); }
  static constexpr int ntw(int p) { return radix(p) == 2 ? 2 : 1; }
};

// butterfly i of the thread in pass P: antenna (of the pair) and index within the antenna
template <int LOG2M, int P>
MIMO_DEV void reg_bfly(int tid, int i, int &g, int &j) {
  using PL = RegFftPlan<LOG2M>;
  constexpr int NB = PL::M / PL::radix(P);
  const int u = tid + i * PL::T;
  g = u / NB;
  j = u % NB;
}

// outputs of pass P (butterfly i at v[i*R .. i*R+R)) -> the pair's LDS images
template <int LOG2M, int P>
MIMO_DEV void reg_pass_store(v2f *buf, const v2f *v, int tid) {
  using PL = RegFftPlan<LOG2M>;
  constexpr int R = PL::radix(P), NS = PL::ns(P), PB = lds_padded_len(PL::M);
#pragma unroll
  for (int i = 0; i < PL::bt(P); i++) {
    int g, j;
    reg_bfly<LOG2M, P>(tid, i, g, j);
    const int o = (j / NS) * NS * R + (j % NS);
#pragma unroll
    for (int r = 0; r < R; r++) buf[g * PB + lds_pad(o + r * NS)] = v[i * R + r];
  }
}

// inputs of pass P from the LDS images, twiddle, radix-R DFT
template <int LOG2M, int P>
MIMO_DEV void reg_pass_load(const v2f *buf, v2f *v, const v2f *w1, int tid) {
  using PL = RegFftPlan<LOG2M>;
  constexpr int R = PL::radix(P), NB = PL::M / R, PB = lds_padded_len(PL::M);
#pragma unroll
  for (int i = 0; i < PL::bt(P); i++) {
    int g, j;
    reg_bfly<LOG2M, P>(tid, i, g, j);
#pragma unroll
    for (int r = 0; r < R; r++) v[i * R + r] = buf[g * PB + lds_pad(j + r * NB)];
    v2f w[R];
    w[1] = w1[PL::ntw(P) == 2 ? (i & 1) : 0];
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
    for (int r = 1; r < R; r++) v[i * R + r] = vmul(v[i * R + r], w[r]);
    dft_small<R, false>(v + i * R);
  }
}

template <int LOG2M, int P>
MIMO_DEV void reg_passes(v2f *lds, v2f *v, const v2f (*w1)[2], int tid) {
  using PL = RegFftPlan<LOG2M>;
  if constexpr (P < PL::NP) {
    int t = tid;                            // opaque per pass: addresses are not hoisted
    asm volatile("" : "+v"(t));
    __syncthreads();                        // readers of the previous images are done
    reg_pass_store<LOG2M, P - 1>(lds, v, t);
    __syncthreads();
    reg_pass_load<LOG2M, P>(lds, v, w1[P], t);
    reg_passes<LOG2M, P + 1>(lds, v, w1, tid);
  }
}

// hard decision on the square-Gray-QAM level grid: the index (as qam_demap) and the decided
// point (as qam_point of that index) from one set of level computations, with the oracle's
// two roundings in (y * inv_scale + L) * 0.5 (no contraction into an FMA)
MIMO_DEV uint32_t qam_slice(float2 y, const Qam &q, float2 &pt) {
#pragma clang fp contract(off)
  const float L = (float)q.L, Lm1 = (float)(q.L - 1);
  const float tI = (y.x * q.inv_scale + L) * 0.5f;
  const float tQ = (y.y * q.inv_scale + L) * 0.5f;
  const float fI = fminf(fmaxf(floorf(tI), 0.0f), Lm1);   // NaN -> 0 (fmaxf), as qam_level
  const float fQ = fminf(fmaxf(floorf(tQ), 0.0f), Lm1);
  pt = make_float2((2.0f * fI - Lm1) * q.scale, (2.0f * fQ - Lm1) * q.scale);
  return (gray_enc((uint32_t)fI) << q.b) | gray_enc((uint32_t)fQ);
}

template <int LOG2M, int NA, bool SISO, int EX = 0>
__global__ __launch_bounds__(1 << (LOG2M - 2))
__attribute__((amdgpu_waves_per_eu(4)))
void decode_reg_kernel(DecodeArgs a) {
  using PL = RegFftPlan<LOG2M>;
  constexpr int M = PL::M, T = PL::T;
  static_assert(NA % 2 == 0, "antenna pairs");
  extern __shared__ __attribute__((aligned(16))) float2 lds_raw[];
  v2f *lds = reinterpret_cast<v2f *>(lds_raw);
  const int tid = threadIdx.x;
  const uint32_t f = blockIdx.y, s = blockIdx.x;
  const FrameInfo &I = a.info[f];
  const uint32_t n_out = (I.status == 0) ? min(I.n_sym, a.max_out) : 0u;
  if (s >= n_out) return;                  // uniform per workgroup
  const int64_t abs0 = I.base + (int64_t)I.i0 + (int64_t)((EX & 1) ? 0 : s) * a.SL + a.cp;
  const bool inb = abs0 >= 0 && abs0 + M <= (int64_t)a.frame_len;

  // per-thread base twiddles of passes 1..NP-1: e^{-2 pi i k/(NS R)}, k = j mod NS
  v2f w1[PL::NP][2];
#pragma unroll
  for (int p = 1; p < PL::NP; p++) {
    const int R = PL::radix(p), NS = PL::ns(p), NB = M / R;
#pragma unroll
    for (int i = 0; i < PL::ntw(p); i++) {
      const int j = (tid + i * T) % NB;
      w1[p][i] = twiddle<false>(a.tw, (j % NS) * (kTwN / (NS * R)));
    }
  }

  v2f X[NA][4];                            // X[r][q]: subcarrier tid + T*q of antenna r
#pragma unroll
  for (int g0 = 0; g0 < NA; g0 += 2) {
    v2f v[8];
    {                                      // pass 0 straight from HBM
      const int g = tid / (M / 8), j = tid % (M / 8);
      const v2f *x = reinterpret_cast<const v2f *>(a.iq + ((uint64_t)I.cap * NA + g0 + g) * a.stride);
#pragma unroll
      for (int r = 0; r < 8; r++) {
        const int64_t n = abs0 + j + r * (M / 8);
        v[r] = (inb || (n >= 0 && n < (int64_t)a.frame_len)) ? x[n] : v2f{0.0f, 0.0f};
      }
      dft_small<8, false>(v);
    }
    if constexpr (!(EX & 32)) reg_passes<LOG2M, 1>(lds, v, w1, tid);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      X[g0][q] = v[q] * a.dn;              // (:561) x dft_normalizer
      X[g0 + 1][q] = v[4 + q] * a.dn;
    }
  }

  // ---- phase A: every load of the apply and demap, then the arithmetic; no stores yet
  const float2 *__restrict__ Wf = a.W + (uint64_t)f * NA * NA * M;
  const float *__restrict__ gf = a.gain + (uint64_t)f * M;
  int jq[4];
  float gn[4];
  v2f gs[4];                               // SISO: G[k][rx][tx]
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int k = tid + T * q;
    jq[q] = a.all_occ ? k : a.occ_index[k];
    if constexpr (SISO) {
      const float2 gg = a.G[(((uint64_t)f * M + k) * NA + a.siso_rx) * NA + a.siso_tx];
      gs[q] = v2f{gg.x, gg.y};
    } else {
      gn[q] = gf[k];
    }
  }
  const uint64_t frame_id = a.frame_id0 + I.ref;
  float e_num[NA], e_den[NA], e_err[NA];
#pragma unroll
  for (int t = 0; t < NA; t++) e_num[t] = e_den[t] = e_err[t] = 0.0f;
  uint32_t dpk[NA];                        // decided indices, byte q = subcarrier q
#pragma unroll
  for (int t = 0; t < NA; t++) dpk[t] = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int k = tid + T * q;
    // reference indices for the EVM: transmitted (HBM, ref_mode 1), regenerated from the seed
    // (ref_mode 2) or the decisions themselves (ref_mode 0)
    uint32_t refq[NA];
#pragma unroll
    for (int t = 0; t < NA; t++) {
      const uint64_t ob = (uint64_t)I.ref * NA * a.max_out * a.M_occ + t * a.o_ts + s * a.o_ss;
      refq[t] = 0xFFFFFFFFu;
      if (a.ref_mode == 1 && jq[q] >= 0) refq[t] = a.ref_idx[ob + jq[q]];
    }
    v2f y[NA];
    if constexpr (SISO) {
#pragma unroll
      for (int t = 0; t < NA; t++) {
        y[t] = v2f{0.0f, 0.0f};
        if (t == (int)a.siso_rx) {
          const float2 z = cdiv(make_float2(X[t][q].x, X[t][q].y), make_float2(gs[q].x, gs[q].y));
          y[t] = v2f{z.x, z.y};
        }
      }
    } else {
      // this subcarrier's weights, TB streams' rows in flight together
      constexpr int TB = NA <= 4 ? NA : 2;
#pragma unroll
      for (int t0 = 0; t0 < NA; t0 += TB) {
        v2f w[TB][NA];
#pragma unroll
        for (int tb = 0; tb < TB; tb++)
#pragma unroll
          for (int r = 0; r < NA; r++)
            if constexpr (EX & 64) w[tb][r] = v2f{gn[q] * (float)(tb + 1), (float)r * 1e-3f};
            else w[tb][r] = reinterpret_cast<const v2f *>(Wf + ((uint64_t)(t0 + tb) * NA + r) * M)[(EX & 4) ? 0 : (EX & 8) ? (k & 255) : k];
#pragma unroll
        for (int tb = 0; tb < TB; tb++) {
          const int t = t0 + tb;
          y[t] = v2f{0.0f, 0.0f};
#pragma unroll
          for (int r = 0; r < NA; r++) {
            y[t] = __builtin_elementwise_fma(w[tb][r].xx, X[r][q], y[t]);
            y[t] = __builtin_elementwise_fma(w[tb][r].yy, v2f{-X[r][q].y, X[r][q].x}, y[t]);
          }
          y[t] = y[t] * gn[q];
        }
      }
    }
#pragma unroll
    for (int t = 0; t < NA; t++) {
      X[t][q] = y[t];                      // subcarrier q of every antenna is consumed
      if (jq[q] < 0) continue;
      const float2 ye = make_float2(y[t].x, y[t].y);
      float2 sp;
      uint32_t d;
      if constexpr (EX & 16) { sp = ye; d = 0; } else d = qam_slice(ye, a.qam, sp);
      dpk[t] |= d << (8 * q);
      uint32_t refi = refq[t];
      if (a.ref_mode == 0) refi = d;
      else if (a.ref_mode == 2)
        refi = (uint32_t)(hash5(a.ref_seed, DOM_DATA, frame_id, t, (uint64_t)s * a.M_occ + jq[q]) &
                          (uint64_t)(a.qam.L * a.qam.L - 1));
      if (refi != d) {                       // symbol error (rare): the transmitted point
        sp = qam_point(refi, a.qam);
        e_err[t] += 1.0f;
      }
      const float er = ye.x - sp.x, ei = ye.y - sp.y;
      e_num[t] += er * er + ei * ei;
      e_den[t] += sp.x * sp.x + sp.y * sp.y;
    }
  }
  // ---- phase B: stores (equalised symbols, indices, per-wave EVM partials)
#pragma unroll
  for (int t = 0; t < NA; t++) {
    const uint64_t ob = (uint64_t)f * NA * a.max_out * a.M_occ + t * a.o_ts + s * a.o_ss;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      if (jq[q] < 0) continue;
      if ((EX & 2) && X[t][q].x != 12345.0f) continue;
      if (a.out_sym) a.out_sym[ob + jq[q]] = make_float2(X[t][q].x, X[t][q].y);
      if (a.out_idx) a.out_idx[ob + jq[q]] = (uint8_t)(dpk[t] >> (8 * q));
    }
  }
  const int lane = tid & 63, wv = tid >> 6;
  double *epw = a.evm_part + ((((uint64_t)f * a.max_out + s) * (T / 64) + wv) * NA) * 3;
#pragma unroll
  for (int t = 0; t < NA; t++) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      e_num[t] += __shfl_xor(e_num[t], off);
      e_den[t] += __shfl_xor(e_den[t], off);
      e_err[t] += __shfl_xor(e_err[t], off);
    }
  }
  if (lane < NA * 3) {
    const int t = lane / 3, c = lane % 3;
    float v = 0.0f;
#pragma unroll
    for (int u = 0; u < NA; u++)
      if (u == t) v = c == 0 ? e_num[u] : (c == 1 ? e_den[u] : e_err[u]);
    epw[lane] = (double)v;
  }
}

// per-frame EVM / symbol-error totals, bitwise reproducible run to run: workgroup (frame,
// chunk) sums a contiguous range of the frame's (symbol, part) entries in a fixed strided order
// (256/C lanes per component, C = 3N components, coalesced) and an LDS pass in fixed order;
// the workgroup that completes a frame's last chunk sums the kEvmChunks chunk partials in
// chunk order (release/acquire on the per-frame counter, which it resets for the next launch)
__global__ __launch_bounds__(256) void evm_kernel(EvmArgs a) {
  __shared__ double red[256];
  __shared__ int s_last;
  const uint32_t f = blockIdx.x, ch = blockIdx.y, tid = threadIdx.x;
  const FrameInfo &I = a.info[f];
  const uint32_t n_out = (I.status == 0) ? min(I.n_sym, a.max_out) : 0u;
  const uint32_t per = a.N * 3, G = 256 / per;
  const uint64_t recs = (n_out == 0) ? 0u : (a.nrec ? (uint64_t)a.nrec[f] : (uint64_t)n_out);
  const uint64_t n = recs * a.parts;                // (record, part) entries, fixed order
  const uint64_t lo = n * ch / kEvmChunks, hi = n * (ch + 1) / kEvmChunks;
  const uint32_t g = tid / per, c = tid % per;
  const double *src = a.evm_part + (uint64_t)f * a.rec_stride * a.parts * per;
  double v = 0.0;
  if (g < G)
    for (uint64_t e = lo + g; e < hi; e += G) v += src[e * per + c];
  red[tid] = v;
  __syncthreads();
  double *cp = a.chunk_part + ((uint64_t)f * kEvmChunks + ch) * per;
  if (tid < per) {
    double t = 0.0;
    for (uint32_t q = 0; q < G; q++) t += red[q * per + tid];
    __hip_atomic_store(cp + tid, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (tid == 0) {
    const uint32_t done = __hip_atomic_fetch_add(a.counter + f, 1u, __ATOMIC_ACQ_REL,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    s_last = (done == kEvmChunks - 1);
  }
  __syncthreads();
  if (!s_last) return;
  if (tid < per) {
    double t = 0.0;
    for (uint32_t q = 0; q < kEvmChunks; q++)
      t += __hip_atomic_load(a.chunk_part + ((uint64_t)f * kEvmChunks + q) * per + tid,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    a.evm_out[(uint64_t)f * per + tid] = t;
  }
  if (tid == 0) __hip_atomic_store(a.counter + f, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the same totals for the persistent / split decodes, whose records per frame are few (one
// per workgroup segment x waves): one workgroup per frame sums them in a fixed strided order
// and an LDS pass in fixed order, with no chunk partials, counters or second phase
__global__ __launch_bounds__(256) void evm_frame_kernel(EvmArgs a) {
  __shared__ double red[256];
  const uint32_t f = blockIdx.x, tid = threadIdx.x;
  const FrameInfo &I = a.info[f];
  const uint32_t n_out = (I.status == 0) ? min(I.n_sym, a.max_out) : 0u;
  const uint32_t per = a.N * 3, G = 256 / per;
  const uint64_t n = (n_out == 0) ? 0u : (uint64_t)a.nrec[f] * a.parts;
  const uint32_t g = tid / per, c = tid % per;
  const double *src = a.evm_part + (uint64_t)f * a.rec_stride * a.parts * per;
  double v = 0.0;
  if (g < G)
    for (uint64_t e = g; e < n; e += G) v += src[e * per + c];
  red[tid] = v;
  __syncthreads();
  if (tid < per) {
    double t = 0.0;
    for (uint32_t q = 0; q < G; q++) t += red[q * per + tid];
    a.evm_out[(uint64_t)f * per + tid] = t;
  }
}

// ------------------------------------------------------------------------------------
template <int LOG2M, int NA>
static uint32_t decode_launch_na(const DecodeArgs &a, uint32_t nf, hipStream_t s) {
  constexpr int M = 1 << LOG2M;
  constexpr int GA0 = (8192 / M) < 1 ? 1 : (8192 / M);
  constexpr int GA = GA0 < NA ? GA0 : NA;
  constexpr int TW = (M * NA / 32) < 64 ? 64 : ((M * NA / 32) > 1024 ? 1024 : (M * NA / 32));
  constexpr int T0 = TW < 256 ? 256 : TW;
  constexpr int T = T0 > M ? M : T0;
  // persistent kernel: 16 complex per thread per item (4 antennas x 4 subcarriers at C3)
  constexpr int TP0 = (NA * M / 16) < 64 ? 64 : ((NA * M / 16) > 1024 ? 1024 : (NA * M / 16));
  constexpr int TP = TP0 > M / 4 ? M / 4 : TP0;
  if constexpr (LOG2M >= 9 && LOG2M <= 12 && (NA == 2 || NA == 4)) {
    // register-resident form, grid (symbol, frame), T = M/4 threads, two LDS images
    const size_t shm = sizeof(float2) * lds_padded_len(M) * 2;
    auto kern = (a.detector == 3) ? decode_reg_kernel<LOG2M, NA, true>
                                  : decode_reg_kernel<LOG2M, NA, false>;
    (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)shm);
    hipLaunchKernelGGL(kern, dim3(a.max_out, nf), dim3(M / 4), shm, s, a);
    return (M / 4) / 64;
  }
  if constexpr (GA == NA && TP >= 64 && LOG2M < 9) {
    if (a.all_occ && nf <= kDecMaxFrames) {
      const size_t shm = sizeof(float2) * (lds_padded_len(M) * NA + M / 2);
      auto pick = [&](auto ref) {
        constexpr int R = decltype(ref)::value;
        return decode_persistent_kernel<LOG2M, NA, TP, false, true, R>;
      };
      auto kern = a.ref_mode == 1 ? pick(std::integral_constant<int, 1>{})
                : a.ref_mode == 2 ? pick(std::integral_constant<int, 2>{})
                                  : pick(std::integral_constant<int, 0>{});
      (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)shm);
      int per_cu = 1;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, TP, shm) != hipSuccess ||
          per_cu < 1)
        per_cu = 1;
      const uint32_t grid = std::min<uint32_t>(nf * a.max_out, a.n_cu * (uint32_t)per_cu);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(TP), shm, s, a);
      return TP / 64;
    }
  }
  if constexpr (LOG2M < 9 || LOG2M > 12 || !(NA == 2 || NA == 4)) {
    const size_t shm = sizeof(float2) * lds_padded_len(M) * GA;
    (void)hipFuncSetAttribute((const void *)decode_kernel<LOG2M, NA, GA, T>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipLaunchKernelGGL((decode_kernel<LOG2M, NA, GA, T>), dim3(a.max_out, nf), dim3(T), shm, s,
                       a);
    return 1;
  }
  return 0;
}

template <int LOG2M>
static uint32_t decode_dispatch(const DecodeArgs &a, int log2M, uint32_t nf, hipStream_t s) {
  if constexpr (LOG2M <= 12) {
    if (log2M == LOG2M) {
      switch (a.N) {
        case 1: return decode_launch_na<LOG2M, 1>(a, nf, s);
        case 2: return decode_launch_na<LOG2M, 2>(a, nf, s);
        case 4: return decode_launch_na<LOG2M, 4>(a, nf, s);
        case 8: return decode_launch_na<LOG2M, 8>(a, nf, s);
        default: return 0;
      }
    }
    return decode_dispatch<LOG2M + 1>(a, log2M, nf, s);
  }
  return 0;
}

uint32_t launch_decode(const DecodeArgs &a, int log2M, uint32_t n_frames, hipStream_t s,
                       bool *per_frame_records, int *path) {
  *per_frame_records = false;
  *path = 0;
  {
    uint32_t parts = launch_decode_stream(a, log2M, n_frames, s);
    if (parts) *path = 1;
    // the folded CFO (cpe == 2: no derotated scratch capture) is applied by the streaming
    // decode only; any other kernel would decode the raw samples
    if (!parts && a.cpe == 2) return 0;
    if (!parts && (parts = launch_decode_split(a, log2M, n_frames, s))) *path = 2;
    if (parts) {
      *per_frame_records = true;
      return parts;
    }
  }
  // the per-symbol kernels read complex64 only: sc16 wire input never falls through to them
  if (a.sc16) return 0;
  const uint32_t parts = decode_dispatch<6>(a, log2M, n_frames, s);
  if (parts) *path = 3;
  return parts;
}

void launch_evm(const EvmArgs &a, uint32_t n_frames, hipStream_t s) {
  if (a.nrec && a.few)   // a few records per frame (the streaming decode's segments)
    hipLaunchKernelGGL(evm_frame_kernel, dim3(n_frames), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(evm_kernel, dim3(n_frames, kEvmChunks), dim3(256), 0, s, a);
}

}  // namespace mimo

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

#include "fft.hpp"
#include "kernels.hpp"

namespace mimo {

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
      const float2 *__restrict__ x = a.iq + ((uint64_t)f * NA + g0 + rr) * a.stride;
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
  const uint64_t frame_id = a.frame_id0 + f;
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
        ref = a.ref_idx[(((uint64_t)f * NA + t) * a.max_out + s) * a.M_occ + j];
      else if (a.ref_mode == 2)
        ref = (uint32_t)(hash5(a.ref_seed, DOM_DATA, frame_id, t,
                               (uint64_t)s * a.M_occ + j) & (uint64_t)(a.qam.L * a.qam.L - 1));
      const float2 sp = qam_point(ref, a.qam);
      const double er = (double)y.x - sp.x, ei = (double)y.y - sp.y;
      e_num[t] += er * er + ei * ei;
      e_den[t] += (double)sp.x * sp.x + (double)sp.y * sp.y;
      e_err[t] += (d != ref) ? 1.0 : 0.0;
      const uint64_t o = (((uint64_t)f * NA + t) * a.max_out + s) * a.M_occ + j;
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
template <int LOG2M, int NA, int T>
__global__ __launch_bounds__(T) void decode_persistent_kernel(DecodeArgs a) {
  constexpr int M = 1 << LOG2M, PB = lds_padded_len(M);
  constexpr int NPAIR = M / 2;                 // complex pairs per antenna body
  constexpr int NIN = NPAIR / T;               // 16-byte loads per thread per antenna
  constexpr int G4 = M / (4 * T);              // 4-subcarrier groups per thread
  static_assert(NIN >= 1 && G4 >= 1, "decode_persistent_kernel needs M >= 4T");
  extern __shared__ __attribute__((aligned(16))) float2 lds[];
  __shared__ double red[3][NA][T / 64];
  const int tid = threadIdx.x;
  const uint32_t total = a.n_frames * a.max_out;
  const bool siso = (a.detector == 3);

  float4 pre[NA][NIN];
  // issue the loads of one item into pre[] (zeros for items without a decodable symbol)
  auto fetch = [&](uint32_t item) {
    bool ok = false;
    int64_t abs0 = 0;
    uint32_t f = 0;
    if (item < total) {
      f = item / a.max_out;
      const uint32_t s = item % a.max_out;
      const FrameInfo &I = a.info[f];
      const uint32_t n_out = (I.status == 0) ? min(I.n_sym, a.max_out) : 0u;
      if (s < n_out) {
        abs0 = I.base + (int64_t)I.i0 + (int64_t)s * a.SL + a.cp;
        ok = abs0 >= 0 && abs0 + M <= (int64_t)a.frame_len;
      }
    }
#pragma unroll
    for (int r = 0; r < NA; r++) {
      const float2 *__restrict__ x = a.iq + ((uint64_t)f * NA + r) * a.stride + abs0;
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
  fetch(item);
  for (; item < total; item += gridDim.x) {
    const uint32_t f = item / a.max_out, s = item % a.max_out;
    const FrameInfo &I = a.info[f];
    const uint32_t n_out = (I.status == 0) ? min(I.n_sym, a.max_out) : 0u;
    double *ep = a.evm_part + (((uint64_t)f * a.max_out + s) * NA) * 3;
    __syncthreads();   // the previous item's LDS reads are done
#pragma unroll
    for (int r = 0; r < NA; r++)
#pragma unroll
      for (int u = 0; u < NIN; u++) {
        const int i = 2 * (tid + u * T);
        lds[r * PB + lds_pad(i)] = make_float2(pre[r][u].x, pre[r][u].y);
        lds[r * PB + lds_pad(i + 1)] = make_float2(pre[r][u].z, pre[r][u].w);
      }
    fetch(item + gridDim.x);   // next item's input in flight during this item's compute
    if (s >= n_out) {          // block-uniform
      if (tid < NA * 3) ep[tid] = 0.0;
      continue;
    }
    __syncthreads();
    fft_lds<LOG2M, T, NA, false>(lds, a.tw);

    // per-thread partials over <= 4*G4 subcarriers stay fp32; waves and items sum in fp64
    float e_num[NA], e_den[NA], e_err[NA];
#pragma unroll
    for (int t = 0; t < NA; t++) e_num[t] = e_den[t] = e_err[t] = 0.0f;
    const uint64_t frame_id = a.frame_id0 + f;
    const float2 *__restrict__ Wf = a.W + (uint64_t)f * NA * NA * M;
    const float *__restrict__ gf = a.gain + (uint64_t)f * M;
#pragma unroll
    for (int g = 0; g < G4; g++) {
      const int k0 = 4 * (tid + g * T);
      float2 X[NA][4];
#pragma unroll
      for (int r = 0; r < NA; r++)
#pragma unroll
        for (int e = 0; e < 4; e++) {
          const float2 v = lds[r * PB + lds_pad(k0 + e)];
          X[r][e] = make_float2(v.x * a.dn, v.y * a.dn);   // (:561) x dft_normalizer
        }
      float gn[4] = {1.0f, 1.0f, 1.0f, 1.0f};
      if (!siso) {
        const float4 g4 = *reinterpret_cast<const float4 *>(gf + k0);
        gn[0] = g4.x; gn[1] = g4.y; gn[2] = g4.z; gn[3] = g4.w;
      }
#pragma unroll
      for (int t = 0; t < NA; t++) {
        float2 y[4];
        if (siso) {
#pragma unroll
          for (int e = 0; e < 4; e++) {
            y[e] = make_float2(0.0f, 0.0f);
            if (t == (int)a.siso_rx) {
              const float2 gg =
                  a.G[(((uint64_t)f * M + k0 + e) * NA + a.siso_rx) * NA + a.siso_tx];
              y[e] = cdiv(X[t][e], gg);
            }
          }
        } else {
#pragma unroll
          for (int r = 0; r < NA; r++) {
            const float4 *wp = reinterpret_cast<const float4 *>(Wf + ((uint64_t)t * NA + r) * M + k0);
            const float4 w01 = wp[0], w23 = wp[1];
            const float2 w[4] = {make_float2(w01.x, w01.y), make_float2(w01.z, w01.w),
                                 make_float2(w23.x, w23.y), make_float2(w23.z, w23.w)};
#pragma unroll
            for (int e = 0; e < 4; e++)
              y[e] = (r == 0) ? cmul(w[e], X[r][e]) : cadd(y[e], cmul(w[e], X[r][e]));
          }
#pragma unroll
          for (int e = 0; e < 4; e++) y[e] = make_float2(y[e].x * gn[e], y[e].y * gn[e]);
        }
        uint32_t packed = 0;
#pragma unroll
        for (int e = 0; e < 4; e++) {
          const int k = k0 + e;
          const uint32_t d = qam_demap(y[e], a.qam);
          uint32_t refi = d;
          if (a.ref_mode == 1)
            refi = a.ref_idx[(((uint64_t)f * NA + t) * a.max_out + s) * a.M_occ + k];
          else if (a.ref_mode == 2)
            refi = (uint32_t)(hash5(a.ref_seed, DOM_DATA, frame_id, t,
                                    (uint64_t)s * a.M_occ + k) &
                              (uint64_t)(a.qam.L * a.qam.L - 1));
          const float2 sp = qam_point(refi, a.qam);
          const float er = y[e].x - sp.x, ei = y[e].y - sp.y;
          e_num[t] += er * er + ei * ei;
          e_den[t] += sp.x * sp.x + sp.y * sp.y;
          e_err[t] += (d != refi) ? 1.0f : 0.0f;
          packed |= d << (8 * e);
        }
        const uint64_t o = (((uint64_t)f * NA + t) * a.max_out + s) * a.M_occ + k0;
        if (a.out_sym) {
          float4 *op = reinterpret_cast<float4 *>(a.out_sym + o);
          op[0] = make_float4(y[0].x, y[0].y, y[1].x, y[1].y);
          op[1] = make_float4(y[2].x, y[2].y, y[3].x, y[3].y);
        }
        if (a.out_idx) *reinterpret_cast<uint32_t *>(a.out_idx + o) = packed;
        __builtin_amdgcn_sched_barrier(0);   // keep stream t+1's W loads after stream t
      }
    }
#pragma unroll
    for (int t = 0; t < NA; t++) {
      double vn = e_num[t], vd = e_den[t], ve = e_err[t];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        vn += __shfl_xor(vn, off);
        vd += __shfl_xor(vd, off);
        ve += __shfl_xor(ve, off);
      }
      if ((tid & 63) == 0) {
        red[0][t][tid >> 6] = vn;
        red[1][t][tid >> 6] = vd;
        red[2][t][tid >> 6] = ve;
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
}

// per-frame EVM / symbol-error totals: fixed-order strided partial sums + LDS tree, so the
// result is bitwise reproducible run to run
__global__ __launch_bounds__(256) void evm_kernel(EvmArgs a) {
  __shared__ double red[256];
  const uint32_t f = blockIdx.x, tid = threadIdx.x;
  const FrameInfo &I = a.info[f];
  const uint32_t n_out = (I.status == 0) ? min(I.n_sym, a.max_out) : 0u;
  const uint32_t per = a.N * 3;
  for (uint32_t c = 0; c < per; c++) {
    double v = 0.0;
    for (uint32_t s = tid; s < n_out; s += 256)
      v += a.evm_part[((uint64_t)f * a.max_out + s) * per + c];
    red[tid] = v;
    __syncthreads();
    for (uint32_t w = 128; w > 0; w >>= 1) {
      if (tid < w) red[tid] += red[tid + w];
      __syncthreads();
    }
    if (tid == 0) a.evm_out[(uint64_t)f * per + c] = red[0];
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------
template <int LOG2M, int NA>
static void decode_launch_na(const DecodeArgs &a, uint32_t nf, hipStream_t s) {
  constexpr int M = 1 << LOG2M;
  constexpr int GA0 = (8192 / M) < 1 ? 1 : (8192 / M);
  constexpr int GA = GA0 < NA ? GA0 : NA;
  constexpr int TW = (M * NA / 32) < 64 ? 64 : ((M * NA / 32) > 1024 ? 1024 : (M * NA / 32));
  constexpr int T0 = TW < 256 ? 256 : TW;
  constexpr int T = T0 > M ? M : T0;
  // persistent kernel: 16 complex per thread per item (4 antennas x 4 subcarriers at C3)
  constexpr int TP0 = (NA * M / 16) < 64 ? 64 : ((NA * M / 16) > 1024 ? 1024 : (NA * M / 16));
  constexpr int TP = TP0 > M / 4 ? M / 4 : TP0;
  if constexpr (GA == NA && TP >= 64) {
    if (a.all_occ) {
      const size_t shm = sizeof(float2) * lds_padded_len(M) * NA;
      (void)hipFuncSetAttribute((const void *)decode_persistent_kernel<LOG2M, NA, TP>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
      const uint32_t per_cu = (uint32_t)std::max<size_t>(1, (160u * 1024u) / (shm + 2048));
      const uint32_t total = nf * a.max_out;
      const uint32_t grid = std::min<uint32_t>(total, a.n_cu * std::min<uint32_t>(per_cu, 4));
      hipLaunchKernelGGL((decode_persistent_kernel<LOG2M, NA, TP>), dim3(grid), dim3(TP), shm,
                         s, a);
      return;
    }
  }
  const size_t shm = sizeof(float2) * lds_padded_len(M) * GA;
  (void)hipFuncSetAttribute((const void *)decode_kernel<LOG2M, NA, GA, T>,
                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  hipLaunchKernelGGL((decode_kernel<LOG2M, NA, GA, T>), dim3(a.max_out, nf), dim3(T), shm, s, a);
}

template <int LOG2M>
static void decode_dispatch(const DecodeArgs &a, int log2M, uint32_t nf, hipStream_t s) {
  if constexpr (LOG2M <= 12) {
    if (log2M == LOG2M) {
      switch (a.N) {
        case 1: decode_launch_na<LOG2M, 1>(a, nf, s); break;
        case 2: decode_launch_na<LOG2M, 2>(a, nf, s); break;
        case 4: decode_launch_na<LOG2M, 4>(a, nf, s); break;
        case 8: decode_launch_na<LOG2M, 8>(a, nf, s); break;
        default: break;
      }
      return;
    }
    decode_dispatch<LOG2M + 1>(a, log2M, nf, s);
  }
}

void launch_decode(const DecodeArgs &a, int log2M, uint32_t n_frames, hipStream_t s) {
  decode_dispatch<6>(a, log2M, n_frames, s);
}

void launch_evm(const EvmArgs &a, uint32_t n_frames, hipStream_t s) {
  hipLaunchKernelGGL(evm_kernel, dim3(n_frames), dim3(256), 0, s, a);
}

}  // namespace mimo

// rub_mimo_amd/csrc/synth_kernels.hip -- transmitter and channel emulator on gfx950.
//
// tx_symbols_kernel: framegen::assemble_mimo_packet (framing.cc:210-235) for many symbols at
//   once: occupied-carrier mapping, unnormalised IFFT, x dft_normalizer (1/sqrt(M_occ)),
//   cyclic prefix, x baseband gain (main.cc:1048-1053). Symbols come from the caller or
//   from the counter-based hash (uniform QAM indices, the bench's synthetic data).
// mix_kernel: the tx_worker frame layout (main.cc:937-1153) -- zeros, sync words
//   (framing.cc:169-208), data, zeros -- through a flat Rayleigh channel plus AWGN.
#include "fft.hpp"
#include "kernels.hpp"

#pragma clang fp contract(off)

namespace mimo {

template <int LOG2M, int T>
__global__ __launch_bounds__(T) void tx_symbols_kernel(TxSymArgs a) {
  constexpr int M = 1 << LOG2M;
  extern __shared__ __attribute__((aligned(16))) float2 lds[];
  const uint32_t sym = blockIdx.x, t = blockIdx.y, f = blockIdx.z;
  const int tid = threadIdx.x;
  for (int i = tid; i < M; i += T) lds[lds_pad(i)] = make_float2(0.0f, 0.0f);
  __syncthreads();
  const uint64_t frame_id = a.frame_id0 + f;
  const uint64_t sbase = (((uint64_t)f * a.N + t) * a.n_sym + sym) * a.M_occ;
  for (uint32_t j = tid; j < a.M_occ; j += T) {
    float2 v;
    if (a.in) {
      v = a.in[((uint64_t)t * a.n_sym + sym) * a.M_occ + j];
    } else {
      const uint32_t idx = (uint32_t)(hash5(a.seed, DOM_DATA, frame_id, t,
                                            (uint64_t)sym * a.M_occ + j) &
                                      (uint64_t)(a.qam.L * a.qam.L - 1));
      if (a.tx_idx) a.tx_idx[sbase + j] = (uint8_t)idx;
      v = qam_point(idx, a.qam);
    }
    lds[lds_pad(a.occ_list[j])] = v;
  }
  __syncthreads();
  fft_lds<LOG2M, T, 1, true>(lds, a.tw);
  const uint32_t SL = M + a.cp;
  float2 *o = a.out + (((uint64_t)f * a.N + t) * a.n_sym + sym) * SL;
  for (uint32_t i = tid; i < SL; i += T) {
    const uint32_t bi = (i < a.cp) ? (M - a.cp + i) : (i - a.cp);
    float2 v = lds[lds_pad(bi)];
    v = make_float2(v.x * a.dn, v.y * a.dn);
    v = make_float2(v.x * a.gain, v.y * a.gain);
    o[i] = v;
  }
}

__global__ __launch_bounds__(256) void mix_kernel(MixArgs a) {
  const uint32_t f = blockIdx.z, r = blockIdx.y;
  const uint64_t frame_id = a.frame_id0 + f;
  const uint32_t N = a.N, SL = a.SL, M = a.M, cp = a.cp;
  const uint64_t u = (a.offset >= 0) ? (uint64_t)a.offset
                                     : hash5(a.seed, DOM_OFFSET, frame_id, 0, 0) % SL;
  const uint64_t lead = (uint64_t)SL * (N * a.nac + 1) + u;
  const uint64_t nsync = (uint64_t)(N * a.nac + 1) * SL;
  const uint64_t dend = lead + nsync + (uint64_t)a.pid * SL;
  float2 H[kMaxStreams];
  for (uint32_t t = 0; t < N; t++) {
    if (a.identity) H[t] = make_float2(r == t ? 1.0f : 0.0f, 0.0f);
    else H[t] = hash_cnormal(hash5(a.seed, DOM_CHAN, frame_id, r * N + t, 0));
    if (a.H_out && blockIdx.x == 0 && threadIdx.x == 0)
      a.H_out[((uint64_t)f * N + r) * N + t] = H[t];
  }
  float2 *out = a.out + ((uint64_t)f * N + r) * a.stride;
  for (uint64_t n = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; n < a.frame_len;
       n += (uint64_t)gridDim.x * blockDim.x) {
    float2 acc = make_float2(0.0f, 0.0f);
    if (n >= lead && n < dend) {
      const uint64_t m = n - lead;
      if (m < nsync) {
        const uint32_t q = (uint32_t)(m / SL), i = (uint32_t)(m % SL);
        const uint32_t bi = (i < cp) ? (M - cp + i) : (i - cp);
        const uint32_t t_on = (q == 0) ? 0u : ((q - 1) % N);
        float2 v = a.code_time[(uint64_t)q * M + bi];
        v = make_float2(v.x * 0.25f, v.y * 0.25f);
        for (uint32_t t = 0; t < N; t++) {
          const float2 x = (t == t_on) ? v : make_float2(0.0f, 0.0f);
          acc = cadd(acc, cmul(H[t], x));
        }
      } else {
        const uint64_t md = m - nsync;
        const uint64_t sym = md / SL, i = md % SL;
        for (uint32_t t = 0; t < N; t++) {
          const float2 x = a.tx_data[(((uint64_t)f * N + t) * a.pid + sym) * SL + i];
          acc = cadd(acc, cmul(H[t], x));
        }
      }
    } else {
      for (uint32_t t = 0; t < N; t++) acc = cadd(acc, cmul(H[t], make_float2(0.0f, 0.0f)));
    }
    const float2 g = hash_cnormal(hash5(a.seed, DOM_NOISE, frame_id, r, n));
    acc.x = acc.x + g.x * a.nstd;
    acc.y = acc.y + g.y * a.nstd;
    out[n] = acc;
  }
}

template <int LOG2M>
static void tx_dispatch(const TxSymArgs &a, int log2M, uint32_t nf, hipStream_t s) {
  if constexpr (LOG2M <= 12) {
    if (log2M == LOG2M) {
      constexpr int M = 1 << LOG2M;
      constexpr int T = M < 256 ? M : 256;
      const size_t shm = sizeof(float2) * lds_padded_len(M);
      (void)hipFuncSetAttribute((const void *)tx_symbols_kernel<LOG2M, T>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
      hipLaunchKernelGGL((tx_symbols_kernel<LOG2M, T>), dim3(a.n_sym, a.N, nf), dim3(T), shm,
                         s, a);
      return;
    }
    tx_dispatch<LOG2M + 1>(a, log2M, nf, s);
  }
}

void launch_tx_symbols(const TxSymArgs &a, int log2M, uint32_t n_frames, hipStream_t s) {
  tx_dispatch<6>(a, log2M, n_frames, s);
}

void launch_mix(const MixArgs &a, uint32_t n_frames, hipStream_t s) {
  uint64_t blocks = (a.frame_len + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(mix_kernel, dim3((uint32_t)blocks, a.N, n_frames), dim3(256), 0, s, a);
}

}  // namespace mimo

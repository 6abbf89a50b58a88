// rub_mimo_amd/csrc/fft_reg.hpp -- register-resident Stockham FFT for one workgroup (gfx950).
//
// One N-point transform, T threads, PTS = N/T points per thread held in registers. Every pass
// has the main radix (16 with 16 points per thread, else 8) except one smaller pass (log2 N
// not a multiple of log2 of it), placed before the last so that the first and the last pass
// have the main radix R and the twiddles of the forward and the inverse plan are the same
// per-thread values (conjugated). In a pass of radix r the thread runs PTS/r butterflies
// j = tid + i*T; butterfly j reads elements j + q*N/r and writes Stockham order. Between
// passes the thread's values go through one padded LDS image (two barriers). The first pass
// may read straight from global memory and the last pass leaves elements j + q*N/R in the
// thread, which is exactly what the first pass of the next transform (of the same plan)
// reads: a forward transform, a pointwise product and an inverse transform chain in registers
// with no exchange between them (search kernels).
#pragma once

#include "fft.hpp"

namespace mimo {

// Main radix: 16 with 16 points per thread (one butterfly per pass, one LDS exchange fewer
// per transform than radix 8 at N = 2^10 .. 2^14), else 8. REG_RADIX8 builds the radix-8 plan
// everywhere (A/B timing).
#ifdef REG_RADIX8
constexpr bool kRegR16 = false;
#else
constexpr bool kRegR16 = true;
#endif

template <int LOG2N, int PTS>
struct RegPlan {
  static constexpr int N = 1 << LOG2N;
  static constexpr int T = N / PTS;
  static constexpr int LR = (kRegR16 && PTS >= 16 && LOG2N >= 9) ? 4 : 3;   // log2 main radix
  static constexpr int RM = 1 << LR;
  static constexpr int P8 = LOG2N / LR;                 // main-radix passes
  static constexpr int TAIL = LOG2N % LR;
  static constexpr int NP = P8 + (TAIL ? 1 : 0);
  // the smaller pass sits before the last one: the first and the last pass have the main radix
  static constexpr int TPOS = P8 < 2 ? P8 : (P8 - 1 < 2 ? P8 - 1 : 2);
  static constexpr int radix(int p) { return (TAIL && p == TPOS) ? (1 << TAIL) : RM; }
  static constexpr int ns(int p) {
    int n = 1;
    for (int q = 0; q < p; q++) n *= radix(q);
    return n;
  }
  static constexpr int bt(int p) { return PTS / radix(p); }   // butterflies per thread
  // distinct base twiddles per thread in pass p: k = (tid + i*T) mod ns(p)
  static constexpr int ntw(int p) {
    if (p == 0) return 0;
    const int n = ns(p);
    return (T % n == 0) ? 1 : bt(p);
  }
  static constexpr int tw_off(int p) {
    int o = 0;
    for (int q = 0; q < p; q++) o += ntw(q);
    return o;
  }
  static constexpr int NTW = tw_off(NP);
};

// this thread's base twiddles e^{-2 pi i k / (NS R)} of every pass, from the kTwN table
template <int LOG2N, int PTS>
MIMO_DEV void reg_twiddles(v2f *w1, const float2 *__restrict__ tw, int tid) {
  using PL = RegPlan<LOG2N, PTS>;
#pragma unroll
  for (int p = 1; p < PL::NP; p++) {
    const int R = PL::radix(p), NS = PL::ns(p);
#pragma unroll
    for (int i = 0; i < PL::ntw(p); i++) {
      const int j = tid + i * PL::T;
      w1[PL::tw_off(p) + i] = twiddle<false>(tw, (j % NS) * (kTwN / (NS * R)));
    }
  }
}

// padded addresses as one base plus compile-time offsets: lds_pad(o + r NS) = lds_pad(o) +
// r NS + floor(r NS / 32) (NS R a power of two: the NS R-aligned group holding o .. o+(R-1)NS
// never straddles a multiple of 32 when NS < 32), lds_pad(j + r NB) = lds_pad(j) + r NB + r NB/32
template <int LOG2N, int PTS, int P>
MIMO_DEV void reg_store(v2f *buf, const v2f *v, int tid) {
  using PL = RegPlan<LOG2N, PTS>;
  constexpr int R = PL::radix(P), NS = PL::ns(P);
#pragma unroll
  for (int i = 0; i < PL::bt(P); i++) {
    const uint32_t j = (uint32_t)tid + i * PL::T;
    const uint32_t o = (j / NS) * NS * R + (j % NS);
    v2f *bp = buf + lds_pad((int)o);
#pragma unroll
    for (int r = 0; r < R; r++) bp[r * NS + (r * NS) / 32] = v[i * R + r];
  }
}

// twiddle and radix-R DFT of the values already in v (pass P)
template <int LOG2N, int PTS, int P, bool INV>
MIMO_DEV void reg_compute(v2f *v, const v2f *w1) {
  using PL = RegPlan<LOG2N, PTS>;
  constexpr int R = PL::radix(P);
#pragma unroll
  for (int i = 0; i < PL::bt(P); i++) {
    if constexpr (P > 0) {
      v2f w[R];
      const v2f b = w1[PL::tw_off(P) + (PL::ntw(P) == 1 ? 0 : i)];
      w[1] = INV ? v2f{b.x, -b.y} : b;
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
#pragma unroll
      for (int r = 1; r < R; r++) v[i * R + r] = vmul(v[i * R + r], w[r]);
    }
    dft_small<R, INV>(v + i * R);
  }
}

template <int LOG2N, int PTS, int P>
MIMO_DEV void reg_load(const v2f *buf, v2f *v, int tid) {
  using PL = RegPlan<LOG2N, PTS>;
  constexpr int R = PL::radix(P), NB = PL::N / R;
  static_assert(NB % 32 == 0, "padded-offset identity");
#pragma unroll
  for (int i = 0; i < PL::bt(P); i++) {
    const uint32_t j = (uint32_t)tid + i * PL::T;
    const v2f *bp = buf + lds_pad((int)j);
#pragma unroll
    for (int r = 0; r < R; r++) v[i * R + r] = bp[r * NB + (r * NB) / 32];
  }
}

// passes P .. NP-1 of a transform whose pass P-1 outputs are in v
template <int LOG2N, int PTS, int P, bool INV>
MIMO_DEV void reg_rest(v2f *buf, v2f *v, const v2f *w1, int tid) {
  using PL = RegPlan<LOG2N, PTS>;
  if constexpr (P < PL::NP) {
    // an opaque copy of the thread index per pass: the LDS addresses are recomputed here
    // instead of being hoisted to the kernel start and held (spilled) across passes
    int t = tid;
    asm volatile("" : "+v"(t));
    __syncthreads();
    reg_store<LOG2N, PTS, P - 1>(buf, v, t);
    __syncthreads();
    reg_load<LOG2N, PTS, P>(buf, v, t);
    reg_compute<LOG2N, PTS, P, INV>(v, w1);
    reg_rest<LOG2N, PTS, P + 1, INV>(buf, v, w1, tid);
  }
}

// Exchange layouts of an 8-point-per-thread plan (PTS = 8, radix 8 first), one per exchange
// (each is a store then a load, so each may place elements as it likes): with lds_pad the
// radix-8 stores of the first two exchanges (elements 8 j + r, and 64 (j/8) + j%8 + 8 r) are
// 2-way bank-conflicted on gfx950 (8-byte stores: 16-lane groups over 32 banks) -- 31% of
// the LDS cycles of the search's 2048-point LS transform (tools/lds/). Both become
// conflict-free:
//   1 (after pass 0): i = 32 a + b at 33 a + (b ^ 4 ((b >> 4) & 1)) -- the store from two bases
//     per thread (the XOR swaps r < 4 and r >= 4 where j & 2), the load j + r NB from one;
//   2 (after pass 1, radix 8 over NS = 8): i + 2 (i >> 5) + 4 (i >> 6) -- x2(o + 8 r) =
//     x2(o) + 8 r + 2 (r >> 2), x2(j + r NB) = x2(j) + 9 r NB / 8 (NB a multiple of 64);
//     footprint N + N/8 (the image stride reg_image_len);
//   0: lds_pad (later exchanges).
template <int LOG2N, int PTS>
constexpr int reg_ex_layout(int e) {
  using PL = RegPlan<LOG2N, PTS>;
  if (PTS != 8 || PL::RM != 8 || PL::radix(0) != 8) return 0;
  if (e == 0) return (PL::N / PL::radix(1)) % 32 == 0 ? 1 : 0;
  if (e == 1 && PL::NP > 2 && PL::radix(1) == 8 && PL::ns(1) == 8 &&
      (PL::N / PL::radix(2)) % 64 == 0)
    return 2;
  return 0;
}
template <int LOG2N, int PTS>
constexpr int reg_image_len() {   // entries per transform image of the layouts above
  return (reg_ex_layout<LOG2N, PTS>(1) == 2) ? (1 << LOG2N) + (1 << LOG2N) / 8
                                              : (1 << LOG2N) + (1 << LOG2N) / 32;
}
MIMO_DEV constexpr int reg_x2(int i) { return i + 2 * (i >> 5) + 4 * (i >> 6); }

template <int LOG2N, int PTS, int P, int LAY>
MIMO_DEV void reg_store_lay(v2f *buf, const v2f *v, int tid) {
  using PL = RegPlan<LOG2N, PTS>;
  constexpr int R = PL::radix(P);
  if constexpr (LAY == 1) {
    static_assert(P == 0 && R == 8 && PL::bt(P) == 1, "x1: pass 0, one radix-8 butterfly");
    const int j = tid;
    const int m = ((j >> 1) & 1) << 2;
    const int B = 33 * (j >> 2) + 8 * (j & 3);
    v2f *lo = buf + B + m, *hi = buf + B - m;
#pragma unroll
    for (int r = 0; r < 4; r++) lo[r] = v[r];
#pragma unroll
    for (int r = 4; r < 8; r++) hi[r] = v[r];
  } else if constexpr (LAY == 2) {
    static_assert(P == 1 && R == 8 && PL::ns(P) == 8 && PL::bt(P) == 1, "x2: pass 1, radix 8");
    const int j = tid;
    v2f *bp = buf + 64 * (j >> 3) + (j & 7) + 8 * (j >> 3);
#pragma unroll
    for (int r = 0; r < 8; r++) bp[8 * r + 2 * (r >> 2)] = v[r];
  } else {
    reg_store<LOG2N, PTS, P>(buf, v, tid);
  }
}

template <int LOG2N, int PTS, int P, int LAY>
MIMO_DEV void reg_load_lay(const v2f *buf, v2f *v, int tid) {
  using PL = RegPlan<LOG2N, PTS>;
  constexpr int R = PL::radix(P), NB = PL::N / R;
  if constexpr (LAY == 1) {
    static_assert(NB % 32 == 0, "x1 loads");
#pragma unroll
    for (int i = 0; i < PL::bt(P); i++) {
      const int j = tid + i * PL::T;
      const v2f *bp = buf + 33 * (j >> 5) + ((j & 31) ^ (((j >> 4) & 1) << 2));
#pragma unroll
      for (int r = 0; r < R; r++) v[i * R + r] = bp[33 * r * (NB / 32)];
    }
  } else if constexpr (LAY == 2) {
    static_assert(NB % 64 == 0, "x2 loads");
#pragma unroll
    for (int i = 0; i < PL::bt(P); i++) {
      const int j = tid + i * PL::T;
      const v2f *bp = buf + reg_x2(j);
#pragma unroll
      for (int r = 0; r < R; r++) v[i * R + r] = bp[9 * r * (NB / 8)];
    }
  } else {
    reg_load<LOG2N, PTS, P>(buf, v, tid);
  }
}

// a workgroup barrier that orders LDS only: waits for this wave's LDS accesses, not for its
// global loads in flight (__syncthreads' release fence would drain those: a prefetch of the
// next item's data would complete at the first exchange)
MIMO_DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// reg_rest with the exchange layouts above (images of reg_image_len entries); KEEPVM: the
// barriers leave global loads in flight (lds_barrier)
template <int LOG2N, int PTS, int P, bool INV, bool KEEPVM = false>
MIMO_DEV void reg_rest_lay(v2f *buf, v2f *v, const v2f *w1, int tid) {
  using PL = RegPlan<LOG2N, PTS>;
  if constexpr (P < PL::NP) {
    int t = tid;
    asm volatile("" : "+v"(t));
    constexpr int LAY = reg_ex_layout<LOG2N, PTS>(P - 1);
    if constexpr (KEEPVM) lds_barrier(); else __syncthreads();
    reg_store_lay<LOG2N, PTS, P - 1, LAY>(buf, v, t);
    if constexpr (KEEPVM) lds_barrier(); else __syncthreads();
    reg_load_lay<LOG2N, PTS, P, LAY>(buf, v, t);
    reg_compute<LOG2N, PTS, P, INV>(v, w1);
    reg_rest_lay<LOG2N, PTS, P + 1, INV, KEEPVM>(buf, v, w1, tid);
  }
}

// reg_rest_lay through two images used in turn (exchange i stores into and loads from
// img[i % 2]): one barrier per exchange instead of two -- the barrier after exchange i's store
// also orders every wave's loads of exchange i - 1 (from the other image) before exchange
// i + 1 stores there. Barriers order LDS only (lds_barrier). A caller chaining transforms
// starts the next one on the image the last exchange did not use (NP - 1 exchanges: swap the
// pair when that is odd).
template <int LOG2N, int PTS, int P, bool INV>
MIMO_DEV void reg_rest_pp(v2f *img0, v2f *img1, v2f *v, const v2f *w1, int tid) {
  using PL = RegPlan<LOG2N, PTS>;
  if constexpr (P < PL::NP) {
    int t = tid;
    asm volatile("" : "+v"(t));
    constexpr int LAY = reg_ex_layout<LOG2N, PTS>(P - 1);
    v2f *buf = ((P - 1) & 1) ? img1 : img0;
    reg_store_lay<LOG2N, PTS, P - 1, LAY>(buf, v, t);
    lds_barrier();
    reg_load_lay<LOG2N, PTS, P, LAY>(buf, v, t);
    reg_compute<LOG2N, PTS, P, INV>(v, w1);
    reg_rest_pp<LOG2N, PTS, P + 1, INV>(img0, img1, v, w1, tid);
  }
}

// LDS writes of this wave visible to its own reads; no code motion across
MIMO_DEV void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// passes P .. NP-1 of a transform held by ONE wave (T = 64 lanes) through that wave's own LDS
// region: no workgroup barrier, only the wave's own store -> load ordering. (A pass's loads are
// consumed by its butterflies before the next store is issued, so the region needs no sync
// ahead of a store.)
template <int LOG2N, int PTS, int P, bool INV>
MIMO_DEV void reg_rest_wave(v2f *buf, v2f *v, const v2f *w1, int lane) {
  using PL = RegPlan<LOG2N, PTS>;
  static_assert(PL::T == 64, "one wave per transform");
  if constexpr (P < PL::NP) {
    int t = lane;
    asm volatile("" : "+v"(t));
    reg_store<LOG2N, PTS, P - 1>(buf, v, t);
    wave_lds_sync();
    reg_load<LOG2N, PTS, P>(buf, v, t);
    reg_compute<LOG2N, PTS, P, INV>(v, w1);
    reg_rest_wave<LOG2N, PTS, P + 1, INV>(buf, v, w1, lane);
  }
}

// passes 1.. of the wave-local 1024-point transform (RegPlan<10, 16>: radix 16, 4, 16) with
// its first exchange in a layout of its own: pass 0 leaves elements 16 l + r in lane l, which
// lds_pad places 2-way bank-conflicted for 8-byte stores (16-lane groups over 32 banks: lanes l
// and l + 1 land on one bank) -- about a sixth of the search kernel's LDS cycles. Element
// i = 32 a + b goes to 33 a + (b ^ 8 ((b >> 4) & 1)) instead: the stores (fixed r) then cover
// all 16 bank pairs, from two bases per lane (the XOR swaps the halves r < 8 and r >= 8 on odd
// lanes), and pass 1's loads (j + 256 r, fixed r) one bijection per 32 lanes. The footprint
// (1055 entries) fits the lds_pad region (1056). Census: tools/lds/search_model.py.
template <bool INV>
MIMO_DEV void wave1024_rest(v2f *buf, v2f *v, const v2f *w1, int lane) {
  using PL = RegPlan<10, 16>;
  static_assert(PL::NP == 3 && PL::radix(0) == 16 && PL::radix(1) == 4 && PL::T == 64,
                "plan 16, 4, 16");
  int t = lane;
  asm volatile("" : "+v"(t));
  {
    const int m = (t & 1) << 3;
    const int B = 33 * (t >> 1) + 16 * (t & 1);
    v2f *lo = buf + B + m, *hi = buf + B - m;
#pragma unroll
    for (int r = 0; r < 8; r++) lo[r] = v[r];
#pragma unroll
    for (int r = 8; r < 16; r++) hi[r] = v[r];
  }
  wave_lds_sync();
  {
    // pass 1: butterfly i reads elements (lane + 64 i) + 256 r
    const v2f *p = buf + 33 * (t >> 5) + ((t & 31) ^ (((t >> 4) & 1) << 3));
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int r = 0; r < 4; r++) v[4 * i + r] = p[66 * i + 264 * r];
  }
  reg_compute<10, 16, 1, INV>(v, w1);
  reg_rest_wave<10, 16, 2, INV>(buf, v, w1, lane);
}

// element index held in v[s] after the last pass (and read by pass 0): j + r*N/R, R the main
// radix (the first and the last pass)
template <int LOG2N, int PTS>
MIMO_DEV int reg_index(int tid, int s) {
  using PL = RegPlan<LOG2N, PTS>;
  constexpr int R = PL::RM;
  return tid + (s / R) * PL::T + (s % R) * (PL::N / R);
}

}  // namespace mimo

// rub_mimo_amd/csrc/decode_stream.hip -- streaming replay decode for gfx950: one persistent
// 1024-thread workgroup per CU walks a contiguous range of the batch's decodable symbols.
//
// Reference: the replay loop of estimate_channel (framing.cc:853-868) calls
// execute_mimo_decode (framing.cc:535-589) once per OFDM symbol: drop the CP, FFT each rx
// antenna, x dft_normalizer, x_t = sum_r W[k][t][r] X_r[k], x normalize_gain[k]; main.cc then
// demaps and counts symbol errors (main.cc:1394-1411).
//
// Why this shape (measured on MI355X at C3, 4x4, M = 2048): the one-workgroup-per-symbol
// kernel (decode_kernels.hip) spends most of its time on per-symbol dependency chains --
// FrameInfo -> IQ loads -> FFT -> 64 weight loads from L2 -> apply -> stores -- with only two
// workgroups per CU to overlap them; with HBM traffic removed it still took 80% of its time.
// Here every chain is broken:
//   * the next symbol's samples and EVM reference indices stream into an LDS staging area by
//     LDS-DMA (global_load_lds_dwordx4, no registers, no VGPR writeback) while the current
//     symbol is transformed; the kernel waits for them with an explicit vmcnt at the top of
//     the next symbol (the DMA is inline asm, invisible to the compiler's waits, which would
//     otherwise drain it at the first barrier);
//   * each thread owns S = 8/N subcarriers k = tid + q T and keeps W[t][r][k] * gain[k] * dn for
//     them in registers for all symbols of a frame (64 VGPRs at 4x4): the weights are read
//     once per workgroup and frame instead of once per symbol (4x the IQ bytes at 4x4);
//   * complex arithmetic is issued as single VOP3P instructions (cmul_pk & co., fft.hpp) and
//     the twiddles of every pass come from an LDS table.
// The FFT runs on all N antennas at once, 8 points per thread per pass (radix 8, one radix
// 2/4 pass, radix-4 last pass), exchanging through one padded LDS image per antenna; a final
// exchange leaves the spectra in natural order so the thread reads its S subcarriers of every
// antenna. Symbol and index stores are coalesced across the wave (512 B / 64 B per
// instruction); symbol errors are counted per wave with a ballot (SGPRs).
//
// EVM/symbol-error sums are kept per thread in fp32 across the symbols of a frame segment and
// written per wave as fp64 at segment ends into evm_part[f][j][wave] (j = the workgroup's
// rank among those covering frame f; nrec[f] of them), so evm_kernel's fixed-order reduction
// stays bitwise reproducible (the item partition is a pure function of the batch).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "fft.hpp"
#include "fft_reg.hpp"
#include "kernels.hpp"

namespace mimo {

#ifdef DS_MARK
#define MARK(s) asm volatile(s)
#else
#define MARK(s)
#endif
// diagnostics build only (-DDS_PROF, RMIMO_DEC_PROF=1): shader-clock split of the symbol loop
// of workgroup wave 0 (top wait, transform, apply, tail) into DecodeArgs::prof
#ifdef DS_PROF
#define DSP(...) __VA_ARGS__
#else
#define DSP(...)
#endif
// staging DMA issued by DS_ROW_DMA waves per antenna row (0: spread over every wave with the
// per-chunk address arithmetic, the earlier round-3 form)
#ifndef DS_ROW_DMA
#define DS_ROW_DMA 1
#endif
constexpr uint32_t kStreamMaxFrames = 192;   // per-frame tables in LDS beside a 157 KB working set
constexpr uint32_t kStreamMaxQam = 256;          // constellation points (256-QAM)

template <int LOG2M, int NA>
struct StreamPlan {
  static constexpr int M = 1 << LOG2M;
  static constexpr int T = NA * M / 8;                 // 8 points per thread in every pass
  static constexpr int S = 8 / NA;                     // subcarriers per thread in the apply
  static constexpr int P8 = (LOG2M - 2) / 3;           // radix-8 passes (pass 0 included)
  static constexpr int TAIL = (LOG2M - 2) % 3;         // then one radix-2/-4 pass if nonzero
  static constexpr int NP = P8 + (TAIL ? 1 : 0) + 1;   // ... and a final radix-4 pass
  // image stride per antenna: the largest exchange layout (x2, M + M/8; see st_store)
  static constexpr int PB = M + M / 8;
  static constexpr int radix(int p) { return p < P8 ? 8 : (p == NP - 1 ? 4 : (1 << TAIL)); }
  static constexpr int ns(int p) {
    int n = 1;
    for (int q = 0; q < p; q++) n *= radix(q);
    return n;
  }
  static constexpr int bt(int p) { return 8 / radix(p); }          // butterflies per thread
  static constexpr int ntw(int p) { return (T % ns(p) == 0) ? 1 : bt(p); }
};

// an opaque copy: values derived from it inside the symbol loop are recomputed where they are
// used instead of being hoisted out of the loop and held (or spilled) across it
MIMO_DEV int opq(int x) {
  asm volatile("" : "+v"(x));
  return x;
}
MIMO_DEV uint32_t opq_s(uint32_t x) {
  asm volatile("" : "+s"(x));
  return x;
}

// LDS addressing. The images are padded one slot per 32 (lds_pad). For every pass the
// elements a thread touches sit at compile-time offsets from one padded base:
//   store: lds_pad(o + r NS) = lds_pad(o) + r NS + floor(r NS / 32), o = (j/NS) NS R + j%NS
//          (for NS >= 32 r NS is a multiple of 32; for NS < 32 the NS R-aligned group that
//          holds o .. o + (R-1) NS never straddles a multiple of 32, and j%NS + r NS < 32
//          wherever NS R >= 32);
//   load:  lds_pad(j + r NB) = lds_pad(j) + r NB + r NB / 32 (NB = M/R a multiple of 32).
// So each butterfly costs one address computation and its R accesses use immediate offsets.
template <int NS, int R>
constexpr int st_off(int r) { return r * NS + (r * NS) / 32; }

// The wave-local 256-point sub-transforms (WavePlan with M/8 = 256) use a second padding,
// pad2(i) = i + i/32 + 4 (i/64): with one slot per 32 the middle pass's stores (elements
// 64 (j/8) + j%8 + 8 r) hit 4-way bank conflicts; pad2 leaves them 2-way and every other
// access of the region conflict-free (searched over additive paddings and XOR swizzles of the
// region's six access patterns; none is conflict-free everywhere). The identities the
// compile-time offsets rely on hold for that plan: pad2(o + r NS) = pad2(o) + pad2(r NS) and
// pad2(j + r NB) = pad2(j) + pad2(r NB) for its stores (o = (j/NS) NS R + j%NS) and loads
// (j < NB, NB = 32 or 64).
MIMO_DEV constexpr int pad2(int i) { return i + (i >> 5) + 4 * (i >> 6); }
template <int PADK>
MIMO_DEV constexpr int padk(int i) { return PADK ? pad2(i) : i + (i >> 5); }   // (lds_pad)

// Per-exchange layouts of the all-antenna plan (LAY; every exchange is a store then a load, so
// each may place elements as it likes). With lds_pad the radix-8 stores of the first two
// exchanges (elements 8 j + r, and 64 (j/8) + j%8 + 8 r) are 2-way bank-conflicted on gfx950
// (8-byte stores: 16-lane groups over 32 banks), about a quarter of the transform's LDS
// cycles; these two are conflict-free for every access (census: tools/lds/stream_plan_model.py):
//   LAY 1 (after pass 0): i = 32 a + b at 33 a + (b ^ 4 ((b >> 4) & 1)) -- the store of 8 j + r
//          from two bases (the XOR swaps r < 4 and r >= 4 where j & 2), the load of j + r NB
//          from one (NB a multiple of 32);
//   LAY 2 (after pass 1): x2(i) = i + 2 (i >> 5) + 4 (i >> 6) -- x2(o + 8 r) = x2(o) + 8 r +
//          2 (r >> 2) for o = 64 (j/8) + j%8, x2(j + r NB) = x2(j) + 9 r NB / 8 (NB a multiple
//          of 64); footprint M + M/8 (PB);
//   LAY 0: lds_pad (padk<PADK>), later exchanges and the final natural-order store.
MIMO_DEV constexpr int x2pad(int i) { return i + 2 * (i >> 5) + 4 * (i >> 6); }
template <int NP>
constexpr int ex_layout(int e) { return e == 0 ? 1 : ((e == 1 && e < NP - 1) ? 2 : 0); }

template <int LOG2M, int NA, int P, int PADK = 0, int LAY = 0>
MIMO_DEV void st_store(v2f *buf, const v2f *v, uint32_t tid) {
  using PL = StreamPlan<LOG2M, NA>;
  constexpr uint32_t R = PL::radix(P), NS = PL::ns(P), NB = PL::M / R;
  static_assert(NB % 32 == 0 && (NS >= 32 || (32 % (NS * R) == 0) || (NS * R) % 32 == 0),
                "padded-offset identity");
  static_assert(!PADK || PL::M == 256, "pad2 identities checked for the 256-point plan only");
  static_assert(LAY != 1 || (P == 0 && R == 8), "x1 stores: pass 0, radix 8");
  static_assert(LAY != 2 || (P == 1 && R == 8 && NS == 8), "x2 stores: pass 1, radix 8");
#pragma unroll
  for (int i = 0; i < PL::bt(P); i++) {
    const uint32_t u = tid + i * PL::T, g = u / NB, j = u % NB;
    if constexpr (LAY == 1) {
      const uint32_t m = ((j >> 1) & 1u) << 2;
      const uint32_t B = g * PL::PB + 33 * (j >> 2) + 8 * (j & 3u);
      v2f *lo = buf + B + m, *hi = buf + B - m;
#pragma unroll
      for (int r = 0; r < 4; r++) lo[r] = v[i * R + r];
#pragma unroll
      for (int r = 4; r < 8; r++) hi[r] = v[i * R + r];
    } else if constexpr (LAY == 2) {
      v2f *bp = buf + g * PL::PB + 64 * (j >> 3) + (j & 7u) + 8 * (j >> 3);
#pragma unroll
      for (int r = 0; r < 8; r++) bp[8 * r + 2 * (r >> 2)] = v[i * R + r];
    } else {
      const uint32_t o = (j / NS) * NS * R + (j % NS);
      v2f *bp = buf + g * PL::PB + padk<PADK>((int)o);
#pragma unroll
      for (int r = 0; r < (int)R; r++)
        bp[PADK ? pad2(r * (int)NS) : st_off<NS, R>(r)] = v[i * R + r];
    }
  }
}

// pass P with its base twiddle from the LDS table (twl: passes 1.. in order, one row of NS
// entries each, [jm] = e^{-2 pi i jm / (NS R)}) and the powers r = 2 .. R-1 in registers: one
// LDS read per butterfly instead of R - 1 (the transform phase is bound by LDS instructions)
template <int LOG2M, int NA, int P, int PADK = 0, int LAY = 0>
MIMO_DEV void st_load_t(const v2f *buf, v2f *v, const v2f *twl, uint32_t tid) {
  using PL = StreamPlan<LOG2M, NA>;
  constexpr uint32_t R = PL::radix(P), NB = PL::M / R, NS = PL::ns(P);
  constexpr int OFF = [] {
    int o = 0;
    for (int q = 1; q < P; q++) o += PL::ns(q);
    return o;
  }();
  static_assert(LAY != 1 || NB % 32 == 0, "x1 loads: NB a multiple of 32");
  static_assert(LAY != 2 || NB % 64 == 0, "x2 loads: NB a multiple of 64");
#pragma unroll
  for (int i = 0; i < PL::bt(P); i++) {
    const uint32_t u = tid + i * PL::T, g = u / NB, j = u % NB;
    if constexpr (LAY == 1) {
      const v2f *bp = buf + g * PL::PB + 33 * (j >> 5) + ((j & 31u) ^ (((j >> 4) & 1u) << 2));
#pragma unroll
      for (int r = 0; r < (int)R; r++) v[i * R + r] = bp[33 * r * (int)(NB / 32)];
    } else if constexpr (LAY == 2) {
      const v2f *bp = buf + g * PL::PB + x2pad((int)j);
#pragma unroll
      for (int r = 0; r < (int)R; r++) v[i * R + r] = bp[9 * r * (int)(NB / 8)];
    } else {
      const v2f *bp = buf + g * PL::PB + padk<PADK>((int)j);
#pragma unroll
      for (int r = 0; r < (int)R; r++)
        v[i * R + r] = bp[PADK ? pad2(r * (int)NB) : r * NB + (r * NB) / 32];
    }
    v2f w[R];
    twiddle_powers<R>(w, twl[OFF + (j % NS)]);
#pragma unroll
    for (int r = 1; r < (int)R; r++) v[i * R + r] = cmul_pk(v[i * R + r], w[r]);
    dft_fwd_pk<R>(v + i * R);
  }
}

// passes P .. NP-1; the outputs of pass P-1 are already stored in the image
template <int LOG2M, int NA, int P>
MIMO_DEV void st_passes2(v2f *img, v2f *v, const v2f *twl, uint32_t tid) {
  using PL = StreamPlan<LOG2M, NA>;
  if constexpr (P < PL::NP) {
    const uint32_t t = (uint32_t)opq((int)tid);   // opaque per pass: addresses not hoisted
    __syncthreads();                        // the image is complete
    st_load_t<LOG2M, NA, P, 0, ex_layout<PL::NP>(P - 1)>(img, v, twl, t);
    if constexpr (P + 1 < PL::NP) {
      __syncthreads();                      // readers of the image are done
      st_store<LOG2M, NA, P, 0, ex_layout<PL::NP>(P)>(img, v, t);
      st_passes2<LOG2M, NA, P + 1>(img, v, twl, tid);
    }
  }
}

// Wave-local form of the transform (M >= 2048, when its LDS layout fits): pass 0 is a radix-8
// DIF step over stride MS = M/8 (thread n of antenna g: b_q = sum_r x[n + r MS] W8^{rq}, then
// c_q[n] = b_q W_M^{nq}); X_g[8k + q] is then the MS-point DFT of c_q over n. The NA * 8
// sub-transforms run on groups of LG = MS/8 lanes inside one wave (Stockham passes of
// StreamPlan<log2 MS, 1>), exchanging through their own LDS region with no workgroup barrier,
// and leave X_g[8k + q] at region (g, q), index k. Three barriers per symbol instead of nine.
// Region stride QS = 4 mod 8 entries: the apply's reads of subcarriers k' = 8k + q (q fastest
// across lanes) hit distinct banks.
template <int LOG2M, int NA>
struct WavePlan {
  static constexpr int M = 1 << LOG2M, MS = M / 8, LG = MS / 8;
  using SP = StreamPlan<LOG2M - 3, 1>;
  // 256 points: sub256_fwd's per-exchange layouts (the region holds the largest, 282 entries;
  // its stride 4 mod 32 keeps the apply's reads conflict-free); else lds_pad over the region
  static constexpr bool X256 = (MS == 256);
  static constexpr int PADK = 0;
  static constexpr int QS = X256 ? 292 : ((padk<PADK>(MS - 1) + 1 + 3) / 8) * 8 + 4;
  static constexpr int GS = 8 * QS;
  static constexpr int TW0 = MS;                         // W_M^n, n < MS (powers q = 2..7 in registers)
  static constexpr int TWS = [] {
    int s = 0;
    for (int p = 1; p < SP::NP; p++) s += SP::ns(p);
    return s;
  }();
};

// LDS writes of this wave visible to its own reads; no code motion across
MIMO_DEV void lds_wave_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// sub-transform passes P .. NP-1 on a lane group (pass P-1's outputs in registers), ending with
// the natural-order store
template <int L2, int P, int PADK>
MIMO_DEV void wave_passes(v2f *buf, v2f *v, const v2f *twl, uint32_t s) {
  using SP = StreamPlan<L2, 1>;
  if constexpr (P < SP::NP) {
    st_store<L2, 1, P - 1, PADK>(buf, v, s);
    lds_wave_sync();
    st_load_t<L2, 1, P, PADK>(buf, v, twl, s);
    wave_passes<L2, P + 1, PADK>(buf, v, twl, s);
  } else {
    lds_wave_sync();
    st_store<L2, 1, SP::NP - 1, PADK>(buf, v, s);
  }
}

// The 256-point sub-transform of one 32-lane group (radix 8, 8, 4; StreamPlan<8, 1>) with a
// layout of its own for each LDS exchange (every exchange is a store then a load, so each may
// place the elements as it likes), chosen so that no access has a bank conflict on gfx950
// (8-byte stores: 16-lane groups over 32 banks; 8-byte loads: 32-lane groups over 64 banks;
// the census and the search are tools/lds/). One region-wide padding (pad2) left both radix-8
// exchanges' stores 2-way conflicted, about a fifth of the kernel's LDS cycles:
//   in:  element i at i (the block pass's store, lane-contiguous)
//   x1:  i = 32 a + b at 33 a + (b ^ 4 (b >> 4)) -- stores 8 s + r from two bases per thread
//        (the XOR flips bit 2 of r on threads with s & 2), loads s + 32 r from one
//   x2:  i + 2 (i >> 5) + 4 (i >> 6)
//   out: i (the apply reads across the regions, stride QS = 4 mod 32)
MIMO_DEV void sub256_fwd(v2f *rg, v2f *v, const v2f *twl, uint32_t s) {
#ifdef DS_ABL_SUBNOLDS   // timing ablation: the sub-transform's arithmetic without its exchanges
#pragma unroll
  for (int r = 0; r < 8; r++) v[r] = rg[s + 32 * r];
#pragma unroll
  for (int p = 0; p < 3; p++) {
    dft_fwd_pk<8>(v);
    v2f w[8];
    twiddle_powers<8>(w, twl[(s + p) & 7u]);
#pragma unroll
    for (int r = 1; r < 8; r++) v[r] = cmul_pk(v[r], w[r]);
  }
#pragma unroll
  for (int r = 0; r < 8; r++) rg[s + 32 * r] = v[r];
  return;
#endif
#ifdef DS_ABL_SUBNOVALU   // timing ablation: the exchanges without the arithmetic
#pragma unroll
  for (int r = 0; r < 8; r++) v[r] = rg[s + 32 * r];
  {
    const uint32_t m = ((s & 3u) >> 1) << 2;
    const uint32_t B = 33 * (s >> 2) + 8 * (s & 3u);
    v2f *lo = rg + B + m, *hi = rg + B - m;
#pragma unroll
    for (int r = 0; r < 4; r++) lo[r] = v[r];
#pragma unroll
    for (int r = 4; r < 8; r++) hi[r] = v[r];
  }
  lds_wave_sync();
  {
    const v2f *p = rg + (s ^ ((s >> 4) << 2));
#pragma unroll
    for (int r = 0; r < 8; r++) v[r] = p[33 * r];
    v2f *q = rg + 64 * (s >> 3) + (s & 7u) + 8 * (s >> 3);
#pragma unroll
    for (int r = 0; r < 8; r++) q[8 * r + 2 * (r >> 2)] = v[r];
  }
  lds_wave_sync();
#pragma unroll
  for (int i = 0; i < 2; i++) {
    const uint32_t u = s + 32 * i;
    const v2f *p = rg + u + 2 * (u >> 5);
#pragma unroll
    for (int r = 0; r < 4; r++) v[4 * i + r] = p[72 * r];
  }
  lds_wave_sync();
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int r = 0; r < 4; r++) rg[s + 32 * i + 64 * r] = v[4 * i + r];
  return;
#endif
  // initial load: x[s + 32 r]
#pragma unroll
  for (int r = 0; r < 8; r++) v[r] = rg[s + 32 * r];
  dft_fwd_pk<8>(v);                                   // pass 0 (no twiddles): element 8 s + r
  {
    const uint32_t m = ((s & 3u) >> 1) << 2;          // 0 or 4
    const uint32_t B = 33 * (s >> 2) + 8 * (s & 3u);
    v2f *lo = rg + B + m, *hi = rg + B - m;
#pragma unroll
    for (int r = 0; r < 4; r++) lo[r] = v[r];
#pragma unroll
    for (int r = 4; r < 8; r++) hi[r] = v[r];
  }
  lds_wave_sync();
  {
    // pass 1 (radix 8, NS 8): elements s + 32 r, twiddle base W_64^{s % 8}
    const v2f *p = rg + (s ^ ((s >> 4) << 2));
#pragma unroll
    for (int r = 0; r < 8; r++) v[r] = p[33 * r];
    v2f w[8];
    twiddle_powers<8>(w, twl[s & 7u]);
#pragma unroll
    for (int r = 1; r < 8; r++) v[r] = cmul_pk(v[r], w[r]);
    dft_fwd_pk<8>(v);
    // its outputs: elements o + 8 r, o = 64 (s / 8) + s % 8, stored at x2's layout
    v2f *q = rg + 64 * (s >> 3) + (s & 7u) + 8 * (s >> 3);
#pragma unroll
    for (int r = 0; r < 8; r++) q[8 * r + 2 * (r >> 2)] = v[r];
  }
  lds_wave_sync();
  {
    // pass 2 (radix 4, NS 64): butterflies u = s, s + 32: elements u + 64 r, twiddle W_256^u
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const uint32_t u = s + 32 * i;
      const v2f *p = rg + u + 2 * (u >> 5);
#pragma unroll
      for (int r = 0; r < 4; r++) v[4 * i + r] = p[72 * r];
      v2f w[4];
      twiddle_powers<4>(w, twl[8 + u]);
#pragma unroll
      for (int r = 1; r < 4; r++) v[4 * i + r] = cmul_pk(v[4 * i + r], w[r]);
      dft_fwd_pk<4>(v + 4 * i);
    }
  }
  lds_wave_sync();
  // final store: element u + 64 r at its natural index
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int r = 0; r < 4; r++) rg[s + 32 * i + 64 * r] = v[4 * i + r];
}

// a wave-uniform complex value held in SGPRs
// the sum over the 64 lanes, in every lane, with no LDS traffic: v_permlane32/16_swap pair lanes
// l and l ^ 32 / l ^ 16, then DPP row_mirror (l ^ 15), row_half_mirror (l ^ 7) and quad_perm
// (l ^ 2, l ^ 1), whose partner sets together cover the 16 lanes of a row
MIMO_DEV float wave_sum_f(float x) {
  const uint32_t b = __float_as_uint(x);
  const auto s32 = __builtin_amdgcn_permlane32_swap(b, b, false, false);
  x = __uint_as_float(s32[0]) + __uint_as_float(s32[1]);
  const uint32_t b16 = __float_as_uint(x);
  const auto s16 = __builtin_amdgcn_permlane16_swap(b16, b16, false, false);
  x = __uint_as_float(s16[0]) + __uint_as_float(s16[1]);
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x140, 0xf, 0xf, false));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x141, 0xf, 0xf, false));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xf, 0xf, false));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xf, 0xf, false));
  return x;
}
MIMO_DEV v2f uni(v2f v) {
  return v2f{__int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v.x))),
             __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v.y)))};
}

MIMO_DEV uint32_t cvt_u32_sat(float x) {   // v_cvt_u32_f32: NaN and negatives -> 0, saturating
  uint32_t r;
  asm("v_cvt_u32_f32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

// the level pair of the hard decision (as qam_slice_pk below) packed as mI * L + mQ, the index
// of the decision in the LDS table of Gray-coded symbol indices (one multiply-add instead of
// the two Gray encodings and the combine)
MIMO_DEV uint32_t qam_level_pair_pk(v2f y, v2f inv_scale, v2f Lf, uint32_t Lm1, uint32_t L) {
#pragma clang fp contract(off)
  const v2f t = (y * inv_scale + Lf) * 0.5f;
  const uint32_t mI = min(cvt_u32_sat(t.x), Lm1), mQ = min(cvt_u32_sat(t.y), Lm1);
  return mI * L + mQ;
}

// hard decision as qam_slice (decode_kernels.hip) / qam_demap (common.hpp): the level is
// floor((y * inv_scale + L) * 0.5) clamped to [0, L-1] (NaN -> 0); truncation of the
// non-negative value by v_cvt_u32_f32 with its saturation gives exactly that clamp
MIMO_DEV uint32_t qam_slice_pk(v2f y, v2f inv_scale, v2f Lf, uint32_t Lm1, uint32_t b) {
#pragma clang fp contract(off)
  const v2f t = (y * inv_scale + Lf) * 0.5f;
  const uint32_t mI = min(cvt_u32_sat(t.x), Lm1), mQ = min(cvt_u32_sat(t.y), Lm1);
  return (gray_enc(mI) << b) | gray_enc(mQ);
}

// LDS-DMA of 16 bytes per lane (global_load_lds_dwordx4: lane l writes lds + 16 l), issued as
// inline asm so that the compiler does not tie it to its own vmcnt waits (it waits for every
// LDS DMA at the next barrier); the kernel waits for it explicitly (s_waitcnt vmcnt) at the
// point of use. M0 is saved and restored around it.
MIMO_DEV void dma16(uint32_t voff, __attribute__((address_space(1))) const void *sbase, uint32_t lds) {
  uint32_t keep;
  // s_nop 4 first: sbase may come straight from a v_readfirstlane (VALU-written SGPR read as
  // a VMEM base needs wait states the compiler does not insert inside an asm statement)
  asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, %2 nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds) : "memory");
}
#ifndef DS_PROF_TID
#define DS_PROF_TID 0
#endif
// index stores non-temporal from this transform size up (see NTI)
#ifndef DS_NTI_MIN_LOG2M
#define DS_NTI_MIN_LOG2M 11
#endif
template <bool NT, typename V, typename P>
MIMO_DEV void out_store(V v, P p) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

constexpr size_t kStreamStaticLds = 8192;   // pfx, fbody, fcr, ptab, gidx, cpe_part, cfo_tab (+ slack)

// dynamic LDS of the kernel: FFT images, staging, reference staging, twiddle table
template <int LOG2M, int NA>
constexpr size_t stream_dyn_lds(bool wave_fft, int ref_mode, bool sc16) {
  using PL = StreamPlan<LOG2M, NA>;
  using WP = WavePlan<LOG2M, NA>;
  size_t tw = 0;
  if (wave_fft) {
    tw = (size_t)WP::TW0 + WP::TWS;
  } else {
    for (int p = 1; p < PL::NP; p++) tw += (size_t)PL::ns(p);
  }
  const size_t img = wave_fft ? (size_t)NA * WP::GS : (size_t)NA * PL::PB;
  const size_t stage = sc16 ? sizeof(short2) * (size_t)(PL::M + 4) * NA
                            : sizeof(float2) * (size_t)(PL::M + 2) * NA;
  return sizeof(float2) * (img + tw) + stage + (ref_mode == 1 ? (size_t)NA * PL::M : 0);
}

// the wave-local transform where its sub-transforms are >= 256 points and its layout fits
template <int LOG2M, int NA, int REF, bool SC16>
constexpr bool stream_wave_fft() {
  return LOG2M >= 11 && stream_dyn_lds<LOG2M, NA>(true, REF, SC16) + kStreamStaticLds <= 163840;
}

// CPE (opt-in CFO path): per-symbol common phase, decision directed and non-recursive. The
// residual frequency offset left by the CFO estimate turns every symbol by a slowly growing
// angle. Each symbol measures its own: c = sum of conj(Q(y)) y over every stream's outputs y
// at the subcarriers k with k even and bit 9 of k clear (Q the hard decision's constellation
// point; oracle cfo_common_phase), reduced over the workgroup in a fixed order,
// and every output of the symbol is turned by conj(c)/|c| before its decision, EVM and
// stores. Nothing carries from one symbol to the next, so a symbol's outputs are a function
// of the frame alone, not of where a workgroup's range starts (oracle/mimo_ref.c restates it,
// cfo_mode 2). Off (CPE = false) the kernel is unchanged.
// the constellation point of the hard decision of y (levels as qam_level_pair_pk; the point
// as qam_point: (2m - (L-1)) * scale in fp32)
MIMO_DEV v2f qam_dec_point_pk(v2f y, v2f inv_scale, v2f Lf, uint32_t Lm1, float scale) {
#pragma clang fp contract(off)
  const v2f t = (y * inv_scale + Lf) * 0.5f;
  const uint32_t mI = min(cvt_u32_sat(t.x), Lm1), mQ = min(cvt_u32_sat(t.y), Lm1);
  return v2f{(float)(int32_t)(2 * mI - Lm1) * scale, (float)(int32_t)(2 * mQ - Lm1) * scale};
}
template <int LOG2M, int NA, int REF, int OUTS, bool SC16 = false, bool CPE = false>
__global__ __launch_bounds__(NA * (1 << LOG2M) / 8) void decode_stream_kernel(DecodeArgs a) {
  using PL = StreamPlan<LOG2M, NA>;
  constexpr int M = PL::M, T = PL::T, S = PL::S, PB = PL::PB, W8 = M / 8;
  // staging row: M + SPC samples from a start aligned to SPC samples, SPC = samples per
  // 16-byte chunk (2 complex64, or 4 sc16 on the wire)
  constexpr int SPC = SC16 ? 4 : 2;
  constexpr int SB = SC16 ? 4 : 8;                // bytes per staged sample
  constexpr int RS = M + SPC;
  constexpr int NBLK = (RS / SPC + 63) / 64;      // wave DMA instructions per staged row
  [[maybe_unused]] constexpr int NWI = (NA * NBLK + T / 64 - 1) / (T / 64);   // ... per wave and symbol
  constexpr int LASTC = RS / SPC - (NBLK - 1) * 64;          // chunks in a row's last block
  static_assert(RS % SPC == 0 && LASTC >= 1 && LASTC <= 64 && 64 * SPC * SB == 1024,
                "row DMA blocks of 1 KB");
  // waves staging each antenna row (at most the waves there are per row)
  constexpr int WPR = DS_ROW_DMA == 0 ? 0 : ((T / 64) / NA < DS_ROW_DMA ? (T / 64) / NA : DS_ROW_DMA);
  static_assert(!DS_ROW_DMA || (WPR >= 1 && NA * WPR <= T / 64), "waves per staged row");
  constexpr int NREF = NA * M / 16;               // 16-byte chunks of the reference indices
  // store instructions per symbol: the wait at the top of a symbol leaves them in flight
  using WP = WavePlan<LOG2M, NA>;
  constexpr bool WF = stream_wave_fft<LOG2M, NA, REF, SC16>();
  constexpr int MS = WP::MS, LG = WP::LG, QS = WP::QS, GS = WP::GS;
  // subcarriers of a thread in the apply: k = S tid + q (adjacent: one S*8-byte symbol store and
  // one S-byte index store per stream) on the wave-FFT layout, else k = tid + q T
  constexpr bool KADJ = WF && S == 2;
  constexpr int SPS = KADJ ? NA : NA * S;          // store instructions per output kind
#ifdef DS_ABL_NOIDX   // timing ablation: no index stores
  constexpr int OUTX = OUTS & 1;
#elif defined(DS_ABL_NOSYM)   // timing ablation: no symbol stores
  constexpr int OUTX = OUTS & 2;
#else
  constexpr int OUTX = OUTS;
#endif
  constexpr int NSTORE = ((OUTX & 1) ? SPS : 0) + ((OUTX & 2) ? SPS : 0);
  // output store policies (measured): symbols non-temporal everywhere (the
  // captures of the next batch stay cached for its S&C); the uint8 indices non-temporal from
  // M = 2048 up, plain below (C2: decode -6%, the next S&C unchanged; at C3 plain index stores
  // cost the next S&C 15%)
  constexpr bool NTS = true, NTI = LOG2M >= DS_NTI_MIN_LOG2M;
  extern __shared__ __attribute__((aligned(16))) float2 lds_raw[];
  v2f *img = reinterpret_cast<v2f *>(lds_raw);    // [NA][PB] FFT exchange ([NA][8][QS] if WF)
  v2f *stg = img + NA * (WF ? GS : PB);                            // [NA][RS] next symbol
  short2 *stg16 = reinterpret_cast<short2 *>(stg);                 // (sc16 staging)
  uint8_t *rstg = reinterpret_cast<uint8_t *>(stg) + (size_t)NA * RS * SB;   // [NA][M] next references
  v2f *twl = reinterpret_cast<v2f *>(rstg + ((REF == 1) ? NA * M : 0));   // twiddle table
  __shared__ uint32_t pfx[kStreamMaxFrames + 1];
  __shared__ int64_t fbody[kStreamMaxFrames];
  __shared__ uint32_t fcr[kStreamMaxFrames];     // capture | reference row << 16
  // constellation by symbol index, and the Gray-coded symbol index by level pair mI * L + mQ
  __shared__ v2f ptab[kStreamMaxQam];
  __shared__ uint8_t gidx[kStreamMaxQam];
  __shared__ v2f cpe_part[CPE ? T / 64 : 1];                       // per-wave phase sums
  constexpr int CTN = W8 < 256 ? W8 : 256;
  __shared__ v2f cfo_tab[CPE ? CTN : 1];                           // folded CFO, in-body phasors
  struct CfoState {
    uint64_t E, j0;   // nu 2^64 (two's complement), i0 + cp: symbol 0's body
    v2f w, rot;       // exp(-j2pi nu W8), the next symbol's body-start phasor
  };
  __shared__ CfoState cfo_st_s[1];
  CfoState *cfo_st = cfo_st_s;
  const int tid = threadIdx.x;
  const uint32_t wv = __builtin_amdgcn_readfirstlane((uint32_t)tid >> 6);
  for (uint32_t e = tid; e < a.qam.L * a.qam.L; e += T) {
    const float2 p = qam_point(e, a.qam);
    ptab[e] = v2f{p.x, p.y};
    const uint32_t mI = e / a.qam.L, mQ = e % a.qam.L;
    gidx[e] = (uint8_t)((gray_enc(mI) << a.qam.b) | gray_enc(mQ));
  }

  // base twiddles of passes 1..NP-1: twl[off(p) + jm] = e^{-2 pi i jm / (NS R)} (the powers
  // r = 2 .. R-1 are formed in registers, st_load_t)
  if constexpr (WF) {
    // W_M^n (n < MS; pass 0's W_M^{nq} are its powers), then the sub-transform plan's passes
    for (int e = tid; e < WP::TW0; e += T) twl[e] = twiddle<false>(a.tw, e * (kTwN / M));
    using SP = typename WP::SP;
    int off = WP::TW0;
#pragma unroll
    for (int p = 1; p < SP::NP; p++) {
      const int R = SP::radix(p), NS = SP::ns(p);
      for (int e = tid; e < NS; e += T) twl[off + e] = twiddle<false>(a.tw, e * (kTwN / (NS * R)));
      off += NS;
    }
  } else {
    int off = 0;
#pragma unroll
    for (int p = 1; p < PL::NP; p++) {
      const int R = PL::radix(p), NS = PL::ns(p);
      for (int e = tid; e < NS; e += T) twl[off + e] = twiddle<false>(a.tw, e * (kTwN / (NS * R)));
      off += NS;
    }
  }
  // decodable symbols of frames < f (status OK, min(n_sym, max_out) each), and each frame's
  // first data-symbol body (held in LDS: FrameInfo reads in the loop would be vector loads
  // whose waits also drain the symbol stores in flight)
  for (uint32_t f0 = 0; f0 <= a.n_frames; f0 += T) {
    const uint32_t f = f0 + tid;
    uint32_t v = 0;
    if (f < a.n_frames) {
      const FrameInfo &I = a.info[f];
      v = (I.status == 0) ? min(I.n_sym, a.max_out) : 0u;
      fbody[f] = I.base + (int64_t)I.i0 + (int64_t)a.cp;
      fcr[f] = I.cap | (I.ref << 16);
    }
    if (f <= a.n_frames) pfx[f] = v;
  }
  __syncthreads();
  if (tid == 0) {
    uint32_t acc = 0;
    for (uint32_t f = 0; f <= a.n_frames; f++) {
      const uint32_t v = pfx[f];
      pfx[f] = acc;
      acc += v;
    }
  }
  __syncthreads();
  const uint32_t total = pfx[a.n_frames];
  const uint32_t chunk = (total + gridDim.x - 1) / gridDim.x;
  const uint32_t i_begin = blockIdx.x * chunk;
  const uint32_t i_end = min(i_begin + chunk, total);
  if (i_begin >= i_end) return;                       // uniform

  uint32_t f = 0;                                     // largest f with pfx[f] <= i_begin
  {
    uint32_t lo = 0, hi = a.n_frames;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (pfx[mid] <= i_begin) lo = mid; else hi = mid;
    }
    f = lo;
  }
  f = __builtin_amdgcn_readfirstlane(f);
  uint32_t s = __builtin_amdgcn_readfirstlane(i_begin - pfx[f]);
  uint32_t n_out_f = __builtin_amdgcn_readfirstlane(pfx[f + 1] - pfx[f]);

  const uint64_t rowstep = rfl64(a.o_ts);             // output elements between streams
  const v2f inv_sc = v2f{a.qam.inv_scale, a.qam.inv_scale};
  const v2f Lf = v2f{(float)a.qam.L, (float)a.qam.L};
  const uint32_t Lm1 = a.qam.L - 1;
  const uint32_t stg_base = (uint32_t)(uintptr_t)stg;
  const uint32_t rstg_base = (uint32_t)(uintptr_t)rstg;

  // staging of symbol (ff, ss): antenna row g is staged as M + SPC samples from the SPC-aligned
  // sample a_g <= its first sample e_g (alignment taken in the whole batch, so rows of any
  // stride stay on the DMA path and every lane moves one aligned 16-byte chunk); returns the
  // offsets e_g - a_g (< SPC), 4 bits per row
  // per-frame bases of the staging (uniform, SGPRs; read from the LDS frame tables once per
  // frame instead of once per symbol): first body sample, row 0's batch offset, reference row
  struct FrameBase {
    int64_t body, row0;
    uint64_t ref;
  };
  auto frame_base = [&](uint32_t ff) -> FrameBase {
    const int64_t b0 = fbody[ff];
    const uint32_t cr = __builtin_amdgcn_readfirstlane(fcr[ff]);
    FrameBase fb;
    fb.body = (int64_t)rfl64((uint64_t)b0);
    fb.row0 = (int64_t)(cr & 0xFFFFu) * NA * (int64_t)a.stride;
    fb.ref = (uint64_t)(cr >> 16) * NA * a.max_out * a.M_occ;
    return fb;
  };
  // the rows' offsets e_g - a_g in SPC-sample chunks are (e0 + g stride) mod SPC: nibble g of
  // (ptn + (e0 mod SPC) * REP) with ptn's nibble g = (g stride) mod SPC (sums < 16, no carries)
  constexpr uint32_t REP = NA == 1 ? 0x1u : (NA == 2 ? 0x11u : (NA == 4 ? 0x1111u : 0x11111111u));
  uint32_t ptn = 0;
#pragma unroll
  for (int g = 0; g < NA; g++) ptn |= (((uint32_t)g * (uint32_t)a.stride) & (SPC - 1)) << (4 * g);
  ptn = __builtin_amdgcn_readfirstlane(ptn);
  // the reference indices of symbol (fb, ss) into rstg ([NA][M] bytes), by waves RW0 .. RW0 +
  // NREF/64 - 1 (with DS_ROW_DMA the waves after the row waves, which stage no samples). Plain
  // kernels: issued with the next symbol's samples and copied to registers (cref) at the top of
  // the symbol. CPE kernels (fewer registers to spare): issued after a symbol's top barrier
  // (every wave is done with the previous symbol's), waited for by those waves before the
  // barrier that precedes the apply, and read there straight from LDS
  constexpr int RW0 = (WPR && NA * WPR + NREF / 64 <= T / 64) ? NA * WPR : 0;
  static_assert(NREF % 64 == 0 && RW0 + NREF / 64 <= T / 64, "reference DMA waves");
  const bool ref_wave = REF == 1 && wv >= (uint32_t)RW0 && wv < (uint32_t)(RW0 + NREF / 64);
  auto fetch_ref = [&](const FrameBase &fb, uint32_t ss) {
    if constexpr (REF == 1) {
      if (ref_wave) {
        const int tr = opq(tid) - RW0 * 64;
        const uint32_t dst = __builtin_amdgcn_readfirstlane(rstg_base + (uint32_t)((wv - RW0) * 64) * 16u);
        const uint32_t t = (uint32_t)tr / (M / 16), q = (uint32_t)tr % (M / 16);
        const auto rb = sgpr_ptr(a.ref_idx + fb.ref + (uint64_t)ss * a.o_ss);
        dma16(t * (uint32_t)a.o_ts + 16 * q, rb, dst);
      }
    }
  };
  // ... and the wait (the reference waves' only loads in flight: with RW0 = 0 they also stage
  // samples, whose DMA this waits for as well)
  auto wait_ref = [&]() {
    if constexpr (REF == 1 && CPE)
      if (ref_wave) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  auto fetch = [&](const FrameBase &fb, uint32_t ss) -> uint32_t {
    const int64_t abs0 = fb.body + (int64_t)((uint64_t)ss * a.SL);
    const int64_t row0 = fb.row0;
    const int64_t e0 = row0 + abs0;                   // batch sample index of row 0's first
    const int t0 = opq(tid);
    const uint32_t odds = (ptn + ((uint32_t)e0 & (SPC - 1)) * REP) & ((SPC - 1) * REP);
#ifdef DS_ABL_NODMA   // timing ablation (tools/abl_decode.sh): no sample loads
    if (true) {
    } else
#endif
    if (abs0 >= SPC && abs0 + RS <= (int64_t)a.frame_len && ((uintptr_t)a.iq & 15u) == 0) {
#if DS_ROW_DMA
      // wave g < NA stages antenna row g: NBLK wave instructions of 64 consecutive 16-byte
      // chunks from the row's aligned start a_g (its last block is the row's one remaining
      // chunk). Only NA waves compute the row base and issue DMAs: the address arithmetic is
      // scalar, and 16 waves doing it at once kept the CU's one scalar unit busy ~2k cycles
      // per symbol while every VALU waited; the other waves start their sub-transforms
      if (wv < (uint32_t)(NA * WPR)) {                // WPR waves per row
        const uint32_t g = wv / WPR, sub = wv % WPR;
        const int64_t ag = (e0 + (int64_t)g * a.stride) & ~(int64_t)(SPC - 1);
        const auto xa = sgpr_ptr(reinterpret_cast<const char *>(a.iq) + ag * SB);
        const uint32_t lane = (uint32_t)(opq(tid) & 63);
        const uint32_t dst0 = __builtin_amdgcn_readfirstlane(stg_base + g * RS * (uint32_t)SB);
#pragma unroll
        for (int j = 0; j < (NBLK + WPR - 1) / WPR; j++) {
          const uint32_t b = sub + (uint32_t)j * WPR;             // uniform
          if (b < (uint32_t)NBLK && (b + 1 < (uint32_t)NBLK || lane < (uint32_t)LASTC))
            dma16(b * 1024u + lane * 16u, xa, dst0 + b * 1024u);
        }
      }
#else
      // base SPC samples before row 0's aligned start: every row's a_g - base is in [0, 2^32).
      // One wave instruction moves 64 consecutive chunks of one row (row g, block b uniform;
      // a row's last block is its one remaining chunk), so the lane offsets are a scalar plus
      // 16 * lane
      const int64_t base = (e0 & ~(int64_t)(SPC - 1)) - SPC;
      const auto xa = sgpr_ptr(reinterpret_cast<const char *>(a.iq) + base * SB);
      const uint32_t lane16 = (uint32_t)(opq(tid) & 63) * 16u;
#pragma unroll
      for (int u = 0; u < NWI; u++) {
        const uint32_t k = wv + (uint32_t)u * (T / 64);
        if (u < NWI - 1 || k < (uint32_t)(NA * NBLK)) {
          const uint32_t g = k / NBLK, b = k % NBLK;
          const uint32_t rowoff = (uint32_t)(((e0 + (int64_t)g * a.stride) & ~(int64_t)(SPC - 1)) - base);
          const uint32_t dst = __builtin_amdgcn_readfirstlane(
              stg_base + (g * RS + b * 64u * SPC) * (uint32_t)SB);
          const uint32_t voff = __builtin_amdgcn_readfirstlane((rowoff + b * 64u * SPC) * (uint32_t)SB);
          if (b + 1 < NBLK || lane16 == 0) dma16(voff + lane16, xa, dst);
        }
      }
#endif
    } else {                                          // edge of the capture: guarded loads
      const char *xf = reinterpret_cast<const char *>(a.iq) + row0 * SB;
      for (int c = t0; c < NA * RS; c += T) {
        const int g = c / RS, q = c % RS;
        const int64_t n = abs0 - (int64_t)((odds >> (4 * g)) & 15u) + q;   // row sample
        const bool in = n >= 0 && n < (int64_t)a.frame_len;
        if constexpr (SC16) {
          stg16[c] = in ? reinterpret_cast<const short2 *>(xf)[(uint64_t)g * a.stride + n]
                        : make_short2(0, 0);
        } else {
          stg[c] = in ? reinterpret_cast<const v2f *>(xf)[(uint64_t)g * a.stride + n]
                      : v2f{0.0f, 0.0f};
        }
      }
    }
    if constexpr (REF == 1 && !CPE) fetch_ref(fb, ss);   // the next symbol's, with its samples
    return odds;
  };
  // this frame's weights * gain * dn for the thread's subcarriers k = tid + q T
  v2f Wr[NA][NA][S];
  auto load_w = [&](uint32_t ff) {
    const int t0 = opq(tid);
    const uint32_t k0 = KADJ ? (uint32_t)t0 * S : (uint32_t)t0;
    constexpr uint32_t KQ = KADJ ? 1 : T;                 // k of slot q = k0 + q KQ
    const v2f *Wf = reinterpret_cast<const v2f *>(a.W) + (uint64_t)ff * NA * NA * M + k0;
    const float *gf = a.gain + (uint64_t)ff * M + k0;
    float gs[S];
#pragma unroll
    for (int q = 0; q < S; q++) gs[q] = gf[q * KQ] * a.dn;
#pragma unroll
    for (int t = 0; t < NA; t++)
#pragma unroll
      for (int r = 0; r < NA; r++)
#pragma unroll
        for (int q = 0; q < S; q++) Wr[t][r][q] = Wf[(t * NA + r) * M + q * KQ] * gs[q];
  };

  // EVM sums: per-thread fp32 error and reference energies, per-wave symbol-error counts
  float e_num[NA], e_den[NA];
  uint32_t n_err[NA];
#pragma unroll
  for (int t = 0; t < NA; t++) {
    e_num[t] = e_den[t] = 0.0f;
    n_err[t] = 0;
  }
  auto flush = [&](uint32_t ff) {      // per-wave EVM partials of this frame segment
    const int t0 = opq(tid), lane = t0 & 63;
    const uint32_t ch = opq_s(chunk);
    const uint32_t jrec = blockIdx.x - pfx[ff] / ch;
    if (t0 == 0 && pfx[ff] >= i_begin)             // first workgroup of the frame
      a.nrec[ff] = (pfx[ff + 1] - 1) / ch - pfx[ff] / ch + 1;
#pragma unroll
    for (int t = 0; t < NA; t++) {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        e_num[t] += __shfl_xor(e_num[t], off);
        e_den[t] += __shfl_xor(e_den[t], off);
      }
    }
    double *ep = a.evm_part + ((((uint64_t)ff * a.max_out + jrec) * (T / 64) + wv) * NA) * 3;
    if (lane < NA * 3) {
      const int t = lane / 3, c = lane % 3;
      float v = 0.0f;
#pragma unroll
      for (int u = 0; u < NA; u++)
        if (u == t) v = c == 0 ? e_num[u] : (c == 1 ? e_den[u] : (float)n_err[u]);
      ep[lane] = (double)v;
    }
#pragma unroll
    for (int t = 0; t < NA; t++) {
      e_num[t] = e_den[t] = 0.0f;
      n_err[t] = 0;
    }
  };

  // folded CFO (a.cpe == 2): the frame's estimate nu = (eps0 + delta) / M cycles per sample
  // about its window base (fp64, from the stage partials), split into the part inside a symbol
  // body (time domain, before the transform: sample j of the body turns by exp(-j 2 pi nu j),
  // the thread's j = t0 % W8 + r W8) and the body start's phasor rot = exp(-j 2 pi nu j_s),
  // j_s = i0 + cp + s SL, computed for every symbol from the frame's 64-bit fixed-point
  // frequency (E = nu 2^64: the phase in turns is the wrapped product E j_s / 2^64, exact for
  // any j_s) -- the derotation the scratch passes of the unfolded path applied, with nothing
  // carried from symbol to symbol
  // (the thread's in-body phasor exp(-j2pi nu t0%W8) comes from an LDS table of the frame,
  // cfo_tab[n] = exp(-j2pi nu n) for n < CTN, times a wave-uniform exp(-j2pi nu CTN hi) when
  // W8 > CTN)
  // (the frame's E, i0 + cp, exp(-j2pi nu W8) and the next symbol's body-start phasor live in
  // LDS, written by thread 0: registers are the scarce resource of this kernel. The phasor of
  // symbol s is formed at the tail of symbol s - 1 (or at the start) and read at pass 0 of
  // symbol s; pass 0 ends at a barrier every wave passes before thread 0 reaches the tail, so
  // one slot serves)
  v2f cfo_hi = v2f{1.0f, 0.0f};
  auto cfo_ph = [](double cyc) {
    double p = -2.0 * cyc;
    p -= 2.0 * rint(p * 0.5);
    float sn, cs;
    sincospif((float)p, &sn, &cs);
    return v2f{cs, sn};
  };
  auto cfo_frame = [&](uint32_t ff) {
    if constexpr (CPE) {
      if (a.cpe == 2) {
        // (eps0 + delta as ls_combine_q_kernel left it: the fixed-point frequency, exact in
        // fp64 as nu = E 2^-64)
        const FrameInfo &J = a.info[ff];
        const int64_t e64 = J.cfo_E;
        const double nu = ldexp((double)e64, -64);
        // (every reader of the previous frame's table passed this symbol's barriers; the next
        // top barrier publishes the new one)
        for (int e = tid; e < CTN; e += T) cfo_tab[e] = cfo_ph(nu * (double)e);
        if constexpr (W8 > CTN) cfo_hi = uni(cfo_ph(nu * (double)((opq(tid) % W8) / CTN * CTN)));
        if (tid == 0) {
          cfo_st->E = (uint64_t)e64;
          cfo_st->j0 = (uint64_t)J.i0 + a.cp;
          cfo_st->w = cfo_ph(nu * (double)W8);
        }
      }
    }
  };
  // thread 0: the body-start phasor of symbol ss of the current frame into LDS
  auto cfo_next = [&](uint32_t ss) {
    if constexpr (CPE) {
      if (a.cpe == 2 && tid == 0) {
        const uint64_t P = cfo_st->E * (cfo_st->j0 + (uint64_t)ss * a.SL);   // turns x 2^64, wrapped
        const float turns = (float)(int32_t)(uint32_t)(P >> 32) * 0x1p-32f;   // [-1/2, 1/2)
        float sn, cs;
        sincospif(-2.0f * turns, &sn, &cs);
        cfo_st->rot = v2f{cs, sn};
      }
    }
  };
  load_w(f);
  cfo_frame(f);
  cfo_next(s);
  FrameBase fbase = frame_base(f);
  uint32_t odd = fetch(fbase, s);
  // the first symbol's staging (issued after the weight loads: the counted wait in the loop
  // assumes only stores behind the DMA)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();                                    // twiddle table and guarded staging
  DSP(unsigned long long ds_t[8] = {0, 0, 0, 0, 0, 0, 0, 0}; unsigned long long ds_c = __builtin_amdgcn_s_memtime();)
  for (uint32_t i = i_begin; i < i_end; i++) {
    // this symbol's staging has landed (the previous symbol's stores may still be in flight)
    MARK(";@@A top");
    DSP(const unsigned long long ds_0 = __builtin_amdgcn_s_memtime(); ds_t[4] += ds_0 - ds_c;)
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NSTORE) : "memory");
    __syncthreads();
    DSP(const unsigned long long ds_1 = __builtin_amdgcn_s_memtime(); ds_t[1] += ds_1 - ds_0;)
    v2f v[8];
    {
      const int t0 = opq(tid);
      if constexpr (SC16) {   // widen the wire samples as they leave the staging area
        const short2 *x = stg16 + (t0 / W8) * RS + ((odd >> (4 * (t0 / W8))) & 15u) + (t0 % W8);
        const Iq<true> cv{nullptr, a.iq_scale};
#pragma unroll
        for (int r = 0; r < 8; r++) {
          const float2 w = cv.cvt(x[r * W8]);
          v[r] = v2f{w.x, w.y};
        }
      } else {
        const v2f *x = stg + (t0 / W8) * RS + ((odd >> (4 * (t0 / W8))) & 15u) + (t0 % W8);
#pragma unroll
        for (int r = 0; r < 8; r++) v[r] = x[r * W8];
      }
    }
    uint32_t cref[(NA * S + 3) / 4];                  // reference indices, byte (t S + q)
    if constexpr (REF == 1 && !CPE) {
      const int t0 = opq(tid);
#pragma unroll
      for (int w = 0; w < (NA * S + 3) / 4; w++) cref[w] = 0;
      if constexpr (KADJ) {   // the thread's S = 2 bytes of stream t are adjacent
#pragma unroll
        for (int t = 0; t < NA; t++) {
          const int e = t * S;
          cref[e / 4] |= (uint32_t)reinterpret_cast<const uint16_t *>(rstg + t * M)[t0] << (8 * (e % 4));
        }
      } else {
#pragma unroll
        for (int t = 0; t < NA; t++)
#pragma unroll
          for (int q = 0; q < S; q++) {
            const int e = t * S + q;
            cref[e / 4] |= (uint32_t)rstg[t * M + t0 + q * T] << (8 * (e % 4));
          }
      }
    }
    if constexpr (CPE) fetch_ref(fbase, s);
    if constexpr (CPE) {
      // folded CFO: the symbol's derotation on its time samples (the body start's phasor
      // times the in-body part)
      if (a.cpe == 2) {
        v2f c = cmul_pk(cfo_tab[(opq(tid) % W8) % CTN], cfo_st->rot);
        if constexpr (W8 > CTN) c = cmul_pk(c, cfo_hi);
        const v2f cfo_w = cfo_st->w;                  // exp(-j2pi nu W8)
#pragma unroll
        for (int r = 0; r < 8; r++) {
          v[r] = cmul_pk(v[r], c);
          c = cmul_pk(c, cfo_w);
        }
      }
    }
    MARK(";@@B pass0");
    dft_fwd_pk<8>(v);
    if constexpr (WF) {     // pass 0's twiddles W_M^{nq}; c_q[n] to region (g, q)
      const uint32_t t0 = (uint32_t)opq(tid);
      const uint32_t n = t0 % MS, g = t0 / MS;
      v2f w[8];
      twiddle_powers<8>(w, twl[n]);
#pragma unroll
      for (int q = 1; q < 8; q++) v[q] = cmul_pk(v[q], w[q]);
      v2f *e = img + g * GS + (WP::X256 ? (int)n : padk<WP::PADK>((int)n));
#pragma unroll
      for (int q = 0; q < 8; q++) e[q * QS] = v[q];
    }
    __syncthreads();                                  // staging consumed by every wave
    DSP(const unsigned long long ds_2 = __builtin_amdgcn_s_memtime(); ds_t[5] += ds_2 - ds_1;)
    MARK(";@@C fetch");
    // the item after this one (uniform) and its staging, in flight during this symbol
    uint32_t fn = f, sn = s + 1, n_out_n = n_out_f;
    uint32_t odd_n = 0;
    FrameBase fbase_n = fbase;
    if (i + 1 < i_end) {
      if (sn >= n_out_f) {
        do { fn++; } while (pfx[fn + 1] == pfx[fn]);
        sn = 0;
        n_out_n = pfx[fn + 1] - pfx[fn];
        fn = __builtin_amdgcn_readfirstlane(fn);
        fbase_n = frame_base(fn);
      }
      fn = __builtin_amdgcn_readfirstlane(fn);
      sn = __builtin_amdgcn_readfirstlane(sn);
      n_out_n = __builtin_amdgcn_readfirstlane(n_out_n);
      odd_n = fetch(fbase_n, sn);
    }
    // passes 1 .. NP-1 through the LDS images (pass 1 needs no leading barrier: the previous
    // symbol's image readers finished before the barrier at the top), then the exchange that
    // leaves the spectra in natural order
    DSP(const unsigned long long ds_2b = __builtin_amdgcn_s_memtime(); ds_t[6] += ds_2b - ds_2;)
    MARK(";@@D subfft");
    if constexpr (WF) {
      // sub-transform (g, q) on lane group t0 / LG, inside one wave
      static_assert(LG % 32 == 0, "lds_pad(s + r LG) = lds_pad(s) + r (LG + LG/32)");
      static_assert(!WP::PADK || LG == 32, "pad2(s + 32 r) = pad2(s) + pad2(32 r) for s < 32");
      const uint32_t t0 = (uint32_t)opq(tid);
      const uint32_t s = t0 & (LG - 1), sg = t0 / LG;
      v2f *rg = img + (sg >> 3) * GS + (sg & 7) * QS;
      if constexpr (WP::X256) {
        sub256_fwd(rg, v, twl + WP::TW0, s);
      } else {
        const v2f *rp = rg + padk<WP::PADK>((int)s);
#pragma unroll
        for (int r = 0; r < 8; r++) v[r] = rp[WP::PADK ? pad2(r * LG) : r * (LG + LG / 32)];
        dft_fwd_pk<8>(v);
        wave_passes<LOG2M - 3, 1, WP::PADK>(rg, v, twl + WP::TW0, s);
      }
      wait_ref();
      __syncthreads();                                // every spectrum in its region

    } else {
      st_store<LOG2M, NA, 0, 0, ex_layout<PL::NP>(0)>(img, v, (uint32_t)opq(tid));
#ifndef DS_ABL_NOFFT   // timing ablation: no passes 1.. and no final exchange
      st_passes2<LOG2M, NA, 1>(img, v, twl, tid);
      {
        const uint32_t t = (uint32_t)opq(tid);
        __syncthreads();
        st_store<LOG2M, NA, PL::NP - 1>(img, v, t);
        wait_ref();
        __syncthreads();
      }
#else
      wait_ref();
      __syncthreads();
#endif
    }

    MARK(";@@E apply");
    DSP(const unsigned long long ds_3 = __builtin_amdgcn_s_memtime(); ds_t[2] += ds_3 - ds_1; ds_t[7] += ds_3 - ds_2b;)
    // apply, demap, EVM, stores: subcarriers k = tid + q T (KADJ: S tid + q) of every stream
    const uint64_t frame_id = a.frame_id0 + (fcr[f] >> 16);
    // output row (f, t, s) = ob0 + t o_ts: uniform, one 64-bit product per symbol
    const uint64_t ob0 = rfl64(((uint64_t)f * NA) * a.max_out * a.M_occ + (uint64_t)s * a.o_ss);
    // one output's apply (stream t, slot q): y = sum_r W[t][r][q] gain dn X_r
    auto apply1 = [&](int t, int q, const v2f *X) -> v2f {
      v2f acc = v2f{0.0f, 0.0f};
#pragma unroll
      for (int r = 0; r < NA; r++) acc = cmac_pk(acc, Wr[t][r][q], X[r]);
      return acc;
    };
    // demap and EVM terms of output acc (stream t, slot q, subcarrier k); returns the decision
    auto finish = [&](int t, int q, uint32_t k, v2f acc) -> uint32_t {
#ifdef DS_ABL_NODEMAP   // timing ablation: no demap / EVM
      return 0u;
#endif
      const uint32_t d = gidx[qam_level_pair_pk(acc, inv_sc, Lf, Lm1, a.qam.L)];
      uint32_t refi;
      if constexpr (REF == 1 && CPE) refi = rstg[t * M + k];
      else if constexpr (REF == 1) refi = (cref[(t * S + q) / 4] >> (8 * ((t * S + q) % 4))) & 0xFFu;
      else if constexpr (REF == 2)
        refi = (uint32_t)(hash5(a.ref_seed, DOM_DATA, frame_id, t, (uint64_t)s * a.M_occ + k) &
                          (uint64_t)(a.qam.L * a.qam.L - 1));
      else refi = d;
      // the reference point (the transmitted one: a decision error costs its distance)
      n_err[t] += (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(refi != d));
      const v2f sp = ptab[refi];
      const v2f er = acc - sp;
      e_num[t] = __builtin_fmaf(er.x, er.x, __builtin_fmaf(er.y, er.y, e_num[t]));
      e_den[t] = __builtin_fmaf(sp.x, sp.x, __builtin_fmaf(sp.y, sp.y, e_den[t]));
      return d;
    };
    // CPE: the symbol's common phase c = sum conj(Q(y)) y over every stream's outputs at the
    // subcarriers k with k even and bit 9 of k clear (per thread in stream-then-slot order, per
    // wave by a lane sum, the waves in order), then every output of the symbol turned by u =
    // conj(c) / |c| before its decision. (The bit-9 rule halves the pass on whole waves: at C3,
    // k = 2 tid, so waves w with w & 4 clear -- two of the four on each SIMD.) (Every stream: each carries its own static phase error from its column of G,
    // which one stream's estimate would impose on the others.) The even outputs are formed
    // twice -- once here for c, once in the apply below -- rather than held across the
    // workgroup reduction: the symbol's outputs and the weights do not fit the registers
    // together (the held form spilled).
    v2f u = v2f{1.0f, 0.0f};
    if constexpr (CPE) {
      v2f c = v2f{0.0f, 0.0f};
      // KADJ: k = S tid + q, even for q = 0; else k = tid + q T (T even), even on even threads
      const bool even_thread = KADJ || ((opq(tid) & 1) == 0);
      if (even_thread) {
#pragma unroll
        for (int q = 0; q < (KADJ ? 1 : S); q++) {
          const uint32_t kk = KADJ ? (uint32_t)opq(tid) * S : (uint32_t)opq(tid) + q * T;
          if ((kk >> 9) & 1u) continue;               // (uniform per wave when KADJ)
          v2f X[NA];
          if constexpr (WF) {
            const v2f *xp = img + (kk & 7u) * QS + (WP::X256 ? (int)(kk >> 3) : padk<WP::PADK>((int)(kk >> 3)));
#pragma unroll
            for (int r = 0; r < NA; r++) X[r] = xp[r * GS];
          } else {
            const v2f *xp = img + lds_pad((int)(uint32_t)opq(tid)) + q * (T + T / 32);
#pragma unroll
            for (int r = 0; r < NA; r++) X[r] = xp[r * PB];
          }
#pragma unroll
          for (int t = 0; t < NA; t++) {
            const v2f y = apply1(t, q, X);
            const v2f pt = qam_dec_point_pk(y, inv_sc, Lf, Lm1, a.qam.scale);
            c = cmac_pk(c, v2f{pt.x, -pt.y}, y);
          }
        }
      }
      c.x = wave_sum_f(c.x);
      c.y = wave_sum_f(c.y);
      if ((tid & 63) == 0) cpe_part[wv] = c;
      __syncthreads();
      c = cpe_part[0];
#pragma unroll
      for (int w = 1; w < T / 64; w++) c += cpe_part[w];
      const float m2 = c.x * c.x + c.y * c.y;
      if (m2 > 0.0f) {
        const float inv = 1.0f / sqrtf(m2);
        u = uni(v2f{c.x * inv, -c.y * inv});
      }
    }
    // one output: the apply, turned by the common phase (CPE)
    auto out1 = [&](int t, int q, const v2f *X) -> v2f {
      const v2f y = apply1(t, q, X);
      if constexpr (CPE) return cmul_pk(y, u);
      else return y;
    };
    if constexpr (KADJ) {
      // the thread's S adjacent subcarriers k = S tid + q: every antenna's X of both, then per
      // stream both outputs and one 16-byte symbol store and one 2-byte index store (per stream
      // the EVM terms accumulate in the same q order as the strided form)
      v2f X[S][NA];
      // (CPE: the q = 0 outputs of every stream first, then X of q = 1 -- X of both slots and
      // the outputs are not held together: the turned apply has fewer registers to spare)
      v2f yq0[CPE ? NA : 1];
#pragma unroll
      for (int q = 0; q < S; q++) {
        const uint32_t kk = (uint32_t)opq(tid) * S + q;
        const v2f *xp = img + (kk & 7u) * QS + (WP::X256 ? (int)(kk >> 3) : padk<WP::PADK>((int)(kk >> 3)));
#pragma unroll
        for (int r = 0; r < NA; r++) X[q][r] = xp[r * GS];
        if constexpr (CPE) {
          if (q == 0) {
#pragma unroll
            for (int t = 0; t < NA; t++) yq0[t] = out1(t, 0, X[0]);
          }
        }
      }
#pragma unroll
      for (int t = 0; t < NA; t++) {
        const uint64_t ob = ob0 + (uint64_t)t * rowstep;
        const auto osym = sgpr_ptr(reinterpret_cast<v2f *>(a.out_sym + ob));
        const auto oidx = sgpr_ptr(a.out_idx + ob);
        const uint32_t kb = (uint32_t)opq(tid) * S;
        v2f y0;
        if constexpr (CPE) y0 = yq0[t];
        else y0 = out1(t, 0, X[0]);
        const v2f y1 = out1(t, 1, X[1]);
        const uint32_t d0 = finish(t, 0, kb, y0);
        const uint32_t d1 = finish(t, 1, kb + 1, y1);
#ifndef DS_ABL_NOSTORE   // timing ablation: no symbol / index stores
        // (outputs are written once and not read back here: non-temporal stores)
        if constexpr (OUTX & 1)
          out_store<NTS>(v4f{y0.x, y0.y, y1.x, y1.y},
                                      (gptr<v4f>)((gptr<char>)osym + kb * (uint32_t)sizeof(v2f)));
        if constexpr (OUTX & 2)
          out_store<NTI>((uint16_t)(d0 | (d1 << 8)), (gptr<uint16_t>)((gptr<char>)oidx + kb));
#endif
      }
    } else {
      auto load_x = [&](int q, v2f *X) {
        if constexpr (WF) {
          const uint32_t kk = (uint32_t)opq(tid) + q * T;
          const v2f *xp = img + (kk & 7u) * QS + (WP::X256 ? (int)(kk >> 3) : padk<WP::PADK>((int)(kk >> 3)));
#pragma unroll
          for (int r = 0; r < NA; r++) X[r] = xp[r * GS];
        } else {
          const v2f *xp = img + lds_pad((int)(uint32_t)opq(tid)) + q * (T + T / 32);
#pragma unroll
          for (int r = 0; r < NA; r++) X[r] = xp[r * PB];
        }
      };
#pragma unroll
      for (int q = 0; q < S; q++) {
        const uint32_t k = (uint32_t)opq(tid) + q * T;
        v2f X[NA];
        load_x(q, X);
#pragma unroll
        for (int t = 0; t < NA; t++) {
          // uniform row bases (SGPRs): the stores take a 32-bit per-lane offset
          const uint64_t ob = ob0 + (uint64_t)t * rowstep;
          const auto osym = sgpr_ptr(reinterpret_cast<v2f *>(a.out_sym + ob));
          const auto oidx = sgpr_ptr(a.out_idx + ob);
          const v2f acc = out1(t, q, X);
          const uint32_t d = finish(t, q, k, acc);
#ifndef DS_ABL_NOSTORE   // timing ablation: no symbol / index stores
          // (OUTX: the stores the DS_ABL_NOIDX / NOSYM ablations keep, as NSTORE counts them)
          if constexpr (OUTX & 1)
            out_store<NTS>(acc, (gptr<v2f>)((gptr<char>)osym + k * (uint32_t)sizeof(v2f)));
          if constexpr (OUTX & 2) out_store<NTI>((uint8_t)d, &oidx[k]);
#endif
        }
      }
    }

    MARK(";@@F tail");
    DSP(ds_c = __builtin_amdgcn_s_memtime(); ds_t[3] += ds_c - ds_3; ds_t[0]++;)
    const bool last = (i + 1 == i_end);
    if (last || fn != f) {
      flush(f);
      if (!last) {
        n_out_f = n_out_n;
        load_w(fn);
        cfo_frame(fn);
      }
    }
    if (!last) cfo_next(sn);
    MARK(";@@G next");
    f = __builtin_amdgcn_readfirstlane(fn);
    s = __builtin_amdgcn_readfirstlane(sn);
    odd = __builtin_amdgcn_readfirstlane(odd_n);
    fbase = fbase_n;
  }
  DSP(if (a.prof && threadIdx.x == DS_PROF_TID) {
    for (int q = 0; q < 8; q++) atomicAdd(&a.prof[q], ds_t[q]);
  })
}

// ------------------------------------------------------------------------------------
// Split decode for 8x8 (C4: one symbol is 8 x 4096 x 8 B = 256 KB, more than LDS, and its
// weights are 2 MB per frame, so neither a symbol nor a frame's W fits a workgroup):
//   1. spectra_kernel: one workgroup per (frame, symbol, antenna) transforms the body in LDS
//      and writes X to a scratch laid out [frame][chunk of 64 subcarriers][symbol][antenna][64]
//      -- the apply of one chunk then reads 4 KB contiguous per symbol;
//   2. apply_split_kernel: one workgroup per (frame, chunk, symbol range) keeps W*gain*dn of
//      its 64 subcarriers in registers (wave h: outputs 2h and 2h+1, 32 VGPRs) and streams
//      the range's symbols through the 8x8 apply, demap, EVM and stores.
// Weights are read once per (chunk, range) instead of once per symbol (the per-symbol kernel
// reads 2 MB of W from L2 for every 256 KB symbol). The two kernels can alternate over groups
// of symbols (a.sym0 .. + a.sym_cap) through one scratch of that many symbols per frame, so
// that a group's spectra are read back while still in the 256 MB Infinity Cache
// (RMIMO_SPLIT_GROUP, off by default: see split_group_symbols). EVM records: symbol group x
// chunk x range per frame (nrec), NA/2 per record.
constexpr uint32_t kSplitSets = 16;   // EVM partial sets per record (<= kMaxEvmParts)
// the split decode's spectra scratch: [F][sym_cap][N][M] complex64, each (symbol, antenna)
// spectrum one contiguous row: the spectra pass writes one sequential 8 M-byte run per item
// (chunked forms [F][M / CH][sym_cap][N][CH] measured slower the smaller CH: C4 decode 1.335 /
// 1.317 / 1.290 / 1.254 ms at CH = 64 / 512 / 1024 / M, profiles/r05/ab/r05_specch.txt)
// float2 offset of subcarrier k of antenna r, scratch slot sl, frame f
MIMO_DEV uint64_t spec_off(const DecodeArgs &a, uint32_t f, uint32_t sl, uint32_t r, uint32_t k) {
  return (((uint64_t)f * a.sym_cap + sl) * a.N + r) * a.M + k;
}

template <int LOG2M, int T, bool SC16>
__global__ __launch_bounds__(T) void spectra_kernel(DecodeArgs a) {
  constexpr int M = 1 << LOG2M;
  extern __shared__ __attribute__((aligned(16))) float2 lds_sp[];
  const uint32_t f = blockIdx.y, sl = blockIdx.x, r = blockIdx.z;
  const uint32_t s = a.sym0 + sl;                     // symbol; sl its scratch slot
  const FrameInfo &I = a.info[f];
  const uint32_t n_out = (I.status == 0) ? min(I.n_sym, a.max_out) : 0u;
  if (s >= n_out) return;                             // uniform
  const int64_t abs0 = I.base + (int64_t)I.i0 + (int64_t)s * a.SL + a.cp;
  const int64_t L = (int64_t)a.frame_len;
  const auto xs = iq_row<SC16>(a.iq, a.iq_scale, ((uint64_t)I.cap * a.N + r) * a.stride);
  const int tid = threadIdx.x;
  if (abs0 >= 0 && abs0 + M <= L && xs.pair_ok() && (abs0 & 1) == 0) {
#pragma unroll
    for (int i = tid; i < M / 2; i += T) {
      const float4 v = xs.pair(abs0 + 2 * i);
      lds_sp[lds_pad(2 * i)] = make_float2(v.x, v.y);
      lds_sp[lds_pad(2 * i + 1)] = make_float2(v.z, v.w);
    }
  } else {
    for (int i = tid; i < M; i += T) {
      const int64_t n = abs0 + i;
      lds_sp[lds_pad(i)] = (n >= 0 && n < L) ? xs.at(n) : make_float2(0.0f, 0.0f);
    }
  }
  __syncthreads();
  fft_lds<LOG2M, T, 1, false>(lds_sp, a.tw);
  float2 *o = a.spec + spec_off(a, f, sl, r, 0);
#pragma unroll
  for (int k = tid; k < M; k += T) o[k] = lds_sp[lds_pad(k)];
}

// Persistent form of spectra_kernel for M = 2^LOG2M >= 2048 (C4: M = 4096): each workgroup
// walks (frame, symbol, antenna) items with a stride of the grid, the next item's body loaded
// straight into registers (PTS = 16 per thread, in the order the first radix-16 pass reads)
// while the current one is transformed (register-resident radix-16 Stockham FFT, two LDS
// exchanges, base twiddles held per thread) and stored from registers (each wave store
// instruction writes 512 contiguous bytes of one 64-subcarrier chunk). The one-item-per-
// workgroup kernel waited on its load, four global twiddle reads and its stores in turn.
template <int LOG2M, bool SC16>
__global__ __launch_bounds__((1 << LOG2M) / 16) void spectra_persist_kernel(DecodeArgs a) {
  using PL = RegPlan<LOG2M, 16>;
  constexpr int M = 1 << LOG2M, T = PL::T;
  static_assert(T % 64 == 0, "whole waves");
  extern __shared__ __attribute__((aligned(16))) float2 lds_sp[];
  v2f *buf = reinterpret_cast<v2f *>(lds_sp);
  const int tid = threadIdx.x;
  v2f w1[PL::NTW > 0 ? PL::NTW : 1];
  reg_twiddles<LOG2M, 16>(w1, a.tw, tid);
  const uint32_t NI = a.N;
  const uint64_t per_frame = (uint64_t)a.sym_cap * NI;
  const uint64_t total = per_frame * a.n_frames;
  const int64_t L = (int64_t)a.frame_len;
  // item -> (frame, scratch slot, antenna); false when its symbol is not decoded
  auto item = [&](uint64_t it, uint32_t &f, uint32_t &sl, uint32_t &r, int64_t &abs0,
                  uint32_t &cap) -> bool {
    f = (uint32_t)(it / per_frame);
    const uint32_t rem = (uint32_t)(it % per_frame);
    sl = rem / NI;
    r = rem % NI;
    const FrameInfo &I = a.info[f];
    const uint32_t n_out = (I.status == 0) ? min(I.n_sym, a.max_out) : 0u;
    abs0 = I.base + (int64_t)I.i0 + (int64_t)(a.sym0 + sl) * a.SL + a.cp;
    cap = I.cap;
    return a.sym0 + sl < n_out;
  };
  auto load = [&](v2f (&x)[16], uint32_t cap, uint32_t r, int64_t abs0) {
    const auto xs = iq_row<SC16>(a.iq, a.iq_scale, ((uint64_t)cap * a.N + r) * a.stride);
    if (abs0 >= 0 && abs0 + M <= L) {
#pragma unroll
      for (int e = 0; e < 16; e++) {
        const float2 t = xs.at(abs0 + reg_index<LOG2M, 16>(tid, e));
        x[e] = v2f{t.x, t.y};
      }
    } else {   // the capture's edge: zero outside it
#pragma unroll
      for (int e = 0; e < 16; e++) {
        const int64_t n = abs0 + reg_index<LOG2M, 16>(tid, e);
        const float2 t = xs.at(n < 0 ? 0 : (n >= L ? L - 1 : n));
        x[e] = (n >= 0 && n < L) ? v2f{t.x, t.y} : v2f{0.0f, 0.0f};
      }
    }
  };
  uint64_t it = blockIdx.x;
  uint32_t f = 0, sl = 0, r = 0, cap = 0;
  int64_t abs0 = 0;
  // the first live item of this workgroup
  while (it < total && !item(it, f, sl, r, abs0, cap)) it += gridDim.x;
  if (it >= total) return;                            // uniform
  v2f v[16], nx[16];
  load(v, cap, r, abs0);
  for (;;) {
    // the next live item's body, in flight during this transform
    uint64_t nit = it + gridDim.x;
    uint32_t nf = 0, nsl = 0, nr = 0, ncap = 0;
    int64_t nabs0 = 0;
    while (nit < total && !item(nit, nf, nsl, nr, nabs0, ncap)) nit += gridDim.x;
    if (nit < total) load(nx, ncap, nr, nabs0);
    reg_compute<LOG2M, 16, 0, false>(v, w1);
    reg_rest<LOG2M, 16, 1, false>(buf, v, w1, tid);
    // X[k], k = tid + T e, into the whole row [F][sym_cap][N][M] (spec_off)
    float2 *o = a.spec + spec_off(a, f, sl, r, 0);
#pragma unroll
    for (int e = 0; e < 16; e++) {
      const uint32_t k = (uint32_t)reg_index<LOG2M, 16>(tid, e);
      o[k] = make_float2(v[e].x, v[e].y);
    }
    if (nit >= total) break;                          // uniform
    it = nit; f = nf; sl = nsl; r = nr;
#pragma unroll
    for (int e = 0; e < 16; e++) v[e] = nx[e];
    // (reg_rest opens with a barrier: this transform's LDS readers finish before the next store)
  }
}

template <int NA, int REF>
__global__ __launch_bounds__(32 * NA) void apply_split_kernel(DecodeArgs a) {
  constexpr int T = 32 * NA;                          // NA/2 waves
  constexpr int PF = 4;                               // symbols in flight per workgroup
  static_assert(NA == 8, "one 16-byte load per thread covers a symbol's 8 x 64 spectra");
  const uint32_t c = blockIdx.x, f = blockIdx.y, part = blockIdx.z;
  const uint32_t NCH = gridDim.x, P = gridDim.z;
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t h = __builtin_amdgcn_readfirstlane((uint32_t)tid >> 6);
  __shared__ v2f ptab[kStreamMaxQam];
  __shared__ __attribute__((aligned(16))) v2f xs[2][NA * 64];    // spectra of one symbol
  __shared__ __attribute__((aligned(16))) uint8_t rs[2][NA * 64];  // its reference indices
  for (uint32_t e = tid; e < a.qam.L * a.qam.L; e += T) {
    const float2 p = qam_point(e, a.qam);
    ptab[e] = v2f{p.x, p.y};
  }
  const FrameInfo &I = a.info[f];
  const uint32_t n_out = (I.status == 0) ? min(I.n_sym, a.max_out) : 0u;
  const uint32_t grp = a.sym0 / a.sym_cap;            // this launch's symbol group
  if (grp == 0 && c == 0 && part == 0 && tid == 0)
    a.nrec[f] = a.sym_groups * NCH * P * (T / 64) / kSplitSets;
  // the group's symbols of this frame, split in P ranges
  const uint32_t ng = n_out > a.sym0 ? min(n_out - a.sym0, a.sym_cap) : 0u;
  const uint32_t s0 = a.sym0 + (uint32_t)((uint64_t)ng * part / P);
  const uint32_t s1 = a.sym0 + (uint32_t)((uint64_t)ng * (part + 1) / P);
  const uint32_t M = a.M, k = c * 64 + lane;
  v2f Wr[2][NA];
  {
    const float gk = a.gain[(uint64_t)f * M + k] * a.dn;
#pragma unroll
    for (int tt = 0; tt < 2; tt++)
#pragma unroll
      for (int r = 0; r < NA; r++) {
        const float2 w = a.W[(((uint64_t)f * NA + 2 * h + tt) * NA + r) * M + k];
        Wr[tt][r] = v2f{w.x * gk, w.y * gk};
      }
  }
  const v2f inv_sc = v2f{a.qam.inv_scale, a.qam.inv_scale};
  const v2f Lf = v2f{(float)a.qam.L, (float)a.qam.L};
  const uint32_t Lm1 = a.qam.L - 1;
  const uint64_t frame_id = a.frame_id0 + I.ref;
  // symbol s of this chunk: 4 KB at spec4 + (s - sym0) * 256 (16 B per thread), reference
  // indices of stream t at ref + t o_ts + s o_ss (16 B per thread for tid < 32)
  // (thread tid: antenna tid / 32, subcarriers c 64 + 2 (tid % 32) + 0, 1; symbols N M apart)
  const float4 *spec4 = reinterpret_cast<const float4 *>(
      a.spec + spec_off(a, f, 0, (uint32_t)tid >> 5, c * 64 + 2 * ((uint32_t)tid & 31u)));
  const uint8_t *refb = (REF == 1) ? a.ref_idx + (uint64_t)I.ref * NA * a.max_out * a.M_occ +
                                         (uint64_t)(tid >> 2) * a.o_ts + c * 64 + (tid & 3) * 16
                                   : nullptr;
  // symbols in flight: slot u holds symbol sb + u; loads are unconditional (past the range
  // they re-read the last symbol) so the slots stay in registers with counted waits
  const uint32_t slast = s1 > s0 ? s1 - 1 : s0;
  float4 pf0, pf1, pf2, pf3;                           // symbol slots (named: no scratch)
  uint4 pr0, pr1, pr2, pr3;
  auto load_sym = [&](float4 &x, uint4 &r, uint32_t s) {
    const uint32_t sc = min(s, slast);
    x = spec4[(uint64_t)(sc - a.sym0) * (NA * a.M / 2)];
    if constexpr (REF == 1)
      if (tid < 32) r = *reinterpret_cast<const uint4 *>(refb + (uint64_t)sc * a.o_ss);
  };
  if (s0 < s1) {
    load_sym(pf0, pr0, s0);
    load_sym(pf1, pr1, s0 + 1);
    load_sym(pf2, pr2, s0 + 2);
    load_sym(pf3, pr3, s0 + 3);
  }
  float e_num[2] = {0.0f, 0.0f}, e_den[2] = {0.0f, 0.0f};
  uint32_t n_err[2] = {0u, 0u};
  // one symbol: slot -> LDS, refill the slot PF symbols ahead, barrier, apply + demap + EVM
  auto one = [&](float4 &x, uint4 &r, uint32_t s, int b) {
    reinterpret_cast<float4 *>(xs[b])[tid] = x;
    if constexpr (REF == 1)
      if (tid < 32) reinterpret_cast<uint4 *>(rs[b])[tid] = r;
    load_sym(x, r, s + PF);
    __syncthreads();                                  // xs[b] complete; xs[b^1] readers done
    if (s >= s1) return;                              // uniform: the range's last block
    v2f X[NA];
#pragma unroll
    for (int q = 0; q < NA; q++) X[q] = xs[b][q * 64 + lane];
#pragma unroll
    for (int tt = 0; tt < 2; tt++) {
      const uint32_t t = 2 * h + tt;
      v2f acc = v2f{0.0f, 0.0f};
#pragma unroll
      for (int q = 0; q < NA; q++) acc = cmac_pk(acc, Wr[tt][q], X[q]);
      const uint32_t d = qam_slice_pk(acc, inv_sc, Lf, Lm1, a.qam.b);
      const uint64_t o = (uint64_t)f * NA * a.max_out * a.M_occ + t * a.o_ts + s * a.o_ss + k;
      uint32_t refi;
      if constexpr (REF == 1) refi = rs[b][t * 64 + lane];
      else if constexpr (REF == 2)
        refi = (uint32_t)(hash5(a.ref_seed, DOM_DATA, frame_id, t, (uint64_t)s * a.M_occ + k) &
                          (uint64_t)(a.qam.L * a.qam.L - 1));
      else refi = d;
      n_err[tt] += (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(refi != d));
      const v2f pt = ptab[refi];
      const v2f er = acc - pt;
      e_num[tt] = __builtin_fmaf(er.x, er.x, __builtin_fmaf(er.y, er.y, e_num[tt]));
      e_den[tt] = __builtin_fmaf(pt.x, pt.x, __builtin_fmaf(pt.y, pt.y, e_den[tt]));
#ifndef SPLIT_ABL_NOSTORE   // timing ablation: no output stores
#ifndef SPLIT_ABL_NOSYM       // (timing ablation: no symbol stores)
      if (a.out_sym) reinterpret_cast<v2f *>(a.out_sym)[o] = acc;
#endif
#ifndef SPLIT_ABL_NOIDX       // (timing ablation: no index stores)
      if (a.out_idx) a.out_idx[o] = (uint8_t)d;
#endif
#endif
    }
  };
  for (uint32_t sb = s0; sb < s1; sb += PF) {
    one(pf0, pr0, sb, 0);
    one(pf1, pr1, sb + 1, 1);
    one(pf2, pr2, sb + 2, 0);
    one(pf3, pr3, sb + 3, 1);
  }
#pragma unroll
  for (int tt = 0; tt < 2; tt++)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      e_num[tt] += __shfl_xor(e_num[tt], off);
      e_den[tt] += __shfl_xor(e_den[tt], off);
    }
  // partial set ((grp * NCH + c) * P + part) * waves + h: this wave's two streams, zeros elsewhere
  const uint64_t set = (((uint64_t)grp * NCH + c) * P + part) * (T / 64) + h;
  double *ep = a.evm_part + ((uint64_t)f * a.rec_stride * kSplitSets + set) * NA * 3;
  if (lane < NA * 3) {
    const uint32_t t = lane / 3, comp = lane % 3;
    float v = 0.0f;
#pragma unroll
    for (int tt = 0; tt < 2; tt++)
      if (t == 2 * h + tt) v = comp == 0 ? e_num[tt] : (comp == 1 ? e_den[tt] : (float)n_err[tt]);
    ep[lane] = (double)v;
  }
}

// The same 8x8 apply over 128-subcarrier chunks: wave w owns output stream w and lane l the
// adjacent subcarriers 2l, 2l+1 of the chunk, so each lane stores 16 bytes of symbols and 2 of
// indices per symbol (a wave writes 1 KB of symbols and one whole 128-byte line of indices).
// The 64-subcarrier form (apply_split_kernel, RMIMO_APPLY_V1=1) wrote 64-byte index segments:
// 98 of its 767 us at C4 x 8 went to the index stores (a store-ablation build), for 11% of
// the bytes. EVM sets: (group, chunk, range, wave), NA per record as before.
template <int NA, int REF>
__global__ __launch_bounds__(64 * NA) void apply_split2_kernel(DecodeArgs a) {
  constexpr int T = 64 * NA;                          // NA waves: one output stream each
  constexpr int PF = 4;                               // symbols in flight per workgroup
  constexpr int CW = 128;                             // subcarriers per chunk
  static_assert(NA == 8, "one 16-byte load per thread covers a symbol's 8 x 128 spectra");
  const uint32_t c2 = blockIdx.x, f = blockIdx.y, part = blockIdx.z;
  const uint32_t NCH2 = gridDim.x, P = gridDim.z;
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t w = __builtin_amdgcn_readfirstlane((uint32_t)tid >> 6);
  __shared__ v2f ptab[kStreamMaxQam];
  __shared__ __attribute__((aligned(16))) v2f xs[2][NA * CW];     // [antenna][subcarrier]
  __shared__ __attribute__((aligned(16))) uint8_t rs[2][NA * CW];   // [stream][subcarrier]
  for (uint32_t e = tid; e < a.qam.L * a.qam.L; e += T) {
    const float2 p = qam_point(e, a.qam);
    ptab[e] = v2f{p.x, p.y};
  }
  const FrameInfo &I = a.info[f];
  const uint32_t n_out = (I.status == 0) ? min(I.n_sym, a.max_out) : 0u;
  const uint32_t grp = a.sym0 / a.sym_cap;            // this launch's symbol group
  if (grp == 0 && c2 == 0 && part == 0 && tid == 0)
    a.nrec[f] = a.sym_groups * NCH2 * P * (T / 64) / kSplitSets;
  const uint32_t ng = n_out > a.sym0 ? min(n_out - a.sym0, a.sym_cap) : 0u;
  const uint32_t s0 = a.sym0 + (uint32_t)((uint64_t)ng * part / P);
  const uint32_t s1 = a.sym0 + (uint32_t)((uint64_t)ng * (part + 1) / P);
  const uint32_t M = a.M, kb = c2 * CW + 2 * lane;    // this lane's subcarriers kb, kb + 1
  v2f Wr[2][NA];
  {
    const float2 g2 = *reinterpret_cast<const float2 *>(a.gain + (uint64_t)f * M + kb);
    const float gk0 = g2.x * a.dn, gk1 = g2.y * a.dn;
#pragma unroll
    for (int r = 0; r < NA; r++) {
      const float4 wv = *reinterpret_cast<const float4 *>(a.W + (((uint64_t)f * NA + w) * NA + r) * M + kb);
      Wr[0][r] = v2f{wv.x * gk0, wv.y * gk0};
      Wr[1][r] = v2f{wv.z * gk1, wv.w * gk1};
    }
  }
  const v2f inv_sc = v2f{a.qam.inv_scale, a.qam.inv_scale};
  const v2f Lf = v2f{(float)a.qam.L, (float)a.qam.L};
  const uint32_t Lm1 = a.qam.L - 1;
  const uint64_t frame_id = a.frame_id0 + I.ref;
  // thread t loads the float4 of antenna t / 64, subcarriers c2 CW + 2 (t % 64) + 0, 1 (symbols
  // N M apart in the scratch); threads < 64 load 16 bytes of reference indices (stream t / 8,
  // bytes 16 (t % 8) ..)
  const uint32_t ant = (uint32_t)tid >> 6, pr = (uint32_t)tid & 63u;
  const float4 *spec4 = reinterpret_cast<const float4 *>(a.spec + spec_off(a, f, 0, ant, c2 * CW + 2 * pr));
  v4f *xdst0 = reinterpret_cast<v4f *>(&xs[0][ant * CW + 2 * pr]);
  v4f *xdst1 = reinterpret_cast<v4f *>(&xs[1][ant * CW + 2 * pr]);
  const uint8_t *refb = (REF == 1) ? a.ref_idx + (uint64_t)I.ref * NA * a.max_out * a.M_occ +
                                         (uint64_t)(tid >> 3) * a.o_ts + c2 * CW + (tid & 7) * 16
                                   : nullptr;
  const uint32_t slast = s1 > s0 ? s1 - 1 : s0;
  float4 pf0, pf1, pf2, pf3;                          // symbol slots (named: no scratch)
  uint4 pr0, pr1, pr2, pr3;
  auto load_sym = [&](float4 &x, uint4 &r, uint32_t s) {
    const uint32_t sc = min(s, slast);
    x = spec4[(uint64_t)(sc - a.sym0) * (NA * a.M / 2)];
    if constexpr (REF == 1)
      if (tid < 64) r = *reinterpret_cast<const uint4 *>(refb + (uint64_t)sc * a.o_ss);
  };
  if (s0 < s1) {
    load_sym(pf0, pr0, s0);
    load_sym(pf1, pr1, s0 + 1);
    load_sym(pf2, pr2, s0 + 2);
    load_sym(pf3, pr3, s0 + 3);
  }
  float e_num = 0.0f, e_den = 0.0f;
  uint32_t n_err = 0u;
  auto one = [&](float4 &x, uint4 &r, uint32_t s, int b) {
    *(b ? xdst1 : xdst0) = v4f{x.x, x.y, x.z, x.w};
    if constexpr (REF == 1)
      if (tid < 64) reinterpret_cast<uint4 *>(rs[b])[tid] = r;
    load_sym(x, r, s + PF);
    __syncthreads();                                  // xs[b] complete; xs[b^1] readers done
    if (s >= s1) return;                              // uniform: the range's last block
    v2f acc[2] = {v2f{0.0f, 0.0f}, v2f{0.0f, 0.0f}};
#pragma unroll
    for (int q = 0; q < NA; q++) {
      const v4f xv = *reinterpret_cast<const v4f *>(&xs[b][q * CW + 2 * lane]);
      acc[0] = cmac_pk(acc[0], Wr[0][q], v2f{xv.x, xv.y});
      acc[1] = cmac_pk(acc[1], Wr[1][q], v2f{xv.z, xv.w});
    }
    uint32_t d[2];
#pragma unroll
    for (int j = 0; j < 2; j++) {
      d[j] = qam_slice_pk(acc[j], inv_sc, Lf, Lm1, a.qam.b);
      uint32_t refi;
      if constexpr (REF == 1) refi = rs[b][w * CW + 2 * lane + j];
      else if constexpr (REF == 2)
        refi = (uint32_t)(hash5(a.ref_seed, DOM_DATA, frame_id, w, (uint64_t)s * a.M_occ + kb + j) &
                          (uint64_t)(a.qam.L * a.qam.L - 1));
      else refi = d[j];
      n_err += (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(refi != d[j]));
      const v2f pt = ptab[refi];
      const v2f er = acc[j] - pt;
      e_num = __builtin_fmaf(er.x, er.x, __builtin_fmaf(er.y, er.y, e_num));
      e_den = __builtin_fmaf(pt.x, pt.x, __builtin_fmaf(pt.y, pt.y, e_den));
    }
    const uint64_t o = (uint64_t)f * NA * a.max_out * a.M_occ + w * a.o_ts + s * a.o_ss + kb;
    // (plain stores: non-temporal ones measured +3.7% on this kernel at C4)
    if (a.out_sym)
      *reinterpret_cast<v4f *>(reinterpret_cast<v2f *>(a.out_sym) + o) =
          v4f{acc[0].x, acc[0].y, acc[1].x, acc[1].y};
    if (a.out_idx) *reinterpret_cast<uint16_t *>(a.out_idx + o) = (uint16_t)(d[0] | (d[1] << 8));
  };
  for (uint32_t sb = s0; sb < s1; sb += PF) {
    one(pf0, pr0, sb, 0);
    one(pf1, pr1, sb + 1, 1);
    one(pf2, pr2, sb + 2, 0);
    one(pf3, pr3, sb + 3, 1);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    e_num += __shfl_xor(e_num, off);
    e_den += __shfl_xor(e_den, off);
  }
  // partial set ((grp * NCH2 + c2) * P + part) * waves + w: this wave's stream, zeros elsewhere
  const uint64_t set = (((uint64_t)grp * NCH2 + c2) * P + part) * (T / 64) + w;
  double *ep = a.evm_part + ((uint64_t)f * a.rec_stride * kSplitSets + set) * NA * 3;
  if (lane < NA * 3) {
    const uint32_t t = lane / 3, comp = lane % 3;
    const float v = t != w ? 0.0f : (comp == 0 ? e_num : (comp == 1 ? e_den : (float)n_err));
    ep[lane] = (double)v;
  }
}

bool decode_split_accepts(const DecodeArgs &a, int log2M) {
  // (the apply reads 16 bytes of reference indices per lane)
  return a.N == 8 && a.detector != 3 && a.all_occ && log2M >= 9 && log2M <= 12 &&
         a.max_out >= (1u << log2M) / 64 && a.qam.L * a.qam.L <= kStreamMaxQam &&
         (a.ref_mode != 1 || ((uintptr_t)a.ref_idx & 15u) == 0);
}

// symbols per group: every symbol in one group (the spectra of the whole batch in the
// scratch). Infinity-Cache-sized groups (e.g. 32, compile with -DDS_SPLIT_GROUP=32) measured
// slower at C4 x 8 -- 2.10 vs 1.58 ms per decode -- because each group's apply re-reads its
// chunk's weights, 16x the weight traffic, and each launch is a quarter of the chip
uint32_t split_group_symbols(uint32_t max_out) {
#ifdef DS_SPLIT_GROUP
  const uint32_t g = DS_SPLIT_GROUP;
#else
  const uint32_t g = max_out;
#endif
  return std::max(1u, std::min(g, max_out));
}

// symbol groups, ranges per (group, chunk) and the EVM records per frame of the split decode:
// ranges of ~8 symbols (four in flight per workgroup) so that each apply launch has enough
// workgroups; records = groups * chunks * ranges * 4 waves / kSplitSets
uint32_t split_plan(uint32_t max_out, int log2M, uint32_t *groups_out, uint32_t *P_out) {
  const uint32_t NCH = (1u << log2M) / 64, cap = split_group_symbols(max_out);
  const uint32_t groups = (max_out + cap - 1) / cap;
  uint32_t P = std::max(1u, std::min(16u, cap / 8));
  while ((groups * NCH * P * 4) % kSplitSets) P++;    // whole records (NCH * 4 >= 32: P as is)
  if (groups_out) *groups_out = groups;
  if (P_out) *P_out = P;
  return groups * NCH * P * 4 / kSplitSets;
}

// workgroups of a kernel resident per CU at this block size and dynamic LDS (a persistent
// grid is that many times the CU count: no workgroup waits for another to finish)
static uint32_t resident_blocks(const void *k, int threads, size_t shm) {
  int n = 1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, threads, shm) != hipSuccess || n < 1) n = 1;
  return (uint32_t)n;
}

// 8x8 split decode; returns the partial sets per record (0: not handled)
uint32_t launch_decode_split(const DecodeArgs &a, int log2M, uint32_t n_frames, hipStream_t s) {
  if (!a.spec || !a.nrec || !decode_split_accepts(a, log2M)) return 0;
  const uint32_t NCH = a.M / 64;
  const uint32_t cap = split_group_symbols(a.max_out);
  uint32_t groups = 0, P = 0;
  if (split_plan(a.max_out, log2M, &groups, &P) > a.rec_stride) return 0;   // EVM space
  constexpr int T1 = 512;
  const size_t shm = sizeof(float2) * lds_padded_len(1 << log2M);
  DecodeArgs g = a;
  g.sym_cap = cap;
  g.sym_groups = groups;
  const dim3 g2(NCH, n_frames, P);
  for (uint32_t k = 0; k < groups; k++) {
    g.sym0 = k * cap;
    const dim3 g1(std::min(cap, a.max_out - g.sym0), n_frames, a.N);
#define SPECTRA(L2)                                                                      \
  do {                                                                                   \
    if (a.sc16) hipLaunchKernelGGL((spectra_kernel<L2, T1, true>), g1, dim3(T1), shm, s, g); \
    else hipLaunchKernelGGL((spectra_kernel<L2, T1, false>), g1, dim3(T1), shm, s, g);       \
  } while (0)
#define SPECTRA_P(L2)                                                                    \
  do {                                                                                   \
    constexpr int TP = (1 << L2) / 16;                                                   \
    auto kp = a.sc16 ? spectra_persist_kernel<L2, true> : spectra_persist_kernel<L2, false>; \
    hipLaunchKernelGGL(kp, dim3(a.n_cu * resident_blocks((const void *)kp, TP, shm)), dim3(TP), \
                       shm, s, g);                                                       \
  } while (0)
#ifdef DS_SPECTRA_ITEM   // A/B build: one workgroup per (symbol, antenna) instead of the persistent form
    constexpr bool one_item = true;
#else
    constexpr bool one_item = false;
#endif
    switch (log2M) {
      case 9: SPECTRA(9); break;
      case 10: SPECTRA(10); break;
      case 11: if (one_item) SPECTRA(11); else SPECTRA_P(11); break;
      default: if (one_item) SPECTRA(12); else SPECTRA_P(12); break;
    }
#undef SPECTRA
#undef SPECTRA_P
    // (the 128-subcarrier form stores 16 bytes of symbols and 2 of indices per lane: the
    // 64-subcarrier form takes outputs without that alignment)
    const bool v1 = ((uintptr_t)a.out_sym & 15u) || ((uintptr_t)a.out_idx & 1u);
    if (v1) {
      if (a.ref_mode == 1) hipLaunchKernelGGL((apply_split_kernel<8, 1>), g2, dim3(256), 0, s, g);
      else if (a.ref_mode == 2) hipLaunchKernelGGL((apply_split_kernel<8, 2>), g2, dim3(256), 0, s, g);
      else hipLaunchKernelGGL((apply_split_kernel<8, 0>), g2, dim3(256), 0, s, g);
    } else {
      const dim3 g3(NCH / 2, n_frames, P);
      if (a.ref_mode == 1) hipLaunchKernelGGL((apply_split2_kernel<8, 1>), g3, dim3(512), 0, s, g);
      else if (a.ref_mode == 2) hipLaunchKernelGGL((apply_split2_kernel<8, 2>), g3, dim3(512), 0, s, g);
      else hipLaunchKernelGGL((apply_split2_kernel<8, 0>), g3, dim3(512), 0, s, g);
    }
  }
  return kSplitSets;
}

// returns the EVM partial sets per record (waves per workgroup), 0 when the configuration is
// not handled here (the caller then uses the per-symbol kernels)
template <int LOG2M, int NA>
static size_t stream_lds_bytes(int ref_mode, bool sc16) {
  const bool wf = ref_mode == 1 ? (sc16 ? stream_wave_fft<LOG2M, NA, 1, true>()
                                        : stream_wave_fft<LOG2M, NA, 1, false>())
                                : (sc16 ? stream_wave_fft<LOG2M, NA, 0, true>()
                                        : stream_wave_fft<LOG2M, NA, 0, false>());
  return stream_dyn_lds<LOG2M, NA>(wf, ref_mode, sc16);
}

bool decode_stream_cpe(const DecodeArgs &a) {
  const bool outs = (a.out_sym != nullptr) == (a.out_idx != nullptr);   // both or neither
  return a.cpe && !a.sc16 && a.ref_mode == 1 && outs;
}

template <int LOG2M, int NA>
static uint32_t stream_launch(const DecodeArgs &a, hipStream_t s) {
  using PL = StreamPlan<LOG2M, NA>;
  const size_t shm = stream_lds_bytes<LOG2M, NA>(a.ref_mode, a.sc16 != 0);
  auto pick_out = [&](auto ref) -> void (*)(DecodeArgs) {
    constexpr int R = decltype(ref)::value;
    const int outs = (a.out_sym ? 1 : 0) | (a.out_idx ? 2 : 0);
    if (R == 1 && decode_stream_cpe(a)) {   // opt-in CFO path
      if constexpr (R == 1)
        return outs == 3 ? decode_stream_kernel<LOG2M, NA, 1, 3, false, true>
                         : decode_stream_kernel<LOG2M, NA, 1, 0, false, true>;
    }
    if (a.sc16) {   // sc16 wire input: every output, EVM against HBM indices or decisions
      if constexpr (R == 2) return nullptr;
      else return outs == 3 ? decode_stream_kernel<LOG2M, NA, R, 3, true> : nullptr;
    }
    switch (outs) {
      case 3: return decode_stream_kernel<LOG2M, NA, R, 3>;
      case 2: return decode_stream_kernel<LOG2M, NA, R, 2>;
      case 1: return decode_stream_kernel<LOG2M, NA, R, 1>;
      default: return decode_stream_kernel<LOG2M, NA, R, 0>;
    }
  };
  auto kern = a.ref_mode == 1 ? pick_out(std::integral_constant<int, 1>{})
            : a.ref_mode == 2 ? pick_out(std::integral_constant<int, 2>{})
                              : pick_out(std::integral_constant<int, 0>{});
  if (!kern) return 0;
  if (hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)shm) != hipSuccess)
    return 0;
  int per_cu = 1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, PL::T, shm) != hipSuccess ||
      per_cu < 1)
    per_cu = 1;
  const uint32_t grid = a.n_cu * (uint32_t)per_cu;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(PL::T), shm, s, a);
  return PL::T / 64;
}

static bool stream_geometry_ok(const DecodeArgs &a, int log2M, uint32_t n_frames) {
  // (capture and reference row of a frame are packed in 16 bits each in LDS)
  if (a.detector == 3 || !a.all_occ || n_frames > kStreamMaxFrames ||
      a.n_caps > 0xFFFFu || a.n_refs > 0xFFFFu ||
      a.qam.L * a.qam.L > kStreamMaxQam)
    return false;
  if (a.ref_mode == 1 && ((uintptr_t)a.ref_idx & 15u)) return false;
  // 32-bit DMA offsets within one frame's antennas and one frame's reference rows
  if ((uint64_t)a.N * a.stride * sizeof(float2) >= (1ull << 32) ||
      (uint64_t)a.N * a.max_out * a.M_occ >= (1ull << 32))
    return false;
  return (a.N == 4 && (log2M == 11 || log2M == 10)) ||
         (a.N == 2 && (log2M == 12 || log2M == 11 || log2M == 10));
}

bool decode_stream_accepts(const DecodeArgs &a, int log2M, uint32_t n_frames) {
  if (!stream_geometry_ok(a, log2M, n_frames)) return false;
  return !a.sc16 || (a.ref_mode != 2 && a.out_sym && a.out_idx);
}

uint32_t launch_decode_stream(const DecodeArgs &a, int log2M, uint32_t n_frames, hipStream_t s) {
  if (!a.nrec || !decode_stream_accepts(a, log2M, n_frames)) return 0;
  if (a.N == 4 && log2M == 11) return stream_launch<11, 4>(a, s);
  if (a.N == 4 && log2M == 10) return stream_launch<10, 4>(a, s);
  if (a.N == 2 && log2M == 12) return stream_launch<12, 2>(a, s);
  if (a.N == 2 && log2M == 11) return stream_launch<11, 2>(a, s);
  if (a.N == 2 && log2M == 10) return stream_launch<10, 2>(a, s);
  return 0;
}

}  // namespace mimo

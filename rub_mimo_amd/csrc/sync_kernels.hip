// rub_mimo_amd/csrc/sync_kernels.hip -- Schmidl-Cox timing metric and plateau rule on gfx950.
//
// Reference: framesync::execute_sc_sync (framing.cc:591-637), a per-sample state machine:
//   p[n] = conj(x[n-M/2]) x[n]  (wdelaycf read-before-push, lag M/2)
//   P[n] = -sum_{M/2} p          (firfilt_crcf, taps -1)
//   R[n] = 0.5 sum_M |x|^2       (firfilt_rrrf, taps 0.5)
//   y[n] = |P|^2 / R^2 ;  plateau: y > 0.95 run with end - start > cp on every antenna;
//   sync_index = floor(sum of run starts / N).
//
// GPU form (throughput, not a per-sample scan). A persistent grid pulls (frame, chunk) items
// from a queue in chunk-major order. An item is kScSpan = 16384 positions: a halo of
// H >= cp+2 positions (run history) and K = kScSpan - H candidate positions. For each antenna
// the workgroup streams the item through an LDS ring of M + 4096 samples (coalesced 16-byte
// loads, the next 4096 samples in flight while the current ones are processed); thread t
// owns 16 consecutive positions per 4096-sample iteration. With the window sums written as
// running differences,
//   P[n] = P[n-1] + p[n] - p[n-M/2],   2R[n] = 2R[n-1] + |x[n]|^2 - |x[n-M]|^2,
// each thread sums its segment's differences, one block scan (fp64) gives every segment its
// starting sums, and the thread walks its 16 positions. The decision is division-free:
// |P|^2 - thr R^2 against band * R^2.
//
// Exactness. Samples whose fp64 metric lies within the band of the threshold -- or whose
// window energy is tiny next to the energy streamed so far, where fp64 cancellation could
// matter -- are provisionally 1 and recomputed exactly as the CPU oracle does (sequential fp32
// sums oldest->newest, no FMA: this file is compiled with -ffp-contract=off) once the item
// still has a candidate. A sequential fp32 sum of M terms is within (M-1)u of the exact
// value, so |y32 - y_exact| <= ~4e-4 for M <= 2048; a 2e-3 band keeps every
// plateau decision -- hence plateau start/end and sync_index -- bit-identical to the oracle.
// An all-zero window (R = 0, the oracle's 0/0) is tracked exactly with a nonzero count.
//
// "Run of cp+2 ones ending at n" is a last-zero prefix max (block scan per iteration).
// Antennas are processed in order and the item stops as soon as no position can still
// qualify on every antenna (provisional ones only enlarge that set, so the early-out is
// safe); noise and data regions cost one antenna, not N. The first qualifying n is
// atomicMin'ed into trig[frame] and the item records each antenna's run start from its LDS
// bits; plateau_kernel completes a run that began before the halo with an exact backward
// scan. Items beyond a frame's current trigger are skipped; results never depend on
// dispatch order (an item is skipped only when a smaller trigger already exists, and the
// kept candidate is the global minimum).
#include <algorithm>
#include <cstdio>

#include "kernels.hpp"

#pragma clang fp contract(off)

// cycle counters of the item kernel (build with -DMIMO_SC_PROFILE and run with RMIMO_SC_PROF=1)
#ifdef MIMO_SC_PROFILE
#define SC_PROF(...) __VA_ARGS__
#else
#define SC_PROF(...)
#endif

namespace mimo {

constexpr int kScT = kScThreads;        // threads per workgroup
constexpr int kScS = 16;                // consecutive positions per thread per iteration
constexpr int kScIt = kScT * kScS;      // 4096 positions per iteration
constexpr int kScIters = kScSpan / kScIt;
constexpr int kAmbMax = kScAmbMax;      // provisional samples per item
static_assert(kScIt == kScIterLen, "iteration length");
constexpr int kResGroup = kScT / 2;     // samples per resolve pass (two lanes each)
constexpr int kResWin = 4;              // resolve workgroups per (item, antenna): windows in parallel
static_assert(kScSpan % kScIt == 0, "item span");

// LDS ring slot -> padded float2 index: 2 float2 of padding per 32 keeps the 16-byte reads
// of 16 consecutive threads (16 positions apart) on distinct banks
MIMO_DEV int ring_pad(int i) { return i + ((i >> 5) << 1); }

// exact restatement of framing.cc:626-637 under the pinned liquid semantics, on the M
// samples s[i] = x[n - M + 1 + i] (LDS). The three accumulation chains are interleaved for
// latency; each keeps its own oldest -> newest order.
MIMO_DEV float sc_exact_lds(const float2 *s, int M) {
  constexpr int U = 8;                 // M/2 is a multiple of 32 for every supported M
  const int M2 = M / 2;
  float Pr = 0.0f, Pi = 0.0f, R = 0.0f;
  float2 d[U], v[U], u[2 * U];         // the next block's operands load while this one sums
#pragma unroll
  for (int k = 0; k < U; k++) { d[k] = s[k]; v[k] = s[M2 + k]; }
#pragma unroll
  for (int k = 0; k < 2 * U; k++) u[k] = s[k];
  for (int j = 0; j < M2; j += U) {
    float2 dc[U], vc[U], uc[2 * U];
#pragma unroll
    for (int k = 0; k < U; k++) { dc[k] = d[k]; vc[k] = v[k]; }
#pragma unroll
    for (int k = 0; k < 2 * U; k++) uc[k] = u[k];
    if (j + U < M2) {
#pragma unroll
      for (int k = 0; k < U; k++) { d[k] = s[j + U + k]; v[k] = s[M2 + j + U + k]; }
#pragma unroll
      for (int k = 0; k < 2 * U; k++) u[k] = s[2 * (j + U) + k];
    }
#pragma unroll
    for (int k = 0; k < U; k++) {      // P: k' = n - M/2 + 1 + j + k
      float pr = dc[k].x * vc[k].x - (-dc[k].y) * vc[k].y;
      float pi = dc[k].x * vc[k].y + (-dc[k].y) * vc[k].x;
      Pr = Pr + (-1.0f) * pr;
      Pi = Pi + (-1.0f) * pi;
      float z0 = uc[2 * k].x * uc[2 * k].x + uc[2 * k].y * uc[2 * k].y;   // R: i = 2(j+k)
      R = R + 0.5f * z0;
      float z1 = uc[2 * k + 1].x * uc[2 * k + 1].x + uc[2 * k + 1].y * uc[2 * k + 1].y;
      R = R + 0.5f * z1;
    }
  }
  return (Pr * Pr + Pi * Pi) / (R * R);
}

// the same straight from global memory (one lane; list overflow and the rare backward scan)
template <bool S>
MIMO_DEV float sc_exact(const Iq<S> x, int64_t n, int64_t M) {
  const int64_t M2 = M / 2;
  float Pr = 0.0f, Pi = 0.0f, R = 0.0f;
  for (int64_t k = n - M2 + 1; k <= n; k++) {
    float2 d = (k - M2 >= 0) ? x.at(k - M2) : make_float2(0.0f, 0.0f);
    float2 v = (k >= 0) ? x.at(k) : make_float2(0.0f, 0.0f);
    float pr = d.x * v.x - (-d.y) * v.y;
    float pi = d.x * v.y + (-d.y) * v.x;
    Pr = Pr + (-1.0f) * pr;
    Pi = Pi + (-1.0f) * pi;
  }
  for (int64_t k = n - M + 1; k <= n; k++) {
    float2 v = (k >= 0) ? x.at(k) : make_float2(0.0f, 0.0f);
    float z = v.x * v.x + v.y * v.y;
    R = R + 0.5f * z;
  }
  return (Pr * Pr + Pi * Pi) / (R * R);
}
MIMO_DEV float sc_exact(const float2 *__restrict__ x, int64_t n, int64_t M) {
  return sc_exact(Iq<false>{x}, n, M);
}


// a double moved across lanes by one DPP control (both halves; lanes with no source, or in a
// row the row mask leaves out, read 0.0)
template <int CTRL, int ROWS = 0xF>
MIMO_DEV double dpp_f64(double x) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), CTRL, ROWS, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), CTRL, ROWS, 0xF, true);
  return __hiloint2double(hi, lo);
}

// wave-inclusive scan of NV doubles on the DPP path (row_shr 1, 2, 4, 8 within rows of 16,
// then row_bcast 15 and 31 across rows): VALU moves, no LDS round trip per step as the
// ds_bpermute of __shfl_up
template <int NV>
MIMO_DEV void wave_scan_f64(double (&x)[NV]) {
#pragma unroll
  for (int k = 0; k < NV; k++) x[k] += dpp_f64<0x111>(x[k]);
#pragma unroll
  for (int k = 0; k < NV; k++) x[k] += dpp_f64<0x112>(x[k]);
#pragma unroll
  for (int k = 0; k < NV; k++) x[k] += dpp_f64<0x114>(x[k]);
#pragma unroll
  for (int k = 0; k < NV; k++) x[k] += dpp_f64<0x118>(x[k]);
#pragma unroll
  for (int k = 0; k < NV; k++) x[k] += dpp_f64<0x142, 0xA>(x[k]);
#pragma unroll
  for (int k = 0; k < NV; k++) x[k] += dpp_f64<0x143, 0xC>(x[k]);
}

// block-wide exclusive scan of NV doubles plus the block totals (one barrier; the caller
// alternates ws between consecutive scans)
template <int NV>
MIMO_DEV void block_scan(double (&v)[NV], double (&tot)[NV], double (*ws)[kScT / 64]) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double inc[NV];
#pragma unroll
  for (int k = 0; k < NV; k++) inc[k] = v[k];
  wave_scan_f64<NV>(inc);
  if (lane == 63) {
#pragma unroll
    for (int k = 0; k < NV; k++) ws[k][wv] = inc[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; k++) {
    double o = 0.0, t = 0.0;
#pragma unroll
    for (int w = 0; w < kScT / 64; w++) {
      const double u = ws[k][w];
      if (w < wv) o += u;
      t += u;
    }
    v[k] = o + (inc[k] - v[k]);
    tot[k] = t;
  }
}

// "run of cp+2 ones ends at n" for the 16 positions sb..sb+15 of this thread. carry is the
// last zero before the iteration (block-uniform, updated to the last zero through it).
MIMO_DEV uint32_t run_cond(uint32_t bits, int64_t sb, long long &carry, int64_t cp,
                           long long *red) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t inv = ~bits & 0xFFFFu;
  const long long lz = inv ? (long long)(sb + 31 - __clz(inv)) : -1;
  long long inc = lz;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const long long o = __shfl_up(inc, off);
    if (lane >= off && o > inc) inc = o;
  }
  long long ex = __shfl_up(inc, 1);
  if (lane == 0) ex = -1;
  if (lane == 63) red[wv] = inc;
  __syncthreads();
  long long before = carry, all = carry;
#pragma unroll
  for (int w = 0; w < kScT / 64; w++) {
    const long long u = red[w];
    if (w < wv && u > before) before = u;
    if (u > all) all = u;
  }
  if (ex > before) before = ex;
  uint32_t cond = 0;
  if (cp + 2 > kScS) {
    // a zero inside the segment is < cp+2 positions back, so only the leading run of ones
    // (bits 0..i all set) can qualify, and only where the last zero before it is old enough
    const uint32_t lead = bits & ~(bits + 1u) & 0xFFFFu;
    const long long i0 = before + cp + 2 - sb;
    cond = i0 <= 0 ? lead : (i0 >= kScS ? 0u : lead & ~((1u << i0) - 1u));
  } else {
#pragma unroll
    for (int i = 0; i < kScS; i++) {
      const uint32_t m = inv & ((2u << i) - 1u);
      const long long lzv = m ? (long long)(sb + 31 - __clz(m)) : before;
      if (lzv <= sb + i - cp - 2) cond |= 1u << i;
    }
  }
  carry = all;
  return cond;
}

// sequential fp32 sum q[0] + q[1] + ... + q[n-1], in that order. Scalar head up to 16-byte
// alignment, then 16-byte reads with the next 16 terms in flight while 16 are added (the
// dependent-add latency, ~7 cycles on gfx950, is the bound: ~9 cycles per term measured).
// Sequential fp32 sums in the oracle's order, oldest -> newest, from an LDS table. The chain
// of dependent adds is the critical path, so the table reads run three 16-term blocks ahead
// (the loop is unrolled by three so the blocks rotate through fixed registers; a read past the
// last block is clamped onto it and never consumed).
MIMO_DEV float seq_sum(const float *q, int n) {
  float acc = 0.0f;
  const int h = min(n, (int)((4u - (((uint32_t)(uintptr_t)q >> 2) & 3u)) & 3u));
  for (int k = 0; k < h; k++) acc = acc + q[k];
  const float4 *qa = reinterpret_cast<const float4 *>(q + h);
  const int m = n - h, nb = m >> 4;
  if (nb > 0) {
    auto ld = [&](float4 (&d)[4], int b) {
      const int bb = b < nb ? b : nb - 1;
#pragma unroll
      for (int i = 0; i < 4; i++) d[i] = qa[4 * bb + i];
    };
    auto add = [&](const float4 (&d)[4]) {
#pragma unroll
      for (int i = 0; i < 4; i++) {
        acc = acc + d[i].x; acc = acc + d[i].y; acc = acc + d[i].z; acc = acc + d[i].w;
      }
    };
    float4 A[4], B[4], C[4];
    ld(A, 0); ld(B, 1); ld(C, 2);
    int b = 0;
    for (; b + 3 <= nb; b += 3) {
      add(A); ld(A, b + 3);
      add(B); ld(B, b + 4);
      add(C); ld(C, b + 5);
    }
    if (b < nb) add(A);
    if (b + 1 < nb) add(B);
  }
  for (int k = h + 16 * nb; k < n; k++) acc = acc + q[k];
  return acc;
}

// two interleaved sequential sums over complex terms (the .x and .y chains), same scheme
MIMO_DEV float2 seq_sum2(const float2 *q, int n) {
  float ax = 0.0f, ay = 0.0f;
  const int h = min(n, (int)((((uint32_t)(uintptr_t)q) >> 3) & 1u));
  for (int k = 0; k < h; k++) { ax = ax + q[k].x; ay = ay + q[k].y; }
  const float4 *qa = reinterpret_cast<const float4 *>(q + h);
  const int m = n - h, nb = m >> 3;
  if (nb > 0) {
    auto ld = [&](float4 (&d)[4], int b) {
      const int bb = b < nb ? b : nb - 1;
#pragma unroll
      for (int i = 0; i < 4; i++) d[i] = qa[4 * bb + i];
    };
    auto add = [&](const float4 (&d)[4]) {
#pragma unroll
      for (int i = 0; i < 4; i++) {
        ax = ax + d[i].x; ay = ay + d[i].y; ax = ax + d[i].z; ay = ay + d[i].w;
      }
    };
    float4 A[4], B[4], C[4];
    ld(A, 0); ld(B, 1); ld(C, 2);
    int b = 0;
    for (; b + 3 <= nb; b += 3) {
      add(A); ld(A, b + 3);
      add(B); ld(B, b + 4);
      add(C); ld(C, b + 5);
    }
    if (b < nb) add(A);
    if (b + 1 < nb) add(B);
  }
  for (int k = h + 8 * nb; k < n; k++) { ax = ax + q[k].x; ay = ay + q[k].y; }
  return make_float2(ax, ay);
}

// two consecutive samples (q even), zero outside [0, L)
template <bool S>
MIMO_DEV float4 ld_pair(const Iq<S> x, int64_t q, int64_t L, bool vec) {
  if (vec && q >= 0 && q + 1 < L) return x.pair(q);
  const float2 v0 = (q >= 0 && q < L) ? x.at(q) : make_float2(0.0f, 0.0f);
  const float2 v1 = (q + 1 >= 0 && q + 1 < L) ? x.at(q + 1) : make_float2(0.0f, 0.0f);
  return make_float4(v0.x, v0.y, v1.x, v1.y);
}
MIMO_DEV float4 ld_pair(const float2 *__restrict__ x, int64_t q, int64_t L, bool vec) {
  return ld_pair(Iq<false>{x}, q, L, vec);
}

// one iteration's 4096 samples from q0 into registers, 16 bytes per lane, when the block is
// inside [0, L) (block-uniform); otherwise false and the ring is filled by guarded loads
template <bool S>
MIMO_DEV bool fetch_block(float4 (&pre)[kScIt / (2 * kScT)], const Iq<S> x,
                          int64_t q0, int64_t L, bool vec) {
  const bool ok = vec && q0 >= 0 && q0 + kScIt <= L;
  const int64_t p0 = (ok ? q0 : 0) + 2 * (int64_t)threadIdx.x;
  // one branch around all loads (a per-element select makes hipcc wait for each load in turn)
  if (ok) {
#pragma unroll
    for (int j = 0; j < kScIt / (2 * kScT); j++) pre[j] = x.pair(p0 + 2 * kScT * j);
  } else {
#pragma unroll
    for (int j = 0; j < kScIt / (2 * kScT); j++) pre[j] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  }
  return ok;
}
MIMO_DEV bool fetch_block(float4 (&pre)[kScIt / (2 * kScT)], const float2 *__restrict__ x,
                          int64_t q0, int64_t L, bool vec) {
  return fetch_block(pre, Iq<false>{x}, q0, L, vec);
}

// conj(d) * v, the oracle's operation order
MIMO_DEV float2 cj_mul(float2 d, float2 v) {
  return make_float2(d.x * v.x - (-d.y) * v.y, d.x * v.y + (-d.y) * v.x);
}

// the recompute tables of one window: tz[i] = 0.5 |x[q0+i]|^2, tp[i] = -conj(x[q0+i-M/2]) x[q0+i]
// (the oracle's tap products, same fp32 operations). Loads are unconditional from clamped
// addresses and masked afterwards: a per-element "load or zero" select makes hipcc branch
// around each load and wait for it before the next (one memory latency per element);
// kTabU iterations' loads are in flight together
constexpr int kTabU = 8;
MIMO_DEV void table_fill(const float2 *__restrict__ x, int64_t q0, int64_t L, int RL, int WCAP,
                         float *tz, float2 *tp) {
  const int tid = threadIdx.x;
  for (int i0 = 0; i0 < WCAP; i0 += kScT * kTabU) {
    float2 v[kTabU], dd[kTabU];
#pragma unroll
    for (int u = 0; u < kTabU; u++) {
      const int64_t k = q0 + i0 + u * kScT + tid, kd = k - RL;
      v[u] = x[k < 0 ? 0 : (k >= L ? L - 1 : k)];
      dd[u] = x[kd < 0 ? 0 : (kd >= L ? L - 1 : kd)];
    }
#pragma unroll
    for (int u = 0; u < kTabU; u++) {
      const int i = i0 + u * kScT + tid;
      const int64_t k = q0 + i, kd = k - RL;
      const float2 vv = (k >= 0 && k < L) ? v[u] : make_float2(0.0f, 0.0f);
      const float2 dv = (kd >= 0 && kd < L) ? dd[u] : make_float2(0.0f, 0.0f);
      if (i < WCAP) {
        float z = vv.x * vv.x + vv.y * vv.y;
        tz[i] = 0.5f * z;
        const float2 pp = cj_mul(dv, vv);
        tp[i] = make_float2((-1.0f) * pp.x, (-1.0f) * pp.y);
      }
    }
  }
}

struct ResolveLds {            // LDS scratch of the exact recompute
  unsigned long long key;
  int ng;
  int res_i[kResGroup];
  float res_v[3][kResGroup];
};

// Exact fp32 recompute of the pending samples pos[i] (antenna ant[i]; pos0 keeps the
// positions, pos[i] becomes -1 once taken), a batch per (antenna, table window). The oracle's
// per-sample terms -pr, -pi (P taps -1) and 0.5|x|^2 (R taps 0.5) are tabled once per window
// with the same fp32 operations; each sample's three sequential sums then run on two lanes
// (R; Pr and Pi interleaved), oldest -> newest exactly as framing.cc:626-637 under the pinned
// liquid semantics. A sample whose exact metric fails the threshold clears its bit in wbits
// ([antenna][iteration][thread] x 16 bits, LDS or global).
MIMO_DEV void resolve_pending(const ScArgs &a, uint32_t f, int64_t w0, long long *pos,
                              const long long *pos0, const uint8_t *ant, int namb,
                              uint16_t *wbits, unsigned char *tables, int table_bytes,
                              ResolveLds &rl) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int M = (int)a.M, RL = M / 2;
  const int64_t L = (int64_t)a.frame_len;
  const int WCAP = (table_bytes / 12) & ~3;
  float *tz = reinterpret_cast<float *>(tables);
  float2 *tp = reinterpret_cast<float2 *>(tables + sizeof(float) * WCAP);
  for (;;) {
    if (tid == 0) { rl.key = ~0ull; rl.ng = 0; }
    __syncthreads();
    for (int i = tid; i < namb; i += kScT)
      if (pos[i] >= 0)
        atomicMin(&rl.key, ((unsigned long long)ant[i] << 48) | (unsigned long long)pos[i]);
    __syncthreads();
    const unsigned long long key = rl.key;
    if (key == ~0ull) break;   // block-uniform
    const int s = (int)(key >> 48);
    const int64_t nmin = (int64_t)(key & ((1ull << 48) - 1));
    const int64_t q0 = nmin - M + 1;       // table index i <-> sample q0 + i
    const float2 *__restrict__ x = a.iq + ((uint64_t)f * a.N + s) * a.stride;
    table_fill(x, q0, L, RL, WCAP, tz, tp);
    // this window's samples (at most kResGroup per pass; the rest wait for the next pass)
    for (int i = tid; i < namb; i += kScT) {
      const int64_t n = pos[i];
      if (n >= 0 && ant[i] == s && n - nmin <= WCAP - M) {
        const int g = atomicAdd(&rl.ng, 1);
        if (g < kResGroup) { rl.res_i[g] = i; pos[i] = -1; }
      }
    }
    __syncthreads();
    const int ng = rl.ng < kResGroup ? rl.ng : kResGroup;
    if (a.prof && tid == 0) {                     // diagnostics (RMIMO_SC_PROF=1)
      atomicAdd(&a.prof[17], 1ull);
      atomicAdd(&a.prof[19], (unsigned long long)ng);
    }
    {
      const int g = lane + 64 * (wv >> 1);
      if (g < ng) {
        const int r = (int)(pos0[rl.res_i[g]] - nmin);
        if ((wv & 1) == 0) {          // R over i = r .. r + M - 1
          rl.res_v[0][g] = seq_sum(tz + r, M);
        } else {                      // P over i = r + M/2 .. r + M - 1
          const float2 P = seq_sum2(tp + r + RL, RL);
          rl.res_v[1][g] = P.x;
          rl.res_v[2][g] = P.y;
        }
      }
    }
    __syncthreads();
    if (tid < ng) {
      const float Pr = rl.res_v[1][tid], Pi = rl.res_v[2][tid], R = rl.res_v[0][tid];
      const float y32 = (Pr * Pr + Pi * Pi) / (R * R);
      if (!((double)y32 > a.thr)) {
        const int64_t o = pos0[rl.res_i[tid]] - w0;
        const int it = (int)(o / kScIt), t = (int)((o % kScIt) / kScS);
        const int bit = (int)(o % kScS) + 16 * (t & 1);
        uint32_t *w32 = reinterpret_cast<uint32_t *>(wbits) + ((s * kScIters + it) * kScT + t) / 2;
        atomicAnd(w32, ~(1u << bit));
      }
    }
    __syncthreads();
  }
}

// Exact fp32 recompute of one window's samples sorted[0 .. cnt) of antenna s (ascending,
// sorted[cnt-1] - sorted[0] <= WCAP - M): the same table and chains as resolve_pending, for a
// window chosen by the caller, so that the windows of one antenna run in parallel workgroups
MIMO_DEV void resolve_window(const ScArgs &a, uint32_t f, int64_t w0, int s,
                             const long long *sorted, int cnt, uint16_t *wbits,
                             unsigned char *tables, int table_bytes, ResolveLds &rl) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int M = (int)a.M, RL = M / 2;
  const int64_t L = (int64_t)a.frame_len;
  const int WCAP = (table_bytes / 12) & ~3;
  float *tz = reinterpret_cast<float *>(tables);
  float2 *tp = reinterpret_cast<float2 *>(tables + sizeof(float) * WCAP);
  const int64_t nmin = sorted[0];
  const int64_t q0 = nmin - M + 1;         // table index i <-> sample q0 + i
  const float2 *__restrict__ x = a.iq + ((uint64_t)f * a.N + s) * a.stride;
  table_fill(x, q0, L, RL, WCAP, tz, tp);
  __syncthreads();
  {
    const int g = lane + 64 * (wv >> 1);
    if (g < cnt) {
      const int r = (int)(sorted[g] - nmin);
      if ((wv & 1) == 0) {          // R over i = r .. r + M - 1
        rl.res_v[0][g] = seq_sum(tz + r, M);
      } else {                      // P over i = r + M/2 .. r + M - 1
        const float2 P = seq_sum2(tp + r + RL, RL);
        rl.res_v[1][g] = P.x;
        rl.res_v[2][g] = P.y;
      }
    }
  }
  __syncthreads();
  if (tid < cnt) {
    const float Pr = rl.res_v[1][tid], Pi = rl.res_v[2][tid], R = rl.res_v[0][tid];
    const float y32 = (Pr * Pr + Pi * Pi) / (R * R);
    if (!((double)y32 > a.thr)) {
      const int64_t o = sorted[tid] - w0;
      const int it = (int)(o / kScIt), t = (int)((o % kScIt) / kScS);
      const int bit = (int)(o % kScS) + 16 * (t & 1);
      uint32_t *w32 = reinterpret_cast<uint32_t *>(wbits) + ((s * kScIters + it) * kScT + t) / 2;
      atomicAnd(w32, ~(1u << bit));
    }
  }
  __syncthreads();
}

// plateau rule for antennas [0, n_done) from their words into acond (candidates only in
// [c0, cend)); returns the block-wide OR of the surviving bits
MIMO_DEV int item_conditions(const uint16_t *wbits, uint16_t (*acond)[kScT], uint32_t n_done,
                             int64_t w0, int64_t c0, int64_t cend, int64_t cp,
                             long long (*run_ws)[kScT / 64], int &par) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int it = 0; it < kScIters; it++) acond[it][tid] = 0xFFFFu;
  for (uint32_t s = 0; s < n_done; s++) {
    long long carry = w0 - 1;
#pragma unroll 1
    for (int it = 0; it < kScIters; it++) {
      const int64_t sb = w0 + (int64_t)it * kScIt + kScS * tid;
      const uint32_t bits = wbits[((int)s * kScIters + it) * kScT + tid];
      par ^= 1;
      const uint32_t cond = run_cond(bits, sb, carry, cp, run_ws[par]);
      const int64_t lo = c0 - sb, hi = cend - sb;
      uint32_t mask = 0;
      if (hi > 0 && lo < kScS) {
        const int l = lo < 0 ? 0 : (int)lo, u = hi > kScS ? kScS : (int)hi;
        mask = ((1u << u) - 1u) & ~((1u << l) - 1u);
      }
      acond[it][tid] = (uint16_t)(acond[it][tid] & cond & mask);
    }
  }
  int surv = 0;
#pragma unroll
  for (int it = 0; it < kScIters; it++) surv |= (acond[it][tid] != 0);
  return __syncthreads_or(surv);
}

// item_conditions for cp + 2 > kScS without block scans: only a thread whose 16 positions are
// ones on every antenna can hold a candidate, and for it the last zero before its segment is
// found by walking the antenna's words backwards -- at most ~(cp + 2) / 16 words: a longer run
// of ones qualifies whatever lies further back. The walk stops at the item start, which counts
// as a zero (item_conditions' carry = w0 - 1), so the result equals run_cond's leading-run
// branch bit for bit.
MIMO_DEV int item_conditions_walk(const uint16_t *wbits, uint16_t (*acond)[kScT], uint32_t n_done,
                                  int64_t w0, int64_t c0, int64_t cend, int64_t cp) {
  const int tid = threadIdx.x;
  int surv = 0;
#pragma unroll 1
  for (int it = 0; it < kScIters; it++) {
    const int64_t sb = w0 + (int64_t)it * kScIt + kScS * tid;
    const int64_t lo = c0 - sb, hi = cend - sb;
    uint32_t mask = 0;
    if (hi > 0 && lo < kScS) {
      const int l = lo < 0 ? 0 : (int)lo, u = hi > kScS ? kScS : (int)hi;
      mask = ((1u << u) - 1u) & ~((1u << l) - 1u);
    }
    uint32_t all = mask;
    for (uint32_t s = 0; s < n_done; s++) all &= wbits[((int)s * kScIters + it) * kScT + tid];
    uint32_t cond = 0;
    if (all) {
      cond = all;
      for (uint32_t s = 0; s < n_done && cond; s++) {
        const uint32_t bits = wbits[((int)s * kScIters + it) * kScT + tid];
        const uint32_t lead = bits & ~(bits + 1u) & 0xFFFFu;
        int64_t before = w0 - 1;
        int wt = tid, wi = it;
        for (;;) {
          if (--wt < 0) {
            wt = kScT - 1;
            if (--wi < 0) break;
          }
          const int64_t wsb = w0 + (int64_t)wi * kScIt + kScS * wt;
          const uint32_t z = ~(uint32_t)wbits[((int)s * kScIters + wi) * kScT + wt] & 0xFFFFu;
          if (z) { before = wsb + 31 - __clz(z); break; }
          if (sb - wsb > cp + 2) { before = wsb - 1; break; }
        }
        const int64_t i0 = before + cp + 2 - sb;
        cond &= i0 <= 0 ? lead : (i0 >= kScS ? 0u : lead & ~((1u << i0) - 1u));
      }
    }
    acond[it][tid] = (uint16_t)cond;
    surv |= (cond != 0);
  }
  return __syncthreads_or(surv);
}

// first qualifying position -> the chunk's record (run starts from the words) and trig[f].
// s_min must be ~0 on entry.
MIMO_DEV void item_record(const ScArgs &a, uint32_t f, uint64_t chunk, int64_t w0,
                          const uint16_t *wbits, const uint16_t (*acond)[kScT],
                          const long long *lo_s, unsigned long long &s_min) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
#pragma unroll
  for (int it = 0; it < kScIters; it++) {
    const uint32_t v = acond[it][tid];
    if (v)
      atomicMin(&s_min, (unsigned long long)(w0 + (int64_t)it * kScIt + kScS * tid +
                                             __ffs((int)v) - 1));
  }
  __syncthreads();
  const unsigned long long cand = s_min;
  if (cand == ~0ull) return;
  ScRecord *rec = a.rec + (uint64_t)f * a.rec_stride + chunk;
  if (wv == 0) {   // run start: one past the last zero below the candidate
    bool found = false;
    if (lane < (int)a.N) {
      const int s = lane;
      const int64_t o = (int64_t)cand - w0;
      int it = (int)(o / kScIt), t = (int)((o % kScIt) / kScS);
      const int i = (int)(o % kScS);
      uint32_t m = ~(uint32_t)wbits[(s * kScIters + it) * kScT + t] & ((1u << i) - 1u);
      while (!m) {   // rare: only for a candidate item
        if (--t < 0) { t = kScT - 1; if (--it < 0) break; }
        m = ~(uint32_t)wbits[(s * kScIters + it) * kScT + t] & 0xFFFFu;
      }
      const long long lzv =
          m ? (long long)(w0 + (int64_t)it * kScIt + kScS * t + 31 - __clz(m)) : -1;
      found = lzv >= lo_s[s];    // a computed zero, not the evaluation boundary
      // found: the run start; otherwise where plateau_kernel's exact backward scan begins
      rec->start[s] = found ? (unsigned long long)(lzv + 1) : (unsigned long long)lo_s[s];
    }
    const unsigned long long fm = __ballot(found);
    if (lane == 0) {
      rec->found = (uint32_t)fm;
      rec->n_cand = cand;
      rec->pos0 = w0;
      atomicMin(&a.trig[f], cand);
      if (a.cand) a.cand[(uint64_t)f * a.nchunks + chunk] = cand;
    }
  }
}

__global__ __launch_bounds__(kScT) __attribute__((amdgpu_waves_per_eu(2))) void sc_kernel(ScArgs a, uint32_t n_frames) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sc_dyn[];
  const int M = (int)a.M, RL = M / 2, RING = M + kScIt;
  float2 *ring = reinterpret_cast<float2 *>(sc_dyn);
  // provisional plateau bits, [antenna][iteration][thread] x 16
  uint16_t *wbits = reinterpret_cast<uint16_t *>(sc_dyn + sizeof(float2) * ring_pad(RING));
  __shared__ uint16_t acond[kScIters][kScT];
  __shared__ double scan_ws[2][5][kScT / 64];
  __shared__ long long run_ws[2][kScT / 64];
  __shared__ unsigned long long s_trig, s_min;
  __shared__ uint32_t s_item;
  __shared__ long long amb_n[kAmbMax];     // -1 once taken by a resolve pass
  __shared__ long long amb_pos[kAmbMax];
  __shared__ uint8_t amb_s[kAmbMax];
  __shared__ int s_namb;
  __shared__ uint32_t s_slot;
  __shared__ ResolveLds rl;
  __shared__ long long s_lo[kMaxStreams];
  __shared__ unsigned long long s_smin, s_smax;

  const int tid = threadIdx.x;
  const int64_t L = (int64_t)a.frame_len, cp = a.cp;
  const int64_t K = (int64_t)a.chunk_len, H = (int64_t)kScSpan - K;
  const uint64_t total = (a.chunk_hi - a.chunk_lo) * n_frames;
  int par = 0;
    SC_PROF(if (a.prof && tid == 0) atomicMin(&a.prof[8], (unsigned long long)wall_clock64());)

  for (;;) {
    if (tid == 0) s_item = atomicAdd(a.queue, 1u);
    __syncthreads();
    const uint64_t item = s_item;
    if (item >= total) {
    SC_PROF(if (a.prof && tid == 0) atomicMax(&a.prof[9], (unsigned long long)wall_clock64());)
      break;
    }
    const uint32_t f = (uint32_t)(item % n_frames);
    const uint64_t chunk = a.chunk_lo + item / n_frames;
    const int64_t c0 = (int64_t)chunk * K;
    if (tid == 0) {
      s_trig = __hip_atomic_load(&a.trig[f], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_min = ~0ull;
      s_namb = 0;
    }
#pragma unroll
    for (int it = 0; it < kScIters; it++) acond[it][tid] = 0xFFFFu;
    __syncthreads();
    if (c0 >= L || (!a.no_skip && s_trig < (unsigned long long)c0)) {  // an earlier trigger exists
    SC_PROF(if (a.prof && tid == 0) atomicAdd(&a.prof[6], 1ull);)
      continue;
    }
    SC_PROF(const long long t_item = clock64();)
    SC_PROF(const long long w_item = wall_clock64();)
    SC_PROF(long long t_rows = 0, t_words = 0, t_ph[5] = {0, 0, 0, 0, 0};)
    const int64_t w0 = c0 - H;                 // first evaluated position
    const int64_t cend = std::min<int64_t>(c0 + K, L);
    int any = 1;
    uint32_t n_done = 0;
    // antenna 0 evaluates the whole item; antenna s > 0 only the iterations covering the
    // survivors of antennas < s (and their cp+2 run history): a plateau region is short
    int it_lo = 0, it_hi = kScIters - 1;

    for (uint32_t s = 0; s < a.N && any; s++) {
    SC_PROF(const long long t_r0 = clock64();)
      const float2 *__restrict__ x = a.iq + ((uint64_t)f * a.N + s) * a.stride;
      const bool vec = ((uintptr_t)x & 15u) == 0;
      const int64_t ib_lo = w0 + (int64_t)it_lo * kScIt;   // first evaluated position
      if (tid == 0) s_lo[s] = ib_lo;
      for (int it = 0; it < kScIters; it++)
        if (it < it_lo || it > it_hi) {
          acond[it][tid] = 0;
          wbits[((int)s * kScIters + it) * kScT + tid] = 0;
        }
      // history [ib_lo - M, ib_lo) -> its ring slots; the first block in flight behind it
      const int wb = (kScIt * it_lo) % RING;
      for (int j = tid; 2 * j < M; j += kScT) {
        int sl = wb + 2 * j;
        if (sl >= RING) sl -= RING;
        *reinterpret_cast<float4 *>(ring + ring_pad(sl)) = ld_pair(x, ib_lo - M + 2 * j, L, vec);
      }
      float4 pre[kScIt / (2 * kScT)];
      bool pf = fetch_block(pre, x, ib_lo, L, vec);
      __syncthreads();
      // window sums ending at ib_lo - 1: P over the last M/2, 2R and the nonzero count over M
      double c[4] = {0.0, 0.0, 0.0, 0.0}, t4[4], tot[5];
      for (int k = tid; k < M; k += kScT) {
        int sl = wb + k;
        if (sl >= RING) sl -= RING;
        const float2 v = ring[ring_pad(sl)];
        const float z = v.x * v.x + v.y * v.y;
        c[2] += (double)z;
        c[3] += (z != 0.0f) ? 1.0 : 0.0;
        if (k >= RL) {
          int sd = sl - RL;
          if (sd < 0) sd += RING;
          const float2 pp = cj_mul(ring[ring_pad(sd)], v);
          c[0] += (double)pp.x;
          c[1] += (double)pp.y;
        }
      }
      block_scan<4>(c, t4, scan_ws[par]);
    SC_PROF(long long t_m = clock64();)
    SC_PROF(t_ph[0] += t_m - t_r0;)
      par ^= 1;
      double Pc_re = t4[0], Pc_im = t4[1], Zc = t4[2], Cc = t4[3], Ac = t4[2];
      long long carry = ib_lo - 1;             // the evaluation boundary reads as a zero

#pragma unroll 1
      for (int it = it_lo; it <= it_hi; it++) {
        const int64_t ib = w0 + (int64_t)it * kScIt;
        {
          const int slot = (M + it * kScIt) % RING + 2 * tid;
          if (pf) {
#pragma unroll
            for (int j = 0; j < kScIt / (2 * kScT); j++) {
              int sl = slot + 2 * kScT * j;
              if (sl >= RING) sl -= RING;
              *reinterpret_cast<float4 *>(ring + ring_pad(sl)) = pre[j];
            }
          } else {   // frame edges: guarded loads straight into the ring
#pragma unroll 1
            for (int j = 0; j < kScIt / (2 * kScT); j++) {
              int sl = slot + 2 * kScT * j;
              if (sl >= RING) sl -= RING;
              *reinterpret_cast<float4 *>(ring + ring_pad(sl)) =
                  ld_pair(x, ib + 2 * (tid + kScT * j), L, vec);
            }
          }
        }
        __syncthreads();
        if (it + 1 <= it_hi) pf = fetch_block(pre, x, ib + kScIt, L, vec);
        const float2 *xn = ring + ring_pad((M + it * kScIt + kScS * tid) % RING);
        const float2 *xr = ring + ring_pad((RL + it * kScIt + kScS * tid) % RING);
        const float2 *xm = ring + ring_pad((it * kScIt + kScS * tid) % RING);
        // phase A: this segment's sum of window differences
        // (plus |dP| and lagged-energy sums that bound y over the segment)
        double d[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
        float bp = 0.0f, bz = 0.0f;
        int dc = 0;
#pragma unroll 2
        for (int i = 0; i < kScS; i += 2) {
          const float4 vn = *reinterpret_cast<const float4 *>(xn + i);
          const float4 vr = *reinterpret_cast<const float4 *>(xr + i);
          const float4 vm = *reinterpret_cast<const float4 *>(xm + i);
#pragma unroll
          for (int h = 0; h < 2; h++) {
            const float2 n_ = h ? make_float2(vn.z, vn.w) : make_float2(vn.x, vn.y);
            const float2 r_ = h ? make_float2(vr.z, vr.w) : make_float2(vr.x, vr.y);
            const float2 m_ = h ? make_float2(vm.z, vm.w) : make_float2(vm.x, vm.y);
            const float2 pn = cj_mul(r_, n_), pl = cj_mul(m_, r_);
            const float zn = n_.x * n_.x + n_.y * n_.y, zl = m_.x * m_.x + m_.y * m_.y;
            const double zn64 = (double)zn;
            d[0] += (double)pn.x - (double)pl.x;
            d[1] += (double)pn.y - (double)pl.y;
            d[2] += zn64 - (double)zl;
            d[4] += zn64;
            dc += (zn != 0.0f ? 1 : 0) - (zl != 0.0f ? 1 : 0);
            bp += (fabsf(pn.x) + fabsf(pn.y)) + (fabsf(pl.x) + fabsf(pl.y));
            bz += zl;
          }
        }
        d[3] = (double)dc;
        SC_PROF({ const long long t2 = clock64(); t_ph[1] += t2 - t_m; t_m = t2; })
        block_scan<5>(d, tot, scan_ws[par]);
        SC_PROF({ const long long t2 = clock64(); t_ph[2] += t2 - t_m; t_m = t2; })
        par ^= 1;
        // phase B: walk the segment
        double Pre = Pc_re + d[0], Pim = Pc_im + d[1], Z = Zc + d[2], C = Cc + d[3];
        const double Aend = Ac + tot[4];       // energy streamed through this iteration
        const double zfloor = 1e-6 * Aend;
        const int64_t sb = ib + kScS * tid;
        uint32_t bits = 0, ovf = 0;
        // Every n of the segment has |P[n]| <= |P_s| + bp and 2R[n] >= Z_s - bz. If that bound
        // keeps y below thr - 2*band everywhere (and the fp64 sums are far from cancellation),
        // all 16 decisions are 0 and the walk is skipped -- the common case away from a sync.
        bool walk = true;
        {
          const double pmax = sqrt(Pre * Pre + Pim * Pim) + 1.001 * (double)bp;
          const double rmin = 0.5 * (Z - 1.001 * (double)bz);
          if (rmin > 0.0 && Z > 16.0 * zfloor && pmax * pmax < (a.thr - 2.0 * a.band) * (rmin * rmin))
            walk = false;
        }
#pragma unroll 1
        for (int i = 0; walk && i < kScS; i += 2) {   // rare: near a plateau
          const float4 vn = *reinterpret_cast<const float4 *>(xn + i);
          const float4 vr = *reinterpret_cast<const float4 *>(xr + i);
          const float4 vm = *reinterpret_cast<const float4 *>(xm + i);
#pragma unroll
          for (int h = 0; h < 2; h++) {
            const float2 n_ = h ? make_float2(vn.z, vn.w) : make_float2(vn.x, vn.y);
            const float2 r_ = h ? make_float2(vr.z, vr.w) : make_float2(vr.x, vr.y);
            const float2 m_ = h ? make_float2(vm.z, vm.w) : make_float2(vm.x, vm.y);
            const float2 pn = cj_mul(r_, n_), pl = cj_mul(m_, r_);
            const float zn = n_.x * n_.x + n_.y * n_.y, zl = m_.x * m_.x + m_.y * m_.y;
            Pre += (double)pn.x - (double)pl.x;
            Pim += (double)pn.y - (double)pl.y;
            Z += (double)zn - (double)zl;
            C += ((zn != 0.0f) ? 1.0 : 0.0) - ((zl != 0.0f) ? 1.0 : 0.0);
            const int64_t n = sb + i + h;
            bool b = false;
            if (n >= 0 && n < L && C > 0.5) {
              const double R = 0.5 * Z, R2 = R * R;
              const double q = Pre * Pre + Pim * Pim - a.thr * R2;
              if (fabs(q) <= a.band * R2 || Z <= zfloor) {
                const int slot = atomicAdd(&s_namb, 1);
                if (slot < kAmbMax) {
                  amb_n[slot] = n;
                  amb_pos[slot] = n;
                  amb_s[slot] = (uint8_t)s;
                  b = true;
                } else {
                  ovf |= 1u << (i + h);   // list full: this lane recomputes it below
                }
              } else {
                b = q > 0.0;
              }
            }
            bits |= (b ? 1u : 0u) << (i + h);
          }
        }
        while (ovf) {   // overflow of the provisional list (pathological input): exact here
          const int i = __ffs((int)ovf) - 1;
          ovf &= ovf - 1u;
          if (!((double)sc_exact(x, sb + i, a.M) > a.thr)) bits &= ~(1u << i);
          if (a.n_exact) atomicAdd(a.n_exact, 1ull);
        }
        Pc_re += tot[0]; Pc_im += tot[1]; Zc += tot[2]; Cc += tot[3]; Ac = Aend;
        wbits[((int)s * kScIters + it) * kScT + tid] = (uint16_t)bits;
        SC_PROF({ const long long t2 = clock64(); t_ph[3] += t2 - t_m; t_m = t2; })
        const uint32_t cond = run_cond(bits, sb, carry, cp, run_ws[par]);
        // candidates only inside [c0, cend)
        const int64_t lo = c0 - sb, hi = cend - sb;
        uint32_t mask = 0;
        if (hi > 0 && lo < kScS) {
          const int l = lo < 0 ? 0 : (int)lo, u = hi > kScS ? kScS : (int)hi;
          mask = ((1u << u) - 1u) & ~((1u << l) - 1u);
        }
        acond[it][tid] = (uint16_t)(acond[it][tid] & cond & mask);
        SC_PROF({ const long long t2 = clock64(); t_ph[4] += t2 - t_m; t_m = t2; })
      }
    SC_PROF(const long long t_r1 = clock64();)
    SC_PROF(t_rows += t_r1 - t_r0;)
      if (tid == 0) { s_smin = ~0ull; s_smax = 0ull; }
      __syncthreads();
      {
        uint64_t lo = ~0ull, hi = 0ull;
#pragma unroll
        for (int it = 0; it < kScIters; it++) {
          const uint32_t v = acond[it][tid];
          if (v) {
            const uint64_t base = (uint64_t)(w0 + (int64_t)it * kScIt + kScS * tid);
            lo = std::min<uint64_t>(lo, base + __ffs((int)v) - 1);
            hi = std::max<uint64_t>(hi, base + 31 - __clz(v));
          }
        }
        if (lo != ~0ull) { atomicMin(&s_smin, (unsigned long long)lo); atomicMax(&s_smax, (unsigned long long)hi); }
      }
      __syncthreads();
      any = (s_smin != ~0ull) ? 1 : 0;
      if (any) {
        const int64_t ra = (int64_t)s_smin - cp - 2, rb = (int64_t)s_smax;
        it_lo = (int)std::max<int64_t>(0, (ra - w0) / kScIt);
        it_hi = (int)std::min<int64_t>(kScIters - 1, (rb - w0) / kScIt);
      }
      n_done = s + 1;
    SC_PROF(t_words += clock64() - t_r1;)
    }

    const int namb = s_namb < kAmbMax ? s_namb : kAmbMax;
    SC_PROF(const long long t_res0 = clock64();)
    if (any && namb > 0) {
      if (a.n_exact && tid == 0) atomicAdd(a.n_exact, (unsigned long long)namb);
      // hand the item to the hot-item kernels (every antenna's windows resolve in parallel);
      // resolve here only when the hot buffer is full
      if (tid == 0) s_slot = a.hot ? atomicAdd(a.hot_count, 1u) : ~0u;
      __syncthreads();
      if (s_slot < a.hot_cap) {
        ScHot *hp = a.hot + s_slot;
        if (tid == 0) {
          hp->f = f; hp->n_done = n_done; hp->namb = (uint32_t)namb;
          hp->chunk = chunk; hp->c0 = c0; hp->w0 = w0; hp->cend = cend;
        }
        if (tid < (int)n_done) hp->lo[tid] = s_lo[tid];
        for (int i = tid; i < namb; i += kScT) { hp->amb_n[i] = amb_pos[i]; hp->amb_s[i] = amb_s[i]; }
        uint32_t *dst = reinterpret_cast<uint32_t *>(hp->wbits);
        const uint32_t *src = reinterpret_cast<const uint32_t *>(wbits);
        for (int i = tid; i < (int)n_done * kScIters * kScT / 2; i += kScT) dst[i] = src[i];
        any = 0;
      } else {
        resolve_pending(a, f, w0, amb_n, amb_pos, amb_s, namb, wbits, sc_dyn,
                        (int)(sizeof(float2) * ring_pad(RING)), rl);
        any = item_conditions(wbits, acond, n_done, w0, c0, cend, cp, run_ws, par);
      }
    }
#ifdef MIMO_SC_PROFILE
    if (a.prof && tid == 0) {
      const long long t_end = clock64();
      atomicAdd(&a.prof[0], 1ull);
      atomicAdd(&a.prof[1], (unsigned long long)n_done);
      atomicAdd(&a.prof[2], (unsigned long long)t_rows);
      atomicAdd(&a.prof[3], (unsigned long long)t_words);
      for (int k = 0; k < 5; k++) atomicAdd(&a.prof[12 + k], (unsigned long long)t_ph[k]);
      atomicAdd(&a.prof[4], (unsigned long long)(t_end - t_res0));
      atomicAdd(&a.prof[5], (unsigned long long)(t_end - t_item));
      const long long w_end = wall_clock64();
      atomicAdd(&a.prof[7], (unsigned long long)(w_end - w_item));
      atomicMax(&a.prof[10], (unsigned long long)(w_end - w_item));
      atomicMax(&a.prof[11], (unsigned long long)w_item);
    }
#endif
    if (any) item_record(a, f, chunk, w0, wbits, acond, s_lo, s_min);
    __syncthreads();
  }
}

// hot items, stage 1: one workgroup per (item, antenna) resolves that antenna's pending samples
// against the capture and clears the failing bits of the item's saved plateau words
__global__ __launch_bounds__(kScT) void sc_resolve_kernel(ScArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char tables[];
  __shared__ long long pos[kAmbMax], sorted[kAmbMax];
  __shared__ int wstart[kAmbMax + 1];
  __shared__ ResolveLds rl;
  __shared__ int s_n, s_nw;
  const uint32_t s = blockIdx.y;
  const int tid = threadIdx.x;
  const int table_bytes = (int)(sizeof(float2) * ring_pad((int)a.M + kScIt));
  const int WCAP = (table_bytes / 12) & ~3;
  const uint32_t count = min(*a.hot_count, a.hot_cap);
  for (uint32_t h = blockIdx.x; h < count; h += gridDim.x) {
    ScHot *hp = a.hot + h;
    if (s >= hp->n_done) continue;
    if (tid == 0) s_n = 0;
    __syncthreads();
    const int namb = (int)min(hp->namb, (uint32_t)kAmbMax);
    for (int i = tid; i < namb; i += kScT)
      if (hp->amb_s[i] == s) pos[atomicAdd(&s_n, 1)] = hp->amb_n[i];
    __syncthreads();
    const int n = s_n;
    if (n == 0) continue;                          // block-uniform
    if (tid == 0 && a.n_exact && blockIdx.z == 0) atomicAdd(a.n_exact, (unsigned long long)n);
    // ascending order (positions of one antenna are distinct), then greedy windows: a window
    // opens at its smallest sample and takes the next ones within WCAP - M, at most kResGroup;
    // every workgroup of this (item, antenna) derives the same windows and takes every
    // gridDim.z-th of them
    for (int i = tid; i < n; i += kScT) {
      int rank = 0;
      for (int j = 0; j < n; j++) rank += (pos[j] < pos[i]) ? 1 : 0;
      sorted[rank] = pos[i];
    }
    __syncthreads();
    if (tid == 0) {
      int nw = 0, k = 0;
      while (k < n) {
        wstart[nw++] = k;
        const long long lo = sorted[k];
        int e = k + 1;
        while (e < n && e - k < kResGroup && sorted[e] - lo <= (long long)(WCAP - (int)a.M)) e++;
        k = e;
      }
      wstart[nw] = n;
      s_nw = nw;
    }
    __syncthreads();
    const int nw = s_nw;
    for (int w = (int)blockIdx.z; w < nw; w += (int)gridDim.z)
      resolve_window(a, hp->f, hp->w0, (int)s, sorted + wstart[w], wstart[w + 1] - wstart[w],
                     hp->wbits, tables, table_bytes, rl);
    __syncthreads();
  }
}

// hot items, stage 2: plateau rule on the corrected words, candidate, record, trigger
__global__ __launch_bounds__(kScT) void sc_finalize_kernel(ScArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t wb[kMaxStreams * kScIters * kScT];
  __shared__ uint16_t acond[kScIters][kScT];
  __shared__ long long run_ws[2][kScT / 64];
  __shared__ long long lo[kMaxStreams];
  __shared__ unsigned long long s_min;
  const uint32_t count = min(*a.hot_count, a.hot_cap);
  for (uint32_t h = blockIdx.x; h < count; h += gridDim.x) {
    const ScHot *hp = a.hot + h;
    const uint32_t n_done = hp->n_done;
    const uint32_t *src = reinterpret_cast<const uint32_t *>(hp->wbits);
    uint32_t *dst = reinterpret_cast<uint32_t *>(wb);
    for (int i = threadIdx.x; i < (int)n_done * kScIters * kScT / 2; i += kScT) dst[i] = src[i];
    if (threadIdx.x < n_done) lo[threadIdx.x] = hp->lo[threadIdx.x];
    if (threadIdx.x == 0) s_min = ~0ull;
    __syncthreads();
    int par = 0;
    const int any = item_conditions(wb, acond, n_done, hp->w0, hp->c0, hp->cend,
                                    (int64_t)a.cp, run_ws, par);
    if (any) item_record(a, hp->f, hp->chunk, hp->w0, wb, acond, lo, s_min);
    __syncthreads();
  }
}

// run starts of trigger n on capture cap (its chunk's record rec), none earlier than `floor`:
// the record's run starts where the chunk saw the run begin, otherwise an exact backward scan
// (64 positions per step, the oracle's fp32 metric). Returns true when a run reaches below
// floor > 0, i.e. began before the re-arm point of a stream frame.
template <bool S>
MIMO_DEV bool trigger_run_starts(const PlateauArgs &a, uint32_t cap, const ScRecord &rec,
                                 int64_t floor, int64_t (&st)[kMaxStreams]) {
  const int lane = threadIdx.x & 63;
  bool spans = false;
  for (uint32_t s = 0; s < a.N; s++) {
    int64_t start = floor;
    if (rec.found & (1u << s)) {
      start = (int64_t)rec.start[s];
    } else {
      // every computed sample of the chunk's range is in the run: walk back exactly
      const auto x = iq_row<S>(a.iq, a.iq_scale, ((uint64_t)cap * a.N + s) * a.stride);
      bool hit = false;
      for (int64_t q0 = (int64_t)rec.start[s] - 1; q0 >= floor; q0 -= 64) {
        const int64_t q = q0 - lane;
        bool zero = false;
        if (q >= floor) zero = !((double)sc_exact(x, q, a.M) > a.thr);
        const unsigned long long bal = __ballot(zero);
        if (bal) {
          const int l = __ffsll((long long)bal) - 1;   // lowest lane = highest position
          start = q0 - l + 1;
          hit = true;
          break;
        }
      }
      if (!hit && floor > 0) spans = true;
    }
    if (start < floor) {
      start = floor;
      spans = true;
    }
    st[s] = start;
  }
  return spans;
}

// A framesync started at capture sample `origin` that triggers at n with run starts st
// (framing.cc:612-623): sync index, window base, completeness and num_samples_processed, all
// relative to origin as that framesync counts them; FrameInfo keeps absolute positions.
// Uniform on every lane; lane 0 writes. Returns the status.
// the fields the estimation stages fill in later (weights_kernel, the CFO stages): zero until
// then, so a frame they skip reports zeros, not the slot's previous contents
MIMO_DEV void frame_clear_estimates(FrameInfo &I) {
  I.noise_var = 0.0f;
  I.i0 = 0;
  I.cfo_eps = 0.0f;
  I.cfo_E = 0;
}

MIMO_DEV int frame_from_trigger(const PlateauArgs &a, FrameInfo &I, uint32_t cap, uint32_t ref,
                                int64_t origin, int64_t n, const int64_t (&st)[kMaxStreams],
                                bool need_base_in_view, uint64_t &nsp_rel) {
  const int lane = threadIdx.x & 63;
  const int64_t L_rel = (int64_t)a.frame_len - origin;
  uint64_t sum = 0;
  for (uint32_t s = 0; s < a.N; s++) sum += (uint64_t)(st[s] - origin);
  const int64_t sync_rel = (int64_t)(sum / a.N);           // framing.cc:618-620
  const int64_t base_rel = sync_rel - (int64_t)a.SL;       // window start
  const int64_t n_e = base_rel + (int64_t)a.win_len;       // estimate_channel runs at this sample
  int status;
  if (need_base_in_view && base_rel < 0) {
    // the fresh framesync's window would hold zeros before the re-arm point, the capture
    // holds real samples there: resume this frame as a fresh capture instead
    status = 3;   // MIMO_FRAME_RESCAN
    nsp_rel = 0;
  } else if (n_e < L_rel) {
    status = 0;
    nsp_rel = (uint64_t)((n_e + 1 < L_rel) ? n_e + 2 : n_e + 1);
  } else {
    status = 2;   // MIMO_FRAME_INCOMPLETE: still saving access codes
    nsp_rel = (uint64_t)L_rel;
  }
  if (lane == 0) {
    I.status = status;
    I.trigger = (uint64_t)n;
    I.sync_index = (uint64_t)(origin + sync_rel);
    I.base = origin + base_rel;
    I.nsp = nsp_rel;
    I.origin = (uint64_t)origin;
    I.cap = cap;
    I.ref = ref;
    if (status != 0) I.n_sym = 0;
    frame_clear_estimates(I);
    for (uint32_t s = 0; s < a.N; s++) {
      I.plateau_start[s] = (uint64_t)st[s];
      I.plateau_end[s] = (uint64_t)n;
    }
  }
  return status;
}

// The plateau rule run exactly from a re-arm point: positions [r, end) of every antenna, 64
// at a time (the oracle's fp32 metric per lane), then the per-sample state machine of
// framing.cc:601-623 over the ballots with in_plateau false at r. For chunks whose recorded
// (first) candidate precedes r -- frames shorter than a chunk -- so its cost is bounded by a
// chunk of small-M work. Returns the trigger (-1: none before end) and the run starts.
template <bool S>
MIMO_DEV int64_t forward_trigger(const PlateauArgs &a, uint32_t cap, int64_t r, int64_t end,
                                 int64_t (&st)[kMaxStreams]) {
  const int lane = threadIdx.x & 63;
  int64_t ps[kMaxStreams], pe[kMaxStreams];
  bool in[kMaxStreams];
  for (uint32_t s = 0; s < a.N; s++) { ps[s] = pe[s] = r; in[s] = false; }
  for (int64_t q0 = r; q0 < end; q0 += 64) {
    unsigned long long bal[kMaxStreams];
    for (uint32_t s = 0; s < a.N; s++) {
      const auto x = iq_row<S>(a.iq, a.iq_scale, ((uint64_t)cap * a.N + s) * a.stride);
      const int64_t q = q0 + lane;
      const bool b = q < end && (double)sc_exact(x, q, a.M) > a.thr;
      bal[s] = __ballot(b);
    }
    const int cnt = (int)((end - q0) < 64 ? (end - q0) : 64);
    for (int i = 0; i < cnt; i++) {
      const int64_t n = q0 + i;
      bool proceed = true;
      for (uint32_t s = 0; s < a.N; s++) {
        if ((bal[s] >> i) & 1ull) {
          if (in[s]) pe[s] = n;
          else { in[s] = true; ps[s] = n; pe[s] = n; }
        } else {
          in[s] = false;
        }
        proceed = proceed && in[s] && (pe[s] - ps[s] > (int64_t)(a.SL - a.M));   // > cp_len
      }
      if (proceed) {
        for (uint32_t s = 0; s < a.N; s++) st[s] = ps[s];
        return n;
      }
    }
  }
  return -1;
}

MIMO_DEV void frame_empty(FrameInfo &I, int status, uint32_t cap, uint32_t ref, int64_t origin,
                          uint64_t nsp_rel) {
  I.status = status;
  I.trigger = ~0ull;
  I.nsp = nsp_rel;
  I.n_sym = 0;
  I.sync_index = 0;
  I.base = 0;
  I.origin = (uint64_t)origin;
  I.cap = cap;
  I.ref = ref;
  frame_clear_estimates(I);
  for (uint32_t s = 0; s < kMaxStreams; s++) {
    I.plateau_start[s] = 0;
    I.plateau_end[s] = 0;
  }
}

// one frame per capture: run starts (from the trigger chunk's record, exact backward scan
// where the run began before that chunk's halo), sync index, completeness
template <bool S>
__global__ __launch_bounds__(64) void plateau_kernel(PlateauArgs a) {
  const uint32_t f = blockIdx.x;
  FrameInfo &I = a.info[f];
  const unsigned long long n = a.trig[f];
  if (n == ~0ull) {
    if (threadIdx.x == 0) frame_empty(I, 1, f, f, 0, a.frame_len);   // MIMO_FRAME_NO_SYNC
    return;
  }
  const ScRecord &rec = a.rec[(uint64_t)f * a.rec_stride + n / a.chunk_len];
  int64_t st[kMaxStreams];
  (void)trigger_run_starts<S>(a, f, rec, 0, st);
  uint64_t nsp;
  (void)frame_from_trigger(a, I, f, f, 0, (int64_t)n, st, false, nsp);
}

// ---- back-to-back frames in one capture (stream re-arm) ------------------------------------
// The reference's framesync stops at STATE_MIMO (framing.cc:494-496) and reset() only rewinds
// the state (:461-464). A stream of frames is received here as a caller of that API would:
// after a frame, a fresh framesync takes the remaining samples, starting at origin
// r_{k+1} = r_k + get_num_samples_processed(). Frame k's S&C therefore runs with zero filter
// history before r_k. The S&C kernels compute the metric with the capture's real history; the
// two agree at every n >= r_k + M - 1, and the walk takes frame k's trigger as the first chunk
// candidate at or after r_k. That is exact when, over Z_k = [r_k, r_k + M - 1), neither metric
// has a sample above the threshold on any antenna -- then every run counted after r_k starts
// past Z_k in both. stream_cert_kernel proves that per (frame, antenna) in fp64 with a margin
// over the fp32 error band; a frame it cannot prove, or one whose run or window reaches
// before r_k, is reported MIMO_FRAME_RESCAN (the caller resumes that capture at r_k as a
// fresh capture) and the slots after it MIMO_FRAME_NONE.
template <bool S>
__global__ __launch_bounds__(64) void stream_walk_kernel(PlateauArgs a) {
  const uint32_t cap = blockIdx.x;
  const int lane = threadIdx.x;
  const int64_t K = (int64_t)a.chunk_len;
  const unsigned long long *cand = a.cand + (uint64_t)cap * a.nchunks;
  FrameInfo *slot = a.info + (uint64_t)cap * a.fpc;
  const uint64_t *rs = a.ref_starts ? a.ref_starts + (uint64_t)cap * a.ref_stride : nullptr;
  int64_t r = 0;
  uint32_t k = 0;
  while (k < a.fpc) {
    FrameInfo &I = slot[k];
    const uint32_t ref_slot = cap * a.fpc + k;
    int64_t st[kMaxStreams];
    int64_t n = -1;
    uint64_t c_from = (uint64_t)(r / K);
    if (c_from < a.nchunks && cand[c_from] != ~0ull && (int64_t)cand[c_from] < r) {
      // chunk(r) recorded an earlier trigger (several frames per chunk): exact scan of the
      // rest of that chunk, then the recorded candidates of the chunks after it
      n = forward_trigger<S>(a, cap, r, std::min<int64_t>((int64_t)(c_from + 1) * K,
                                                       (int64_t)a.frame_len), st);
      c_from++;
    }
    uint64_t cf = ~0ull;                   // first chunk at or after c_from with a candidate
    for (uint64_t c0 = n >= 0 ? a.nchunks : c_from; c0 < a.nchunks; c0 += 64) {
      const uint64_t c = c0 + lane;
      const unsigned long long b = __ballot(c < a.nchunks && cand[c] != ~0ull);
      if (b) {
        cf = c0 + __ffsll((long long)b) - 1;
        break;
      }
    }
    if (n < 0 && cf == ~0ull) {            // no trigger in the rest of the capture
      if (lane == 0) frame_empty(I, 1, cap, ref_slot, r, a.frame_len - r);
      k++;
      break;
    }
    bool spans = false;
    if (n < 0) {
      n = (int64_t)cand[cf];
      spans = trigger_run_starts<S>(a, cap, a.rec[(uint64_t)cap * a.rec_stride + cf], r, st);
    }
    if (spans) {
      if (lane == 0) frame_empty(I, 3, cap, ref_slot, r, 0);
      k++;
      break;
    }
    // transmitted frame holding this sync index (reference rows for the EVM)
    uint32_t ref = ref_slot;
    if (rs) {
      uint64_t sum = 0;
      for (uint32_t s = 0; s < a.N; s++) sum += (uint64_t)(st[s] - r);
      const uint64_t sync_abs = (uint64_t)r + sum / a.N;
      uint32_t j = 0;
      while (j + 1 < a.ref_stride && rs[j + 1] != ~0ull && rs[j + 1] <= sync_abs) j++;
      ref = cap * a.ref_stride + j;
    }
    uint64_t nsp_rel = 0;
    const int status = frame_from_trigger(a, I, cap, ref, r, n, st, k > 0, nsp_rel);
    k++;
    if (status != 0) break;
    r += (int64_t)nsp_rel;
  }
  for (uint32_t kk = k + lane; kk < a.fpc; kk += 64)
    frame_empty(slot[kk], 4, cap, cap * a.fpc + kk, r, 0);   // MIMO_FRAME_NONE
}

// Re-arm certificate of slot k >= 1 on antenna s: over n in Z = [r, r + M - 1) both the
// capture-history metric (P over the M/2 products ending at n, R over the last M samples)
// and the fresh framesync's metric (samples before r read as zero: P sums products m >=
// r + M/2, R samples m >= r) stay clearly below the threshold. Running fp64 sums per thread
// segment, seeded by one block scan of the segments' differences (as sc_exact_kernel).
template <bool S>
__global__ __launch_bounds__(kScT) void stream_cert_kernel(PlateauArgs a) {
  __shared__ double ws[2][6][kScT / 64];
  __shared__ int s_fail;
  const uint32_t k = blockIdx.x + 1, s = blockIdx.y, cap = blockIdx.z;
  const FrameInfo &I = a.info[(uint64_t)cap * a.fpc + k];
  if (I.status != 0 && I.status != 2) return;
  const int tid = threadIdx.x;
  const int64_t M = a.M, M2 = M / 2, r = (int64_t)I.origin;
  const int64_t L = (int64_t)a.frame_len;
  const auto x = iq_row<S>(a.iq, a.iq_scale, ((uint64_t)cap * a.N + s) * a.stride);
  auto ld = [&](int64_t q) { return (q >= 0 && q < L) ? x.at(q) : make_float2(0.0f, 0.0f); };
  if (tid == 0) s_fail = 0;
  // capture-history sums ending at r - 1 and the region's energy (the cancellation guard)
  double c[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0}, tot[6];
  for (int64_t i = tid; i < M; i += kScT) {
    const int64_t m = r - M + i;
    const float2 v = ld(m);
    const float z = v.x * v.x + v.y * v.y;
    c[2] += (double)z;
    if (i >= M2) {
      const float2 pp = cj_mul(ld(m - M2), v);
      c[0] += (double)pp.x;
      c[1] += (double)pp.y;
    }
    const float2 w = ld(r + i);
    c[3] += (double)(w.x * w.x + w.y * w.y);
  }
  block_scan<6>(c, tot, ws[0]);
  const double Pc0r = tot[0], Pc0i = tot[1], Zc0 = tot[2];
  const double E = tot[2] + tot[3];
  // this thread's positions n = r + j, j in [j0, j1)
  const int64_t G = (M - 1 + kScT - 1) / kScT;
  const int64_t j0 = std::min<int64_t>(M - 1, tid * G), j1 = std::min<int64_t>(M - 1, j0 + G);
  double d[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  for (int64_t j = j0; j < j1; j++) {
    const int64_t n = r + j;
    const float2 vn = ld(n), vh = ld(n - M2), vm = ld(n - M);
    const float2 pn = cj_mul(vh, vn), pl = cj_mul(ld(n - M), vh);
    const float zn = vn.x * vn.x + vn.y * vn.y, zl = vm.x * vm.x + vm.y * vm.y;
    d[0] += (double)pn.x - (double)pl.x;
    d[1] += (double)pn.y - (double)pl.y;
    d[2] += (double)zn - (double)zl;
    if (j >= M2) { d[3] += (double)pn.x; d[4] += (double)pn.y; }
    d[5] += (double)zn;
  }
  block_scan<6>(d, tot, ws[1]);
  double Pcr = Pc0r + d[0], Pci = Pc0i + d[1], Zc = Zc0 + d[2];
  double Pfr = d[3], Pfi = d[4], Zf = d[5];
  const double lim = a.thr - 2.0 * a.band - 1e-3;
  auto fails = [&](double pr, double pi, double z) {
    const double R = 0.5 * z;
    if (E == 0.0) return false;                 // all-zero region: y is 0/0 (false) throughout
    if (R < 1e-9 * E) return true;              // too close to cancellation to certify
    return pr * pr + pi * pi > lim * R * R;
  };
  bool bad = false;
  for (int64_t j = j0; j < j1; j++) {
    const int64_t n = r + j;
    const float2 vn = ld(n), vh = ld(n - M2), vm = ld(n - M);
    const float2 pn = cj_mul(vh, vn), pl = cj_mul(vm, vh);
    const float zn = vn.x * vn.x + vn.y * vn.y, zl = vm.x * vm.x + vm.y * vm.y;
    Pcr += (double)pn.x - (double)pl.x;
    Pci += (double)pn.y - (double)pl.y;
    Zc += (double)zn - (double)zl;
    if (j >= M2) { Pfr += (double)pn.x; Pfi += (double)pn.y; }
    Zf += (double)zn;
    bad = bad || fails(Pcr, Pci, Zc) || fails(Pfr, Pfi, Zf);
  }
  if (bad) s_fail = 1;
  __syncthreads();
  if (tid == 0 && s_fail) atomicOr(&a.certfail[cap], 1ull << k);
}

// the first uncertified slot of each capture becomes RESCAN (resume at its origin), the
// slots after it NONE
__global__ __launch_bounds__(64) void stream_fixup_kernel(PlateauArgs a) {
  const uint32_t cap = blockIdx.x;
  const unsigned long long m = a.certfail[cap];
  if (!m) return;
  const uint32_t k0 = (uint32_t)(__ffsll((long long)m) - 1);
  FrameInfo *slot = a.info + (uint64_t)cap * a.fpc;
  for (uint32_t k = k0 + threadIdx.x; k < a.fpc; k += 64) {
    FrameInfo &I = slot[k];
    if (k == k0) {
      I.status = 3;
      I.n_sym = 0;
      I.nsp = 0;
    } else {
      I.status = 4;
      I.n_sym = 0;
      I.nsp = 0;
    }
  }
}

// ======================================================================================
// Screened S&C (default path). The per-chunk item kernel above scans every chunk of every
// frame and walks the antennas of a plateau chunk one after another in one workgroup; here
//  1. sc_screen_kernel streams antenna 0 once and proves, per block of B positions, that
//     y[n] < thr for every n of the block, from block sums alone: with Sp, Sz, Ap the block
//     sums of p = conj(x[k-M/2]) x[k], |x[k]|^2 and |Re p| + |Im p| (M/2 = D*B),
//       |P[n]| <= |sum_{j=1..D} Sp[b-j]| + Ap[b] + Ap[b-D]
//       2R[n]  >= sum_{j=1..2D-1} Sz[b-j]
//     (fp32 block sums: the bounds are widened by 1e-4 of the absolute sums and the test
//     uses thr - 0.01, far outside the fp32 error of both the sums and the oracle's y).
//     Chunks whose candidate range meets an unproven block are appended to a work list
//     with the first/last unproven position;
//  2. sc_exact_kernel evaluates every (listed chunk, antenna) in parallel, exactly as the item
//     kernel does for one antenna (fp64 running sums, band, deferred near-threshold samples),
//     over the iterations that cover the unproven range and its cp+2 run history;
//  3. sc_resolve_kernel / sc_finalize_kernel (above) resolve the deferred samples and apply
//     the plateau rule per chunk; plateau_kernel completes run starts and the sync index.
// Positions outside the evaluated iterations carry zero bits: for antenna 0 that is exact
// (proven), for the others it only affects run starts, which item_record / plateau_kernel
// then take from an exact backward scan, as for a run that began before a chunk's halo.
// ======================================================================================

// one step of the transposing butterfly: of v[0 .. N) a lane keeps the half selected by its
// lane bit OFF and adds the partner's copy of that half (compile-time indices throughout), with
// no LDS traffic. Offsets 32 and 16 pair lanes l and l ^ OFF through v_permlane32/16_swap: one
// swap of (v[i], v[i + N/2]) leaves a lane its own kept value and the partner's copy of it, so
// the kept sum is the two results added. Offsets 8 and 4 pair lanes through DPP row_mirror
// (l <-> 15 - l in a row) and row_half_mirror (l <-> 7 - l in 8), which flip the same lane bit:
// a lane then holds the sum over lanes l ^ {0, 7, 8, 15} of every row, and the quad sums that
// follow (l ^ {0, 1, 2, 3}) cover each of the 64 lanes once.
template <int CTRL>
MIMO_DEV float dpp_mov(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xf, 0xf, false));
}
template <int OFF, int N>
MIMO_DEV void tr_reduce_step(float *v, int lane) {
  static_assert(OFF == 32 || OFF == 16 || OFF == 8 || OFF == 4, "lane bits 5..2");
  if constexpr (OFF >= 16) {
#pragma unroll
    for (int i = 0; i < N / 2; i++) {
      const uint32_t a = __float_as_uint(v[i]), b = __float_as_uint(v[i + N / 2]);
      const auto r = OFF == 32 ? __builtin_amdgcn_permlane32_swap(a, b, false, false)
                               : __builtin_amdgcn_permlane16_swap(a, b, false, false);
      v[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
  } else {
    const bool up = (lane & OFF) != 0;
#pragma unroll
    for (int i = 0; i < N / 2; i++) {
      const float send = up ? v[i] : v[i + N / 2];
      const float keep = up ? v[i + N / 2] : v[i];
      v[i] = keep + dpp_mov<OFF == 8 ? 0x140 : 0x141>(send);   // row_mirror / row_half_mirror
    }
  }
}

// block sums of antenna 0 over a span, the screen test, and the chunk list
template <bool S, int SPAN>
__global__ __launch_bounds__(kScrT) __attribute__((amdgpu_waves_per_eu(6))) void sc_screen_kernel(ScreenArgs a) {
  constexpr int B = kScrB;
  static_assert(SPAN <= kScrSpan && SPAN % (kScrB * kScrBPI * (kScrT / 64)) == 0, "screen span");
  __shared__ float4 recs[SPAN / B + 2 * (kScrMaxD)];
  // per chunk the test can touch (chunk_len >= kScrSpan / 2: at most three), the first and last
  // unproven position, gathered before the global list update
  constexpr int kScrChunks = 4;
  __shared__ unsigned long long s_cmin[kScrChunks], s_cmax[kScrChunks];
  const uint32_t f = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int D = (int)(a.M / 2) / B, RL = (int)a.M / 2;
  if (a.trig && a.trig[f] != ~0ull) return;           // triggered in an earlier phase
  if (tid < kScrChunks) {
    s_cmin[tid] = ~0ull;
    s_cmax[tid] = 0ull;
  }
  const int64_t L = a.chunk_hi ? std::min<int64_t>((int64_t)a.frame_len,
                                                   (int64_t)(a.chunk_hi * a.chunk_len))
                               : (int64_t)a.frame_len;   // end of this phase's positions
  const int64_t LF = (int64_t)a.frame_len;
  const int64_t q0 = (int64_t)a.chunk_lo * (int64_t)a.chunk_len + (int64_t)blockIdx.x * SPAN;
  if (q0 >= L) return;
  const int NB = SPAN / B + 2 * D;
  const int64_t h0 = q0 - (int64_t)2 * D * B;     // first block of the history
  const auto x = iq_row<S>(a.iq, a.iq_scale, (uint64_t)f * a.N * a.stride);   // antenna 0
  const bool vec = x.pair_ok();
  // block sums: a wave per block, two positions per lane (B = 128); kScrBPI blocks per wave
  // iteration with all their loads issued before the first use (one memory latency per
  // iteration instead of per block)
  for (int j0 = wv * kScrBPI; j0 < NB; j0 += (kScrT / 64) * kScrBPI) {
    float4 cur[kScrBPI], del[kScrBPI];
    const int64_t nb = h0 + (int64_t)j0 * B;
    if (vec && nb - RL >= 0 && nb + (int64_t)kScrBPI * B <= LF && j0 + kScrBPI <= NB) {
#pragma unroll
      for (int b = 0; b < kScrBPI; b++) {
        cur[b] = x.pair(nb + 2 * lane + (int64_t)b * B);
        del[b] = x.pair(nb - RL + 2 * lane + (int64_t)b * B);
      }
    } else {
#pragma unroll
      for (int b = 0; b < kScrBPI; b++) {
        const int64_t n = nb + (int64_t)b * B + 2 * lane;
        cur[b] = ld_pair(x, n, LF, vec);
        del[b] = ld_pair(x, n - RL, LF, vec);
      }
    }
    // per-lane partials v[4 b + c] (c: Re P, Im P, |x|^2, |Re p| + |Im p|), then a transposing
    // butterfly: at offsets 32, 16, 8, 4 a lane keeps half of its values and adds the
    // partner's copy of them (8 + 4 + 2 + 1 exchanges for 16 sums instead of 16 x 6); lanes
    // then hold value (lane >> 2) summed over 16 lanes, and the quad sums finish it
    float v[4 * kScrBPI];
#pragma unroll
    for (int b = 0; b < kScrBPI; b++) {
      const float2 c0 = make_float2(cur[b].x, cur[b].y), c1 = make_float2(cur[b].z, cur[b].w);
      const float2 d0 = make_float2(del[b].x, del[b].y), d1 = make_float2(del[b].z, del[b].w);
      const float2 p0 = cj_mul(d0, c0), p1 = cj_mul(d1, c1);
      v[4 * b + 0] = p0.x + p1.x;
      v[4 * b + 1] = p0.y + p1.y;
      v[4 * b + 2] = (c0.x * c0.x + c0.y * c0.y) + (c1.x * c1.x + c1.y * c1.y);
      v[4 * b + 3] = (fabsf(p0.x) + fabsf(p0.y)) + (fabsf(p1.x) + fabsf(p1.y));
    }
    static_assert(4 * kScrBPI == 16, "transposing reduction of 16 values over 64 lanes");
    tr_reduce_step<32, 16>(v, lane);
    tr_reduce_step<16, 8>(v, lane);
    tr_reduce_step<8, 4>(v, lane);
    tr_reduce_step<4, 2>(v, lane);
    float tot = v[0];
    tot += dpp_mov<0x4E>(tot);   // quad_perm [2, 3, 0, 1]: lane ^ 2
    tot += dpp_mov<0xB1>(tot);   // quad_perm [1, 0, 3, 2]: lane ^ 1
    {
      const int q = lane >> 2, b = q >> 2, c = q & 3;   // value q = 4 b + c
      if ((lane & 3) == 0 && j0 + b < NB) reinterpret_cast<float *>(&recs[j0 + b])[c] = tot;
    }
  }
  __syncthreads();
  const int64_t K = (int64_t)a.chunk_len;
  const int64_t lo_all = (int64_t)a.chunk_lo * K;
  const int64_t c_base = q0 / K;                       // the first chunk the test can touch
  for (int j = 2 * D + tid; j < NB; j += kScrT) {
    const int64_t n0 = h0 + (int64_t)j * B;
    if (n0 >= L) break;
    // positions n < M/2 of a capture that starts at the framesync's origin: every lagged
    // sample x[k - M/2] of P[n] is the empty delay line's zero, so P[n] = 0 and y[n] is 0 (or
    // the oracle's 0/0, compared false) -- never above the threshold. (Block sums cannot show
    // it for the first block, whose energy lower bound is zero, and every capture's chunk 0
    // used to become an exact-pass item for that block alone.)
    if (a.empty_history && n0 + B <= (int64_t)RL) continue;
    // (one pass over the 2D records: each read once; the same sums in the same order)
    double pr = 0.0, pi = 0.0, apw = 0.0, rz = 0.0, azw = 0.0;
    for (int u = 1; u <= 2 * D; u++) {
      const float4 r = recs[j - u];
      if (u <= D) {
        pr += (double)r.x;
        pi += (double)r.y;
        apw += (double)r.w;
      }
      if (u < 2 * D) rz += (double)r.z;
      azw += (double)r.z;
    }
    const double ab = (double)recs[j].w, ad = (double)recs[j - D].w;
    const double pup = sqrt(pr * pr + pi * pi) + ab + ad + 1e-4 * (apw + ab + ad);
    const double rlow = 0.5 * (rz - 1e-4 * (azw + (double)recs[j].z));
    const bool proven = rlow > 0.0 && pup * pup < a.thr_screen * (rlow * rlow);
    if (proven) continue;
    // unproven block: its positions in [lo_all, L) may be candidates -- gathered per chunk in
    // LDS first, so each chunk the workgroup touches costs one set of global atomics (a chain
    // of returning atomics per unproven block kept a workgroup alive ~20 us)
    const int64_t s0 = n0 < lo_all ? lo_all : n0;
    const int64_t s1 = (n0 + B < L ? n0 + B : L) - 1;
    if (s1 < s0) continue;
    for (int64_t c = s0 / K; c <= s1 / K; c++) {
      const int64_t u0 = s0 > c * K ? s0 : c * K, u1 = s1 < (c + 1) * K - 1 ? s1 : (c + 1) * K - 1;
      atomicMin(&s_cmin[c - c_base], (unsigned long long)u0);
      atomicMax(&s_cmax[c - c_base], (unsigned long long)u1);
    }
  }
  __syncthreads();
  if (tid < kScrChunks && s_cmin[tid] != ~0ull) {
    const int64_t c = c_base + tid;
    const uint64_t ci = (uint64_t)f * a.nchunks + (uint64_t)c;
    atomicMin(&a.fmin[ci], s_cmin[tid]);
    atomicMax(&a.fmax[ci], s_cmax[tid]);
    if (atomicOr(&a.flag[ci], 1u) == 0u) {
      const uint32_t slot = atomicAdd(a.count, 1u);
      if (slot < a.cap) {
        ScHot *hp = a.hot + slot;
        hp->f = f;
        hp->n_done = a.N;
        hp->namb = 0;
        hp->arrived = 0;
        hp->chunk = (uint64_t)c;
        hp->c0 = c * K;
        hp->w0 = c * K - ((int64_t)kScSpan - K);
        hp->cend = (c + 1) * K < L ? (c + 1) * K : L;
      }
    }
  }
}

// Ring slot of position p in the exact kernel's LDS ring, which holds positions
// [ib - M, ib + kScIt) of the current iteration at slots (M + p - w0) mod RING.
MIMO_DEV int ring_slot(int64_t p, int64_t w0, int M, int RING) {
  return (int)(((int64_t)M + (p - w0)) % RING);
}

constexpr int kLocAmb = kScT / 2;   // near-threshold samples resolved per iteration pass
// positions spanned by one exact-recompute window: the tables hold M + kResSpread positions,
// sized so that two workgroups fit a CU at M = 2048 (a plateau's two near-threshold edges,
// ~cp + 115 positions apart, still share one window)
constexpr int kResSpread = 512;

// one (listed chunk, antenna): the item kernel's antenna pass over the iterations covering the
// chunk's unproven range (and its cp+2 run history). Near-threshold samples are resolved in
// place with the oracle's exact fp32 chains from the ring (two lanes per sample); the last
// antenna workgroup of an item to finish then applies the plateau rule to the item's words
// (item_conditions / item_record, as sc_finalize_kernel) -- no separate resolve/finalize pass.
template <bool S>
__global__ __launch_bounds__(kScT) __attribute__((amdgpu_waves_per_eu(2)))
void sc_exact_kernel(ScArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sc_dyn[];
  const int M = (int)a.M, RL = M / 2, RING = M + kScIt;
  float2 *ring = reinterpret_cast<float2 *>(sc_dyn);
  __shared__ double scan_ws[2][5][kScT / 64];
  __shared__ long long s_amb[kLocAmb], s_sorted[kLocAmb];
  __shared__ float s_rv[kLocAmb][3];
  // exact-recompute tables after the ring: rtz[i] = 0.5|x|^2 at table position i < W and
  // rtp[i - M/2] = -conj(x[k-M/2]) x[k] for M/2 <= i < W (only those are summed)
  float *rtz = reinterpret_cast<float *>(sc_dyn + sizeof(float2) * ring_pad(RING));
  float2 *rtp = reinterpret_cast<float2 *>(rtz + ((M + kResSpread + 3) & ~3));
  __shared__ int s_namb, s_last;
  // the plateau step's word copy and conditions alias the ring (dead after the iterations)
  uint16_t *fwb = reinterpret_cast<uint16_t *>(sc_dyn);
  uint16_t(*acond)[kScT] = reinterpret_cast<uint16_t(*)[kScT]>(fwb + kMaxStreams * kScIters * kScT);
  __shared__ long long run_ws[2][kScT / 64];
  __shared__ long long flo[kMaxStreams];
  __shared__ unsigned long long s_min;
  const uint32_t count_raw = *a.hot_count;
  const uint32_t count = min(count_raw, a.hot_cap);
  const uint32_t item0 = a.item_lo ? *a.item_lo : 0u;   // items of earlier screen phases: done
  // the next screen phase appends after this phase's items: their count, for its exact launch
  // (the kernel boundary orders this store before the next screen's appends)
  if (a.snap && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *a.snap = count_raw;
  // one (item, antenna) pass per workgroup (blockIdx.x the antenna), walking the item's unproven
  // iterations in turn (splitting them over 2 or 4 workgroups, each with its own M-sample
  // history setup, measured 1.5-2.2x slower: DESIGN.md)
  const uint32_t s = blockIdx.x;
  uint32_t slot = item0 + blockIdx.y;
  // the first slot's record is read before the count is known (it is inside the allocation
  // whatever the count, and used only if the slot is live): in phase 1 (item0 = 0) its loads
  // go out with the count's instead of one memory latency after it
  const ScHot *hs = a.hot + min(slot, a.hot_cap - 1u);
  uint32_t f_n = hs->f;
  int64_t w0_n = hs->w0;
  uint64_t chunk_n = hs->chunk;
  for (; slot < count; slot += gridDim.y) {
  ScHot *hp = a.hot + slot;
  const int tid = threadIdx.x;
  if (tid == 0) s_namb = 0;
  const unsigned long long t_item = a.prof ? (unsigned long long)wall_clock64() : 0ull;
  if (a.prof && tid == 0) atomicMin(&a.prof[0], t_item);
  unsigned long long t_res = 0;
  uint32_t n_win = 0, n_smp = 0;   // diagnostics: resolve windows and samples of this pass
  bool multi_win = false;          // diagnostics: an iteration of this pass had >= 2 windows
  const uint32_t f = f_n;
  const int64_t L = (int64_t)a.frame_len;
  const int64_t w0 = w0_n;
  const uint64_t ci = (uint64_t)f * a.nchunks + chunk_n;
  const int64_t fmin = (int64_t)a.fmin[ci], fmax = (int64_t)a.fmax[ci];
  const unsigned long long t_rec = a.prof ? (unsigned long long)wall_clock64() + (fmin & 0) : 0ull;
  int it_lo = (int)std::max<int64_t>(0, (fmin - (int64_t)a.cp - 2 - w0) / kScIt);
  int it_hi = (int)std::min<int64_t>(kScIters - 1, (fmax - w0) / kScIt);
  const auto x = iq_row<S>(a.iq, a.iq_scale, ((uint64_t)f * a.N + s) * a.stride);
  const bool vec = x.pair_ok();
  if (tid == 0) hp->lo[s] = w0 + (int64_t)it_lo * kScIt;   // first evaluated position
  for (int it = 0; it < kScIters; it++)
    if (it < it_lo || it > it_hi) hp->wbits[((int)s * kScIters + it) * kScT + tid] = 0;
  const int64_t ib_lo = w0 + (int64_t)it_lo * kScIt;
  {
  // the first two blocks' loads, then the history [ib_lo - M, ib_lo) -> its ring slots: all in
  // flight together (the window sums below wait for the history only). Block it_lo + j goes
  // through register set j & 1 (pre, pre2): each iteration refills the set it consumed two
  // blocks ahead, so an iteration's ring fill no longer waits one memory latency on the load
  // the previous iteration issued (the second iteration of a pass did, ~5 us)
  float4 pre[kScIt / (2 * kScT)], pre2[kScIt / (2 * kScT)];
  bool pf = fetch_block(pre, x, ib_lo, L, vec);
  bool pf2 = it_hi > it_lo ? fetch_block(pre2, x, ib_lo + kScIt, L, vec) : false;
  const int wb = (kScIt * it_lo) % RING;
  if (vec && ib_lo - M >= 0 && ib_lo <= L) {
    // all history pairs in flight together, then the ring writes
    constexpr int HU = 4;
    for (int j0 = 0; 2 * j0 < M; j0 += kScT * HU) {
      float4 hv[HU];
#pragma unroll
      for (int u = 0; u < HU; u++) {
        const int j = j0 + u * kScT + tid;
        hv[u] = x.pair(ib_lo - M + 2 * (2 * j < M ? j : 0));
      }
#pragma unroll
      for (int u = 0; u < HU; u++) {
        const int j = j0 + u * kScT + tid;
        if (2 * j < M) {
          int sl = wb + 2 * j;
          if (sl >= RING) sl -= RING;
          *reinterpret_cast<float4 *>(ring + ring_pad(sl)) = hv[u];
        }
      }
    }
  } else {
    for (int j = tid; 2 * j < M; j += kScT) {
      int sl = wb + 2 * j;
      if (sl >= RING) sl -= RING;
      *reinterpret_cast<float4 *>(ring + ring_pad(sl)) = ld_pair(x, ib_lo - M + 2 * j, L, vec);
    }
  }
  __syncthreads();
  // window sums ending at ib_lo - 1: P over the last M/2, 2R and the nonzero count over M
  double c[4] = {0.0, 0.0, 0.0, 0.0}, t4[4], tot[5];
  for (int k = tid; k < M; k += kScT) {
    int sl = wb + k;
    if (sl >= RING) sl -= RING;
    const float2 v = ring[ring_pad(sl)];
    const float z = v.x * v.x + v.y * v.y;
    c[2] += (double)z;
    c[3] += (z != 0.0f) ? 1.0 : 0.0;
    if (k >= RL) {
      int sd = sl - RL;
      if (sd < 0) sd += RING;
      const float2 pp = cj_mul(ring[ring_pad(sd)], v);
      c[0] += (double)pp.x;
      c[1] += (double)pp.y;
    }
  }
  int par = 0;
  block_scan<4>(c, t4, scan_ws[par]);
  par ^= 1;
  double Pc_re = t4[0], Pc_im = t4[1], Zc = t4[2], Cc = t4[3], Ac = t4[2];
  const unsigned long long t_setup = a.prof ? (unsigned long long)wall_clock64() : 0ull;
  if (a.prof && tid == 0) {
    atomicAdd(&a.prof[20], t_rec - t_item);
    atomicAdd(&a.prof[21], t_setup - t_rec);
    atomicAdd(&a.prof[23], (unsigned long long)(it_hi - it_lo + 1));
    atomicMax(&a.prof[25], t_item);
    atomicAdd(&a.prof[26], t_item);
  }
  unsigned long long pq_ring = 0, pq_scan = 0, pq_walk = 0, pq_first = 0;
#pragma unroll 1
  for (int it = it_lo; it <= it_hi; it++) {
    const int64_t ib = w0 + (int64_t)it * kScIt;
    const unsigned long long tq0 = a.prof ? (unsigned long long)wall_clock64() : 0ull;
    const bool odd = ((it - it_lo) & 1) != 0;                  // uniform: register set
    const bool pf_used = odd ? pf2 : pf;
    {
      const int sl0 = (M + it * kScIt) % RING + 2 * tid;
      if (pf_used) {
        if (odd) {
#pragma unroll
          for (int j = 0; j < kScIt / (2 * kScT); j++) {
            int sl = sl0 + 2 * kScT * j;
            if (sl >= RING) sl -= RING;
            *reinterpret_cast<float4 *>(ring + ring_pad(sl)) = pre2[j];
          }
        } else {
#pragma unroll
          for (int j = 0; j < kScIt / (2 * kScT); j++) {
            int sl = sl0 + 2 * kScT * j;
            if (sl >= RING) sl -= RING;
            *reinterpret_cast<float4 *>(ring + ring_pad(sl)) = pre[j];
          }
        }
      } else {   // frame edges: guarded loads straight into the ring
#pragma unroll 1
        for (int j = 0; j < kScIt / (2 * kScT); j++) {
          int sl = sl0 + 2 * kScT * j;
          if (sl >= RING) sl -= RING;
          *reinterpret_cast<float4 *>(ring + ring_pad(sl)) =
              ld_pair(x, ib + 2 * (tid + kScT * j), L, vec);
        }
      }
    }
    __syncthreads();
    const unsigned long long tq1 = a.prof ? (unsigned long long)wall_clock64() : 0ull;
    if (it + 2 <= it_hi) {                        // two blocks ahead, into the set just used
      if (odd) pf2 = fetch_block(pre2, x, ib + 2 * kScIt, L, vec);
      else pf = fetch_block(pre, x, ib + 2 * kScIt, L, vec);
    }
    const float2 *xn = ring + ring_pad((M + it * kScIt + kScS * tid) % RING);
    const float2 *xr = ring + ring_pad((RL + it * kScIt + kScS * tid) % RING);
    const float2 *xm = ring + ring_pad((it * kScIt + kScS * tid) % RING);
    double d[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    float bp = 0.0f, bz = 0.0f;
    int dc = 0;
#pragma unroll 2
    for (int i = 0; i < kScS; i += 2) {
      const float4 vn = *reinterpret_cast<const float4 *>(xn + i);
      const float4 vr = *reinterpret_cast<const float4 *>(xr + i);
      const float4 vm = *reinterpret_cast<const float4 *>(xm + i);
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const float2 n_ = h ? make_float2(vn.z, vn.w) : make_float2(vn.x, vn.y);
        const float2 r_ = h ? make_float2(vr.z, vr.w) : make_float2(vr.x, vr.y);
        const float2 m_ = h ? make_float2(vm.z, vm.w) : make_float2(vm.x, vm.y);
        const float2 pn = cj_mul(r_, n_), pl = cj_mul(m_, r_);
        const float zn = n_.x * n_.x + n_.y * n_.y, zl = m_.x * m_.x + m_.y * m_.y;
        const double zn64 = (double)zn;
        d[0] += (double)pn.x - (double)pl.x;
        d[1] += (double)pn.y - (double)pl.y;
        d[2] += zn64 - (double)zl;
        d[4] += zn64;
        dc += (zn != 0.0f ? 1 : 0) - (zl != 0.0f ? 1 : 0);
        bp += (fabsf(pn.x) + fabsf(pn.y)) + (fabsf(pl.x) + fabsf(pl.y));
        bz += zl;
      }
    }
    d[3] = (double)dc;
    block_scan<5>(d, tot, scan_ws[par]);
    par ^= 1;
    const unsigned long long tq2 = a.prof ? (unsigned long long)wall_clock64() : 0ull;
    double Pre = Pc_re + d[0], Pim = Pc_im + d[1], Z = Zc + d[2], C = Cc + d[3];
    const double Aend = Ac + tot[4];
    const double zfloor = 1e-6 * Aend;
    const int64_t sb = ib + kScS * tid;
    uint32_t bits = 0, ovf = 0;
    bool walk = true;
    {
      const double pmax = sqrt(Pre * Pre + Pim * Pim) + 1.001 * (double)bp;
      const double rmin = 0.5 * (Z - 1.001 * (double)bz);
      if (rmin > 0.0 && Z > 16.0 * zfloor && pmax * pmax < (a.thr - 2.0 * a.band) * (rmin * rmin))
        walk = false;
    }
#pragma unroll 1
    for (int i = 0; walk && i < kScS; i += 2) {
      const float4 vn = *reinterpret_cast<const float4 *>(xn + i);
      const float4 vr = *reinterpret_cast<const float4 *>(xr + i);
      const float4 vm = *reinterpret_cast<const float4 *>(xm + i);
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const float2 n_ = h ? make_float2(vn.z, vn.w) : make_float2(vn.x, vn.y);
        const float2 r_ = h ? make_float2(vr.z, vr.w) : make_float2(vr.x, vr.y);
        const float2 m_ = h ? make_float2(vm.z, vm.w) : make_float2(vm.x, vm.y);
        const float2 pn = cj_mul(r_, n_), pl = cj_mul(m_, r_);
        const float zn = n_.x * n_.x + n_.y * n_.y, zl = m_.x * m_.x + m_.y * m_.y;
        Pre += (double)pn.x - (double)pl.x;
        Pim += (double)pn.y - (double)pl.y;
        Z += (double)zn - (double)zl;
        C += ((zn != 0.0f) ? 1.0 : 0.0) - ((zl != 0.0f) ? 1.0 : 0.0);
        const int64_t n = sb + i + h;
        bool b = false;
        if (n >= 0 && n < L && C > 0.5) {
          const double R = 0.5 * Z, R2 = R * R;
          const double q = Pre * Pre + Pim * Pim - a.thr * R2;
          if (fabs(q) <= a.band * R2 || Z <= zfloor) {
            const int k = atomicAdd(&s_namb, 1);
            if (k < kLocAmb) {
              s_amb[k] = n;
              b = true;                // provisional: resolved below, from the ring
            } else {
              ovf |= 1u << (i + h);   // list full: this lane recomputes it below
            }
          } else {
            b = q > 0.0;
          }
        }
        bits |= (b ? 1u : 0u) << (i + h);
      }
    }
    while (ovf) {   // overflow of the deferred list (pathological input): exact here
      const int i = __ffs((int)ovf) - 1;
      ovf &= ovf - 1u;
      if (!((double)sc_exact(x, sb + i, a.M) > a.thr)) bits &= ~(1u << i);
      if (a.n_exact) atomicAdd(a.n_exact, 1ull);
    }
    __syncthreads();
    const unsigned long long tq3 = a.prof ? (unsigned long long)wall_clock64() : 0ull;
    if (a.prof) {   // per-pass sums, added once per pass (atomics here would time themselves)
      pq_ring += tq1 - tq0;
      pq_scan += tq2 - tq1;
      pq_walk += tq3 - tq2;
      if (it == it_lo) pq_first += tq1 - tq0;
      if (tid == 0 && !pf_used) atomicAdd(&a.prof[24], 1ull);   // diagnostics: guarded ring fills
    }
    const int namb = (a.diag & 8) ? 0 : min(s_namb, kLocAmb);          // uniform
    const unsigned long long t_r0 = a.prof ? (unsigned long long)wall_clock64() : 0ull;
    const uint32_t n_win0 = n_win;
    if (namb > 0) {
      // exact fp32 recompute of this iteration's near-threshold samples (the oracle's chains,
      // as resolve_window): ascending order, then windows of <= kResSpread positions; per
      // window the per-sample terms are tabled from the ring by every thread, then each
      // sample's R chain runs on a lane of waves 0-1 and its P chains on a lane of waves 2-3
      for (int i = tid; i < namb; i += kScT) {
        int rank = 0;
        for (int j = 0; j < namb; j++) rank += (s_amb[j] < s_amb[i]) ? 1 : 0;
        s_sorted[rank] = s_amb[i];
      }
      __syncthreads();
      for (int k = 0; k < namb;) {                    // uniform
        const int64_t nmin = s_sorted[k];
        int e = k + 1;
        while (e < namb && s_sorted[e] - nmin < kResSpread) e++;
        const int64_t q0 = nmin - M + 1;              // table index i <-> position q0 + i
        const int W = (int)(s_sorted[e - 1] - nmin) + M;
        // ring slots of positions q0 + i and q0 + i - RL: one 64-bit remainder per window, then
        // a conditional wrap per entry (i < W < RING) -- a remainder per entry was ~2 us
        const int sq = ring_slot(q0, w0, M, RING);
        const int sqd = sq >= RL ? sq - RL : sq - RL + RING;
        for (int i = tid; i < W; i += kScT) {
          const int sl = sq + i < RING ? sq + i : sq + i - RING;
          const float2 vv = ring[ring_pad(sl)];
          const float z = vv.x * vv.x + vv.y * vv.y;
          rtz[i] = 0.5f * z;
          if (i >= RL) {
            const int sd = sqd + i < RING ? sqd + i : sqd + i - RING;
            const float2 dv = ring[ring_pad(sd)];
            const float2 pp = cj_mul(dv, vv);
            rtp[i - RL] = make_float2((-1.0f) * pp.x, (-1.0f) * pp.y);
          }
        }
        __syncthreads();
        {
          const int g = k + (tid & (kLocAmb - 1));
          if (g < e) {
            const int r = (int)(s_sorted[g] - nmin);
            if (tid < kLocAmb) {
              s_rv[g][0] = seq_sum(rtz + r, M);
            } else {
              const float2 P = seq_sum2(rtp + r, RL);
              s_rv[g][1] = P.x;
              s_rv[g][2] = P.y;
            }
          }
        }
        __syncthreads();
        k = e;
        n_win++;
      }
      n_smp += namb;
      for (int g = 0; g < namb; g++) {
        const int64_t o = s_sorted[g] - sb;
        if (o >= 0 && o < kScS) {
          const float Pr = s_rv[g][1], Pi = s_rv[g][2], R = s_rv[g][0];
          const float y32 = (Pr * Pr + Pi * Pi) / (R * R);
          if (!((double)y32 > a.thr)) bits &= ~(1u << (int)o);
        }
      }
      if (tid == 0 && a.n_exact) atomicAdd(a.n_exact, (unsigned long long)namb);
      __syncthreads();
      if (tid == 0) s_namb = 0;
      if (a.prof) t_res += (unsigned long long)wall_clock64() - t_r0;
    }
    if (a.prof && tid == 0 && n_win > n_win0) {   // diagnostics: windows of this iteration
      atomicMax(&a.prof[27], (unsigned long long)(n_win - n_win0));
      if (n_win - n_win0 >= 2) {
        atomicAdd(&a.prof[28], 1ull);
        multi_win = true;
      }
    }
    Pc_re += tot[0]; Pc_im += tot[1]; Zc += tot[2]; Cc += tot[3]; Ac = Aend;
    hp->wbits[((int)s * kScIters + it) * kScT + tid] = (uint16_t)bits;
    __syncthreads();   // every lane's phase B reads of the ring precede the next block's writes
  }
  if (a.prof && tid == 0) {
    atomicAdd(&a.prof[22], (unsigned long long)wall_clock64() - t_setup - t_res);
    atomicAdd(&a.prof[16], pq_ring);
    atomicAdd(&a.prof[17], pq_scan);
    atomicAdd(&a.prof[18], pq_walk);
    atomicAdd(&a.prof[19], pq_first);
  }
  }
  // the item's last antenna pass: plateau rule over every antenna's words
  if (a.prof && tid == 0) {
    const unsigned long long t = (unsigned long long)wall_clock64();
    atomicMax(&a.prof[1], t);
    atomicAdd(&a.prof[3], t - t_item);
    atomicAdd(&a.prof[4], 1ull);
    atomicAdd(&a.prof[7], t_res);
    // slowest pass: duration (10 ns), iterations, resolve time (10 ns), packed
    const unsigned long long dur = t - t_item;
    atomicMax(&a.prof[13], (dur << 32) | ((unsigned long long)(it_hi - it_lo + 1) << 24) |
                               (t_res & 0xFFFFFFull));
    atomicMax(&a.prof[14], ((unsigned long long)n_win << 32) | n_smp);
    if (multi_win) atomicMax(&a.prof[29], dur);
    atomicAdd(&a.prof[15], (unsigned long long)n_smp);
  }
  __threadfence();
  __syncthreads();
  if (tid == 0)
    s_last = (__hip_atomic_fetch_add(&hp->arrived, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
              hp->n_done - 1u) ? 1 : 0;
  __syncthreads();
  if (s_last && !(a.diag & 16)) {
    // the acquire of the arrival counter (agent scope) invalidated this CU's L1: plain 16-byte
    // loads see every antenna pass's words
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    const uint32_t n_done = hp->n_done;
    const uint4 *src = reinterpret_cast<const uint4 *>(hp->wbits);
    uint4 *dst = reinterpret_cast<uint4 *>(fwb);
    for (int i = tid; i < (int)n_done * kScIters * kScT / 8; i += kScT) dst[i] = src[i];
    if (tid < (int)n_done) flo[tid] = hp->lo[tid];
    if (tid == 0) s_min = ~0ull;
    __syncthreads();
    const unsigned long long tf0 = a.prof ? (unsigned long long)wall_clock64() : 0ull;
    int par = 0;
    const int any = (int64_t)a.cp + 2 > kScS
                        ? item_conditions_walk(fwb, acond, n_done, hp->w0, hp->c0, hp->cend,
                                               (int64_t)a.cp)
                        : item_conditions(fwb, acond, n_done, hp->w0, hp->c0, hp->cend,
                                          (int64_t)a.cp, run_ws, par);
    const unsigned long long tf1 = a.prof ? (unsigned long long)wall_clock64() : 0ull;
    if (any) item_record(a, hp->f, hp->chunk, hp->w0, fwb, acond, flo, s_min);
    if (a.prof && tid == 0) {
      atomicAdd(&a.prof[10], tf1 - tf0);
      atomicAdd(&a.prof[11], (unsigned long long)wall_clock64() - tf1);
      atomicAdd(&a.prof[12], any ? 1ull : 0ull);
      const unsigned long long t = (unsigned long long)wall_clock64();
      atomicMax(&a.prof[2], t);
      atomicAdd(&a.prof[6], 1ull);
    }
  }
  __syncthreads();
  if (slot + gridDim.y < count) {   // the next slot's record (uniform)
    const ScHot *hn = a.hot + slot + gridDim.y;
    f_n = hn->f;
    w0_n = hn->w0;
    chunk_n = hn->chunk;
  }
  }
}

size_t sc_lds_bytes(uint32_t M, uint32_t N) {
  const int ring = (int)M + kScIt;
  return sizeof(float2) * (size_t)(ring + ((ring >> 5) << 1)) +
         sizeof(uint16_t) * (size_t)N * kScIters * kScT;
}

void launch_sc(const ScArgs &a, uint32_t n_frames, uint32_t n_cu, hipStream_t s) {
  const size_t shm = sc_lds_bytes(a.M, a.N);
  static size_t set_shm = 0;
  static int per_cu = 0;
  if (shm != set_shm) {
    (void)hipFuncSetAttribute((const void *)sc_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)shm);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, sc_kernel, kScT, shm) !=
            hipSuccess || per_cu < 1)
      per_cu = 1;
    set_shm = shm;
  }
  const uint64_t total = (a.chunk_hi - a.chunk_lo) * (uint64_t)n_frames;
  const uint32_t grid = (uint32_t)std::min<uint64_t>(total, (uint64_t)n_cu * per_cu);
  if (grid) hipLaunchKernelGGL(sc_kernel, dim3(grid), dim3(kScT), shm, s, a, n_frames);
  if (a.prof) fprintf(stderr, "sc grid %u (per_cu %d, n_cu %u, lds %zu)\n", grid, per_cu, n_cu, shm);
}

size_t sc_table_bytes(uint32_t M) {
  const int ring = (int)M + kScIt;
  return sizeof(float2) * (size_t)(ring + ((ring >> 5) << 1));
}

void launch_sc_hot(const ScArgs &a, hipStream_t s) {
  if (!a.hot || !a.hot_cap) return;
  const size_t shm = sc_table_bytes(a.M);
  static size_t set_shm = 0;
  if (shm != set_shm) {
    (void)hipFuncSetAttribute((const void *)sc_resolve_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    set_shm = shm;
  }
  const uint32_t gx = std::min<uint32_t>(a.hot_cap, 256);
  static const int diag = [] { const char *e = getenv("RMIMO_SC_DIAG"); return e ? atoi(e) : 0; }();
  ScArgs ad = a;
  if (diag & 4) ad.hot_cap = 0;      // diagnostics: same grid, every workgroup exits at once
  // (item slot, antenna, window slot): the windows of one antenna in parallel
  const uint32_t gxr = std::min<uint32_t>(a.hot_cap, 64);
  if (!(diag & 1))
    hipLaunchKernelGGL(sc_resolve_kernel, dim3(gxr, a.N, kResWin), dim3(kScT), shm, s, ad);
  if (!(diag & 2)) hipLaunchKernelGGL(sc_finalize_kernel, dim3(gx), dim3(kScT), 0, s, a);
}

void launch_sc_finalize(const ScArgs &a, hipStream_t s) {
  if (a.hot && a.hot_cap)
    hipLaunchKernelGGL(sc_finalize_kernel, dim3(std::min<uint32_t>(a.hot_cap, 256)), dim3(kScT), 0,
                       s, a);
}

__global__ __launch_bounds__(256) void fill_kernel(FillArgs a) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (int k = 0; k < a.count; k++) {
    uint32_t *p = a.p[k];
    const uint32_t v = a.v[k];
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n[k]; i += stride)
      p[i] = v;
  }
}

void launch_fill(const FillArgs &a, hipStream_t s) {
  uint64_t mx = 0;
  for (int k = 0; k < a.count; k++) mx = std::max<uint64_t>(mx, a.n[k]);
  if (!mx) return;
  const uint32_t grid = (uint32_t)std::min<uint64_t>((mx + 255) / 256, 1024);
  hipLaunchKernelGGL(fill_kernel, dim3(grid), dim3(256), 0, s, a);
}

__global__ void sc_snapshot_kernel(uint32_t *dst, const uint32_t *src) { *dst = *src; }

void launch_sc_snapshot(uint32_t *dst, const uint32_t *src, hipStream_t s) {
  hipLaunchKernelGGL(sc_snapshot_kernel, dim3(1), dim3(1), 0, s, dst, src);
}

void launch_sc_screen(const ScreenArgs &a, uint32_t n_frames, hipStream_t s) {
  const uint64_t end = a.chunk_hi ? std::min<uint64_t>(a.frame_len, a.chunk_hi * a.chunk_len)
                                  : (uint64_t)a.frame_len;
  const uint64_t span = end - std::min<uint64_t>(end, a.chunk_lo * a.chunk_len);
  // positions per workgroup: 8192 up to M = 2048 (twice the workgroups; a phase-1 screen of
  // 64 C3 captures is ~830 workgroups at 16384, under one per SIMD), 16384 above (the 2D-block
  // history, M positions, would be half of an 8192 span)
  const int sp = a.M <= 2048 ? 8192 : kScrSpan;
  const uint32_t gx = (uint32_t)((span + sp - 1) / sp);
  if (!gx) return;
  if (sp == 8192) {
    if (a.sc16)
      hipLaunchKernelGGL((sc_screen_kernel<true, 8192>), dim3(gx, n_frames), dim3(kScrT), 0, s, a);
    else
      hipLaunchKernelGGL((sc_screen_kernel<false, 8192>), dim3(gx, n_frames), dim3(kScrT), 0, s, a);
  } else if (a.sc16) {
    hipLaunchKernelGGL((sc_screen_kernel<true, kScrSpan>), dim3(gx, n_frames), dim3(kScrT), 0, s, a);
  } else {
    hipLaunchKernelGGL((sc_screen_kernel<false, kScrSpan>), dim3(gx, n_frames), dim3(kScrT), 0, s, a);
  }
}

void launch_sc_exact(const ScArgs &a, hipStream_t s) {
  const size_t shm = sc_table_bytes(a.M) +
                     sizeof(float) * (size_t)((a.M + kResSpread + 3) & ~3u) +
                     sizeof(float2) * (size_t)(a.M / 2 + kResSpread);
  static size_t set_shm[2] = {0, 0};
  const int v = a.sc16 ? 1 : 0;
  auto kern = a.sc16 ? sc_exact_kernel<true> : sc_exact_kernel<false>;
  if (shm != set_shm[v]) {
    (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)shm);
    set_shm[v] = shm;
  }
  hipLaunchKernelGGL(kern, dim3(a.N, std::min<uint32_t>(a.hot_cap, 256)), dim3(kScT), shm, s, a);
}

__global__ __launch_bounds__(256) void sc_trace_kernel(const float2 *iq, uint64_t stride,
                                                       uint32_t M, int64_t lo, int64_t n,
                                                       float *out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  out[(uint64_t)blockIdx.y * n + i] = sc_exact(iq + (uint64_t)blockIdx.y * stride, lo + i, M);
}

void launch_sc_trace(const float2 *iq, uint64_t stride, uint32_t rows, uint32_t M, int64_t lo,
                     int64_t hi, float *out, hipStream_t s) {
  if (hi <= lo || rows == 0) return;
  const int64_t n = hi - lo;
  hipLaunchKernelGGL(sc_trace_kernel, dim3((uint32_t)((n + 255) / 256), rows), dim3(256), 0, s,
                     iq, stride, M, lo, n, out);
}

void launch_plateau(const PlateauArgs &a, uint32_t n_frames, hipStream_t s) {
  if (a.sc16) hipLaunchKernelGGL(plateau_kernel<true>, dim3(n_frames), dim3(64), 0, s, a);
  else hipLaunchKernelGGL(plateau_kernel<false>, dim3(n_frames), dim3(64), 0, s, a);
}

void launch_stream_walk(const PlateauArgs &a, uint32_t n_caps, hipStream_t s) {
  if (a.sc16) hipLaunchKernelGGL(stream_walk_kernel<true>, dim3(n_caps), dim3(64), 0, s, a);
  else hipLaunchKernelGGL(stream_walk_kernel<false>, dim3(n_caps), dim3(64), 0, s, a);
  if (a.fpc > 1) {
    if (a.sc16)
      hipLaunchKernelGGL(stream_cert_kernel<true>, dim3(a.fpc - 1, a.N, n_caps), dim3(kScT), 0,
                         s, a);
    else
      hipLaunchKernelGGL(stream_cert_kernel<false>, dim3(a.fpc - 1, a.N, n_caps), dim3(kScT), 0,
                         s, a);
    hipLaunchKernelGGL(stream_fixup_kernel, dim3(n_caps), dim3(64), 0, s, a);
  }
}

}  // namespace mimo

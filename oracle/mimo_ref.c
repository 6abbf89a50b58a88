/*
 * oracle/mimo_ref.c -- TEST INFRASTRUCTURE ONLY. See mimo_ref.h for scope and pinning.
 *
 * Compiled with -ffp-contract=off so every fp32 operation is a single IEEE rounding,
 * which the GPU path reproduces bit for bit where parity must be exact (S&C metric).
 * Each function cites the reference lines it restates.
 */
#include "mimo_ref.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ====================================================================================
 * liquid msequence (used at mimo/main.cc:1268-1270, framing.cc:1075, 1240)
 * ==================================================================================== */
void ref_msequence_init(ref_msequence *ms, uint32_t m, uint32_t g, uint32_t a) {
  ms->m = m;
  ms->g = g >> 1;
  ms->a = 0;
  for (uint32_t i = 0; i < m; i++) { /* initial state is bit-reversed (0001 -> 1000) */
    ms->a <<= 1;
    ms->a |= (a & 1u);
    a >>= 1;
  }
  ms->n = (m >= 32) ? 0xFFFFFFFFu : ((1u << m) - 1u);
  ms->v = ms->a;
  ms->b = 0;
}

static uint32_t parity32(uint32_t x) {
  x ^= x >> 16; x ^= x >> 8; x ^= x >> 4; x ^= x >> 2; x ^= x >> 1;
  return x & 1u;
}

uint32_t ref_msequence_advance(ref_msequence *ms) {
  ms->b = parity32(ms->v & ms->g);
  ms->v = ((ms->v << 1) | ms->b) & ms->n;
  return ms->b;
}

uint32_t ref_msequence_generate_symbol(ref_msequence *ms, uint32_t bps) {
  uint32_t s = 0;
  for (uint32_t i = 0; i < bps; i++) { s <<= 1; s |= ref_msequence_advance(ms); }
  return s;
}

void ref_msequence_reset(ref_msequence *ms) { ms->v = ms->a; }

uint64_t ref_msequence_period(uint32_t m, uint32_t g, uint32_t a) {
  ref_msequence ms;
  ref_msequence_init(&ms, m, g, a);
  uint32_t v0 = ms.v;
  uint64_t lim = (1ull << m) + 1;
  for (uint64_t k = 1; k <= lim; k++) {
    ref_msequence_advance(&ms);
    if (ms.v == v0) return k;
  }
  return 0;
}

void ref_msequence_draw_bits(uint32_t m, uint32_t g, uint32_t a, uint32_t count,
                             uint8_t *out) {
  ref_msequence ms;
  ref_msequence_init(&ms, m, g, a);
  for (uint32_t i = 0; i < count; i++)
    out[i] = (uint8_t)(ref_msequence_generate_symbol(&ms, 1) & 1u);
}

/* ====================================================================================
 * sctype helpers, framing.cc:949-1030
 * ==================================================================================== */
void ref_init_default_sctype(uint8_t *p, uint32_t M) { /* framing.cc:949-954 */
  for (uint32_t i = 0; i < M; i++) p[i] = REF_SC_DATA;
}

void ref_init_liquid_sctype(uint8_t *p, uint32_t M) { /* framing.cc:956-997 */
  uint32_t M2 = M / 2;
  uint32_t G = M / 10; /* ADD_NULL_CARRIERS */
  if (G < 2) G = 2;
  uint32_t P = (M > 34) ? 8 : 4, P2 = P / 2;
  for (uint32_t i = 0; i < M; i++) p[i] = REF_SC_NULL;
  for (uint32_t i = 1; i + G < M2; i++) p[i] = (((i + P2) % P) == 0) ? REF_SC_PILOT : REF_SC_DATA;
  for (uint32_t i = 1; i + G < M2; i++) {
    uint32_t k = M - i;
    p[k] = (((i + P2) % P) == 0) ? REF_SC_PILOT : REF_SC_DATA;
  }
}

int ref_validate_sctype(const uint8_t *p, uint32_t M, uint32_t *M_null, uint32_t *M_pilot,
                        uint32_t *M_data) { /* framing.cc:1000-1030, error code not exit */
  uint32_t n0 = 0, n1 = 0, n2 = 0;
  for (uint32_t i = 0; i < M; i++) {
    if (p[i] == REF_SC_NULL) n0++;
    else if (p[i] == REF_SC_PILOT) n1++;
    else if (p[i] == REF_SC_DATA) n2++;
    else return -1;
  }
  *M_null = n0; *M_pilot = n1; *M_data = n2;
  return 0;
}

/* ====================================================================================
 * FFT: unnormalised DFT, FFTW convention (forward e^{-i}, backward e^{+i}).
 * Stockham radix-4 (+ one radix-2) on split re/im arrays; twiddles computed in double.
 * ==================================================================================== */
typedef struct {
  uint32_t n, npass;
  uint32_t radix[32], ns[32];
  float *twr[32][3], *twi[32][3]; /* per pass, r = 1..R-1, index k in [0, Ns) (forward) */
  float *br, *bi, *cr, *ci;       /* work buffers */
} fft_plan;

#define FFT_PLAN_CACHE 16
static __thread fft_plan *g_plans[FFT_PLAN_CACHE]; /* per thread: plans own work buffers */

static fft_plan *fft_get_plan(uint32_t n) {
  for (int i = 0; i < FFT_PLAN_CACHE; i++)
    if (g_plans[i] && g_plans[i]->n == n) return g_plans[i];
  fft_plan *pl = (fft_plan *)calloc(1, sizeof(fft_plan));
  pl->n = n;
  uint32_t lg = 0;
  while ((1u << lg) < n) lg++;
  uint32_t ns = 1, np = 0;
  while (ns < n) {
    uint32_t r = ((n / ns) % 4 == 0) ? 4 : 2;
    pl->radix[np] = r;
    pl->ns[np] = ns;
    for (uint32_t q = 1; q < r; q++) {
      pl->twr[np][q - 1] = (float *)malloc(sizeof(float) * ns);
      pl->twi[np][q - 1] = (float *)malloc(sizeof(float) * ns);
      for (uint32_t k = 0; k < ns; k++) {
        double ang = -2.0 * M_PI * (double)(q * k) / (double)(ns * r);
        pl->twr[np][q - 1][k] = (float)cos(ang);
        pl->twi[np][q - 1][k] = (float)sin(ang);
      }
    }
    ns *= r;
    np++;
  }
  pl->npass = np;
  pl->br = (float *)malloc(sizeof(float) * n);
  pl->bi = (float *)malloc(sizeof(float) * n);
  pl->cr = (float *)malloc(sizeof(float) * n);
  pl->ci = (float *)malloc(sizeof(float) * n);
  for (int i = 0; i < FFT_PLAN_CACHE; i++)
    if (!g_plans[i]) { g_plans[i] = pl; return pl; }
  /* cache full: evict slot 0 (leak-free enough for test use) */
  g_plans[0] = pl;
  return pl;
}

void ref_fft(ref_cf32 *x, uint32_t n, int inverse) {
  if (n <= 1) return;
  fft_plan *pl = fft_get_plan(n);
  float *xr = pl->br, *xi = pl->bi, *yr = pl->cr, *yi = pl->ci;
  for (uint32_t i = 0; i < n; i++) { xr[i] = x[i].re; xi[i] = inverse ? -x[i].im : x[i].im; }
  /* inverse transform = conj(FFT(conj(x))) : exact sign flips */
  for (uint32_t ps = 0; ps < pl->npass; ps++) {
    uint32_t R = pl->radix[ps], Ns = pl->ns[ps], nr = n / R;
    if (R == 4) {
      const float *w1r = pl->twr[ps][0], *w1i = pl->twi[ps][0];
      const float *w2r = pl->twr[ps][1], *w2i = pl->twi[ps][1];
      const float *w3r = pl->twr[ps][2], *w3i = pl->twi[ps][2];
      for (uint32_t b = 0; b < nr / Ns; b++) {
        const float *a0r = xr + b * Ns, *a0i = xi + b * Ns;
        const float *a1r = a0r + nr, *a1i = a0i + nr;
        const float *a2r = a1r + nr, *a2i = a1i + nr;
        const float *a3r = a2r + nr, *a3i = a2i + nr;
        float *o0r = yr + b * Ns * 4, *o0i = yi + b * Ns * 4;
        float *o1r = o0r + Ns, *o1i = o0i + Ns, *o2r = o1r + Ns, *o2i = o1i + Ns;
        float *o3r = o2r + Ns, *o3i = o2i + Ns;
        for (uint32_t k = 0; k < Ns; k++) {
          float x0r = a0r[k], x0i = a0i[k];
          float t1r = a1r[k], t1i = a1i[k], t2r = a2r[k], t2i = a2i[k];
          float t3r = a3r[k], t3i = a3i[k];
          float x1r = t1r * w1r[k] - t1i * w1i[k], x1i = t1r * w1i[k] + t1i * w1r[k];
          float x2r = t2r * w2r[k] - t2i * w2i[k], x2i = t2r * w2i[k] + t2i * w2r[k];
          float x3r = t3r * w3r[k] - t3i * w3i[k], x3i = t3r * w3i[k] + t3i * w3r[k];
          float b0r = x0r + x2r, b0i = x0i + x2i, b1r = x0r - x2r, b1i = x0i - x2i;
          float b2r = x1r + x3r, b2i = x1i + x3i;
          float b3r = x1i - x3i, b3i = x3r - x1r; /* (x1-x3)*(-i) */
          o0r[k] = b0r + b2r; o0i[k] = b0i + b2i;
          o2r[k] = b0r - b2r; o2i[k] = b0i - b2i;
          o1r[k] = b1r + b3r; o1i[k] = b1i + b3i;
          o3r[k] = b1r - b3r; o3i[k] = b1i - b3i;
        }
      }
    } else {
      const float *w1r = pl->twr[ps][0], *w1i = pl->twi[ps][0];
      for (uint32_t b = 0; b < nr / Ns; b++) {
        const float *a0r = xr + b * Ns, *a0i = xi + b * Ns;
        const float *a1r = a0r + nr, *a1i = a0i + nr;
        float *o0r = yr + b * Ns * 2, *o0i = yi + b * Ns * 2;
        float *o1r = o0r + Ns, *o1i = o0i + Ns;
        for (uint32_t k = 0; k < Ns; k++) {
          float t1r = a1r[k], t1i = a1i[k];
          float x1r = t1r * w1r[k] - t1i * w1i[k], x1i = t1r * w1i[k] + t1i * w1r[k];
          o0r[k] = a0r[k] + x1r; o0i[k] = a0i[k] + x1i;
          o1r[k] = a0r[k] - x1r; o1i[k] = a0i[k] - x1i;
        }
      }
    }
    float *t;
    t = xr; xr = yr; yr = t;
    t = xi; xi = yi; yi = t;
  }
  for (uint32_t i = 0; i < n; i++) { x[i].re = xr[i]; x[i].im = inverse ? -xi[i] : xi[i]; }
}

/* ====================================================================================
 * S0 / S1 generation, framing.cc:1054-1111 (USE_NEW_INIT_S0) and 1214-1262 (BPSK S1)
 * ==================================================================================== */
void ref_init_S0(const uint8_t *p, uint32_t M, const uint8_t *bits, ref_cf32 *S0,
                 ref_cf32 *s0) {
  uint32_t M_S0 = 0;
  for (uint32_t i = 0; i < M; i++) {
    uint32_t s = bits[i] & 1u; /* msequence_generate_symbol(ms,1)&1 drawn for every i */
    if (p[i] == REF_SC_NULL) { S0[i].re = 0.0f; S0[i].im = 0.0f; }
    else if ((i % 2) == 0) { S0[i].re = s ? 1.0f : -1.0f; S0[i].im = 0.0f; M_S0++; }
    else { S0[i].re = 0.0f; S0[i].im = 0.0f; }
  }
  float dn = (float)sqrt(1.0 / (double)(float)M_S0); /* framing.cc:1100 */
  memcpy(s0, S0, sizeof(ref_cf32) * M);
  ref_fft(s0, M, 1);
  for (uint32_t i = 0; i < M; i++) { s0[i].re = s0[i].re * dn; s0[i].im = s0[i].im * dn; }
}

void ref_init_S1(const uint8_t *p, uint32_t M, uint32_t nac, const uint8_t *bits,
                 ref_cf32 *S1, ref_cf32 *s1) {
  float dn = (float)sqrt(1.0 / (double)(float)M); /* framing.cc:1228: sqrt(1/M), not M_S1 */
  for (uint32_t j = 0; j < nac; j++) {
    ref_cf32 *Sj = S1 + (size_t)M * j, *sj = s1 + (size_t)M * j;
    for (uint32_t i = 0; i < M; i++) {
      uint32_t s = bits[(size_t)j * M + i] & 1u;
      if (p[i] == REF_SC_NULL) { Sj[i].re = 0.0f; Sj[i].im = 0.0f; }
      else { Sj[i].re = s ? 1.0f : -1.0f; Sj[i].im = 0.0f; } /* BPSK_CONSTELLATION[s] */
    }
    memcpy(sj, Sj, sizeof(ref_cf32) * M);
    ref_fft(sj, M, 1);
    for (uint32_t i = 0; i < M; i++) { sj[i].re = sj[i].re * dn; sj[i].im = sj[i].im * dn; }
  }
}

/* ====================================================================================
 * complex helpers (std::complex<float> semantics without FMA)
 * ==================================================================================== */
static inline ref_cf32 cmul(ref_cf32 a, ref_cf32 b) {
  ref_cf32 r;
  r.re = a.re * b.re - a.im * b.im;
  r.im = a.re * b.im + a.im * b.re;
  return r;
}
static inline ref_cf32 cadd(ref_cf32 a, ref_cf32 b) {
  ref_cf32 r = {a.re + b.re, a.im + b.im};
  return r;
}
static inline ref_cf32 csub(ref_cf32 a, ref_cf32 b) {
  ref_cf32 r = {a.re - b.re, a.im - b.im};
  return r;
}
static inline ref_cf32 cconj(ref_cf32 a) {
  ref_cf32 r = {a.re, -a.im};
  return r;
}
static inline ref_cf32 cneg(ref_cf32 a) {
  ref_cf32 r = {-a.re, -a.im};
  return r;
}
/* a / b : (a * conj b) / |b|^2 -- exact for b = +-1 */
static inline ref_cf32 cdiv(ref_cf32 a, ref_cf32 b) {
  float d = b.re * b.re + b.im * b.im;
  ref_cf32 r;
  r.re = (a.re * b.re + a.im * b.im) / d;
  r.im = (a.im * b.re - a.re * b.im) / d;
  return r;
}

/* ====================================================================================
 * 2x2 invert, framing.cc:1344-1367 (INVERT_TO_UNITY false)
 * W, G row-major 2x2: W[0]=W00 W[1]=W01 W[2]=W10 W[3]=W11
 * ==================================================================================== */
float ref_invert2(ref_cf32 W[4], const ref_cf32 G[4]) {
  ref_cf32 det = csub(cmul(G[0], G[3]), cmul(G[1], G[2]));
  ref_cf32 det_inv = cconj(det);
  W[0] = cmul(det_inv, G[3]);
  W[3] = cmul(det_inv, G[0]);
  W[2] = cmul(cneg(det_inv), G[2]);
  W[1] = cmul(cneg(det_inv), G[1]);
  return 1.0f / (det.re * det.re + det.im * det.im);
}

/* ====================================================================================
 * square Gray QAM (build's definition; the reference used liquid ARB32OPT, main.cc:1203)
 * ==================================================================================== */
static uint32_t qam_bits_per_dim(uint32_t order) {
  uint32_t b = 0;
  while ((1u << (2 * b)) < order) b++;
  return b;
}
static inline uint32_t gray_enc(uint32_t m) { return m ^ (m >> 1); }
static inline uint32_t gray_dec(uint32_t g) {
  uint32_t m = g;
  for (uint32_t s = 1; s < 16; s <<= 1) m ^= m >> s;
  return m;
}
static float qam_scale(uint32_t order) {
  uint32_t L = 1u << qam_bits_per_dim(order);
  return (float)(1.0 / sqrt(2.0 * ((double)L * L - 1.0) / 3.0));
}
static float qam_inv_scale(uint32_t order) {
  uint32_t L = 1u << qam_bits_per_dim(order);
  return (float)sqrt(2.0 * ((double)L * L - 1.0) / 3.0);
}

ref_cf32 ref_qam_point(uint32_t index, uint32_t order) {
  uint32_t b = qam_bits_per_dim(order), L = 1u << b;
  uint32_t mI = gray_dec(index >> b), mQ = gray_dec(index & (L - 1));
  float sc = qam_scale(order);
  ref_cf32 r;
  r.re = (float)(int32_t)(2 * mI - (L - 1)) * sc;
  r.im = (float)(int32_t)(2 * mQ - (L - 1)) * sc;
  return r;
}

static inline uint32_t qam_level(float v, uint32_t L) {
  float t = (v + (float)L) * 0.5f;
  if (t != t) return 0; /* NaN -> level 0 */
  float f = floorf(t);
  int32_t m = (f < 0.0f) ? 0 : ((f > (float)(L - 1)) ? (int32_t)(L - 1) : (int32_t)f);
  return (uint32_t)m;
}

uint32_t ref_qam_demap(ref_cf32 y, uint32_t order) {
  uint32_t b = qam_bits_per_dim(order), L = 1u << b;
  float is = qam_inv_scale(order);
  uint32_t mI = qam_level(y.re * is, L), mQ = qam_level(y.im * is, L);
  return (gray_enc(mI) << b) | gray_enc(mQ);
}

/* ====================================================================================
 * counter-based PRNG (shared bit-for-bit with the GPU synthesiser)
 * ==================================================================================== */
static inline uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
uint64_t ref_hash5(uint64_t seed, uint64_t dom, uint64_t a, uint64_t b, uint64_t c) {
  uint64_t h = mix64(seed ^ (dom * 0xD6E8FEB86659FD93ull));
  h = mix64(h ^ a);
  h = mix64(h ^ b);
  h = mix64(h ^ c);
  return h;
}
static ref_cf32 hash_cnormal(uint64_t h) { /* CN(0,1) via Box-Muller */
  float u1 = (float)((h >> 40) + 1ull) * 5.9604644775390625e-08f;
  float u2 = (float)((h >> 16) & 0xFFFFFFull) * 5.9604644775390625e-08f;
  float r = sqrtf(-2.0f * logf(u1));
  float th = 6.283185307179586f * u2;
  ref_cf32 g;
  g.re = r * cosf(th) * 0.70710678118654752f;
  g.im = r * sinf(th) * 0.70710678118654752f;
  return g;
}
enum { DOM_DATA = 1, DOM_CHAN = 2, DOM_NOISE = 3, DOM_OFFSET = 4 };

/* ====================================================================================
 * framegen, framing.cc:79-266
 * ==================================================================================== */
struct ref_framegen {
  uint32_t M, cp, SL, N, nac, M_null, M_pilot, M_data;
  uint8_t *p;
  float dn;
  ref_cf32 *S0, *s0, *S1, *s1; /* S1/s1: [N][nac*M] */
  ref_cf32 *X;
};

ref_framegen *ref_framegen_create(uint32_t M, uint32_t cp, uint32_t N, uint32_t nac,
                                  const uint8_t *p, const uint8_t *s0_bits,
                                  const uint8_t *s1_bits) {
  ref_framegen *fg = (ref_framegen *)calloc(1, sizeof(*fg));
  fg->M = M; fg->cp = cp; fg->SL = M + cp; fg->N = N; fg->nac = nac;
  fg->p = (uint8_t *)malloc(M);
  memcpy(fg->p, p, M);
  if (ref_validate_sctype(p, M, &fg->M_null, &fg->M_pilot, &fg->M_data) != 0) {
    free(fg->p); free(fg); return NULL;
  }
  fg->S0 = (ref_cf32 *)malloc(sizeof(ref_cf32) * M);
  fg->s0 = (ref_cf32 *)malloc(sizeof(ref_cf32) * M);
  ref_init_S0(p, M, s0_bits, fg->S0, fg->s0);
  fg->dn = 1.0f / sqrtf((float)(fg->M_pilot + fg->M_data)); /* framing.cc:115 */
  fg->S1 = (ref_cf32 *)malloc(sizeof(ref_cf32) * (size_t)N * nac * M);
  fg->s1 = (ref_cf32 *)malloc(sizeof(ref_cf32) * (size_t)N * nac * M);
  for (uint32_t t = 0; t < N; t++)
    ref_init_S1(p, M, nac, s1_bits + (size_t)t * nac * M, fg->S1 + (size_t)t * nac * M,
                fg->s1 + (size_t)t * nac * M);
  fg->X = (ref_cf32 *)malloc(sizeof(ref_cf32) * M);
  return fg;
}

void ref_framegen_destroy(ref_framegen *fg) {
  if (!fg) return;
  free(fg->p); free(fg->S0); free(fg->s0); free(fg->S1); free(fg->s1); free(fg->X);
  free(fg);
}

uint32_t ref_framegen_write_sync_words(ref_framegen *fg, ref_cf32 **tx) { /* :169-208 */
  uint32_t M = fg->M, cp = fg->cp, idx = 0;
  uint32_t total = (fg->nac * fg->N + 1) * (M + cp);
  for (uint32_t s = 0; s < fg->N; s++) memset(tx[s], 0, sizeof(ref_cf32) * total);
  memcpy(tx[0] + idx, fg->s0 + M - cp, sizeof(ref_cf32) * cp); idx += cp;
  memcpy(tx[0] + idx, fg->s0, sizeof(ref_cf32) * M); idx += M;
  for (uint32_t ac = 0; ac < fg->nac; ac++) {
    for (uint32_t s = 0; s < fg->N; s++) {
      const ref_cf32 *code = fg->s1 + (size_t)s * fg->nac * M + (size_t)M * ac;
      memcpy(tx[s] + idx, code + M - cp, sizeof(ref_cf32) * cp); idx += cp;
      memcpy(tx[s] + idx, code, sizeof(ref_cf32) * M); idx += M;
    }
  }
  return idx;
}

uint32_t ref_framegen_assemble_mimo_packet(ref_framegen *fg, ref_cf32 **tx,
                                           ref_cf32 *const *in) { /* :210-235 */
  uint32_t M = fg->M, cp = fg->cp;
  for (uint32_t s = 0; s < fg->N; s++) {
    for (uint32_t i = 0, j = 0; i < M; i++) {
      if (fg->p[i] == REF_SC_NULL) { fg->X[i].re = 0.0f; fg->X[i].im = 0.0f; }
      else fg->X[i] = in[s][j++];
    }
    ref_fft(fg->X, M, 1);
    for (uint32_t i = 0; i < M; i++) { fg->X[i].re *= fg->dn; fg->X[i].im *= fg->dn; }
    memcpy(tx[s], fg->X + M - cp, sizeof(ref_cf32) * cp);
    memcpy(tx[s] + cp, fg->X, sizeof(ref_cf32) * M);
  }
  return M + cp;
}

/* ====================================================================================
 * synthetic capture: tx_worker layout (main.cc:937-1153) + flat Rayleigh + AWGN
 *   [lead zeros SL*(N*nac+1)+u][sync (N*nac+1)*SL][pid data symbols][tail zeros]
 *   all x BASEBAND_GAIN 0.25 (main.cc:1048-1053, config.h:59)
 * ==================================================================================== */
static uint32_t synth_offset(const ref_synth_cfg *c) {
  uint32_t SL = c->M + c->cp;
  if (c->offset >= 0) return (uint32_t)c->offset;
  return (uint32_t)(ref_hash5(c->seed, DOM_OFFSET, c->frame, 0, 0) % SL);
}

uint64_t ref_synth_frame_len(const ref_synth_cfg *c) {
  uint64_t SL = c->M + c->cp;
  return SL * (2ull * c->N * c->nac + 2 + c->pid + c->tail_syms) + synth_offset(c);
}

uint64_t ref_synth_frame(const ref_synth_cfg *c, const uint8_t *p, const uint8_t *s0_bits,
                         const uint8_t *s1_bits, ref_cf32 *const *rx, uint8_t *tx_idx,
                         ref_cf32 *Hout) {
  uint32_t M = c->M, cp = c->cp, SL = M + cp, N = c->N;
  uint64_t L = ref_synth_frame_len(c);
  uint64_t lead = (uint64_t)SL * (N * c->nac + 1) + synth_offset(c);
  ref_framegen *fg = ref_framegen_create(M, cp, N, c->nac, p, s0_bits, s1_bits);
  if (!fg) return 0;
  uint32_t Mocc = fg->M_pilot + fg->M_data;
  /* TX signal per antenna */
  ref_cf32 **tx = (ref_cf32 **)malloc(sizeof(ref_cf32 *) * N);
  for (uint32_t t = 0; t < N; t++) tx[t] = (ref_cf32 *)calloc(L, sizeof(ref_cf32));
  ref_cf32 **tmp = (ref_cf32 **)malloc(sizeof(ref_cf32 *) * N);
  for (uint32_t t = 0; t < N; t++) tmp[t] = tx[t] + lead;
  uint32_t nsync = ref_framegen_write_sync_words(fg, tmp);
  ref_cf32 **in = (ref_cf32 **)malloc(sizeof(ref_cf32 *) * N);
  for (uint32_t t = 0; t < N; t++) in[t] = (ref_cf32 *)malloc(sizeof(ref_cf32) * Mocc);
  for (uint32_t s = 0; s < c->pid; s++) {
    for (uint32_t t = 0; t < N; t++) {
      for (uint32_t j = 0; j < Mocc; j++) {
        uint32_t k = (uint32_t)(ref_hash5(c->seed, DOM_DATA, c->frame, t,
                                          (uint64_t)s * Mocc + j) & (c->qam - 1));
        if (tx_idx) tx_idx[((size_t)t * c->pid + s) * Mocc + j] = (uint8_t)k;
        in[t][j] = ref_qam_point(k, c->qam);
      }
      tmp[t] = tx[t] + lead + nsync + (uint64_t)s * SL;
    }
    ref_framegen_assemble_mimo_packet(fg, tmp, in);
  }
  for (uint32_t t = 0; t < N; t++)
    for (uint64_t n = lead; n < lead + nsync + (uint64_t)c->pid * SL; n++) {
      tx[t][n].re *= 0.25f; tx[t][n].im *= 0.25f;
    }
  /* channel */
  ref_cf32 H[64];
  for (uint32_t r = 0; r < N; r++)
    for (uint32_t t = 0; t < N; t++) {
      if (c->identity_channel) { H[r * N + t].re = (r == t) ? 1.0f : 0.0f; H[r * N + t].im = 0.0f; }
      else H[r * N + t] = hash_cnormal(ref_hash5(c->seed, DOM_CHAN, c->frame, r * N + t, 0));
      if (Hout) Hout[r * N + t] = H[r * N + t];
    }
  float nstd = (float)sqrt(0.0625 * pow(10.0, -(double)c->snr_db / 10.0));
  for (uint32_t r = 0; r < N; r++) {
    for (uint64_t n = 0; n < L; n++) {
      ref_cf32 acc = {0.0f, 0.0f};
      for (uint32_t t = 0; t < N; t++) acc = cadd(acc, cmul(H[r * N + t], tx[t][n]));
      ref_cf32 g = hash_cnormal(ref_hash5(c->seed, DOM_NOISE, c->frame, r, n));
      acc.re = acc.re + g.re * nstd;
      acc.im = acc.im + g.im * nstd;
      rx[r][n] = acc;
    }
  }
  for (uint32_t t = 0; t < N; t++) { free(tx[t]); free(in[t]); }
  free(tx); free(in); free(tmp);
  ref_framegen_destroy(fg);
  return L;
}

/* ====================================================================================
 * exact S&C metric, framing.cc:626-637 with the pinned liquid semantics
 * ==================================================================================== */
static inline ref_cf32 xat(const ref_cf32 *x, int64_t k) {
  ref_cf32 z = {0.0f, 0.0f};
  return (k < 0) ? z : x[k];
}

float ref_sc_metric_at(const ref_cf32 *x, uint64_t n, uint32_t M) {
  uint32_t M2 = M / 2;
  float Pr = 0.0f, Pi = 0.0f, R = 0.0f;
  for (int64_t k = (int64_t)n - M2 + 1; k <= (int64_t)n; k++) { /* oldest -> newest */
    ref_cf32 d = xat(x, k - M2), v = xat(x, k);
    float pr = d.re * v.re - (-d.im) * v.im; /* conj(d) * v */
    float pi = d.re * v.im + (-d.im) * v.re;
    Pr = Pr + (-1.0f) * pr;
    Pi = Pi + (-1.0f) * pi;
  }
  for (int64_t k = (int64_t)n - M + 1; k <= (int64_t)n; k++) {
    ref_cf32 v = xat(x, k);
    float z = v.re * v.re + v.im * v.im;
    R = R + 0.5f * z;
  }
  return (Pr * Pr + Pi * Pi) / (R * R);
}

/* ====================================================================================
 * framesync, framing.cc:268-944
 * ==================================================================================== */
struct ref_framesync {
  ref_rx_cfg cfg;
  uint32_t M, M2, cp, SL, N, nac;
  uint8_t *p;
  int32_t *occ; /* sc -> occupied index or -1 */
  uint32_t M_null, M_pilot, M_data, M_occ;
  uint64_t acb_len, tx_sig_len, win_len;
  float dn;
  ref_cf32 *S0, *s0, *S1, *s1; /* S1/s1 [N][nac*M] */
  /* S&C state per stream */
  ref_cf32 *dly;  /* [N][M2] */
  ref_cf32 *xc;   /* [N][M2] cross-correlator window (p values) */
  float *nz;      /* [N][M]  normaliser window (|x|^2) */
  uint32_t dly_pos, xc_pos, nz_pos;
  ref_cf32 *win;  /* [N][win_len] ring */
  uint64_t win_head;
  uint64_t *plateau_start, *plateau_end;
  int *in_plateau;
  uint64_t sync_index, nsp, trigger;
  int state;
  /* opt-in CFO (cfo_mode): estimates, and the decode's derotation of the current symbol */
  double cfo_eps0, cfo_delta, cfo_nu;
  uint64_t cfo_body;
  /* channel */
  ref_cf32 *G, *W; /* [M][N][N] */
  float *gain;     /* [M_occ] */
  float noise_var;
  uint32_t *corr_idx; float *corr_max; uint32_t *s0_idx; float *s0_max;
  /* decode */
  ref_cf32 *sym; uint32_t sym_count;
  ref_cf32 *outs; uint32_t n_out, cap_out;
  /* trace */
  float *trace; uint64_t trace_len, trace_cap;
  float *ctrace, *s0trace;
  /* CPU-baseline phase clocks (wall seconds), see ref_framesync_get_phase_times */
  double t_phase[4];
};

static double wall_now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static int is_occ(const ref_framesync *fs, uint32_t sc) { return fs->p[sc] != REF_SC_NULL; }

ref_framesync *ref_framesync_create(const ref_rx_cfg *cfg, const uint8_t *p,
                                    const uint8_t *s0_bits, const uint8_t *s1_bits) {
  ref_framesync *fs = (ref_framesync *)calloc(1, sizeof(*fs));
  fs->cfg = *cfg;
  uint32_t M = cfg->M, N = cfg->N;
  fs->M = M; fs->M2 = M / 2; fs->cp = cfg->cp; fs->SL = M + cfg->cp; fs->N = N;
  fs->nac = cfg->nac;
  fs->acb_len = (uint64_t)fs->SL * (cfg->nac * N + 4);   /* framing.cc:284 */
  fs->tx_sig_len = (uint64_t)cfg->pid_max * fs->SL;     /* framing.cc:285 */
  fs->win_len = fs->acb_len + fs->tx_sig_len;           /* framing.cc:387-388 */
  fs->p = (uint8_t *)malloc(M);
  memcpy(fs->p, p, M);
  if (ref_validate_sctype(p, M, &fs->M_null, &fs->M_pilot, &fs->M_data) != 0) {
    free(fs->p); free(fs); return NULL;
  }
  fs->M_occ = fs->M_data + fs->M_pilot;
  fs->occ = (int32_t *)malloc(sizeof(int32_t) * M);
  for (uint32_t i = 0, j = 0; i < M; i++) fs->occ[i] = (p[i] != REF_SC_NULL) ? (int32_t)j++ : -1;
  fs->dn = 1.0f / sqrtf((float)fs->M_occ); /* framing.cc:330 */
  size_t MNN = (size_t)M * N * N;
  fs->G = (ref_cf32 *)calloc(MNN, sizeof(ref_cf32));
  fs->W = (ref_cf32 *)calloc(MNN, sizeof(ref_cf32));
  for (uint32_t sc = 0; sc < M; sc++) /* framing.cc:302-319 */
    for (uint32_t r = 0; r < N; r++)
      for (uint32_t t = 0; t < N; t++)
        if (p[sc] != REF_SC_NULL && r == t) {
          fs->G[(sc * N + r) * N + t].re = 1.0f;
          fs->W[(sc * N + r) * N + t].re = 1.0f;
        }
  fs->gain = (float *)malloc(sizeof(float) * (fs->M_occ ? fs->M_occ : 1));
  for (uint32_t j = 0; j < fs->M_occ; j++) fs->gain[j] = 1.0f;
  fs->S0 = (ref_cf32 *)malloc(sizeof(ref_cf32) * M);
  fs->s0 = (ref_cf32 *)malloc(sizeof(ref_cf32) * M);
  fs->S1 = (ref_cf32 *)malloc(sizeof(ref_cf32) * (size_t)N * cfg->nac * M);
  fs->s1 = (ref_cf32 *)malloc(sizeof(ref_cf32) * (size_t)N * cfg->nac * M);
  for (uint32_t t = 0; t < N; t++)
    ref_init_S1(p, M, cfg->nac, s1_bits + (size_t)t * cfg->nac * M,
                fs->S1 + (size_t)t * cfg->nac * M, fs->s1 + (size_t)t * cfg->nac * M);
  ref_init_S0(p, M, s0_bits, fs->S0, fs->s0);
  fs->dly = (ref_cf32 *)calloc((size_t)N * fs->M2, sizeof(ref_cf32));
  fs->xc = (ref_cf32 *)calloc((size_t)N * fs->M2, sizeof(ref_cf32));
  fs->nz = (float *)calloc((size_t)N * M, sizeof(float));
  fs->win = (ref_cf32 *)calloc((size_t)N * fs->win_len, sizeof(ref_cf32));
  fs->plateau_start = (uint64_t *)calloc(N, sizeof(uint64_t));
  fs->plateau_end = (uint64_t *)calloc(N, sizeof(uint64_t));
  fs->in_plateau = (int *)calloc(N, sizeof(int));
  size_t nacN = (size_t)N * cfg->nac;
  fs->corr_idx = (uint32_t *)calloc((size_t)N * nacN, sizeof(uint32_t));
  fs->corr_max = (float *)calloc((size_t)N * nacN, sizeof(float));
  fs->s0_idx = (uint32_t *)calloc(N, sizeof(uint32_t));
  fs->s0_max = (float *)calloc(N, sizeof(float));
  fs->sym = (ref_cf32 *)calloc((size_t)N * fs->SL, sizeof(ref_cf32));
  fs->noise_var = cfg->noise_var;
  fs->state = REF_STATE_SEEK_PLATEAU;
  return fs;
}

void ref_framesync_destroy(ref_framesync *fs) {
  if (!fs) return;
  free(fs->p); free(fs->occ); free(fs->G); free(fs->W); free(fs->gain);
  free(fs->S0); free(fs->s0); free(fs->S1); free(fs->s1);
  free(fs->dly); free(fs->xc); free(fs->nz); free(fs->win);
  free(fs->plateau_start); free(fs->plateau_end); free(fs->in_plateau);
  free(fs->corr_idx); free(fs->corr_max); free(fs->s0_idx); free(fs->s0_max);
  free(fs->sym); free(fs->outs); free(fs->trace); free(fs->ctrace); free(fs->s0trace);
  free(fs);
}

static void win_push(ref_framesync *fs, const ref_cf32 *x) { /* windowcf_push, all streams */
  for (uint32_t s = 0; s < fs->N; s++) fs->win[(size_t)s * fs->win_len + fs->win_head] = x[s];
  fs->win_head = (fs->win_head + 1) % fs->win_len;
}

/* framing.cc:626-637: wdelay read-before-push (lag M/2), firfilt push+execute */
static float sc_metric_stream(ref_framesync *fs, ref_cf32 x, uint32_t s) {
  uint32_t M = fs->M, M2 = fs->M2;
  ref_cf32 *dly = fs->dly + (size_t)s * M2, *xc = fs->xc + (size_t)s * M2;
  float *nz = fs->nz + (size_t)s * M;
  ref_cf32 d = dly[fs->dly_pos];
  dly[fs->dly_pos] = x;
  ref_cf32 pv;
  pv.re = d.re * x.re - (-d.im) * x.im;
  pv.im = d.re * x.im + (-d.im) * x.re;
  xc[fs->xc_pos] = pv;
  float Pr = 0.0f, Pi = 0.0f;
  for (uint32_t i = 1; i <= M2; i++) { /* oldest -> newest */
    ref_cf32 q = xc[(fs->xc_pos + i) % M2];
    Pr = Pr + (-1.0f) * q.re;
    Pi = Pi + (-1.0f) * q.im;
  }
  float z = x.re * x.re + x.im * x.im;
  nz[fs->nz_pos] = z;
  float R = 0.0f;
  for (uint32_t i = 1; i <= M; i++) R = R + 0.5f * nz[(fs->nz_pos + i) % M];
  return (Pr * Pr + Pi * Pi) / (R * R);
}

static void trace_push(ref_framesync *fs, const float *y) {
  if (fs->trace_len + 1 > fs->trace_cap) {
    fs->trace_cap = fs->trace_cap ? fs->trace_cap * 2 : 4096;
    fs->trace = (float *)realloc(fs->trace, sizeof(float) * fs->trace_cap * fs->N);
  }
  memcpy(fs->trace + fs->trace_len * fs->N, y, sizeof(float) * fs->N);
  fs->trace_len++;
}

static void execute_sc_sync(ref_framesync *fs, const ref_cf32 *x) { /* framing.cc:591-624 */
  float y[64];
  int proceed = 1;
  win_push(fs, x);
  for (uint32_t s = 0; s < fs->N; s++) {
    y[s] = sc_metric_stream(fs, x[s], s);
    if ((double)y[s] > fs->cfg.threshold) {
      if (fs->in_plateau[s]) fs->plateau_end[s] = fs->nsp;
      else {
        fs->in_plateau[s] = 1;
        fs->plateau_start[s] = fs->nsp;
        fs->plateau_end[s] = fs->nsp;
      }
    } else {
      fs->in_plateau[s] = 0;
    }
    proceed = proceed && (fs->plateau_end[s] - fs->plateau_start[s] > fs->cp) &&
              fs->in_plateau[s];
  }
  fs->dly_pos = (fs->dly_pos + 1) % fs->M2;
  fs->xc_pos = (fs->xc_pos + 1) % fs->M2;
  fs->nz_pos = (fs->nz_pos + 1) % fs->M;
  if (fs->cfg.trace_sc) trace_push(fs, y);
  if (proceed) {
    fs->trigger = fs->nsp;
    for (uint32_t s = 0; s < fs->N; s++) fs->sync_index += fs->plateau_start[s];
    fs->sync_index /= fs->N;
    fs->state = REF_STATE_SAVE_ACCESS_CODES;
  }
}

static void emit_symbol(ref_framesync *fs, const ref_cf32 *X /* [N][M_occ] */) {
  size_t per = (size_t)fs->N * fs->M_occ;
  if (fs->n_out + 1 > fs->cap_out) {
    fs->cap_out = fs->cap_out ? fs->cap_out * 2 : 64;
    fs->outs = (ref_cf32 *)realloc(fs->outs, sizeof(ref_cf32) * per * fs->cap_out);
  }
  memcpy(fs->outs + per * fs->n_out, X, sizeof(ref_cf32) * per);
  fs->n_out++;
}

/* ====================================================================================
 * Opt-in CFO -- a BUILD EXTENSION, not the reference: framing.cc:486 leaves the frequency
 * offset as a FIXME and never derotates. This restates the CFO stages of rub_mimo_amd's
 * batched receive (cfo_kernels.hip, the derotating loads of est_kernels.hip,
 * ls_combine_q_kernel, decode_stream.hip) so that path has an oracle. On the window buf
 * (index j = absolute sample - base, base = sync_index - SL), every sum in fp64:
 *  1. eps0 = arg(sum_r sum_{n<M/2} conj(x[t0+n]) x[t0+n+M/2]) / pi, t0 = trigger - M + 1: the S&C
 *     window that ends at the trigger lies in the M/2-periodic S0 on every antenna;
 *  2. search and LS read x1[j] = x[j] exp(-j 2 pi eps0 j / M);
 *  3. delta = arg(P1) / (2 pi), P1 = exp(-j 2 pi eps0) sum over the data symbols s < PID+2,
 *     antennas and prefix interiors (n in [4, cp-4)) of conj(x[k]) x[k+M], k = i0 + s SL + n,
 *     k + M inside the window (i0 = corr[N-1][last] + M, framing.cc:857);
 *  4. each access code's LS terms X/S1 turned by exp(-j 2 pi delta (c + M/2) / M), c its window;
 *  5. the decode reads x[j] exp(-j 2 pi (eps0 + delta) j / M);
 *  6. cfo_mode 2: per symbol, c = sum conj(Q(y)) y over the outputs y of every stream at the
 *     occupied indices j with j even and bit 9 of j clear (Q the hard decision's point; the
 *     GPU's rule: it halves that pass on whole waves), and every output of the symbol turned
 *     by conj(c) / |c|. (Every stream: each stream's output carries its own static phase error
 *     from its column of G, and one stream's would turn the others by it.)
 * ==================================================================================== */
static ref_cf32 cfo_turn(ref_cf32 v, double nu, uint64_t j) {
  double ph = -2.0 * nu * (double)j; /* units of pi */
  ph -= 2.0 * rint(ph * 0.5);
  float c = (float)cos(M_PI * ph), s = (float)sin(M_PI * ph);
  ref_cf32 r;
  r.re = v.re * c - v.im * s;
  r.im = v.re * s + v.im * c;
  return r;
}

static void cfo_common_phase(const ref_framesync *fs, ref_cf32 *out /* [N][M_occ] */) {
  double cr = 0.0, ci = 0.0;
  for (size_t i = 0; i < (size_t)fs->N * fs->M_occ; i++) { /* every stream, the j above */
    if (((i % fs->M_occ) & 1) || (((i % fs->M_occ) >> 9) & 1)) continue;
    ref_cf32 y = out[i];
    ref_cf32 p = ref_qam_point(ref_qam_demap(y, fs->cfg.qam), fs->cfg.qam);
    cr += (double)p.re * y.re + (double)p.im * y.im; /* conj(p) y */
    ci += (double)p.re * y.im - (double)p.im * y.re;
  }
  double m = sqrt(cr * cr + ci * ci);
  if (m == 0.0) return;
  ref_cf32 u = {(float)(cr / m), (float)(-ci / m)};
  for (size_t i = 0; i < (size_t)fs->N * fs->M_occ; i++) out[i] = cmul(out[i], u);
}

/* stage 1 on the window: eps0, and x1 = buf derotated by it (stages 1-2) */
static double cfo_stage1(const ref_framesync *fs, const ref_cf32 *buf, ref_cf32 *x1) {
  const uint32_t M = fs->M, N = fs->N;
  const uint64_t base = fs->nsp - fs->win_len;
  const int64_t t0 = (int64_t)(fs->trigger - base) - (int64_t)M + 1;
  double re = 0.0, im = 0.0;
  for (uint32_t r = 0; r < N; r++)
    for (uint32_t n = 0; n < M / 2; n++) {
      int64_t k = t0 + (int64_t)n;
      if (k < 0 || (uint64_t)(k + M / 2) >= fs->win_len) continue;
      ref_cf32 u = buf[(size_t)r * fs->win_len + k], v = buf[(size_t)r * fs->win_len + k + M / 2];
      re += (double)u.re * v.re + (double)u.im * v.im;
      im += (double)u.re * v.im - (double)u.im * v.re;
    }
  double eps0 = (re == 0.0 && im == 0.0) ? 0.0 : atan2(im, re) / M_PI;
  for (uint32_t r = 0; r < N; r++)
    for (uint64_t j = 0; j < fs->win_len; j++)
      x1[(size_t)r * fs->win_len + j] = cfo_turn(buf[(size_t)r * fs->win_len + j], eps0 / M, j);
  return eps0;
}

/* stage 3 (after the search): delta from the data prefixes of the raw window */
static double cfo_stage3(const ref_framesync *fs, const ref_cf32 *buf, uint64_t i0, double eps0) {
  const uint32_t M = fs->M, N = fs->N, cp = fs->cp, SL = fs->SL, margin = 4;
  const uint32_t inner = cp > 2 * margin ? cp - 2 * margin : 0;
  double re = 0.0, im = 0.0;
  for (uint32_t s = 0; s < fs->cfg.pid_max + 2; s++)
    for (uint32_t r = 0; r < N; r++)
      for (uint32_t n = 0; n < inner; n++) {
        uint64_t k = i0 + (uint64_t)s * SL + margin + n;
        if (k + M >= fs->win_len) continue;
        ref_cf32 u = buf[(size_t)r * fs->win_len + k], v = buf[(size_t)r * fs->win_len + k + M];
        re += (double)u.re * v.re + (double)u.im * v.im;
        im += (double)u.re * v.im - (double)u.im * v.re;
      }
  const double c = cos(-2.0 * M_PI * eps0), sn = sin(-2.0 * M_PI * eps0);
  const double r2 = re * c - im * sn, i2 = re * sn + im * c;
  return (r2 == 0.0 && i2 == 0.0) ? 0.0 : atan2(i2, r2) / (2.0 * M_PI);
}

/* framing.cc:535-589 (MIMO) and 508-533 (SISO) */
static void decode_symbol(ref_framesync *fs, ref_cf32 *X /* scratch [N][M] */,
                          ref_cf32 *out /* [N][M_occ] */) {
  uint32_t M = fs->M, N = fs->N, cp = fs->cp;
  for (uint32_t r = 0; r < N; r++) {
    memcpy(X + (size_t)r * M, fs->sym + (size_t)r * fs->SL + cp, sizeof(ref_cf32) * M);
    if (fs->cfg.cfo_mode) /* opt-in CFO: the body at window index cfo_body derotated by eps */
      for (uint32_t n = 0; n < M; n++)
        X[(size_t)r * M + n] = cfo_turn(X[(size_t)r * M + n], fs->cfo_nu, fs->cfo_body + n);
    if (fs->cfg.detector == REF_DET_SISO && r != fs->cfg.siso_rx) continue;
    ref_fft(X + (size_t)r * M, M, 0);
    for (uint32_t k = 0; k < M; k++) {
      X[(size_t)r * M + k].re = X[(size_t)r * M + k].re * fs->dn;
      X[(size_t)r * M + k].im = X[(size_t)r * M + k].im * fs->dn;
    }
  }
  memset(out, 0, sizeof(ref_cf32) * N * fs->M_occ);
  if (fs->cfg.detector == REF_DET_SISO) {
    uint32_t rx = fs->cfg.siso_rx, tx = fs->cfg.siso_tx;
    for (uint32_t sc = 0, j = 0; sc < M; sc++)
      if (is_occ(fs, sc)) {
        out[(size_t)rx * fs->M_occ + j] =
            cdiv(X[(size_t)rx * M + sc], fs->G[((size_t)sc * N + rx) * N + tx]);
        j++;
      }
    return;
  }
  for (uint32_t sc = 0, j = 0; sc < M; sc++) {
    if (!is_occ(fs, sc)) continue;
    for (uint32_t t = 0; t < N; t++) {
      const ref_cf32 *w = fs->W + ((size_t)sc * N + t) * N;
      ref_cf32 acc = cmul(w[0], X[sc]);
      for (uint32_t r = 1; r < N; r++) acc = cadd(acc, cmul(w[r], X[(size_t)r * M + sc]));
      out[(size_t)t * fs->M_occ + j] = acc;
    }
    j++;
  }
  for (uint32_t t = 0; t < N; t++) /* volk_32fc_32f_multiply_32fc by normalize_gain */
    for (uint32_t j = 0; j < fs->M_occ; j++) {
      out[(size_t)t * fs->M_occ + j].re *= fs->gain[j];
      out[(size_t)t * fs->M_occ + j].im *= fs->gain[j];
    }
  if (fs->cfg.cfo_mode == 2) cfo_common_phase(fs, out);
}

/* complex double Gauss-Jordan with partial pivoting: solve A X = B, A n x n, B n x n */
typedef struct { double re, im; } cd;
static int cd_solve(int n, cd *A, cd *B) {
  for (int c = 0; c < n; c++) {
    int piv = c;
    double best = A[c * n + c].re * A[c * n + c].re + A[c * n + c].im * A[c * n + c].im;
    for (int r = c + 1; r < n; r++) {
      double m = A[r * n + c].re * A[r * n + c].re + A[r * n + c].im * A[r * n + c].im;
      if (m > best) { best = m; piv = r; }
    }
    if (piv != c)
      for (int k = 0; k < n; k++) {
        cd t = A[c * n + k]; A[c * n + k] = A[piv * n + k]; A[piv * n + k] = t;
        t = B[c * n + k]; B[c * n + k] = B[piv * n + k]; B[piv * n + k] = t;
      }
    cd d = A[c * n + c];
    double dd = d.re * d.re + d.im * d.im;
    if (dd == 0.0) return -1;
    cd inv = {d.re / dd, -d.im / dd};
    for (int k = 0; k < n; k++) {
      cd a = A[c * n + k], b = B[c * n + k];
      A[c * n + k].re = a.re * inv.re - a.im * inv.im; A[c * n + k].im = a.re * inv.im + a.im * inv.re;
      B[c * n + k].re = b.re * inv.re - b.im * inv.im; B[c * n + k].im = b.re * inv.im + b.im * inv.re;
    }
    for (int r = 0; r < n; r++) {
      if (r == c) continue;
      cd f = A[r * n + c];
      if (f.re == 0.0 && f.im == 0.0) continue;
      for (int k = 0; k < n; k++) {
        cd a = A[c * n + k], b = B[c * n + k];
        A[r * n + k].re -= f.re * a.re - f.im * a.im; A[r * n + k].im -= f.re * a.im + f.im * a.re;
        B[r * n + k].re -= f.re * b.re - f.im * b.im; B[r * n + k].im -= f.re * b.im + f.im * b.re;
      }
    }
  }
  return 0;
}

/* NxN ZF (W = G^-1) / MMSE (W = (G^H G + s2 I)^-1 G^H), fp64, stored fp32 */
static void solve_weights(uint32_t N, const ref_cf32 *G, ref_cf32 *W, int mmse, double s2) {
  cd A[64], B[64];
  if (!mmse) {
    for (uint32_t i = 0; i < N * N; i++) {
      A[i].re = G[i].re; A[i].im = G[i].im;
      B[i].re = 0.0; B[i].im = 0.0;
    }
    for (uint32_t i = 0; i < N; i++) B[i * N + i].re = 1.0;
  } else {
    for (uint32_t a = 0; a < N; a++)
      for (uint32_t b = 0; b < N; b++) {
        double sr = 0.0, si = 0.0; /* (G^H G)[a][b] = sum_r conj(G[r][a]) G[r][b] */
        for (uint32_t r = 0; r < N; r++) {
          double gar = G[r * N + a].re, gai = G[r * N + a].im;
          double gbr = G[r * N + b].re, gbi = G[r * N + b].im;
          sr += gar * gbr + gai * gbi;
          si += gar * gbi - gai * gbr;
        }
        A[a * N + b].re = sr + ((a == b) ? s2 : 0.0);
        A[a * N + b].im = si;
        B[a * N + b].re = G[b * N + a].re; /* G^H [a][b] = conj(G[b][a]) */
        B[a * N + b].im = -G[b * N + a].im;
      }
  }
  if (cd_solve((int)N, A, B) != 0) {
    for (uint32_t i = 0; i < N * N; i++) { W[i].re = 0.0f; W[i].im = 0.0f; }
    return;
  }
  for (uint32_t i = 0; i < N * N; i++) { W[i].re = (float)B[i].re; W[i].im = (float)B[i].im; }
}

/* Parseval variant of the access-code search (CPU-baseline mode, not the reference's loop).
 * The brute-force metric at lag i is |sum_k FFT(x[i..i+M))[k] conj(C[k])|^2 / M^2 with C the
 * code spectrum; by Parseval (unnormalised DFT) that sum is M sum_n x[i+n] conj(c[n]) with
 * c = IDFT(C)/M, the time-domain code. One overlap-save FFT of P >= SL+M-1 per (rx, code)
 * yields all SL lags: r = IDFT_P(FFT_P(x seg) conj(FFT_P(c))) / P, metric |r[i]|^2. First
 * maximum wins over ascending i, as framing.cc:720-741. */
static void search_parseval(ref_framesync *fs, const ref_cf32 *buf) {
  uint32_t M = fs->M, N = fs->N, SL = fs->SL, nac = fs->nac, nacN = nac * N;
  uint32_t P = 1;
  while (P < SL + M - 1) P <<= 1;
  uint32_t ncode = nacN + 1; /* code 0: S0; code 1 + ac: S1 of (tx, code) */
  ref_cf32 *Z = (ref_cf32 *)malloc(sizeof(ref_cf32) * (size_t)ncode * P);
  ref_cf32 *Y = (ref_cf32 *)malloc(sizeof(ref_cf32) * P);
  for (uint32_t q = 0; q < ncode; q++) {
    const ref_cf32 *S = q == 0 ? fs->S0
                               : fs->S1 + (size_t)((q - 1) % N) * nac * M +
                                     (size_t)((q - 1) / N) * M;
    ref_cf32 *z = Z + (size_t)q * P;
    memset(z, 0, sizeof(ref_cf32) * P);
    memcpy(z, S, sizeof(ref_cf32) * M);
    ref_fft(z, M, 1);                     /* M * c[n] */
    for (uint32_t n = 0; n < M; n++) { z[n].re /= (float)M; z[n].im /= (float)M; }
    ref_fft(z, P, 0);
  }
  for (uint32_t r = 0; r < N; r++) {
    const ref_cf32 *b = buf + (size_t)r * fs->win_len;
    for (uint32_t q = 0; q < ncode; q++) {
      uint64_t base = (uint64_t)SL * q;
      memset(Y, 0, sizeof(ref_cf32) * P);
      for (uint32_t n = 0; n < SL + M - 1 && base + n < fs->win_len; n++) Y[n] = b[base + n];
      ref_fft(Y, P, 0);
      const ref_cf32 *z = Z + (size_t)q * P;
      for (uint32_t k = 0; k < P; k++) Y[k] = cmul(Y[k], cconj(z[k]));
      ref_fft(Y, P, 1);
      float inv = 1.0f / (float)P;
      for (uint32_t i = 0; i < SL; i++) {
        float re = Y[i].re * inv, im = Y[i].im * inv;
        float v = re * re + im * im;
        if (q == 0) {
          if (fs->s0trace) fs->s0trace[(size_t)r * SL + i] = v;
          if (v > fs->s0_max[r]) { fs->s0_max[r] = v; fs->s0_idx[r] = i; }
        } else {
          uint32_t ac = q - 1; /* ac = code * N + tx */
          if (fs->ctrace) fs->ctrace[((size_t)r * nacN + ac) * SL + i] = v;
          if (v > fs->corr_max[r * nacN + ac]) {
            fs->corr_idx[r * nacN + ac] = (uint32_t)(i + base);
            fs->corr_max[r * nacN + ac] = v;
          }
        }
      }
    }
  }
  free(Y);
  free(Z);
}

static void estimate_channel(ref_framesync *fs) { /* framing.cc:653-886 */
  uint32_t M = fs->M, N = fs->N, SL = fs->SL, nac = fs->nac, nacN = nac * N;
  /* windowcf_read: linear oldest -> newest */
  ref_cf32 *buf = (ref_cf32 *)malloc(sizeof(ref_cf32) * (size_t)N * fs->win_len);
  for (uint32_t s = 0; s < N; s++)
    for (uint64_t j = 0; j < fs->win_len; j++)
      buf[(size_t)s * fs->win_len + j] =
          fs->win[(size_t)s * fs->win_len + (fs->win_head + j) % fs->win_len];
  ref_cf32 *X = (ref_cf32 *)malloc(sizeof(ref_cf32) * (size_t)N * M);
  /* opt-in CFO stage 1: search and LS read the window derotated by eps0 */
  ref_cf32 *raw = buf;
  fs->cfo_eps0 = fs->cfo_delta = fs->cfo_nu = 0.0;
  if (fs->cfg.cfo_mode) {
    buf = (ref_cf32 *)malloc(sizeof(ref_cf32) * (size_t)N * fs->win_len);
    fs->cfo_eps0 = cfo_stage1(fs, raw, buf);
  }
  for (uint32_t i = 0; i < (size_t)N * nacN; i++) { fs->corr_max[i] = 0.0f; fs->corr_idx[i] = 0; }
  for (uint32_t s = 0; s < N; s++) { fs->s0_max[s] = 0.0f; fs->s0_idx[s] = 0; }
  double t0 = wall_now();
  /* brute-force access-code search, framing.cc:702-744 (USE_NEW_CHANNEL_EST) */
  float MM = (float)(M * M);
  if (fs->cfg.trace_corr) {
    fs->ctrace = (float *)realloc(fs->ctrace, sizeof(float) * (size_t)N * nacN * SL);
    fs->s0trace = (float *)realloc(fs->s0trace, sizeof(float) * (size_t)N * SL);
  }
  if (fs->cfg.search_mode == 1) search_parseval(fs, buf);
  for (uint32_t i = 0; fs->cfg.search_mode != 1 && i < SL; i++) {
    for (uint32_t r = 0; r < N; r++) {
      const ref_cf32 *b = buf + (size_t)r * fs->win_len;
      memcpy(X, b + i, sizeof(ref_cf32) * M);
      ref_fft(X, M, 0);
      ref_cf32 acc = {0.0f, 0.0f};
      for (uint32_t k = 0; k < M; k++) acc = cadd(acc, cmul(X[k], cconj(fs->S0[k])));
      float v = (acc.re * acc.re + acc.im * acc.im) / MM;
      if (fs->s0trace) fs->s0trace[(size_t)r * SL + i] = v;
      if (v > fs->s0_max[r]) { fs->s0_max[r] = v; fs->s0_idx[r] = i; }
      for (uint32_t code = 0; code < nac; code++)
        for (uint32_t tx = 0; tx < N; tx++) {
          uint32_t ac = code * N + tx;
          uint32_t sample = i + SL * (ac + 1);
          memcpy(X, b + sample, sizeof(ref_cf32) * M);
          ref_fft(X, M, 0);
          const ref_cf32 *S = fs->S1 + (size_t)tx * nac * M + (size_t)code * M;
          ref_cf32 a2 = {0.0f, 0.0f};
          for (uint32_t k = 0; k < M; k++) a2 = cadd(a2, cmul(X[k], cconj(S[k])));
          float cv = (a2.re * a2.re + a2.im * a2.im) / MM;
          if (fs->ctrace) fs->ctrace[((size_t)r * nacN + ac) * SL + i] = cv;
          if (cv > fs->corr_max[r * nacN + ac]) {
            fs->corr_idx[r * nacN + ac] = sample;
            fs->corr_max[r * nacN + ac] = cv;
          }
        }
    }
  }
  double t1 = wall_now();
  /* LS estimate, framing.cc:801-824 (+ training-residual noise variance, build extension) */
  if (!fs->cfg.keep_identity_bias)
    for (size_t i = 0; i < (size_t)M * N * N; i++) { fs->G[i].re = 0.0f; fs->G[i].im = 0.0f; }
  double *sv = (double *)calloc((size_t)M * N * N * 3, sizeof(double));
  if (fs->cfg.cfo_mode) { /* opt-in CFO stage 3: the residual from the data prefixes */
    const uint64_t i0 = (uint64_t)fs->corr_idx[(N - 1) * nacN + nacN - 1] + M;
    fs->cfo_delta = cfo_stage3(fs, raw, i0, fs->cfo_eps0);
    fs->cfo_nu = (fs->cfo_eps0 + fs->cfo_delta) / (double)M;
  }
  for (uint32_t code = 0; code < nac; code++)
    for (uint32_t r = 0; r < N; r++)
      for (uint32_t tx = 0; tx < N; tx++) {
        uint32_t ac = code * N + tx;
        memcpy(X, buf + (size_t)r * fs->win_len + fs->corr_idx[r * nacN + ac],
               sizeof(ref_cf32) * M);
        ref_fft(X, M, 0);
        const ref_cf32 *S = fs->S1 + (size_t)tx * nac * M + (size_t)code * M;
        /* opt-in CFO stage 4: the code's terms turned by delta at its window centre */
        double rc = 1.0, rs = 0.0;
        if (fs->cfg.cfo_mode) {
          double ph = -2.0 * (fs->cfo_delta / (double)M) *
                      ((double)fs->corr_idx[r * nacN + ac] + 0.5 * (double)M);
          ph -= 2.0 * rint(ph * 0.5);
          rc = cos(M_PI * ph);
          rs = sin(M_PI * ph);
        }
        for (uint32_t k = 0; k < M; k++) {
          if (!is_occ(fs, k)) continue;
          ref_cf32 q = cdiv(X[k], S[k]);
          if (fs->cfg.cfo_mode) {
            ref_cf32 q2 = {(float)(q.re * rc - q.im * rs), (float)(q.re * rs + q.im * rc)};
            q = q2;
          }
          size_t gi = ((size_t)k * N + r) * N + tx;
          fs->G[gi] = cadd(fs->G[gi], q);
          sv[gi * 3 + 0] += q.re;
          sv[gi * 3 + 1] += q.im;
          sv[gi * 3 + 2] += (double)q.re * q.re + (double)q.im * q.im;
        }
      }
  float scale = fs->dn / (float)nac;
  for (uint32_t r = 0; r < N; r++)
    for (uint32_t tx = 0; tx < N; tx++)
      for (uint32_t sc = 0; sc < M; sc++)
        if (is_occ(fs, sc)) {
          size_t gi = ((size_t)sc * N + r) * N + tx;
          fs->G[gi].re = fs->G[gi].re * scale;
          fs->G[gi].im = fs->G[gi].im * scale;
        }
  if (nac >= 2) {
    double acc = 0.0;
    for (uint32_t sc = 0; sc < M; sc++) {
      if (!is_occ(fs, sc)) continue;
      for (uint32_t e = 0; e < N * N; e++) {
        size_t gi = (size_t)sc * N * N + e;
        double mr = sv[gi * 3 + 0], mi = sv[gi * 3 + 1];
        acc += sv[gi * 3 + 2] - (mr * mr + mi * mi) / (double)nac;
      }
    }
    double dn = (double)fs->dn;
    double est = acc * dn * dn / ((double)fs->M_occ * N * N * (nac - 1));
    if (fs->cfg.noise_var < 0.0f) fs->noise_var = (float)est;
  }
  free(sv);
  /* weights, framing.cc:826-831 (+ NxN ZF/MMSE extension) */
  for (uint32_t sc = 0, j = 0; sc < M; sc++) {
    if (!is_occ(fs, sc)) continue;
    ref_cf32 *G = fs->G + (size_t)sc * N * N, *W = fs->W + (size_t)sc * N * N;
    if (fs->cfg.detector == REF_DET_ZF2 || fs->cfg.detector == REF_DET_SISO) {
      if (N == 2) fs->gain[j] = ref_invert2(W, G);
    } else {
      solve_weights(N, G, W, fs->cfg.detector == REF_DET_MMSE, (double)fs->noise_var);
      fs->gain[j] = 1.0f;
    }
    j++;
  }
  double t2 = wall_now();
  /* replay decode of the window, framing.cc:853-868 (opt-in CFO: the raw window, each body
   * derotated by eps0 + delta in decode_symbol) */
  if (fs->cfg.cfo_mode) {
    free(buf);
    buf = raw;
  }
  ref_cf32 *out = (ref_cf32 *)malloc(sizeof(ref_cf32) * (size_t)N * (fs->M_occ ? fs->M_occ : 1));
  fs->sym_count = 0;
  for (uint64_t i = (uint64_t)fs->corr_idx[(N - 1) * nacN + nacN - 1] + M; i < fs->win_len; i++) {
    for (uint32_t s = 0; s < N; s++)
      fs->sym[(size_t)s * SL + fs->sym_count] = buf[(size_t)s * fs->win_len + i];
    fs->sym_count++;
    if (fs->sym_count < SL) continue;
    fs->cfo_body = i + 1 - SL + fs->cp; /* window index of the body's first sample */
    decode_symbol(fs, X, out);
    emit_symbol(fs, out);
    fs->sym_count = 0;
  }
  free(out);
  free(X);
  free(buf);
  double t3 = wall_now();
  fs->t_phase[1] += t1 - t0;
  fs->t_phase[2] += t2 - t1;
  fs->t_phase[3] += t3 - t2;
}

static void execute_save_access_codes(ref_framesync *fs, const ref_cf32 *x) { /* :639-651 */
  if (fs->nsp - fs->sync_index < fs->tx_sig_len + fs->acb_len - fs->SL) {
    win_push(fs, x);
    return;
  }
  estimate_channel(fs);
  fs->state = REF_STATE_MIMO;
}

int ref_framesync_execute(ref_framesync *fs, const ref_cf32 *const *in, uint32_t n) {
  ref_cf32 x[64];
  int brk = 0;
  double te0 = wall_now(), sub0 = fs->t_phase[1] + fs->t_phase[2] + fs->t_phase[3];
  for (uint32_t i = 0; i < n; i++) { /* framing.cc:481-504 */
    for (uint32_t s = 0; s < fs->N; s++) x[s] = in[s][i];
    switch (fs->state) {
      case REF_STATE_SEEK_PLATEAU: execute_sc_sync(fs, x); break;
      case REF_STATE_SAVE_ACCESS_CODES: execute_save_access_codes(fs, x); break;
      case REF_STATE_MIMO: brk = 1; break;
      default: return -1;
    }
    fs->nsp++;
    if (brk) break;
  }
  fs->t_phase[0] += (wall_now() - te0) -
                    (fs->t_phase[1] + fs->t_phase[2] + fs->t_phase[3] - sub0);
  return fs->state;
}

void ref_framesync_get_phase_times(const ref_framesync *fs, double *t4) {
  for (int i = 0; i < 4; i++) t4[i] = fs->t_phase[i];
}

void ref_framesync_reset(ref_framesync *fs) { fs->state = REF_STATE_SEEK_PLATEAU; }

void ref_framesync_get_cfo(const ref_framesync *fs, double *eps2) {
  eps2[0] = fs->cfo_eps0;
  eps2[1] = fs->cfo_delta;
}

/* Test helper (not a reference entry point): advance a fresh framesync over samples [0, p0)
 * with the S&C state updates of framing.cc:626-637 (window ring, wdelaycf read-before-push,
 * the two firfilt histories) but without the per-sample dot products and the plateau rule on
 * samples [0, p0 - 1); sample p0 - 1 then runs through execute_sc_sync in full. The metric of
 * every later sample depends only on those histories, so it equals the full run's bit for bit.
 * The plateau state at p0 equals the full run's when no antenna is in a run after sample
 * p0 - 1 (its y at or below the threshold), which is checked (-2 otherwise): a run open at
 * p0 - 1 would carry a start this walk never saw. What it cannot see is a trigger before p0,
 * which the full run would have taken; callers start p0 where the capture holds no frame. */
int ref_framesync_fast_forward(ref_framesync *fs, const ref_cf32 *const *in, uint64_t p0) {
  if (fs->state != REF_STATE_SEEK_PLATEAU || fs->nsp != 0 || p0 == 0 || fs->cfg.trace_sc) return -1;
  ref_cf32 x[64];
  const uint32_t M = fs->M, M2 = fs->M2;
  for (uint64_t i = 0; i + 1 < p0; i++) {
    for (uint32_t s = 0; s < fs->N; s++) x[s] = in[s][i];
    win_push(fs, x);
    for (uint32_t s = 0; s < fs->N; s++) {
      ref_cf32 *dly = fs->dly + (size_t)s * M2, *xc = fs->xc + (size_t)s * M2;
      float *nz = fs->nz + (size_t)s * M;
      const ref_cf32 d = dly[fs->dly_pos];
      dly[fs->dly_pos] = x[s];
      ref_cf32 pv;
      pv.re = d.re * x[s].re - (-d.im) * x[s].im;
      pv.im = d.re * x[s].im + (-d.im) * x[s].re;
      xc[fs->xc_pos] = pv;
      nz[fs->nz_pos] = x[s].re * x[s].re + x[s].im * x[s].im;
    }
    fs->dly_pos = (fs->dly_pos + 1) % M2;
    fs->xc_pos = (fs->xc_pos + 1) % M2;
    fs->nz_pos = (fs->nz_pos + 1) % M;
    fs->nsp++;
  }
  for (uint32_t s = 0; s < fs->N; s++) x[s] = in[s][p0 - 1];
  execute_sc_sync(fs, x);
  fs->nsp++;
  for (uint32_t s = 0; s < fs->N; s++)
    if (fs->in_plateau[s]) return -2;
  return fs->state == REF_STATE_SEEK_PLATEAU ? 0 : -2;
}

/* CPU-baseline helper (not a reference entry point): put a fresh framesync in the state the
 * plateau rule leaves it in when it fires at sample `trigger` with `sync_index`
 * (framing.cc:617-623): the window ring holds samples up to `trigger` (zeros before 0), the
 * sample count is trigger + 1, the state SAVE_ACCESS_CODES. Executing the samples from
 * trigger + 1 on then runs search, LS, weights and decode exactly as the full run does. */
int ref_framesync_skip_to_sync(ref_framesync *fs, const ref_cf32 *const *in, uint64_t trigger,
                               uint64_t sync_index) {
  if (fs->state != REF_STATE_SEEK_PLATEAU || fs->nsp != 0) return -1;
  uint64_t start = trigger + 1 > fs->win_len ? trigger + 1 - fs->win_len : 0;
  fs->win_head = start % fs->win_len;
  ref_cf32 x[64];
  for (uint64_t i = start; i <= trigger; i++) {
    for (uint32_t s = 0; s < fs->N; s++) x[s] = in[s][i];
    win_push(fs, x);
  }
  fs->nsp = trigger + 1;
  fs->trigger = trigger;
  fs->sync_index = sync_index;
  fs->state = REF_STATE_SAVE_ACCESS_CODES;
  return 0;
}
uint64_t ref_framesync_get_sync_index(const ref_framesync *fs) { return fs->sync_index; }
uint64_t ref_framesync_get_num_samples_processed(const ref_framesync *fs) { return fs->nsp; }
uint64_t ref_framesync_get_plateau_start(const ref_framesync *fs, uint32_t s) {
  return fs->plateau_start[s];
}
uint64_t ref_framesync_get_plateau_end(const ref_framesync *fs, uint32_t s) {
  return fs->plateau_end[s];
}
int ref_framesync_get_state(const ref_framesync *fs) { return fs->state; }
void ref_framesync_get_corr(const ref_framesync *fs, uint32_t *corr_idx, float *corr_max,
                            uint32_t *s0_idx, float *s0_max) {
  size_t n = (size_t)fs->N * fs->N * fs->nac;
  if (corr_idx) memcpy(corr_idx, fs->corr_idx, sizeof(uint32_t) * n);
  if (corr_max) memcpy(corr_max, fs->corr_max, sizeof(float) * n);
  if (s0_idx) memcpy(s0_idx, fs->s0_idx, sizeof(uint32_t) * fs->N);
  if (s0_max) memcpy(s0_max, fs->s0_max, sizeof(float) * fs->N);
}
void ref_framesync_get_G(const ref_framesync *fs, ref_cf32 *G) {
  memcpy(G, fs->G, sizeof(ref_cf32) * (size_t)fs->M * fs->N * fs->N);
}
void ref_framesync_get_W(const ref_framesync *fs, ref_cf32 *W) {
  memcpy(W, fs->W, sizeof(ref_cf32) * (size_t)fs->M * fs->N * fs->N);
}
void ref_framesync_get_gain(const ref_framesync *fs, float *gain) {
  memcpy(gain, fs->gain, sizeof(float) * fs->M_occ);
}
float ref_framesync_get_noise_var(const ref_framesync *fs) { return fs->noise_var; }
uint32_t ref_framesync_num_symbols(const ref_framesync *fs) { return fs->n_out; }
void ref_framesync_get_symbols(const ref_framesync *fs, ref_cf32 *out, uint32_t max_syms) {
  uint32_t n = fs->n_out < max_syms ? fs->n_out : max_syms;
  memcpy(out, fs->outs, sizeof(ref_cf32) * (size_t)n * fs->N * fs->M_occ);
}
uint64_t ref_framesync_sc_trace_len(const ref_framesync *fs) { return fs->trace_len; }
void ref_framesync_get_sc_trace(const ref_framesync *fs, uint32_t s, float *out) {
  for (uint64_t i = 0; i < fs->trace_len; i++) out[i] = fs->trace[i * fs->N + s];
}
uint32_t ref_framesync_M_occ(const ref_framesync *fs) { return fs->M_occ; }
int ref_framesync_get_corr_trace(const ref_framesync *fs, float *corr, float *s0) {
  if (!fs->ctrace) return -1;
  size_t nacN = (size_t)fs->N * fs->nac;
  memcpy(corr, fs->ctrace, sizeof(float) * fs->N * nacN * fs->SL);
  memcpy(s0, fs->s0trace, sizeof(float) * fs->N * fs->SL);
  return 0;
}

/* main.cc:1394-1461 generalised: square-QAM hard decision + EVM */
void ref_demap_evm(const ref_cf32 *sym, uint32_t n_sym, uint32_t N, uint32_t M_occ,
                   uint32_t qam, const uint8_t *tx_idx, uint8_t *rx_idx, double *evm_num,
                   double *evm_den, uint64_t *errors) {
  for (uint32_t t = 0; t < N; t++) { evm_num[t] = 0.0; evm_den[t] = 0.0; errors[t] = 0; }
  for (uint32_t s = 0; s < n_sym; s++)
    for (uint32_t t = 0; t < N; t++)
      for (uint32_t j = 0; j < M_occ; j++) {
        ref_cf32 y = sym[((size_t)s * N + t) * M_occ + j];
        uint32_t d = ref_qam_demap(y, qam);
        size_t oi = ((size_t)t * n_sym + s) * M_occ + j;
        if (rx_idx) rx_idx[oi] = (uint8_t)d;
        uint32_t ref = tx_idx ? tx_idx[oi] : d;
        if (d != ref) errors[t]++;
        ref_cf32 sp = ref_qam_point(ref, qam);
        double er = (double)y.re - sp.re, ei = (double)y.im - sp.im;
        evm_num[t] += er * er + ei * ei;
        evm_den[t] += (double)sp.re * sp.re + (double)sp.im * sp.im;
      }
}

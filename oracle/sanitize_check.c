/*
 * oracle/sanitize_check.c -- TEST INFRASTRUCTURE ONLY. A driver that runs the oracle
 * (mimo_ref.c) end to end on small frames so that it can be built and run under
 * AddressSanitizer + UndefinedBehaviorSanitizer (oracle/Makefile target `sanitize`,
 * tests/test_oracle.py::test_oracle_under_asan_ubsan). Every path a test or the bench's CPU
 * baseline drives is exercised: msequence draws, sctype helpers, S0/S1, framegen, the
 * synthesiser, framesync fed in one call and in ragged chunks (brute-force and Parseval
 * search, all detectors, S&C and search traces), the skip-to-sync baseline helper, reset,
 * the exact S&C metric and demap/EVM. Exit status 0 and no sanitizer report = clean.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mimo_ref.h"

static int fails = 0, synced = 0;
#define CHECK(c)                                                       \
  do {                                                                 \
    if (!(c)) {                                                        \
      fprintf(stderr, "sanitize_check: %s failed (line %d)\n", #c, __LINE__); \
      fails++;                                                         \
    }                                                                  \
  } while (0)

/* S1 generator polynomials of the first streams (degree-13 primitive, as codes.py) */
static const uint32_t kS1Poly[8] = {020033, 020047, 020065, 020123, 020145, 020157, 020213, 020215};

static void one_case(uint32_t M, uint32_t cp, uint32_t N, uint32_t nac, uint32_t pid,
                     uint32_t qam, int det, int search_mode, int liquid, uint32_t chunk,
                     uint64_t seed) {
  uint8_t *p = malloc(M);
  if (liquid) ref_init_liquid_sctype(p, M); else ref_init_default_sctype(p, M);
  uint32_t n0, n1, n2;
  CHECK(ref_validate_sctype(p, M, &n0, &n1, &n2) == 0);
  const uint32_t m_occ = n1 + n2;
  uint8_t *b0 = malloc(M), *b1 = malloc((size_t)N * nac * M);
  ref_msequence_draw_bits(12, 010123, 1, M, b0);
  for (uint32_t t = 0; t < N; t++) ref_msequence_draw_bits(13, kS1Poly[t], 1, nac * M, b1 + (size_t)t * nac * M);

  ref_synth_cfg sc = {M, cp, N, nac, pid, qam, seed, 0, -1, 30.0f, 3, 0};
  const uint64_t L = ref_synth_frame_len(&sc);
  ref_cf32 **rx = malloc(sizeof(ref_cf32 *) * N);
  for (uint32_t r = 0; r < N; r++) rx[r] = calloc(L, sizeof(ref_cf32));
  uint8_t *tx_idx = malloc((size_t)N * pid * m_occ);
  ref_cf32 *H = malloc(sizeof(ref_cf32) * N * N);
  CHECK(ref_synth_frame(&sc, p, b0, b1, rx, tx_idx, H) == L);

  ref_rx_cfg rc;
  memset(&rc, 0, sizeof(rc));
  rc.M = M; rc.cp = cp; rc.N = N; rc.nac = nac; rc.pid_max = pid;
  rc.detector = det; rc.noise_var = -1.0f; rc.keep_identity_bias = 1;
  rc.threshold = 0.95; rc.trace_sc = 1; rc.trace_corr = 1; rc.search_mode = search_mode;
  ref_framesync *fs = ref_framesync_create(&rc, p, b0, b1);
  CHECK(fs != NULL);
  /* fed in ragged chunks (execute keeps its state across calls) */
  const ref_cf32 **in = malloc(sizeof(ref_cf32 *) * N);
  uint64_t pos = 0;
  uint32_t step = chunk;
  while (pos < L) {
    const uint32_t c = (uint32_t)((L - pos) < step ? (L - pos) : step);
    for (uint32_t r = 0; r < N; r++) in[r] = rx[r] + pos;
    ref_framesync_execute(fs, in, c);
    pos += c;
    step = step * 7 % 1013 + 1;
  }
  const int st = ref_framesync_get_state(fs);
  if (st == REF_STATE_MIMO) {
    synced++;
    const uint32_t ns = ref_framesync_num_symbols(fs);
    CHECK(ns == pid + 2);
    ref_cf32 *sym = malloc(sizeof(ref_cf32) * (size_t)ns * N * m_occ);
    ref_framesync_get_symbols(fs, sym, ns);
    double num[8], den[8];
    uint64_t err[8];
    uint8_t *ri = malloc((size_t)N * pid * m_occ);
    ref_demap_evm(sym, pid, N, m_occ, qam, tx_idx, ri, num, den, err);
    CHECK(den[0] > 0.0);
    uint32_t *ci = malloc(sizeof(uint32_t) * N * N * nac);
    float *cm = malloc(sizeof(float) * N * N * nac);
    uint32_t si[8];
    float sm[8];
    ref_framesync_get_corr(fs, ci, cm, si, sm);
    const uint32_t SL = M + cp;
    float *ctr = malloc(sizeof(float) * (size_t)N * N * nac * SL);
    float *str = malloc(sizeof(float) * (size_t)N * SL);
    CHECK(ref_framesync_get_corr_trace(fs, ctr, str) == 0);
    ref_cf32 *G = malloc(sizeof(ref_cf32) * (size_t)M * N * N);
    ref_cf32 *W = malloc(sizeof(ref_cf32) * (size_t)M * N * N);
    float *gain = malloc(sizeof(float) * m_occ);
    ref_framesync_get_G(fs, G);
    ref_framesync_get_W(fs, W);
    ref_framesync_get_gain(fs, gain);
    (void)ref_framesync_get_noise_var(fs);
    const uint64_t tl = ref_framesync_sc_trace_len(fs);
    float *y = malloc(sizeof(float) * (tl ? tl : 1));
    ref_framesync_get_sc_trace(fs, 0, y);
    double t4[4];
    ref_framesync_get_phase_times(fs, t4);
    /* the CPU-baseline helper from the trigger, then reset and a one-shot run */
    const uint64_t si0 = ref_framesync_get_sync_index(fs);
    ref_rx_cfg rc2 = rc;
    rc2.trace_sc = 0; rc2.trace_corr = 0;
    ref_framesync *fs2 = ref_framesync_create(&rc2, p, b0, b1);
    for (uint32_t r = 0; r < N; r++) in[r] = rx[r];
    uint64_t trig = 0;
    for (uint32_t s = 0; s < N; s++) {
      const uint64_t e = ref_framesync_get_plateau_end(fs, s);
      if (e > trig) trig = e;
    }
    (void)ref_framesync_skip_to_sync(fs2, in, trig, si0);
    for (uint32_t r = 0; r < N; r++) in[r] = rx[r] + trig + 1;
    CHECK(ref_framesync_execute(fs2, in, (uint32_t)(L - trig - 1)) == REF_STATE_MIMO);
    CHECK(ref_framesync_get_sync_index(fs2) == si0);
    ref_framesync_reset(fs2);
    ref_framesync_destroy(fs2);
    (void)ref_sc_metric_at(rx[0], si0, M);
    free(sym); free(ri); free(ci); free(cm); free(ctr); free(str); free(G); free(W);
    free(gain); free(y);
  }
  ref_framesync_destroy(fs);
  /* framegen (TX) */
  ref_framegen *fg = ref_framegen_create(M, cp, N, nac, p, b0, b1);
  ref_cf32 **tx = malloc(sizeof(ref_cf32 *) * N);
  ref_cf32 **din = malloc(sizeof(ref_cf32 *) * N);
  for (uint32_t t = 0; t < N; t++) {
    tx[t] = calloc((size_t)(nac * N + 1) * (M + cp), sizeof(ref_cf32));
    din[t] = calloc(m_occ, sizeof(ref_cf32));
    for (uint32_t j = 0; j < m_occ; j++) din[t][j] = ref_qam_point((j * 7 + t) % qam, qam);
  }
  CHECK(ref_framegen_write_sync_words(fg, tx) == (nac * N + 1) * (M + cp));
  CHECK(ref_framegen_assemble_mimo_packet(fg, tx, din) == M + cp);
  ref_framegen_destroy(fg);
  for (uint32_t t = 0; t < N; t++) { free(tx[t]); free(din[t]); }
  free(tx); free(din);
  for (uint32_t r = 0; r < N; r++) free(rx[r]);
  free(rx); free(in); free(tx_idx); free(H); free(p); free(b0); free(b1);
}

int main(void) {
  ref_msequence ms;
  ref_msequence_init(&ms, 12, 010123, 1);
  for (int i = 0; i < 100; i++) (void)ref_msequence_generate_symbol(&ms, 3);
  ref_msequence_reset(&ms);
  CHECK(ref_msequence_period(12, 010123, 1) == 4095);
  ref_cf32 G[4] = {{1.0f, 0.5f}, {0.2f, -0.1f}, {-0.3f, 0.4f}, {0.9f, 0.0f}}, W[4];
  CHECK(ref_invert2(W, G) > 0.0f);
  for (uint32_t q = 4; q <= 256; q *= 4)
    for (uint32_t i = 0; i < q; i++) CHECK(ref_qam_demap(ref_qam_point(i, q), q) == i);
  one_case(64, 16, 1, 4, 8, 4, REF_DET_SISO, 0, 0, 333, 3);
  one_case(64, 16, 2, 4, 8, 16, REF_DET_ZF2, 0, 0, 97, 5);
  one_case(128, 16, 2, 3, 6, 16, REF_DET_ZF2, 0, 1, 1000, 9);
  one_case(64, 16, 4, 2, 6, 64, REF_DET_MMSE, 1, 0, 250, 7);
  one_case(128, 16, 4, 2, 5, 16, REF_DET_ZF, 0, 0, 4096, 11);
  one_case(64, 8, 8, 2, 4, 16, REF_DET_MMSE, 1, 0, 777, 13);
  CHECK(synced >= 4);   /* most cases reach the detector (Rayleigh draws may not sync) */
  if (fails) {
    fprintf(stderr, "sanitize_check: %d check(s) failed\n", fails);
    return 1;
  }
  printf("sanitize_check OK (%d of 6 frames synced)\n", synced);
  return 0;
}

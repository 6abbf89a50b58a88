/*
 * oracle/mimo_ref.h -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * Plain-C CPU restatement of the reference receive path in
 *   /root/reference/mimo/framing.cc  (rx_beamforming::framegen / framesync, S0/S1 init,
 *                                     sctype helpers, 2x2 invert)
 *   /root/reference/mimo/main.cc     (TX frame layout of tx_worker, callback, demap/SER)
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Parity vs the reference binaries is UNPINNED: the reference needs liquid-dsp, FFTW3f,
 * VOLK, UHD and Boost (all absent here) and ships no tests, fixtures or golden vectors.
 * The restatement is pinned instead by (1) reference-derived known answers asserted in
 * tests/test_oracle.py and (2) an independent numpy model (oracle/numpy_model.py) that
 * produced the committed fixtures under tests/golden/.
 *
 * Pinned third-party semantics:
 *   - liquid msequence: g>>=1, initial state bit-reversed, advance = parity(v&g) shifted in.
 *   - liquid wdelaycf read-before-push: effective lag exactly M/2.
 *   - liquid firfilt_{crcf,rrrf}: sequential fp32 dot product oldest->newest, no FMA.
 *   - liquid windowcf: last-N ring, zero initialised.
 *   - FFTW3f: unnormalised +-exp transforms (own radix-4/2 FFT, double-precision twiddles).
 *   - VOLK conjugate dot product: sequential sum of a*conj(b).
 */
#ifndef MIMO_REF_H
#define MIMO_REF_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { float re, im; } ref_cf32;

/* subcarrier types, liquid OFDMFRAME_SCTYPE_* */
enum { REF_SC_NULL = 0, REF_SC_PILOT = 1, REF_SC_DATA = 2 };

/* receiver states, framing.h:34-39 */
enum { REF_STATE_SEEK_PLATEAU = 0, REF_STATE_SAVE_ACCESS_CODES = 1, REF_STATE_WAIT = 2,
       REF_STATE_MIMO = 3 };

/* detectors: 0 = reference 2x2 ZF (framing.cc:1344-1367), 1 = NxN ZF, 2 = NxN MMSE,
 * 3 = SISO division (framing.cc:508-533) */
enum { REF_DET_ZF2 = 0, REF_DET_ZF = 1, REF_DET_MMSE = 2, REF_DET_SISO = 3 };

/* ---------------- liquid msequence restatement ---------------- */
typedef struct { uint32_t m, g, a, n, v, b; } ref_msequence;
void     ref_msequence_init(ref_msequence *ms, uint32_t m, uint32_t g, uint32_t a);
uint32_t ref_msequence_advance(ref_msequence *ms);
uint32_t ref_msequence_generate_symbol(ref_msequence *ms, uint32_t bps);
void     ref_msequence_reset(ref_msequence *ms);
uint64_t ref_msequence_period(uint32_t m, uint32_t g, uint32_t a);
/* draw `count` bits msequence_generate_symbol(ms,1)&1 from a fresh generator */
void     ref_msequence_draw_bits(uint32_t m, uint32_t g, uint32_t a, uint32_t count,
                                 uint8_t *out);

/* ---------------- sctype helpers, framing.cc:949-1051 ---------------- */
void ref_init_default_sctype(uint8_t *p, uint32_t M);      /* USE_ALL_CARRIERS variant */
void ref_init_liquid_sctype(uint8_t *p, uint32_t M);       /* guard/pilot variant */
int  ref_validate_sctype(const uint8_t *p, uint32_t M, uint32_t *M_null, uint32_t *M_pilot,
                         uint32_t *M_data);

/* ---------------- FFT (unnormalised, FFTW sign convention) ---------------- */
void ref_fft(ref_cf32 *x, uint32_t n, int inverse);

/* ---------------- S0 / S1, framing.cc:1054-1111, 1214-1262 ---------------- */
void ref_init_S0(const uint8_t *p, uint32_t M, const uint8_t *bits, ref_cf32 *S0,
                 ref_cf32 *s0);
void ref_init_S1(const uint8_t *p, uint32_t M, uint32_t nac, const uint8_t *bits,
                 ref_cf32 *S1, ref_cf32 *s1);

/* ---------------- 2x2 invert, framing.cc:1344-1367 ---------------- */
float ref_invert2(ref_cf32 W[4], const ref_cf32 G[4]);

/* ---------------- square Gray QAM ---------------- */
ref_cf32 ref_qam_point(uint32_t index, uint32_t order);
uint32_t ref_qam_demap(ref_cf32 y, uint32_t order);

/* ---------------- counter-based PRNG shared with the GPU synthesiser ---------------- */
uint64_t ref_hash5(uint64_t seed, uint64_t dom, uint64_t a, uint64_t b, uint64_t c);

/* ---------------- framegen (TX), framing.cc:79-266 ---------------- */
typedef struct ref_framegen ref_framegen;
ref_framegen *ref_framegen_create(uint32_t M, uint32_t cp, uint32_t N, uint32_t nac,
                                  const uint8_t *p, const uint8_t *s0_bits,
                                  const uint8_t *s1_bits /* N*nac*M */);
void     ref_framegen_destroy(ref_framegen *fg);
uint32_t ref_framegen_write_sync_words(ref_framegen *fg, ref_cf32 **tx);
uint32_t ref_framegen_assemble_mimo_packet(ref_framegen *fg, ref_cf32 **tx,
                                           ref_cf32 *const *in);

/* ---------------- synthetic capture (tx_worker layout + channel + AWGN) ---------------- */
typedef struct {
  uint32_t M, cp, N, nac, pid, qam;
  uint64_t seed, frame;
  int32_t  offset;      /* lead offset u; <0 -> drawn from the PRNG in [0, SL) */
  float    snr_db;      /* per stream at each rx antenna; noise var = 0.0625*10^(-snr/10) */
  uint32_t tail_syms;   /* zero symbols after the data (default 3) */
  int      identity_channel; /* 1: H = I (no fading) */
} ref_synth_cfg;
uint64_t ref_synth_frame_len(const ref_synth_cfg *c);
/* rx: N planar buffers of frame_len complex; tx_idx: N*pid*M_occ (may be NULL);
 * H: N*N complex row-major [rx][tx] (may be NULL). Returns frame length. */
uint64_t ref_synth_frame(const ref_synth_cfg *c, const uint8_t *p, const uint8_t *s0_bits,
                         const uint8_t *s1_bits, ref_cf32 *const *rx, uint8_t *tx_idx,
                         ref_cf32 *H);

/* ---------------- framesync (RX), framing.cc:268-944 ---------------- */
typedef struct {
  uint32_t M, cp, N, nac, pid_max;
  int      detector;          /* REF_DET_* */
  float    noise_var;         /* MMSE sigma^2; <0 -> estimate from training residuals */
  int      keep_identity_bias;/* 1 (reference): G starts at identity, framing.cc:309-311 */
  uint32_t siso_tx, siso_rx;
  double   threshold;         /* PLATEAU_THREASHOLD 0.95, config.h:87 */
  int      trace_sc;          /* keep per-sample y (DEBUG_LOG f_sc files) */
  int      trace_corr;        /* keep search metrics (DEBUG_LOG corr_* files) */
  int      search_mode;       /* 0: brute-force FFT per lag, framing.cc:702-744 (faithful);
                                 1: Parseval variant (CPU-baseline mode 3 of BASELINE.md, labelled):
                                 one overlap-save FFT correlation per (rx, code); same metric up
                                 to fp32 rounding */
  int      cfo_mode;          /* build extension, not in the reference (framing.cc:486 FIXME):
                                 0 off (the reference); 1 the CFO stages of rub_mimo_amd's
                                 batched path (S0 coarse, prefix fine, derotated search, LS
                                 and decode); 2 the same plus the per-symbol common phase.
                                 See "Opt-in CFO" in mimo_ref.c */
  uint32_t qam;               /* QAM order of the hard decision (cfo_mode 2 only) */
} ref_rx_cfg;

typedef struct ref_framesync ref_framesync;
ref_framesync *ref_framesync_create(const ref_rx_cfg *cfg, const uint8_t *p,
                                    const uint8_t *s0_bits, const uint8_t *s1_bits);
void     ref_framesync_destroy(ref_framesync *fs);
int      ref_framesync_execute(ref_framesync *fs, const ref_cf32 *const *in, uint32_t n);
void     ref_framesync_reset(ref_framesync *fs);
/* CPU-baseline helper: state after the plateau rule fired at `trigger` (see mimo_ref.c) */
int      ref_framesync_fast_forward(ref_framesync *fs, const ref_cf32 *const *in, uint64_t p0);
int      ref_framesync_skip_to_sync(ref_framesync *fs, const ref_cf32 *const *in,
                                    uint64_t trigger, uint64_t sync_index);
uint64_t ref_framesync_get_sync_index(const ref_framesync *fs);
uint64_t ref_framesync_get_num_samples_processed(const ref_framesync *fs);
uint64_t ref_framesync_get_plateau_start(const ref_framesync *fs, uint32_t s);
uint64_t ref_framesync_get_plateau_end(const ref_framesync *fs, uint32_t s);
int      ref_framesync_get_state(const ref_framesync *fs);
/* corr_indices [N][N*nac] (window index), s0 index [N], max values */
void     ref_framesync_get_corr(const ref_framesync *fs, uint32_t *corr_idx, float *corr_max,
                                uint32_t *s0_idx, float *s0_max);
void     ref_framesync_get_G(const ref_framesync *fs, ref_cf32 *G /* [M][N][N] */);
void     ref_framesync_get_W(const ref_framesync *fs, ref_cf32 *W /* [M][N][N] */);
void     ref_framesync_get_gain(const ref_framesync *fs, float *gain /* [M_occ] */);
float    ref_framesync_get_noise_var(const ref_framesync *fs);
uint32_t ref_framesync_num_symbols(const ref_framesync *fs);
/* symbols: [n_sym][N][M_occ] complex in callback order */
void     ref_framesync_get_symbols(const ref_framesync *fs, ref_cf32 *out, uint32_t max_syms);
uint64_t ref_framesync_sc_trace_len(const ref_framesync *fs);
void     ref_framesync_get_sc_trace(const ref_framesync *fs, uint32_t s, float *out);
uint32_t ref_framesync_M_occ(const ref_framesync *fs);
/* wall seconds spent per phase since create: [0] S&C + plateau, [1] access-code search,
 * [2] LS + weights, [3] replay decode (FFT, detect, gain) */
void     ref_framesync_get_phase_times(const ref_framesync *fs, double *t4);
/* cfo_mode != 0: the estimates of the last estimate_channel in subcarrier spacings: [0] eps0
 * (S0 coarse), [1] delta (prefix fine); the frame's offset is eps0 + delta */
void     ref_framesync_get_cfo(const ref_framesync *fs, double *eps2);
/* search metric traces by lag i in [0,SL): corr [N][N*nac][SL], s0 [N][SL] */
int      ref_framesync_get_corr_trace(const ref_framesync *fs, float *corr, float *s0);

/* exact fp32 S&C metric at absolute sample n of a contiguous capture x (x[k<0]=0):
 * the sequential firfilt order of framing.cc:626-637 */
float ref_sc_metric_at(const ref_cf32 *x, uint64_t n, uint32_t M);

/* demap + EVM over kept symbols, main.cc:1394-1461 (square QAM instead of ARB32OPT).
 * sym: [n_sym][N][M_occ]; tx_idx: [N][n_sym*M_occ] or NULL (decision directed).
 * out per stream s: evm_num[s], evm_den[s], errors[s]; rx_idx: [N][n_sym*M_occ] or NULL */
void ref_demap_evm(const ref_cf32 *sym, uint32_t n_sym, uint32_t N, uint32_t M_occ,
                   uint32_t qam, const uint8_t *tx_idx, uint8_t *rx_idx, double *evm_num,
                   double *evm_den, uint64_t *errors);

#ifdef __cplusplus
}
#endif
#endif

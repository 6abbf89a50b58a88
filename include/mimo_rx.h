/*
 * include/mimo_rx.h -- C-ABI of librub_mimo_amd.so, the MI355X (gfx950) OFDM-MIMO receive
 * pipeline. Plain pointers and sizes only; no torch or C++ types cross this boundary.
 *
 * Each entry point replaces a piece of the reference C++ API in /root/reference/mimo/framing.h
 * (cited per function). The C++ facade include/framing.h re-exposes the reference classes
 * rx_beamforming::framesync / framegen on top of these calls, so mimo/main.cc-style callers
 * compile unchanged.
 *
 * Conventions
 *   - complex samples are interleaved fp32 (re, im) = std::complex<float> = gr_complex.
 *   - antenna buffers are planar: one array per antenna (framing.cc:481-484 reads in_buff[s][i]).
 *   - every function returns MIMO_OK (0) or a negative MIMO_ERR_*; nothing calls exit()
 *     (the reference exits at framing.cc:497-499, 1020-1022).
 *   - a handle owns one HIP stream (or the caller's) and is single-caller-thread.
 *   - device pointers (d_*) are HIP device memory (e.g. torch tensor data_ptr()).
 */
#ifndef RUB_MIMO_AMD_MIMO_RX_H
#define RUB_MIMO_AMD_MIMO_RX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MIMO_OK 0
#define MIMO_ERR_ARG (-1)
#define MIMO_ERR_HIP (-2)
#define MIMO_ERR_STATE (-3)
#define MIMO_ERR_NOMEM (-4)
#define MIMO_ERR_SCTYPE (-5)
#define MIMO_ERR_UNSUPPORTED (-6)

#define MIMO_MAX_STREAMS 8

/* framesync_states_t, framing.h:34-39 */
enum { MIMO_STATE_SEEK_PLATEAU = 0, MIMO_STATE_SAVE_ACCESS_CODES = 1, MIMO_STATE_WAIT = 2,
       MIMO_STATE_MIMO = 3 };

/* detectors: ZF2 = reference 2x2 adjugate*conj(det) + gain 1/|det|^2 (framing.cc:1344-1367);
 * ZF / MMSE = NxN in fp64, stored fp32; SISO = X/G[rx][tx] on one stream (framing.cc:508-533) */
enum { MIMO_DET_ZF2 = 0, MIMO_DET_ZF = 1, MIMO_DET_MMSE = 2, MIMO_DET_SISO = 3 };

/* per-frame status of the batched path. RESCAN (back-to-back streams only): the re-arm at this
 * frame's origin could not be proven equal to a fresh framesync there (a plateau or window
 * reaching back across the re-arm point); the caller resumes the capture at `origin` as a
 * fresh capture. NONE: an unused frame slot after the end of a stream. */
enum { MIMO_FRAME_OK = 0, MIMO_FRAME_NO_SYNC = 1, MIMO_FRAME_INCOMPLETE = 2,
       MIMO_FRAME_RESCAN = 3, MIMO_FRAME_NONE = 4 };

/* subcarrier types, liquid OFDMFRAME_SCTYPE_{NULL,PILOT,DATA} */
enum { MIMO_SC_NULL = 0, MIMO_SC_PILOT = 1, MIMO_SC_DATA = 2 };

/* Receiver configuration: the framesync constructor arguments (framing.h:189-196) plus the
 * config.h constants the reference reads at compile time (PID_MAX, PLATEAU_THREASHOLD). */
typedef struct mimo_rx_config {
  uint32_t M;                 /* _M, number of subcarriers (power of two, 64..4096) */
  uint32_t cp_len;            /* _cp_len */
  uint32_t num_streams;       /* _num_streams (1..8) */
  uint32_t num_access_codes;  /* _num_access_codes */
  uint32_t pid_max;           /* PID_MAX (config.h:92): data symbols per frame window */
  const uint8_t *p;           /* _p, M subcarrier types; copied */
  const uint8_t *s0_bits;     /* M draws msequence_generate_symbol(ms_S0,1)&1 (framing.cc:1075) */
  const uint8_t *s1_bits;     /* num_streams*num_access_codes*M draws, stream-major
                                 (framing.cc:1240, one generator per stream) */
  int32_t detector;           /* MIMO_DET_* (INVERT_CHANNEL, config.h:102) */
  float noise_var;            /* MMSE sigma^2; < 0: estimate from the training residuals */
  int32_t keep_identity_bias; /* 1 = reference: G starts at identity (framing.cc:309-311) */
  uint32_t siso_tx, siso_rx;  /* set_siso_tx / set_siso_rx (framing.h:211-212) */
  double plateau_threshold;   /* PLATEAU_THREASHOLD (config.h:87), 0.95 */
  uint32_t qam_order;         /* square Gray QAM for the fused demap/EVM stage (4..256) */
  int32_t cfo_correct;        /* batched path, opt-in (absent from the reference: FIXME at
                                 framing.cc:486): 1 = estimate each synced frame's CFO (eps0
                                 from the S0 half-period correlation ending at its trigger,
                                 delta from the data symbols' cyclic prefixes, both summed
                                 over the antennas) and derotate before search, LS and decode
                                 (in the loads where the fused search and the streaming
                                 decode run, else into a device scratch copy; the caller's
                                 capture is not modified); where the streaming decode takes
                                 the batch with reference indices from HBM, each symbol's
                                 common phase is also measured from its own decisions and
                                 removed (mimo_rx_get_cfo_mode). The stages are restated in
                                 oracle/mimo_ref.c (cfo_mode). 0 = off (the reference's
                                 behaviour). Scratch-path batches with frames_per_capture > 1
                                 are refused with MIMO_ERR_UNSUPPORTED. */
} mimo_rx_config;

typedef struct mimo_rx mimo_rx;

/* callback, framing.h:30-31: eq[t] points at M_occ equalised symbols of stream t, valid
 * only during the call (framing.cc:587). */
typedef void (*mimo_rx_symbol_cb)(const float *const *eq, uint32_t n_streams, uint32_t m_occ,
                                  void *user);

/* framesync::framesync (framing.cc:268-436). hip_stream: hipStream_t or NULL (own stream). */
int mimo_rx_create(const mimo_rx_config *cfg, void *hip_stream, mimo_rx **out);
/* framesync::~framesync (framing.cc:916-943) */
int mimo_rx_destroy(mimo_rx *h);
/* the mimo_callback argument of the constructor (framing.h:196) */
int mimo_rx_set_callback(mimo_rx *h, mimo_rx_symbol_cb cb, void *user);
/* framesync::execute (framing.cc:471-506): host planar complex64 input, any chunking;
 * state persists across calls; *state_out receives the framesync_states_t. */
int mimo_rx_execute(mimo_rx *h, const float *const *iq_planar, uint32_t n_ant, uint64_t n,
                    int32_t *state_out);
/* framesync::reset (framing.cc:461-464): back to STATE_SEEK_PLATEAU */
int mimo_rx_reset(mimo_rx *h);
int mimo_rx_set_siso(mimo_rx *h, uint32_t siso_tx, uint32_t siso_rx);
int mimo_rx_get_state(const mimo_rx *h, int32_t *state);
/* get_sync_index / get_num_samples_processed / get_plateau_start|end (framing.h:200-206) */
int mimo_rx_get_sync_index(const mimo_rx *h, uint64_t *out);
int mimo_rx_get_num_samples_processed(const mimo_rx *h, uint64_t *out);
int mimo_rx_get_plateau(const mimo_rx *h, uint32_t stream, uint64_t *start, uint64_t *end);
/* get_G (framing.h:201): [M][N][N] complex64 ([sc][rx][tx]); W likewise ([sc][out][rx]) */
int mimo_rx_get_G(mimo_rx *h, float *G);
int mimo_rx_get_W(mimo_rx *h, float *W);
/* normalize_gain (framing.cc:404-409), M_occ floats */
int mimo_rx_get_gain(mimo_rx *h, float *gain);
int mimo_rx_get_noise_var(mimo_rx *h, float *out);
/* corr_indices [N][N*nac] (window index, framing.cc:737) and s0_corr_index [N] (:720) */
int mimo_rx_get_corr(mimo_rx *h, uint32_t *corr_idx, uint32_t *s0_idx);
int mimo_rx_get_m_occ(const mimo_rx *h, uint32_t *m_occ);

/* ---------------- batched device-resident frames (the hot path the bench times) ---------
 * n_frames independent captures, each num_streams planar antenna arrays of frame_len
 * complex64 at d_iq + (f*num_streams + s)*stride (complex units). Every frame runs the whole
 * receive chain (S&C + plateau, access-code search, LS, weights, decode, demap, EVM) with
 * no host synchronisation.
 *
 * frames_per_capture = K > 1 makes each capture a stream of back-to-back frames (a live
 * 20 MS/s stream, BASELINE config C5): frame k + 1 is what a fresh framesync (framing.cc:268)
 * finds in the samples after frame k, i.e. starting at origin
 *   r_{k+1} = r_k + get_num_samples_processed()   (framing.cc:471-506, r_0 = 0).
 * The reference itself stops at STATE_MIMO and its reset() keeps stale filter state
 * (framing.cc:461-464, 494-496), so this re-arm is defined as that fresh construction. Frame
 * slots are then [capture][K]: outputs, results and d_ref_idx rows are per slot. */
typedef struct mimo_batch {
  const void *d_iq;
  uint64_t stride;        /* complex samples between antenna arrays (>= frame_len) */
  uint64_t frame_len;
  uint32_t n_frames;
  uint32_t max_out_syms;  /* symbols kept per frame (main.cc keeps PID_MAX, main.cc:106) */
  void *d_out_sym;        /* [n_frames][N][max_out_syms][M_occ] complex64 (out_layout), or NULL */
  void *d_out_idx;        /* same layout, uint8 demapped index, or NULL */
  int32_t ref_mode;       /* 0: decision-directed EVM; 1: d_ref_idx; 2: synthetic hash */
  const void *d_ref_idx;  /* ref_mode 1: same layout as d_out_idx */
  uint64_t ref_seed;      /* ref_mode 2: seed of mimo_synth_frames */
  uint64_t frame_id0;     /* ref_mode 2: frame id of frame 0 */
  uint32_t frames_per_capture;  /* 0 or 1: one frame per capture; K > 1: back-to-back streams */
  uint32_t ref_stride;          /* entries per capture in d_ref_starts (0: frames_per_capture) */
  /* streams with ref_mode 1/2, or NULL: [n_frames][ref_stride] capture sample where each
   * transmitted frame starts (UINT64_MAX after the last). A decoded frame whose sync index
   * lies in [start_j, start_{j+1}) takes reference row / frame id capture*ref_stride + j;
   * NULL: its slot. */
  const uint64_t *d_ref_starts;
  /* MIMO_SAMPLE_FC32 (0): d_iq holds complex64. MIMO_SAMPLE_SC16 (1): d_iq holds the UHD sc16
   * wire format (interleaved int16 I/Q, mimo/config.h:52; 4 bytes per sample, strides and
   * lengths still in samples), read as float(i16) * sc16_scale -- bit-identical to widening
   * with mimo_ingest_sc16 first. The S&C, fused search + LS and streaming decode kernels read
   * it directly (C3-type geometries); other configurations widen it into an internal buffer. */
  uint32_t sample_format;
  float sc16_scale;
  /* MIMO_LAYOUT_STREAM_MAJOR (0): d_out_sym, d_out_idx and d_ref_idx are
   * [n_frames][N][max_out_syms][M_occ]. MIMO_LAYOUT_SYMBOL_MAJOR (1): [n_frames][max_out_syms][N][M_occ],
   * each symbol's N stream rows together -- the order the reference's callback hands them out in
   * (one call per symbol with the N stream arrays, framing.cc:587) -- and a sequential write
   * stream per decode workgroup (fewer concurrent HBM write streams: the C3 decode ~7% faster) */
  uint32_t out_layout;
  /* MIMO_STAGES_ALL (0): the whole receive chain. MIMO_STAGES_FRONT (1): S&C, plateau, search,
   * LS and weights only; MIMO_STAGES_DECODE (2): the replay decode and EVM only, of the batch
   * the same handle last ran MIMO_STAGES_FRONT on (same arguments). The two halves may run on
   * different streams (the caller orders them with events), e.g. batch i's decode on one CU
   * partition beside batch i+1's front stages on another handle and partition. Not with
   * cfo_correct. */
  uint32_t stages;
} mimo_batch;

enum { MIMO_SAMPLE_FC32 = 0, MIMO_SAMPLE_SC16 = 1 };
enum { MIMO_LAYOUT_STREAM_MAJOR = 0, MIMO_LAYOUT_SYMBOL_MAJOR = 1 };
enum { MIMO_STAGES_ALL = 0, MIMO_STAGES_FRONT = 1, MIMO_STAGES_DECODE = 2 };

/* Positions are those a framesync started at `origin` reports (origin 0 for one frame per
 * capture): add origin for the capture sample. */
typedef struct mimo_frame_result {
  int32_t status;                          /* MIMO_FRAME_* */
  uint32_t n_sym;                          /* decode callbacks (PID+2 in the reference) */
  uint64_t trigger;                        /* sample where the plateau rule fired */
  uint64_t sync_index;
  uint64_t num_samples_processed;          /* as one framesync::execute over the frame */
  uint64_t plateau_start[MIMO_MAX_STREAMS];
  uint64_t plateau_end[MIMO_MAX_STREAMS];
  float noise_var;
  float cfo_eps;                           /* cfo_correct: estimated CFO, subcarrier spacings */
  double evm_num[MIMO_MAX_STREAMS];        /* sum |y - s|^2 over kept symbols */
  double evm_den[MIMO_MAX_STREAMS];        /* sum |s|^2 */
  uint64_t errors[MIMO_MAX_STREAMS];       /* symbol errors (ref_mode 1/2) */
  uint64_t origin;                         /* capture sample where this frame's framesync began */
  uint32_t capture;                        /* capture (stream) index */
  uint32_t ref_frame;                      /* reference row / frame id offset used for the EVM */
} mimo_frame_result;

int mimo_rx_process_batch(mimo_rx *h, const mimo_batch *b, void *hip_stream);
/* copies the last batch's per-frame results to host (synchronises the stream); n_frames
 * counts frame slots (captures x frames_per_capture) */
int mimo_rx_batch_results(mimo_rx *h, mimo_frame_result *out, uint32_t n_frames);
/* per-frame detail of the last batch, host copies: corr [F][N][N*nac], G [F][M][N][N] */
int mimo_rx_batch_corr(mimo_rx *h, uint32_t *corr_idx, uint32_t *s0_idx, uint32_t n_frames);
int mimo_rx_batch_G(mimo_rx *h, float *G, uint32_t n_frames);
int mimo_rx_batch_W(mimo_rx *h, float *W, uint32_t n_frames);

/* stage timing with HIP events on the handle's launch stream (for the roofline line).
 * stages: 0 S&C, 1 plateau, 2 search, 3 LS, 4 weights, 5 decode, 6 EVM reduce; an sc16 batch
 * that is widened internally (not read in place) adds its widening launch to stage 0 */
#define MIMO_NUM_STAGES 7
int mimo_rx_set_timing(mimo_rx *h, int enable);
/* sums of stage durations (ms) and launch counts since the last call; synchronises */
int mimo_rx_get_stage_times(mimo_rx *h, double *ms, uint32_t *launches);
/* S&C samples whose fp64 metric fell within the decision band and were recomputed with the
 * oracle's exact fp32 order, since the last call (diagnostic; synchronises) */
int mimo_rx_get_sc_exact_count(mimo_rx *h, uint64_t *out);
/* the replay-decode kernel family the last batch or execute launched (diagnostic, no sync):
 * STREAM = decode_stream_kernel (persistent, 2x2/4x4), SPLIT = spectra_kernel +
 * apply_split_kernel (8x8 at M >= 512), SYMBOL = the per-symbol kernels, NONE = no decode yet */
enum { MIMO_DECODE_NONE = 0, MIMO_DECODE_STREAM = 1, MIMO_DECODE_SPLIT = 2,
       MIMO_DECODE_SYMBOL = 3 };
int mimo_rx_get_decode_path(const mimo_rx *h, int32_t *path);
/* persistent grids (the streaming and split decodes) sized for n_cu CUs instead of the device's
 * count (diagnostic: a handle whose stream is CU-masked; 0 restores the device's count). Call
 * before the handle's first batch (captured graphs keep the grid they were captured with). */
int mimo_rx_set_grid_cus(mimo_rx *h, uint32_t n_cu);
/* roofline probe (diagnostic, no reference counterpart): the streaming decode's memory pattern
 * without its arithmetic -- per symbol N rows of M + 2 complex64 samples staged by LDS-DMA and
 * N x M uint8 reference indices, N x M complex64 + N x M uint8 written symbol-major, on the
 * decode's persistent grid -- over n_frames x spf symbols of the caller's captures ([n_caps][N]
 * [stride] complex64), reference rows and output buffers ([n_frames][spf][N][M]); reps timed
 * launches after one warm-up, the mean in *ms_per_launch. N x M in {4 x 2048, 4 x 1024,
 * 2 x 4096, 2 x 2048, 2 x 1024} (the streaming decode's geometries, every subcarrier occupied).
 * Returns 0, or 1 (arguments), 2 (HIP), 3 (geometry). */
int mimo_probe_decode_pattern(const void *d_iq, uint64_t stride, uint32_t n_caps, uint32_t N,
                              uint32_t M, uint32_t cp, uint32_t n_frames, uint32_t spf,
                              const void *d_ref, void *d_out_sym, void *d_out_idx, int reps,
                              void *hip_stream, float *ms_per_launch);
/* the CFO stages the last batch ran (diagnostic, no sync): 0 off, 1 estimate and derotation,
 * 2 the same plus the per-symbol common phase (the streaming decode's CPE variant) -- the
 * oracle's cfo_mode for the same batch */
int mimo_rx_get_cfo_mode(const mimo_rx *h, int32_t *mode);
/* streaming execute: the device capture's capacity and the samples it holds per antenna
 * (diagnostic). While seeking, only the samples a later trigger can still reach are kept
 * (the reference's bounded window ring, framing.cc:387-388), so the capture stays near the
 * window size however long an unsynchronised stream runs. */
int mimo_rx_get_stream_capacity(const mimo_rx *h, uint64_t *capacity, uint64_t *held);
/* DEBUG_LOG (mimo/config.h:84-86, off by default here): the streaming execute writes the
 * reference's debug traces into directory `dir` (NULL or "" turns them off):
 *   f_sc_<k>.dat     float32 Schmidl-Cox metric y of every sample processed while seeking,
 *                    antenna k from 1, appended per call (framing.cc:390-402, 598-600);
 *   corr_<k>_<ac>.dat  float32 search metric over window indices [0, ACB - M), ac from 1, and
 *                    corr_<k>_0.dat for S0 (framing.cc:675-696, 716-737, 873-883).
 * The files mimo/apps/plot.py reads. Opening happens here (the reference opens them in its
 * constructor); they are closed by the next call or mimo_rx_destroy. */
int mimo_rx_set_debug_log(mimo_rx *h, const char *dir);

/* ---------------- transmitter: framegen (framing.h:42-103) ---------------- */
typedef struct mimo_tx mimo_tx;
int mimo_tx_create(uint32_t M, uint32_t cp_len, uint32_t num_streams,
                   uint32_t num_access_codes, const uint8_t *p, const uint8_t *s0_bits,
                   const uint8_t *s1_bits, mimo_tx **out);
int mimo_tx_destroy(mimo_tx *h);
/* framegen::write_sync_words (framing.cc:169-208): host buffers, (nac*N+1)*SL each */
int mimo_tx_write_sync_words(mimo_tx *h, float *const *tx, uint32_t *n_written);
/* framegen::assemble_mimo_packet (framing.cc:210-235): in[t] M_occ symbols -> SL samples */
int mimo_tx_assemble_mimo_packet(mimo_tx *h, float *const *tx, const float *const *in,
                                 uint32_t *n_written);
int mimo_tx_get_codes(mimo_tx *h, float *s0 /* M */, float *s1 /* N*nac*M */);

/* ---------------- synthetic captures on the GPU (tx_worker layout + channel + AWGN) -----
 * [lead zeros SL*(N*nac+1)+u][sync words][pid data symbols][tail zeros], x0.25 baseband
 * gain (main.cc:1048-1053), flat Rayleigh H ~ CN(0,1) per frame, AWGN. */
typedef struct mimo_synth_config {
  uint32_t M, cp_len, num_streams, num_access_codes, pid, qam_order;
  uint64_t seed;
  float snr_db;
  uint32_t tail_syms;
  int32_t identity_channel;
  int32_t offset;         /* lead offset u; < 0: drawn per frame from the seed in [0, SL) */
  const uint8_t *p, *s0_bits, *s1_bits;
} mimo_synth_config;
/* length of frame `frame_id` (depends on its offset u) */
int mimo_synth_frame_len(const mimo_synth_config *c, uint64_t frame_id, uint64_t *len);
/* writes n_frames captures into d_out (layout of mimo_batch; samples past a frame's own
 * length are zero-padded noise), optional d_tx_idx [F][N][pid][M_occ] and d_H [F][N][N] */
int mimo_synth_frames(const mimo_synth_config *c, uint64_t frame_id0, uint32_t n_frames,
                      void *d_out, uint64_t stride, uint64_t frame_len, void *d_tx_idx,
                      void *d_H, void *hip_stream);

/* ---------------- helpers (setup-time, host) ---------------- */
int mimo_sctype_default(uint8_t *p, uint32_t M);   /* ofdmframe_init_default_sctype */
int mimo_sctype_liquid(uint8_t *p, uint32_t M);    /* compiled-out guard/pilot variant */
int mimo_sctype_validate(const uint8_t *p, uint32_t M, uint32_t *M_null, uint32_t *M_pilot,
                         uint32_t *M_data);        /* ofdmframe_validate_sctype */
int mimo_msequence_draw_bits(uint32_t m, uint32_t g, uint32_t a, uint32_t count,
                             uint8_t *out);        /* liquid msequence draws */
/* 2x2 invert (framing.cc:1344-1367) on host arrays: returns gain */
float mimo_invert2(float *W /* 4 complex */, const float *G /* 4 complex */);

/* device memory / stream helpers so callers need no HIP headers */
int mimo_dev_alloc(void **ptr, size_t bytes);
int mimo_dev_free(void *ptr);
int mimo_memcpy_h2d(void *dst, const void *src, size_t bytes, void *hip_stream);
int mimo_memcpy_d2h(void *dst, const void *src, size_t bytes, void *hip_stream);
int mimo_memcpy_d2d(void *dst, const void *src, size_t bytes, void *hip_stream);
int mimo_memset_d(void *dst, int value, size_t bytes, void *hip_stream);
/* Capture ingest at the wire format (UHD sc16, mimo/config.h:52) instead of the host fc32
 * the reference's rx worker receives (mimo/main.cc:837-848). d_sc16 holds n_arrays rows of n
 * interleaved int16 I/Q samples, src_stride samples apart; row r is widened to complex64
 * float(i16)*scale at d_fc32 + r*dst_stride (complex units), i.e. straight into the planar
 * layout of mimo_batch. Rows must not overlap. Asynchronous on hip_stream. */
int mimo_ingest_sc16(const void *d_sc16, uint64_t src_stride, void *d_fc32, uint64_t dst_stride,
                     uint32_t n_arrays, uint64_t n, float scale, void *hip_stream);
/* ---------------- pinned-host capture ring ----------------
 * Replaces the rx worker's malloc'd fc32 rx_buffer and its /tmp round trip
 * (mimo/main.cc:842-848, 872-898, 906-918): the recv loop writes UHD sc16 wire samples
 * (CPU format "sc16", mimo/config.h:52) straight into pinned host chunks, and every commit is
 * uploaded asynchronously (one 2-D copy on the ring's own HIP stream) into a device capture
 * [n_ant][stride] of sc16 samples -- the layout mimo_batch takes with sample_format =
 * MIMO_SAMPLE_SC16. A chunk is reused only after its upload has completed, so n_chunks >= 2
 * overlaps the next recv with the previous upload. One producer thread calls acquire/commit;
 * the consumer calls bind/publish (both may run concurrently with the producer). */
typedef struct mimo_ring mimo_ring;
int mimo_ring_create(uint32_t n_ant, uint32_t chunk_samples, uint32_t n_chunks, mimo_ring **out);
int mimo_ring_destroy(mimo_ring *r);   /* waits for the uploads in flight */
/* target of the following commits: d_capture rows of `capacity` samples, `stride` apart
 * (samples; capacity <= stride); write position 0. The uploads are not ordered against
 * readers of d_capture: rebinding a capture that a published batch may still be reading needs
 * the caller to synchronise first, or mimo_ring_bind_after. */
int mimo_ring_bind(mimo_ring *r, void *d_capture, uint64_t stride, uint64_t capacity);
/* mimo_ring_bind, and the uploads into the new binding wait (on the device) for the work
 * enqueued on consumer_stream so far: a capture can be refilled while its batch runs */
int mimo_ring_bind_after(mimo_ring *r, void *d_capture, uint64_t stride, uint64_t capacity,
                         void *consumer_stream);
/* the next chunk: rows[a] = host pointer of antenna a's chunk_samples interleaved int16 I/Q
 * (UHD's per-channel buffer vector, main.cc:874); waits for that chunk's previous upload */
int mimo_ring_acquire(mimo_ring *r, void **rows, uint32_t *max_samples);
/* n <= max_samples samples were written to every row of the acquired chunk: upload them at
 * the write position (MIMO_ERR_ARG past capacity or with no bound capture) */
int mimo_ring_commit(mimo_ring *r, uint32_t n);
/* make hip_stream wait, on the device, for every upload committed so far; *n_written = the
 * bound capture's samples per antenna so far */
int mimo_ring_publish(mimo_ring *r, void *hip_stream, uint64_t *n_written);

/* Carrier-frequency offset (absent from the reference: FIXME at framing.cc:486). Over the S0
 * body starting at sample `start` of each antenna row (period M/2, framing.cc:1054-1111),
 * P = sum_{n<M/2} conj(x[start+n]) x[start+n+M/2]; eps = arg(P)/pi in subcarrier spacings.
 * eps[0..n_ant-1] per antenna, eps[n_ant] from the sum of the antennas' P. Synchronous. */
int mimo_cfo_estimate(const void *d_iq, uint64_t stride, uint32_t n_ant, uint64_t start,
                      uint32_t M, double *eps, void *hip_stream);
/* x[n] *= exp(-j 2 pi (eps/M) (n - n0)) for n < n on every row, in place. Asynchronous. */
int mimo_cfo_derotate(void *d_iq, uint64_t stride, uint32_t n_ant, uint64_t n, int64_t n0,
                      double eps, uint32_t M, void *hip_stream);
int mimo_stream_sync(void *hip_stream);
int mimo_device_count(int *n);
const char *mimo_last_error(void);
const char *mimo_version(void);

#ifdef __cplusplus
}
#endif
#endif

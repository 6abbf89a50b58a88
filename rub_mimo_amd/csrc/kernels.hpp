// rub_mimo_amd/csrc/kernels.hpp -- launch interfaces of the gfx950 kernels (host side).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.hpp"

namespace mimo {

// Schmidl-Cox metric + plateau rule, framing.cc:591-637 (see sync_kernels.hip)
struct ScRecord {             // a chunk's trigger candidate and the run starts it saw
  unsigned long long n_cand;
  unsigned long long start[kMaxStreams];
  long long pos0;             // first sample the chunk computed
  uint32_t found;             // bit s: start[s] is final (a zero bit inside the chunk)
  uint32_t pad;
};
// an S&C work item spans kScSpan positions: a halo of >= cp+2 (run history, multiple of 16)
// and the chunk's candidate positions; 256 threads own 16 positions each per 4096-position
// iteration
constexpr int kScSpan = 16384;
constexpr int kScThreads = 256;
constexpr int kScIterLen = 4096;
constexpr int kScAmbMax = 256;   // near-threshold samples deferred per item
inline uint64_t sc_chunk_len(uint32_t cp) { return kScSpan - ((uint64_t)cp + 2 + 15) / 16 * 16; }
size_t sc_lds_bytes(uint32_t M, uint32_t N);
size_t sc_table_bytes(uint32_t M);

// an item whose plateau candidates hinge on near-threshold samples, handed from the item
// kernel to the resolve and finalize kernels
struct ScHot {
  uint32_t f, n_done, namb, arrived;   // arrived: antenna passes done (sc_exact_kernel)
  uint64_t chunk;
  int64_t c0, w0, cend;
  int64_t lo[kMaxStreams];                          // first evaluated position per antenna
  int64_t amb_n[kScAmbMax];
  uint8_t amb_s[kScAmbMax];
  uint16_t wbits[kMaxStreams * (kScSpan / kScIterLen) * kScThreads];
};

struct ScArgs {
  const float2 *iq;
  int sc16;                 // iq holds sc16 wire samples (float(i16) * iq_scale)
  float iq_scale;
  uint64_t stride;          // complex samples between antenna arrays
  uint64_t frame_len;
  uint32_t N, M, cp;
  double thr, band;
  uint64_t chunk_len;        // candidate positions per chunk (sc_chunk_len)
  uint64_t chunk_lo, chunk_hi;
  unsigned long long *trig; // [F], min trigger sample (UINT64_MAX = none yet)
  ScRecord *rec;            // [F][rec_stride] per-chunk candidates
  uint64_t rec_stride;
  unsigned long long *n_exact;  // count of exact fp32 recomputes (null: not counted)
  uint32_t *queue;          // [0] work-queue head, [1] hot-item count; zeroed before launch
  uint32_t *hot_count;
  const uint32_t *item_lo;  // screened path: first hot item of this exact launch, or null (0)
  ScHot *hot;               // [hot_cap] (null: resolve inside the item kernel)
  uint32_t hot_cap;
  unsigned long long *prof; // diagnostics: [items, antenna passes, row, words, resolve, total
                            // cycles, skipped items] (null: off)
  // screened path: chunk geometry and the screen's first/last unproven position per chunk
  uint64_t nchunks;
  const unsigned long long *fmin, *fmax;   // [F][nchunks]
  // back-to-back streams: every chunk's first candidate ([F][nchunks], ~0 = none) for the
  // stream walk, and no skipping of chunks past a capture's earliest trigger
  unsigned long long *cand;
  int no_skip;
  uint32_t diag;            // diagnostics (RMIMO_SC_DIAG bits 8/16: skip in-place resolve/finalize)
  uint32_t *snap;           // sc_exact_kernel: copy of *hot_count (the items of this phase), or null
};

// S&C screen over antenna 0 (sc_screen_kernel): blocks of kScrB positions, kScrSpan positions
// per workgroup plus 2D blocks of history (D = M/2 / kScrB <= kScrMaxD)
constexpr int kScrT = 256;
constexpr int kScrB = 128;
constexpr int kScrSpan = 16384;
constexpr int kScrMaxD = 32;               // M <= 8192
constexpr int kScrBPI = 4;                 // blocks per wave iteration (loads in flight)
struct ScreenArgs {
  const float2 *iq;
  int sc16;                 // iq holds sc16 wire samples (float(i16) * iq_scale)
  float iq_scale;
  uint64_t stride, frame_len;
  uint32_t N, M;
  double thr_screen;                       // thr - 0.01
  uint64_t chunk_len, chunk_lo, nchunks;
  uint64_t chunk_hi;                       // screen chunks [chunk_lo, chunk_hi) (0: nchunks)
  const unsigned long long *trig;          // [F] skip frames already triggered, or null
  uint32_t *flag;                          // [F][nchunks] chunk listed
  unsigned long long *fmin, *fmax;         // [F][nchunks] first / last unproven position
  uint32_t *count;                         // listed chunks (= hot items)
  ScHot *hot;                              // [cap] one per listed chunk
  uint32_t cap;
  // capture sample 0 is the framesync origin (batched path): the delay line is empty there,
  // so every lagged sample of positions n < M/2 is zero and P[n] = 0 (framing.cc:598-637)
  uint32_t empty_history;
};
// several small 32-bit-word fills in one launch (the per-batch resets of the S&C queues,
// flags and trigger words: one kernel instead of one memset node each)
constexpr int kMaxFill = 10;
struct FillArgs {
  uint32_t *p[kMaxFill];
  uint64_t n[kMaxFill];       // words
  uint32_t v[kMaxFill];
  int count;
};
void launch_fill(const FillArgs &a, hipStream_t s);
// true when the geometry allows the screen (M/2 a multiple of kScrB, M <= 8192)
inline bool sc_screen_ok(uint32_t M) { return M / 2 >= (uint32_t)kScrB && (M / 2) % kScrB == 0 && M / 2 / kScrB <= (uint32_t)kScrMaxD; }
// copies one device word (the hot-item count after a screen phase)
void launch_sc_snapshot(uint32_t *dst, const uint32_t *src, hipStream_t s);
void launch_sc_screen(const ScreenArgs &a, uint32_t n_frames, hipStream_t s);
void launch_sc_exact(const ScArgs &a, hipStream_t s);
// persistent grid of n_cu x (resident blocks per CU) over the F x chunks items
void launch_sc(const ScArgs &a, uint32_t n_frames, uint32_t n_cu, hipStream_t s);
void launch_sc_hot(const ScArgs &a, hipStream_t s);
void launch_sc_finalize(const ScArgs &a, hipStream_t s);   // plateau rule per hot item   // resolve + finalize the hot items

struct PlateauArgs {
  const unsigned long long *trig;
  const ScRecord *rec;
  uint64_t rec_stride, chunk_len;
  const float2 *iq;
  int sc16;
  float iq_scale;
  uint64_t stride, frame_len;
  uint32_t N, M, SL;
  double thr, band;
  uint64_t win_len;         // ACB + TX (framing.cc:284-285, 387-388)
  FrameInfo *info;
  // back-to-back streams (frames_per_capture > 1): info is [capture][fpc] slots
  uint32_t fpc;
  uint64_t nchunks;
  const unsigned long long *cand;          // [capture][nchunks] first candidate per chunk
  unsigned long long *certfail;            // [capture] bit k: slot k's re-arm certificate failed
  const uint64_t *ref_starts;              // [capture][ref_stride] transmitted frame starts
  uint32_t ref_stride;                     // or null
};
// one frame per capture: trigger -> run starts, sync index, window
void launch_plateau(const PlateauArgs &a, uint32_t n_frames, hipStream_t s);
// back-to-back frames per capture: the re-arm walk over the chunk candidates, the re-arm
// certificates of frames k >= 1 and the chain fix-up (see sync_kernels.hip)
void launch_stream_walk(const PlateauArgs &a, uint32_t n_caps, hipStream_t s);
// DEBUG_LOG: the oracle-exact fp32 metric y of positions [lo, hi) of every antenna row
// (framing.cc:598-600), out[row][i]
void launch_sc_trace(const float2 *iq, uint64_t stride, uint32_t rows, uint32_t M, int64_t lo,
                     int64_t hi, float *out, hipStream_t s);

// access-code search, framing.cc:702-744 (est_kernels.hip)
struct SearchArgs {
  const float2 *iq;
  int sc16;
  float iq_scale;
  uint64_t stride, frame_len;
  uint32_t N, M, SL, n_slots;      // n_slots = N*nac + 1 (slot 0 = S0)
  uint32_t lagc, n_lagc;           // lags per transform, transforms per slot
  const float2 *codespec;          // [n_slots][F]
  const float2 *codespec_w;        // [n_slots][F], bin B k + q at q 1024 + k (B = F/1024), or null
  const float *vscale;             // [n_slots]
  const FrameInfo *info;
  unsigned long long *keys;        // [F][N][n_slots] packed (value, ~index)
  const float2 *tw;
  // fused search + LS terms (search_ls_kernel): slot pairs, one lag chunk per slot
  const int8_t *s1sign;            // [N][nac][M]
  float2 *lsq;                     // [F][N][N][nac][M] X/S1 per access code
  uint32_t nac;
  uint32_t xcd_order;              // search_ls_kernel: slot pair slowest within each XCD
  const double *cfo_part;          // opt-in CFO, folded: derotate the loads by stage 1 (or null)
  float *corr_trace;               // DEBUG_LOG: [F][N][n_slots][SL] every lag's metric (or null)
};
void launch_search(const SearchArgs &a, int log2F, uint32_t n_frames, hipStream_t s);
// true when (log2F, log2M) has a search_ls_kernel instance (it then ran)
bool launch_search_ls(const SearchArgs &a, int log2F, int log2M, uint32_t n_frames, hipStream_t s);
bool search_ls_supported(int log2F, int log2M);
// the wave-local form of search_ls_kernel (F >= 1024) is on (default; RMIMO_SEARCH_WAVE=0 turns it off)
bool search_ls_wave_enabled();

// LS estimate, framing.cc:797-824 (+ training residual noise variance)
struct LsArgs {
  const float2 *iq;
  uint64_t stride, frame_len;
  int sc16;                        // capture at the sc16 wire format (ls_window_kernel)
  float iq_scale;
  uint32_t N, M, nac, n_slots;
  const unsigned long long *keys;
  const int8_t *s1sign;            // [N][nac][M]
  const int8_t *s1sign_w;          // [N][nac][M/8][8]: sign of subcarrier lt + (M/8) e at 8 lt + e
                                   // (ls_window_kernel's thread order, one 8-byte load per code)
  const int32_t *occ_index;        // [M] -> j or -1
  int keep_bias;
  float scale;                     // dft_normalizer / float(nac) (framing.cc:821)
  const FrameInfo *info;
  float2 *G;                       // [F][M][N][N]
  double *part;                    // [F][N*N][n_groups][3][M] per-group sums (ls_kernel)
  uint32_t n_groups;               // ceil(nac / kLsCodesPerGroup)
  double *nv_part;                 // [F][n_nvp] residual-variance partials
  uint32_t n_nvp;                  // ceil(M / 256)
  const float2 *tw;
  const float2 *lsq;               // search_ls_kernel's X/S1 terms (ls_combine_q_kernel)
  const double *cfo_part;          // opt-in CFO: rotate code c's term by the stage-2 residual
  uint32_t M_cfo;                  // (M, window-relative; null: off)
  int cfo_fold;                    // ls_window_kernel with CFO: derotate the window loads by the
                                   // stage-1 estimate too (folded CFO; else the capture is)
};
constexpr uint32_t kLsCodesPerGroup = 4;   // access codes FFT'd per LS workgroup
void launch_ls(const LsArgs &a, int log2M, uint32_t n_frames, hipStream_t s);
void launch_ls_combine_q(const LsArgs &a, uint32_t n_frames, hipStream_t s);
// the LS estimate straight from the access-code windows at the search's keys, no terms in HBM
// (ls_window_kernel; 512 <= M <= 4096, CFO with nac <= 256): false when the geometry has no
// instance
bool launch_ls_window(const LsArgs &a, int log2M, uint32_t n_frames, hipStream_t s);

// per-subcarrier weights, framing.cc:826-831 -> 1344-1367 (+ NxN ZF/MMSE)
struct WeightArgs {
  uint32_t N, M, M_occ, nac, SL, n_slots;
  int detector;
  float noise_var;                 // < 0: estimate
  double nv_norm;                  // dn^2 / (M_occ*N*N*(nac-1)), 0 if nac < 2
  const int32_t *occ_index;
  const float2 *G;
  float2 *W;                       // [F][N(out)][N(rx)][M]
  float *gain;                     // [F][M]
  const double *nv_part;
  uint32_t n_nvp;
  const unsigned long long *keys;
  uint64_t win_len;
  FrameInfo *info;
};
void launch_weights(const WeightArgs &a, uint32_t n_frames, hipStream_t s);

// opt-in CFO of the batched path (cfo_kernels.hip)
struct CfoBatchArgs {
  const float2 *iq;
  float2 *out;                     // scratch capture, same layout as iq
  uint64_t stride, frame_len, len; // len: window samples derotated from each frame's base
  uint64_t win;                    // the framesync window (ACB + TX): stage 2 reads inside it
  uint32_t N, M, cp, SL;
  uint32_t n_codes;                // access-code symbols (N * nac) after S0
  uint32_t n_data;                 // data symbols in a window (PID + 2)
  uint32_t n_slots;
  int rot_window;                  // stage 2 derotates the whole window (LS not yet run)
  int fold;                        // the search, LS and decode loads derotate: estimates only
  FrameInfo *info;
  const unsigned long long *keys;  // search keys (stage 2 timing)
  double *part;                    // [F][2 stages][blocks][2] partial correlations
};
size_t cfo_batch_part_doubles(uint32_t n_frames);
// stage 1 (after S&C): coarse estimate, window derotated into `out`; stage 2 (after the
// weights): fine residual from the data symbols' prefixes, data region of `out` in place
void launch_cfo_batch(const CfoBatchArgs &a, uint32_t n_frames, int stage, hipStream_t s);
void launch_cfo_batch_rot2(const CfoBatchArgs &a, uint32_t n_frames, hipStream_t s);

// replay decode, framing.cc:535-589 / 508-533 fused with square-QAM demap + EVM
struct DecodeArgs {
  const float2 *iq;
  int sc16;                 // iq holds sc16 wire samples (float(i16) * iq_scale)
  float iq_scale;
  uint64_t stride, frame_len;
  uint32_t N, M, cp, SL, M_occ;
  int detector;
  uint32_t siso_tx, siso_rx;
  float dn;                        // 1/sqrtf(M_occ) (framing.cc:330)
  const int32_t *occ_index;
  const float2 *W;
  const float *gain;
  const float2 *G;
  const FrameInfo *info;
  uint32_t max_out;
  float2 *out_sym;                 // frame slot f at f N max_out M_occ, or null
  uint8_t *out_idx;                // same layout or null
  // element strides inside a frame slot (out_sym, out_idx, ref_idx): between streams and
  // between symbols. MIMO_LAYOUT_STREAM_MAJOR [F][N][max_out][M_occ]: (max_out M_occ, M_occ);
  // MIMO_LAYOUT_SYMBOL_MAJOR [F][max_out][N][M_occ]: (M_occ, N M_occ)
  uint64_t o_ts, o_ss;
  int ref_mode;
  const uint8_t *ref_idx;
  uint64_t ref_seed, frame_id0;
  Qam qam;
  double *evm_part;                // [F][max_out][parts][N][3]
  const float2 *tw;
  uint32_t n_frames;
  uint32_t n_caps, n_refs;         // captures and reference rows the frames point into
  int all_occ;                     // every subcarrier occupied (j == k): vector stores
  uint32_t n_cu;                   // compute units (persistent grid size)
  unsigned long long *prof;        // diagnostics: [items, load, fft, apply, reduce] cycles
  uint32_t *nrec;                  // [F] EVM records per frame (decode_stream_kernel) or null
  float2 *spec;                    // split decode (8x8) spectra scratch [F][sym_cap][N][M]
  uint32_t sym0, sym_cap, sym_groups;   // split decode: this launch's symbol group (set inside)
  uint32_t rec_stride;             // EVM records per frame in evm_part (max_out, or the split's)
  int cpe;                         // opt-in CFO: decision-directed common-phase tracking; 2 =
                                   // folded: the kernel also derotates by the frame's estimate
  const double *cfo_part;          // folded CFO: the stage partials (cfo_stage_eps)
};
// returns the number of EVM partial sets written per symbol (see EvmArgs::parts), 0 when no
// kernel takes the configuration (nothing launched: an sc16 batch the streaming kernel does not
// take); sets *per_frame_records when the streaming kernel wrote nrec[f] records per frame
// instead, and *path to the kernel family launched (MIMO_DECODE_*: 1 stream, 2 split, 3 symbol)
uint32_t launch_decode(const DecodeArgs &a, int log2M, uint32_t n_frames, hipStream_t s,
                       bool *per_frame_records, int *path);
// decode_stream.hip: persistent streaming form (0 when the configuration is not handled)
uint32_t launch_decode_stream(const DecodeArgs &a, int log2M, uint32_t n_frames, hipStream_t s);
// true when launch_decode_stream takes this configuration (nrec aside): the sc16 wire input
// is decoded only there
bool decode_stream_accepts(const DecodeArgs &a, int log2M, uint32_t n_frames);
// true when launch_decode_stream runs its CPE variant for these arguments (folded CFO
// derotation and the per-symbol common phase)
bool decode_stream_cpe(const DecodeArgs &a);
// decode_stream.hip: 8x8 split form (spectra to a scratch, then a chunked apply, optionally
// alternating over symbol groups); 0 when the configuration is not handled or a.spec is null.
// The scratch holds split_group_symbols(max_out) symbols per frame.
uint32_t launch_decode_split(const DecodeArgs &a, int log2M, uint32_t n_frames, hipStream_t s);
// one-pass 8x8 decode by residue class (M = 4096): accepts / launches (0: not handled), and
// the EVM records per frame it may write (rec_stride must hold them)
bool decode_split_accepts(const DecodeArgs &a, int log2M);
uint32_t split_group_symbols(uint32_t max_out);
// the split decode's symbol groups, symbol ranges per (group, chunk) and EVM records per frame
uint32_t split_plan(uint32_t max_out, int log2M, uint32_t *groups, uint32_t *P);
constexpr uint32_t kMaxEvmParts = 16;

struct EvmArgs {
  uint32_t N, max_out;
  uint32_t parts;                  // partial sets per symbol (launch_decode's return value)
  const FrameInfo *info;
  const double *evm_part;
  double *evm_out;                 // [F][N][3]
  double *chunk_part;              // [F][kEvmChunks][N][3]
  int few;                         // nrec records are few per frame: one workgroup per frame
  uint32_t *counter;               // [F] chunks done, zero between launches (self-resetting)
  const uint32_t *nrec;            // [F] records per frame (streaming decode) or null: n_sym
  uint32_t rec_stride;             // records per frame in evm_part (DecodeArgs::rec_stride)
};
constexpr uint32_t kEvmChunks = 16;
void launch_evm(const EvmArgs &a, uint32_t n_frames, hipStream_t s);

// code tables: S0/S1 -> IFFT*dn (framing.cc:1054-1111, 1214-1262) -> zero-pad FFT_F
struct CodesArgs {
  uint32_t M, N, nac, n_slots;
  const uint8_t *p;                // [M]
  const uint8_t *s0_bits;          // [M]
  const uint8_t *s1_bits;          // [N][nac*M]
  float dn_s0, dn_s1;
  float2 *code_time;               // [n_slots][M]
  float2 *codespec;                // [n_slots][F] (null: skip)
  float2 *codespec_w;              // [n_slots][F] permuted for the wave-local search (or null)
  const float2 *tw;
};
void launch_codes(const CodesArgs &a, int log2M, int log2F, hipStream_t s);

// transmitter: assemble_mimo_packet (framing.cc:210-235) for many symbols
struct TxSymArgs {
  uint32_t N, M, cp, M_occ;
  float dn;                        // 1/sqrtf(M_pilot+M_data) (framing.cc:115)
  float gain;                      // baseband gain (1 for framegen, 0.25 in tx_worker)
  const int32_t *occ_list;         // [M_occ] -> sc
  // symbol source: explicit (in != null) [N][n_sym][M_occ] or hashed QAM
  const float2 *in;
  uint32_t n_sym;
  uint64_t seed, frame_id0;
  Qam qam;
  uint8_t *tx_idx;                 // hashed mode: [F][N][n_sym][M_occ] or null
  float2 *out;                     // [F][N][n_sym][SL]
  const float2 *tw;
};
void launch_tx_symbols(const TxSymArgs &a, int log2M, uint32_t n_frames, hipStream_t s);

struct MixArgs {
  uint32_t N, M, cp, SL, nac, pid;
  uint64_t seed, frame_id0;
  int32_t offset;                  // < 0: per-frame hashed offset
  int identity;
  float nstd;
  const float2 *code_time;         // [n_slots][M]
  const float2 *tx_data;           // [F][N][pid][SL]
  float2 *out;                     // [F][N][stride]
  uint64_t stride, frame_len;
  float2 *H_out;                   // [F][N][N] or null
};
void launch_mix(const MixArgs &a, uint32_t n_frames, hipStream_t s);

// sc16 wire samples (interleaved int16 I/Q) -> planar complex64 rows (ingest_kernels.hip);
// false when the grid would not fit
// CFO (cfo_kernels.hip): per-row sum conj(x[n]) x[n+half] over [start, start+half) into
// d_out[2*row..], fp64; derotation by exp(-j 2 pi nu (n - n0))
bool launch_cfo_corr(const void *x, uint64_t stride, uint32_t rows, uint64_t start,
                     uint32_t half, double *d_out, hipStream_t s);
bool launch_cfo_derotate(void *x, uint64_t stride, uint32_t rows, uint64_t n, int64_t n0,
                         double nu, hipStream_t s);
// host side: record msg as this thread's mimo_last_error() and return code (engine.cpp)
int host_fail(int code, const char *msg);

bool launch_sc16_to_fc32(const void *src, uint64_t src_stride, void *dst, uint64_t dst_stride,
                         uint32_t rows, uint64_t n, float scale, hipStream_t s);

}  // namespace mimo

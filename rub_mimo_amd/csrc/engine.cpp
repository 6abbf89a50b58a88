// rub_mimo_amd/csrc/engine.cpp -- host side of librub_mimo_amd.so: the C-ABI of
// include/mimo_rx.h, device tables and workspaces, and the stage orchestration.
//
// Two drivers share the same kernels:
//   * mimo_rx_process_batch: n_frames device-resident captures, every stage launched once
//     for the whole batch on one stream, no host synchronisation (the bench's step).
//   * mimo_rx_execute: the reference's streaming framesync::execute (framing.cc:471-506)
//     over host chunks of any size -- samples are appended to a device capture buffer, the
//     S&C kernels run over the new chunks only, and the channel estimate + replay decode run
//     once the window [sync_index - SL, sync_index - SL + ACB + TX) is complete; decoded
//     symbols are handed to the callback one OFDM symbol at a time (framing.cc:587).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../../include/mimo_rx.h"
#include "kernels.hpp"

using namespace mimo;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(x)                                                                       \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess)                                                               \
      return fail(MIMO_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_));        \
  } while (0)

template <class T>
struct DevBuf {
  T *p = nullptr;
  size_t n = 0;
  DevBuf() = default;
  DevBuf(const DevBuf &) = delete;
  DevBuf &operator=(const DevBuf &) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  hipError_t ensure(size_t cnt) {
    if (cnt <= n && p) return hipSuccess;
    release();
    hipError_t e = hipMalloc(reinterpret_cast<void **>(&p), sizeof(T) * std::max<size_t>(cnt, 1));
    if (e == hipSuccess) n = cnt;
    return e;
  }
};

int ilog2(uint32_t v) {
  int l = 0;
  while ((1u << l) < v) l++;
  return ((1u << l) == v) ? l : -1;
}

// twiddle table tw[k] = exp(-2 pi i k / kTwN), shared by all handles (device 0 of the caller)
std::mutex g_tw_mu;
float2 *g_tw = nullptr;
int g_tw_dev = -1;

int get_twiddles(float2 **out) {
  std::lock_guard<std::mutex> lk(g_tw_mu);
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  if (!g_tw || g_tw_dev != dev) {
    std::vector<float2> h(kTwN);
    for (int k = 0; k < kTwN; k++) {
      const double a = -2.0 * M_PI * (double)k / (double)kTwN;
      h[k] = make_float2((float)std::cos(a), (float)std::sin(a));
    }
    float2 *d = nullptr;
    HIPCHK(hipMalloc(&d, sizeof(float2) * kTwN));
    HIPCHK(hipMemcpy(d, h.data(), sizeof(float2) * kTwN, hipMemcpyHostToDevice));
    g_tw = d;
    g_tw_dev = dev;
  }
  *out = g_tw;
  return MIMO_OK;
}

Qam make_qam(uint32_t order) {
  Qam q;
  uint32_t b = 0;
  while ((1u << (2 * b)) < order) b++;
  q.b = b;
  q.L = 1u << b;
  const double e = 2.0 * ((double)q.L * q.L - 1.0) / 3.0;
  q.scale = (float)(1.0 / std::sqrt(e));
  q.inv_scale = (float)std::sqrt(e);
  return q;
}

int validate_sctype(const uint8_t *p, uint32_t M, uint32_t *n0, uint32_t *n1, uint32_t *n2) {
  uint32_t a = 0, b = 0, c = 0;
  for (uint32_t i = 0; i < M; i++) {
    if (p[i] == MIMO_SC_NULL) a++;
    else if (p[i] == MIMO_SC_PILOT) b++;
    else if (p[i] == MIMO_SC_DATA) c++;
    else return fail(MIMO_ERR_SCTYPE, "invalid subcarrier type " + std::to_string(p[i]));
  }
  *n0 = a; *n1 = b; *n2 = c;
  return MIMO_OK;
}

struct StageTimer {
  bool on = false;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> ev;
  hipEvent_t begin(hipStream_t s) {
    if (!on) return nullptr;
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    (void)hipEventRecord(e, s);
    return e;
  }
  void end(int stage, hipEvent_t b, hipStream_t s) {
    if (!on || !b) return;
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return;
    (void)hipEventRecord(e, s);
    ev.push_back({stage, {b, e}});
  }
};

// code tables common to the receiver and the transmitter
struct Codes {
  DevBuf<float2> code_time;   // [n_slots][M]
  DevBuf<float2> codespec;    // [n_slots][F]
  DevBuf<float2> codespec_w;  // [n_slots][F], the wave-local search's bin order
};

int build_codes(Codes &c, uint32_t M, uint32_t N, uint32_t nac, const uint8_t *p,
                const uint8_t *s0_bits, const uint8_t *s1_bits, int log2F, bool spectra,
                hipStream_t s) {
  const uint32_t n_slots = N * nac + 1;
  uint32_t n0, n1, n2;
  int rc = validate_sctype(p, M, &n0, &n1, &n2);
  if (rc) return rc;
  uint32_t m_s0 = 0;
  for (uint32_t i = 0; i < M; i += 2)
    if (p[i] != MIMO_SC_NULL) m_s0++;
  if (m_s0 == 0) return fail(MIMO_ERR_SCTYPE, "ofdmframe_init_S0: no subcarriers enabled");
  DevBuf<uint8_t> dp, d0, d1;
  HIPCHK(dp.ensure(M));
  HIPCHK(d0.ensure(M));
  HIPCHK(d1.ensure((size_t)N * nac * M));
  HIPCHK(hipMemcpyAsync(dp.p, p, M, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(d0.p, s0_bits, M, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(d1.p, s1_bits, (size_t)N * nac * M, hipMemcpyHostToDevice, s));
  HIPCHK(c.code_time.ensure((size_t)n_slots * M));
  const uint32_t F = 1u << log2F;
  if (spectra) HIPCHK(c.codespec.ensure((size_t)n_slots * F));
  if (spectra && F >= 1024) HIPCHK(c.codespec_w.ensure((size_t)n_slots * F));
  CodesArgs a{};
  a.M = M; a.N = N; a.nac = nac; a.n_slots = n_slots;
  a.p = dp.p; a.s0_bits = d0.p; a.s1_bits = d1.p;
  a.dn_s0 = (float)std::sqrt(1.0 / (double)(float)m_s0);   // framing.cc:1100
  a.dn_s1 = (float)std::sqrt(1.0 / (double)(float)M);      // framing.cc:1228
  a.code_time = c.code_time.p;
  a.codespec = spectra ? c.codespec.p : nullptr;
  a.codespec_w = (spectra && F >= 1024) ? c.codespec_w.p : nullptr;
  int rc2 = get_twiddles(const_cast<float2 **>(&a.tw));
  if (rc2) return rc2;
  launch_codes(a, ilog2(M), log2F, s);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(s));  // the staging buffers die with this scope
  return MIMO_OK;
}

}  // namespace

// ======================================================================================
struct mimo_rx {
  // configuration (framesync ctor arguments + config.h constants)
  uint32_t M = 0, cp = 0, SL = 0, N = 0, nac = 0, pid = 0;
  uint32_t M_null = 0, M_pilot = 0, M_data = 0, M_occ = 0;
  int log2M = 0, log2F = 0;
  uint32_t F = 0, lagc = 0, n_lagc = 0, n_slots = 0;
  bool search_ls = false;               // fused search + LS (search_ls_kernel) for this geometry
  bool cfo = false;                     // opt-in CFO estimate + derotation (batched path)
  int cur_sc16 = 0;                     // the batch being launched reads sc16 wire samples
  float cur_scale = 1.0f;
  uint32_t cur_layout = 0;              // its output layout (MIMO_LAYOUT_*)
  DevBuf<float2> spec;                  // 8x8 split decode: spectra scratch
  DevBuf<float2> wide;                  // sc16 batches the fused kernels do not take: widened
  DevBuf<float2> cfo_iq;                // derotated scratch capture
  DevBuf<double> cfo_eps;
  uint32_t n_cu = 256;
  int det = 0;
  float noise_var = -1.0f;
  int keep_bias = 1;
  uint32_t siso_tx = 0, siso_rx = 0;
  double thr = 0.95;
  Qam qam{};
  uint64_t acb = 0, txl = 0, win_len = 0;
  float dn = 1.0f, ls_scale = 1.0f;
  double nv_norm = 0.0;
  std::vector<uint8_t> p;
  std::vector<int32_t> occ_index;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  // device tables
  float2 *tw = nullptr;
  Codes codes;
  DevBuf<float> vscale;
  DevBuf<int8_t> s1sign, s1sign_w;   // signs [N][nac][M]; ls_window_kernel's order
  DevBuf<int32_t> occ;
  // workspace
  uint32_t cap_frames = 0;
  uint64_t cap_chunks = 0;
  uint64_t cap_evm = 0;
  DevBuf<unsigned long long> trig, keys;
  DevBuf<ScRecord> rec;
  DevBuf<FrameInfo> info;
  DevBuf<float2> G, W;
  DevBuf<float> gain;
  DevBuf<double> nvp, evm_part, evm_out, lspart, evm_chunk;
  DevBuf<float2> lsq;                   // fused search + LS: X/S1 per access code
  DevBuf<uint32_t> evm_cnt;             // per-frame chunk counters of evm_kernel (self-resetting)
  DevBuf<uint32_t> nrec;                // per-frame EVM records of the streaming decode
  size_t cap_lspart = 0;
  DevBuf<unsigned long long> n_exact;   // S&C exact fp32 recomputes (diagnostic)
  DevBuf<uint32_t> queue;               // S&C work-queue head, hot-item count
  DevBuf<ScHot> hot;                    // S&C items awaiting exact resolution
  DevBuf<uint32_t> scr_flag;            // S&C screen: chunk listed [F][nchunks]
  DevBuf<unsigned long long> scr_min, scr_max;   // first / last unproven position per chunk
  DevBuf<unsigned long long> cand;      // streams: first S&C candidate per chunk [cap][chunks]
  DevBuf<unsigned long long> certfail;  // streams: re-arm certificate failures [cap] (bit = slot)
  uint32_t cap_hot = 0;
  DevBuf<unsigned long long> sc_prof;   // RMIMO_SC_PROF=1 cycle counters
  uint32_t last_frames = 0, last_max_out = 0;
  int last_decode_path = MIMO_DECODE_NONE;   // kernel family of the last decode launch
  int last_cfo_mode = 0;                     // CFO stages of the last batch (get_cfo_mode)
  // streaming state (facade). The device capture holds samples [origin, origin + total) of
  // the stream since construction/reset (positions inside it are capture-relative).
  DevBuf<float2> capbuf;
  uint64_t cap_len = 0, total = 0, origin = 0;
  uint64_t trim_clo = ~0ull;   // stream position of the S&C chunk of the last trim probe
  DevBuf<uint32_t> probe;               // trim probe: per antenna, a proven metric zero
  // DEBUG_LOG files of the streaming execute (framing.cc:390-402, 598-600, 675-696, 873-883)
  std::string dbg_dir;
  std::vector<FILE *> dbg_fsc;
  DevBuf<float> dbg_y, dbg_corr;
  float *cur_corr_trace = nullptr;
  int state = MIMO_STATE_SEEK_PLATEAU;
  uint64_t nsp = 0;
  bool have_sync = false, have_est = false;
  FrameInfo sinfo{};
  DevBuf<float2> symbuf;
  std::vector<float2> symhost;
  mimo_rx_symbol_cb cb = nullptr;
  void *user = nullptr;
  StageTimer timer;
  // captured batch pipelines (see mimo_rx_process_batch): a few recent batch keys, so that
  // callers alternating between capture buffers (double-buffered ingest) replay graphs too
  struct GraphEntry {
    mimo_batch key{};
    hipStream_t stream = nullptr;
    std::array<const void *, 27> sig{};
    hipGraphExec_t exec = nullptr;
    uint64_t used = 0;            // 0: empty slot
  };
  std::array<GraphEntry, 4> graphs{};
  uint64_t graph_tick = 0;
};

struct mimo_tx {
  uint32_t M = 0, cp = 0, SL = 0, N = 0, nac = 0, M_occ = 0;
  int log2M = 0;
  float dn = 1.0f;
  hipStream_t stream = nullptr;
  Codes codes;
  std::vector<float2> s0, s1;  // host copies of the time-domain codes
  DevBuf<int32_t> occ_list;
  DevBuf<float2> din, dout;
  float2 *tw = nullptr;
};

namespace {

// Per-frame arrays grow with F; the per-chunk trigger records grow with F * chunks. A
// growing single-frame record array (streaming capture) keeps its earlier records: chunks
// already final are never recomputed, and trig[] is untouched when only the capture grows.
int ensure_workspace(mimo_rx *h, uint32_t F, uint64_t chunks, uint64_t evm_entries) {
  if (F > h->cap_frames) {
    const uint32_t nf = F;
    HIPCHK(h->trig.ensure(nf));
    HIPCHK(h->keys.ensure((size_t)nf * h->N * h->n_slots));
    HIPCHK(h->info.ensure(nf));
    HIPCHK(h->G.ensure((size_t)nf * h->M * h->N * h->N));
    HIPCHK(h->W.ensure((size_t)nf * h->M * h->N * h->N));
    HIPCHK(h->gain.ensure((size_t)nf * h->M));
    HIPCHK(h->nvp.ensure((size_t)nf * h->N * h->N * ((h->M + 255) / 256)));   // ls_combine blocks
    HIPCHK(h->evm_out.ensure((size_t)nf * h->N * 3));
    HIPCHK(h->evm_chunk.ensure((size_t)nf * kEvmChunks * h->N * 3));
    HIPCHK(h->evm_cnt.ensure(nf));
    HIPCHK(h->nrec.ensure(nf));
    HIPCHK(hipMemset(h->evm_cnt.p, 0, sizeof(uint32_t) * nf));
    h->cap_frames = nf;
    HIPCHK(h->rec.ensure((size_t)nf * h->cap_chunks));
  }
  if (chunks > h->cap_chunks) {
    const uint64_t nc = std::max<uint64_t>(chunks, h->cap_chunks * 2);
    ScRecord *np = nullptr;
    HIPCHK(hipMalloc(&np, sizeof(ScRecord) * (size_t)h->cap_frames * nc));
    // frame 0's records survive: the streaming execute path (one frame) never recomputes a
    // final chunk, whatever batch sizes the handle ran before
    if (h->rec.p && h->cap_chunks)
      HIPCHK(hipMemcpy(np, h->rec.p, sizeof(ScRecord) * h->cap_chunks, hipMemcpyDeviceToDevice));
    h->rec.release();
    h->rec.p = np;
    h->rec.n = (size_t)h->cap_frames * nc;
    h->cap_chunks = nc;
  }
  if (evm_entries > h->cap_evm) {
    HIPCHK(h->evm_part.ensure(evm_entries));
    h->cap_evm = evm_entries;
  }
  return MIMO_OK;
}

// Decision band of the fp64 S&C metric: a first-order bound on |y_fp32 - y| for the oracle's
// sequential fp32 sums (framing.cc:626-637), for y <= 1 (|P| <= R always):
//   |dy| <= 2 sqrt(2) (M/2 + 2) u sqrt(y) + 2 (M + 1) u y + 4 u y,   u = 2^-24,
// with a 25% margin for the neglected O((M u)^2) terms. Outside the band the fp64 decision
// equals the oracle's; inside it the sample is recomputed exactly.
static double sc_band(uint32_t M) {
  const double u = 0x1p-24;
  return 1.25 * u * (std::sqrt(2.0) * (M + 4.0) + 2.0 * M + 6.0);
}

// S&C + plateau over chunks [chunk_lo, end) of every capture; with fpc > 1 frames per capture
// the stream walk assigns F * fpc frame slots
int run_sync(mimo_rx *h, const float2 *iq, uint64_t stride, uint32_t F, uint64_t frame_len,
             uint64_t chunk_lo, bool reset_trig, hipStream_t s, uint32_t fpc = 1,
             const uint64_t *ref_starts = nullptr, uint32_t ref_stride = 0,
             bool zero_keys = false) {
  const uint64_t K = sc_chunk_len(h->cp);
  const uint64_t nchunks = (frame_len + K - 1) / K;
  const bool stream = fpc > 1;
  int rc = ensure_workspace(h, F * fpc, nchunks, 0);
  if (rc) return rc;
  FillArgs fa{};
  auto add_fill = [&fa](void *p, uint64_t bytes, uint32_t v) {
    fa.p[fa.count] = reinterpret_cast<uint32_t *>(p);
    fa.n[fa.count] = bytes / 4;
    fa.v[fa.count] = v;
    fa.count++;
  };
  if (reset_trig) add_fill(h->trig.p, sizeof(unsigned long long) * F, 0xFFFFFFFFu);
  // the search's argmax keys, zeroed here instead of by a memset ahead of the search
  if (zero_keys) add_fill(h->keys.p, sizeof(unsigned long long) * F * fpc * h->N * h->n_slots, 0u);
  if (stream) {
    HIPCHK(h->cand.ensure((size_t)F * nchunks));
    HIPCHK(h->certfail.ensure(F));
    add_fill(h->cand.p, sizeof(unsigned long long) * F * nchunks, 0xFFFFFFFFu);
    add_fill(h->certfail.p, sizeof(unsigned long long) * F, 0u);
  }
  if (chunk_lo >= nchunks) launch_fill(fa, s);
  if (chunk_lo < nchunks) {
    ScArgs a{};
    a.iq = iq; a.stride = stride; a.frame_len = frame_len;
    a.sc16 = h->cur_sc16; a.iq_scale = h->cur_scale;
    a.N = h->N; a.M = h->M; a.cp = h->cp;
    a.thr = h->thr;
    a.band = sc_band(h->M);
    static const int diag_env = [] { const char *e = getenv("RMIMO_SC_DIAG"); return e ? atoi(e) : 0; }();
    a.diag = (uint32_t)diag_env;
    a.chunk_len = K; a.chunk_lo = chunk_lo; a.chunk_hi = nchunks;
    a.trig = h->trig.p; a.rec = h->rec.p; a.rec_stride = h->cap_chunks;
    a.cand = stream ? h->cand.p : nullptr;
    a.no_skip = stream ? 1 : 0;
    if (!h->n_exact.p) {
      HIPCHK(h->n_exact.ensure(1));
      HIPCHK(hipMemsetAsync(h->n_exact.p, 0, sizeof(unsigned long long), s));
    }
    a.n_exact = h->n_exact.p;
    if (!h->queue.p) HIPCHK(h->queue.ensure(3));
    add_fill(h->queue.p, 3 * sizeof(uint32_t), 0u);
    a.queue = h->queue.p;
    a.hot_count = h->queue.p + 1;
    // screened path where the geometry allows it (else the per-chunk item kernel): one hot item
    // per listed chunk
    const bool screen = sc_screen_ok(h->M);
    const uint64_t n_list = (nchunks - chunk_lo) * (uint64_t)F;
    const uint32_t hot_cap = screen ? (uint32_t)n_list : 8 * F + 32;
    if (hot_cap > h->cap_hot) {
      HIPCHK(h->hot.ensure(hot_cap));
      h->cap_hot = hot_cap;
    }
    a.nchunks = nchunks;
    if (screen) {
      const size_t nf = (size_t)F * nchunks;
      HIPCHK(h->scr_flag.ensure(nf));
      HIPCHK(h->scr_min.ensure(nf));
      HIPCHK(h->scr_max.ensure(nf));
      add_fill(h->scr_flag.p, sizeof(uint32_t) * nf, 0u);
      add_fill(h->scr_min.p, sizeof(unsigned long long) * nf, 0xFFFFFFFFu);
      add_fill(h->scr_max.p, sizeof(unsigned long long) * nf, 0u);
      a.fmin = h->scr_min.p;
      a.fmax = h->scr_max.p;
    }
    a.hot = h->hot.p;
    a.hot_cap = hot_cap;
    launch_fill(fa, s);   // trigger words, queue heads and screen flags in one launch
    static const bool prof_env = [] { const char *e = getenv("RMIMO_SC_PROF"); return e && e[0] == '1'; }();
    if (prof_env) {
      if (!h->sc_prof.p) HIPCHK(h->sc_prof.ensure(32));
      HIPCHK(hipMemsetAsync(h->sc_prof.p, 0, 32 * sizeof(unsigned long long), s));
      HIPCHK(hipMemsetAsync(h->sc_prof.p + 8, 0xFF, sizeof(unsigned long long), s));
      if (screen) HIPCHK(hipMemsetAsync(h->sc_prof.p, 0xFF, sizeof(unsigned long long), s));
      a.prof = h->sc_prof.p;
    }
    hipEvent_t e = h->timer.begin(s);
    if (screen) {
      ScreenArgs sa{};
      sa.iq = iq; sa.stride = stride; sa.frame_len = frame_len;
      sa.sc16 = h->cur_sc16; sa.iq_scale = h->cur_scale;
      sa.N = h->N; sa.M = h->M;
      sa.thr_screen = h->thr - 0.01;
      sa.chunk_len = K; sa.chunk_lo = chunk_lo; sa.nchunks = nchunks;
      sa.flag = h->scr_flag.p; sa.fmin = h->scr_min.p; sa.fmax = h->scr_max.p;
      sa.count = a.hot_count; sa.hot = a.hot; sa.cap = a.hot_cap;
      // batches: every capture starts at its (first) framesync's origin; the streaming execute's
      // capture may begin mid-stream after a trim (its history is not empty)
      sa.empty_history = reset_trig ? 1u : 0u;
      if (a.diag & 32) a.diag |= 16;   // diagnostics: finalize as a separate kernel
      // Two phases for one frame per capture: the first chunks of every capture (a
      // frame's S0 plateau sits near its capture's start), then the rest only for captures with
      // no trigger yet. A trigger found in phase 1 is the capture's first (every earlier chunk
      // was evaluated) and phase 2 evaluates exactly the chunks one pass would have for the
      // others, so results are those of one pass; the screen's reads of antenna 0 past the
      // trigger of a synced capture are skipped. RMIMO_SC_PHASES=1: one pass.
      // Phase 1 ends one chunk past the S0 pair of a frame that starts its capture as the
      // reference's tx_worker lays frames out (main.cc:937-1153: SL (N nac + 1) + u zeros,
      // u < SL, then the two S0 symbols), the M-sample metric delay included.
      static const bool one_phase = [] { const char *e = getenv("RMIMO_SC_PHASES"); return e && e[0] == '1'; }();
      const uint64_t s0_end = (uint64_t)h->SL * ((uint64_t)h->N * h->nac + 4) + h->M;
      const uint64_t c1 = (!stream && chunk_lo == 0 && !one_phase && nchunks >= 16)
                              ? std::min<uint64_t>(nchunks, std::max<uint64_t>(2, (s0_end + K - 1) / K + 1))
                              : nchunks;
      sa.chunk_hi = c1;
      launch_sc_screen(sa, F, s);
      ScArgs a1 = a;
      if (c1 < nchunks) a1.snap = h->queue.p + 2;   // phase-1 items: done after this launch
      launch_sc_exact(a1, s);   // resolves and finalises its items itself
      if (a.diag & 32) launch_sc_finalize(a, s);
      if (c1 < nchunks) {
        sa.chunk_lo = c1;
        sa.chunk_hi = nchunks;
        sa.trig = h->trig.p;
        launch_sc_screen(sa, F, s);
        ScArgs a2 = a;
        a2.item_lo = h->queue.p + 2;
        launch_sc_exact(a2, s);
        if (a.diag & 32) launch_sc_finalize(a2, s);
      }
    } else {
      launch_sc(a, F, h->n_cu, s);
      launch_sc_hot(a, s);
    }
    static const bool cnt_env = [] { const char *e = getenv("RMIMO_SC_COUNT"); return e && e[0] == '1'; }();
    hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(s, &cst);
    if (cnt_env && cst == hipStreamCaptureStatusNone) {   // diagnostics: S&C work-list size
      uint32_t q[2] = {0, 0};
      HIPCHK(hipMemcpyAsync(q, h->queue.p, sizeof(q), hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      fprintf(stderr, "sc_count hot_items %u (screen %d, frames %u, chunks %llu)\n", q[1],
              screen ? 1 : 0, F, (unsigned long long)nchunks);
      static const bool items_env = [] { const char *e = getenv("RMIMO_SC_COUNT"); return e[1] == '+'; }();
      if (items_env && screen) {   // per item: frame, chunk, unproven range and its iterations
        const uint32_t n = std::min(q[1], hot_cap);
        std::vector<ScHot> hv(n);
        std::vector<unsigned long long> mn((size_t)F * nchunks), mx((size_t)F * nchunks);
        HIPCHK(hipMemcpyAsync(hv.data(), h->hot.p, sizeof(ScHot) * n, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(mn.data(), h->scr_min.p, sizeof(unsigned long long) * mn.size(),
                              hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(mx.data(), h->scr_max.p, sizeof(unsigned long long) * mx.size(),
                              hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        for (uint32_t i = 0; i < n; i++) {
          const ScHot &it = hv[i];
          const size_t ci = (size_t)it.f * nchunks + it.chunk;
          const long long lo = (long long)mn[ci] - it.w0, hi = (long long)mx[ci] - it.w0;
          const long long a0 = std::max<long long>(0, (lo - (long long)h->cp - 2) / kScIterLen);
          const long long a1 = std::min<long long>(kScSpan / kScIterLen - 1, hi / kScIterLen);
          fprintf(stderr, "sc_item %u f %u chunk %llu w0 %lld c0 %lld unproven [%lld, %lld] (%lld) "
                  "iterations %lld-%lld\n", i, it.f, (unsigned long long)it.chunk, (long long)it.w0,
                  (long long)it.c0, lo, hi, hi - lo + 1, a0, a1);
        }
      }
    }
    h->timer.end(0, e, s);
    if (prof_env && screen) {   // diagnostics: exact-kernel timeline (wall clock, 100 MHz)
      unsigned long long v[32];
      HIPCHK(hipMemcpyAsync(v, h->sc_prof.p, sizeof(v), hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      fprintf(stderr, "exact_prof passes %llu last_pass_end %.2f us finalize_end %.2f us "
              "avg_pass %.2f us avg_resolve %.2f us finalizes %llu cond %.2f us record %.2f us "
              "(%llu with candidates) slowest pass %.2f us (%llu iterations, resolve %.2f us) "
              "max windows/pass %llu (samples %llu) total samples %llu\n", v[4],
              (double)(v[1] - v[0]) / 100.0, (double)(v[2] - v[0]) / 100.0,
              v[4] ? (double)v[3] / v[4] / 100.0 : 0.0, v[4] ? (double)v[7] / v[4] / 100.0 : 0.0,
              v[6], v[6] ? (double)v[10] / v[6] / 100.0 : 0.0,
              v[12] ? (double)v[11] / v[12] / 100.0 : 0.0, v[12], (double)(v[13] >> 32) / 100.0,
              (v[13] >> 24) & 0xFF, (double)(v[13] & 0xFFFFFF) / 100.0, v[14] >> 32,
              v[14] & 0xFFFFFFFFull, v[15]);
      const double np = v[4] ? (double)v[4] : 1.0;
      fprintf(stderr, "exact_split record %.2f us setup %.2f us iterations %.2f us (%.2f per pass) "
              "start offset avg %.2f max %.2f us | per iteration: ring %.2f scan %.2f walk %.2f us "
              "(first iteration's ring %.2f us per pass; guarded fills %llu)\n",
              v[20] / np / 100.0, v[21] / np / 100.0,
              v[22] / np / 100.0, v[23] / np, (v[26] / np - (double)v[0]) / 100.0,
              (double)(v[25] - v[0]) / 100.0, v[23] ? v[16] / (double)v[23] / 100.0 : 0.0,
              v[23] ? v[17] / (double)v[23] / 100.0 : 0.0, v[23] ? v[18] / (double)v[23] / 100.0 : 0.0,
              v[19] / np / 100.0, v[24]);
      fprintf(stderr, "exact_windows max per iteration %llu, iterations with >= 2 windows %llu "
              "(their passes' max duration %.2f us)\n", v[27], v[28], (double)v[29] / 100.0);
    } else if (prof_env) {   // diagnostics: per-item cycle split of the S&C kernel
      unsigned long long v[20];
      HIPCHK(hipMemcpyAsync(v, h->sc_prof.p, sizeof(v), hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      const double it = v[0] ? (double)v[0] : 1.0;
      fprintf(stderr, "sc_prof items %llu skipped %llu antenna_passes %llu cycles/item rows %.0f "
              "words %.0f resolve %.0f total %.0f wall_us/item %.2f span_us %.2f max_item_us %.2f "
              "last_start_us %.2f\n", v[0], v[6], v[1],
              v[2] / it, v[3] / it, v[4] / it, v[5] / it, v[7] / it / 100.0,
              (double)(v[9] - v[8]) / 100.0, v[10] / 100.0, (double)(v[11] - v[8]) / 100.0);
      fprintf(stderr, "sc_prof phases/item warm %.0f A %.0f scan %.0f B %.0f run %.0f | resolve "
              "passes %llu chain cycles/pass %.0f samples/pass %.1f\n",
              v[12] / it, v[13] / it, v[14] / it, v[15] / it, v[16] / it, v[17],
              v[17] ? (double)v[18] / v[17] : 0.0, v[17] ? (double)v[19] / v[17] : 0.0);
    }
  }
  PlateauArgs pa{};
  pa.trig = h->trig.p; pa.rec = h->rec.p; pa.rec_stride = h->cap_chunks; pa.chunk_len = K;
  pa.iq = iq; pa.stride = stride; pa.frame_len = frame_len;
  pa.sc16 = h->cur_sc16; pa.iq_scale = h->cur_scale;
  pa.N = h->N; pa.M = h->M; pa.SL = h->SL; pa.thr = h->thr; pa.win_len = h->win_len;
  pa.band = sc_band(h->M);
  pa.info = h->info.p;
  pa.fpc = fpc; pa.nchunks = nchunks;
  pa.cand = stream ? h->cand.p : nullptr;
  pa.certfail = stream ? h->certfail.p : nullptr;
  pa.ref_starts = ref_starts;
  pa.ref_stride = ref_stride ? ref_stride : fpc;
  hipEvent_t e = h->timer.begin(s);
  if (stream) launch_stream_walk(pa, F, s);
  else launch_plateau(pa, F, s);
  h->timer.end(1, e, s);
  HIPCHK(hipGetLastError());
  return MIMO_OK;
}

int run_estimate(mimo_rx *h, const float2 *iq, uint64_t stride, uint32_t F, uint64_t frame_len,
                 hipStream_t s, bool keys_zeroed = false, CfoBatchArgs *cfo = nullptr) {
  if (!keys_zeroed)
    HIPCHK(hipMemsetAsync(h->keys.p, 0, sizeof(unsigned long long) * F * h->N * h->n_slots, s));
  SearchArgs sa{};
  sa.iq = iq; sa.stride = stride; sa.frame_len = frame_len;
  sa.sc16 = h->cur_sc16; sa.iq_scale = h->cur_scale;
  sa.N = h->N; sa.M = h->M; sa.SL = h->SL; sa.n_slots = h->n_slots;
  sa.lagc = h->lagc; sa.n_lagc = h->n_lagc;
  sa.codespec = h->codes.codespec.p; sa.vscale = h->vscale.p;
  sa.codespec_w = h->codes.codespec_w.p;
  sa.info = h->info.p; sa.keys = h->keys.p; sa.tw = h->tw;
  sa.corr_trace = h->cur_corr_trace;
  LsArgs la{};
  la.iq = iq; la.stride = stride; la.frame_len = frame_len;
  la.N = h->N; la.M = h->M; la.nac = h->nac; la.n_slots = h->n_slots;
  la.keys = h->keys.p; la.s1sign = h->s1sign.p; la.occ_index = h->occ.p;
  la.s1sign_w = h->s1sign_w.p;
  la.keep_bias = h->keep_bias; la.scale = h->ls_scale; la.info = h->info.p;
  la.n_groups = (h->nac + kLsCodesPerGroup - 1) / kLsCodesPerGroup;
  la.n_nvp = h->N * h->N * ((h->M + 255) / 256);
  la.G = h->G.p; la.nv_part = h->nvp.p; la.tw = h->tw;
  la.sc16 = h->cur_sc16; la.iq_scale = h->cur_scale;
  // LS straight from the windows (ls_window_kernel) after a search that only finds the keys
  // (the opt-in CFO's stage 2 between them, its residual rotating each code's term in the LS
  // kernel), unless RMIMO_LS_FORM=terms: the search's fused terms and ls_combine_q_kernel, the
  // parity tests' reference for this form
  static const bool ls_terms = [] { const char *e = getenv("RMIMO_LS_FORM"); return e && strcmp(e, "terms") == 0; }();
  const bool ls_win = h->search_ls && !ls_terms && h->log2M >= 9 && h->log2M <= 12 &&
                      (!cfo || h->nac <= 256);
  if (h->search_ls && ls_win) {
    sa.xcd_order = 1;
    sa.cfo_part = (cfo && cfo->fold) ? cfo->part : nullptr;   // folded CFO: derotating loads
    hipEvent_t e = h->timer.begin(s);
    launch_search_ls(sa, h->log2F, h->log2M, F, s);   // keys only (sa.lsq null)
    h->timer.end(2, e, s);
    if (cfo) {   // opt-in CFO stage 2: residual from the data prefixes
      cfo->keys = h->keys.p; cfo->n_slots = h->n_slots; cfo->rot_window = 0;
      launch_cfo_batch(*cfo, F, 2, s);
      la.cfo_part = cfo->part;
      la.cfo_fold = cfo->fold;
    }
    e = h->timer.begin(s);
    if (!launch_ls_window(la, h->log2M, F, s))   // (ls_win admits only what it launches)
      return fail(MIMO_ERR_UNSUPPORTED, "ls_window_kernel: no instance for this geometry");
    h->timer.end(3, e, s);
  } else if (h->search_ls) {
    // search of slot pairs with the LS terms fused in, then the fixed-order LS combine
    HIPCHK(h->lsq.ensure((size_t)F * h->N * h->N * h->nac * h->M));
    sa.s1sign = h->s1sign.p; sa.lsq = h->lsq.p; sa.nac = h->nac;
    sa.cfo_part = (cfo && cfo->fold) ? cfo->part : nullptr;   // folded CFO: derotating loads
    sa.xcd_order = 1;
    la.lsq = h->lsq.p;
    hipEvent_t e = h->timer.begin(s);
    launch_search_ls(sa, h->log2F, h->log2M, F, s);
    h->timer.end(2, e, s);
    if (cfo) {   // opt-in CFO stage 2: residual from the data prefixes; LS terms rotated below
      cfo->keys = h->keys.p; cfo->n_slots = h->n_slots; cfo->rot_window = 0;
      launch_cfo_batch(*cfo, F, 2, s);
      la.cfo_part = cfo->part;
    }
    e = h->timer.begin(s);
    launch_ls_combine_q(la, F, s);
    h->timer.end(3, e, s);
  } else {
    hipEvent_t e = h->timer.begin(s);
    launch_search(sa, h->log2F, F, s);
    h->timer.end(2, e, s);
    if (cfo) {   // opt-in CFO stage 2 before a separate LS pass: the whole window in place
      cfo->keys = h->keys.p; cfo->n_slots = h->n_slots; cfo->rot_window = 1;
      launch_cfo_batch(*cfo, F, 2, s);
    }
    {
      const size_t need = (size_t)F * h->N * h->N * la.n_groups * 3 * h->M;
      if (need > h->cap_lspart) {
        HIPCHK(h->lspart.ensure(need));
        h->cap_lspart = need;
      }
    }
    la.part = h->lspart.p;
    e = h->timer.begin(s);
    launch_ls(la, h->log2M, F, s);
    h->timer.end(3, e, s);
  }
  WeightArgs wa{};
  wa.N = h->N; wa.M = h->M; wa.M_occ = h->M_occ; wa.nac = h->nac; wa.SL = h->SL;
  wa.n_slots = h->n_slots; wa.detector = h->det; wa.noise_var = h->noise_var;
  wa.nv_norm = h->nv_norm; wa.occ_index = h->occ.p; wa.G = h->G.p; wa.W = h->W.p;
  wa.gain = h->gain.p; wa.nv_part = h->nvp.p; wa.n_nvp = la.n_nvp; wa.keys = h->keys.p;
  wa.win_len = h->win_len;
  wa.info = h->info.p;
  hipEvent_t e = h->timer.begin(s);
  launch_weights(wa, F, s);
  h->timer.end(4, e, s);
  HIPCHK(hipGetLastError());
  return MIMO_OK;
}

int run_decode(mimo_rx *h, const float2 *iq, uint64_t stride, uint32_t F, uint64_t frame_len,
               uint32_t max_out, float2 *out_sym, uint8_t *out_idx, int ref_mode,
               const uint8_t *ref_idx, uint64_t ref_seed, uint64_t frame_id0, hipStream_t s,
               uint32_t n_caps = 0, const double *cfo_fold_part = nullptr) {
  if (max_out == 0) {
    int rc0 = ensure_workspace(h, F, 0, 0);
    return rc0;
  }
  DecodeArgs d{};
  d.iq = iq; d.stride = stride; d.frame_len = frame_len;
  d.sc16 = h->cur_sc16; d.iq_scale = h->cur_scale;
  d.N = h->N; d.M = h->M; d.cp = h->cp; d.SL = h->SL; d.M_occ = h->M_occ;
  d.detector = h->det; d.siso_tx = h->siso_tx; d.siso_rx = h->siso_rx; d.dn = h->dn;
  d.occ_index = h->occ.p; d.W = h->W.p; d.gain = h->gain.p; d.G = h->G.p; d.info = h->info.p;
  d.max_out = max_out; d.out_sym = out_sym; d.out_idx = out_idx;
  if (h->cur_layout == MIMO_LAYOUT_SYMBOL_MAJOR) {   // [F][max_out][N][M_occ]
    d.o_ts = h->M_occ;
    d.o_ss = (uint64_t)h->N * h->M_occ;
  } else {                                         // [F][N][max_out][M_occ]
    d.o_ts = (uint64_t)max_out * h->M_occ;
    d.o_ss = h->M_occ;
  }
  d.ref_mode = ref_mode; d.ref_idx = ref_idx; d.ref_seed = ref_seed; d.frame_id0 = frame_id0;
  d.qam = h->qam; d.evm_part = h->evm_part.p; d.tw = h->tw;
  d.n_frames = F; d.n_cu = h->n_cu;
  d.n_caps = n_caps ? n_caps : F; d.n_refs = F;
  d.all_occ = (h->M_occ == h->M) ? 1 : 0;
  static const bool dprof = [] { const char *e = getenv("RMIMO_DEC_PROF"); return e && e[0] == '1'; }();
  if (dprof) {
    if (!h->sc_prof.p) HIPCHK(h->sc_prof.ensure(28));
    HIPCHK(hipMemsetAsync(h->sc_prof.p, 0, 8 * sizeof(unsigned long long), s));
    d.prof = h->sc_prof.p;
  }
  hipEvent_t e = h->timer.begin(s);
  d.nrec = h->nrec.p;
  d.cpe = h->cfo ? (cfo_fold_part ? 2 : 1) : 0;
  d.cfo_part = cfo_fold_part;
  d.rec_stride = max_out;
  if (decode_split_accepts(d, h->log2M)) {
    // [F][group][N][M] complex64 spectra of the 8x8 split decode (one symbol group)
    if (h->spec.ensure((size_t)F * split_group_symbols(max_out) * h->N * h->M) != hipSuccess)
      return fail(MIMO_ERR_NOMEM, "split decode scratch");
    d.spec = h->spec.p;
    d.rec_stride = std::max(d.rec_stride, split_plan(max_out, h->log2M, nullptr, nullptr));
  }
  {
    const int rc0 = ensure_workspace(h, F, 0, (uint64_t)F * d.rec_stride * h->N * 3 * kMaxEvmParts);
    if (rc0) return rc0;
  }
  d.evm_part = h->evm_part.p;
  bool per_frame = false;
  int path = MIMO_DECODE_NONE;
  const uint32_t parts = launch_decode(d, h->log2M, F, s, &per_frame, &path);
  h->timer.end(5, e, s);
  h->last_decode_path = path;
  h->last_cfo_mode = !h->cfo ? 0 : (path == MIMO_DECODE_STREAM && decode_stream_cpe(d) ? 2 : 1);
  static const bool cfo_dbg = [] { const char *e = getenv("RMIMO_CFO_DEBUG"); return e && e[0] == '1'; }();
  if (cfo_dbg && h->cfo) {   // diagnostics: the per-frame CFO state the decode read
    std::vector<FrameInfo> fi(F);
    HIPCHK(hipMemcpyAsync(fi.data(), h->info.p, sizeof(FrameInfo) * F, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    for (uint32_t f = 0; f < F; f++)
      fprintf(stderr, "cfo_dbg f %u status %d base %lld i0 %u eps %.9f E %lld\n", f, (int)fi[f].status,
              (long long)fi[f].base, fi[f].i0, (double)fi[f].cfo_eps, (long long)fi[f].cfo_E);
  }
  if (!parts)   // run_batch widens every sc16 batch the streaming decode does not take
    return fail(MIMO_ERR_UNSUPPORTED, "no decode kernel takes this configuration");
  if (dprof) {   // diagnostics: per-item cycle split of the decode kernel
    unsigned long long v[8];
    HIPCHK(hipMemcpyAsync(v, h->sc_prof.p, sizeof(v), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    const double it = v[0] ? (double)v[0] : 1.0;
    fprintf(stderr, "dec_prof items %llu cycles/item load %.0f fft %.0f apply %.0f reduce %.0f "
            "| stream split: pass0 %.0f fetch %.0f subfft %.0f\n",
            v[0], v[1] / it, v[2] / it, v[3] / it, v[4] / it, v[5] / it, v[6] / it, v[7] / it);
  }
  EvmArgs ea{};
  ea.N = h->N; ea.max_out = max_out; ea.parts = parts; ea.info = h->info.p;
  ea.evm_part = h->evm_part.p;
  ea.rec_stride = d.rec_stride;
  ea.evm_out = h->evm_out.p;
  ea.chunk_part = h->evm_chunk.p;
  ea.counter = h->evm_cnt.p;
  ea.nrec = per_frame ? h->nrec.p : nullptr;
  // per workgroup segment (streaming, residue-class), not per chunk x range
  ea.few = (path == MIMO_DECODE_STREAM) ? 1 : 0;
  e = h->timer.begin(s);
  launch_evm(ea, F, s);
  h->timer.end(6, e, s);
  HIPCHK(hipGetLastError());
  return MIMO_OK;
}

}  // namespace

// ======================================================================================
// the error slot of this thread, for the other host translation units (ring.cpp)
int mimo::host_fail(int code, const char *msg) { return fail(code, msg); }

extern "C" {

const char *mimo_last_error(void) { return g_err.c_str(); }
const char *mimo_version(void) { return "rub_mimo_amd 0.1.0 (gfx950)"; }

static void close_debug_files(mimo_rx *h) {
  for (FILE *f : h->dbg_fsc)
    if (f) fclose(f);
  h->dbg_fsc.clear();
}

int mimo_rx_create(const mimo_rx_config *cfg, void *hip_stream, mimo_rx **out) {
  if (!cfg || !out || !cfg->p || !cfg->s0_bits || !cfg->s1_bits)
    return fail(MIMO_ERR_ARG, "mimo_rx_create: null argument");
  *out = nullptr;
  const int l2 = ilog2(cfg->M);
  if (l2 < 6 || l2 > 12) return fail(MIMO_ERR_UNSUPPORTED, "M must be a power of two in [64, 4096]");
  const uint32_t N = cfg->num_streams;
  if (!(N == 1 || N == 2 || N == 4 || N == 8))
    return fail(MIMO_ERR_UNSUPPORTED, "num_streams must be 1, 2, 4 or 8");
  if (cfg->cp_len == 0 || cfg->cp_len > cfg->M / 2)
    return fail(MIMO_ERR_ARG, "cp_len must be in [1, M/2]");
  if (cfg->num_access_codes == 0) return fail(MIMO_ERR_ARG, "num_access_codes must be > 0");
  if (cfg->detector < 0 || cfg->detector > 3) return fail(MIMO_ERR_ARG, "bad detector");
  if ((cfg->detector == MIMO_DET_ZF2) && N != 2)
    return fail(MIMO_ERR_ARG, "the reference invert() is 2x2 only (framing.cc:1346)");
  if (cfg->detector == MIMO_DET_SISO && (cfg->siso_tx >= N || cfg->siso_rx >= N))
    return fail(MIMO_ERR_ARG, "siso_tx/siso_rx out of range");
  const uint32_t q = cfg->qam_order;
  if (!(q == 4 || q == 16 || q == 64 || q == 256))
    return fail(MIMO_ERR_ARG, "qam_order must be 4, 16, 64 or 256");
  mimo_rx *h = new mimo_rx();
  h->M = cfg->M; h->cp = cfg->cp_len; h->SL = h->M + h->cp; h->N = N;
  h->nac = cfg->num_access_codes; h->pid = cfg->pid_max;
  h->log2M = l2;
  h->p.assign(cfg->p, cfg->p + h->M);
  int rc = validate_sctype(h->p.data(), h->M, &h->M_null, &h->M_pilot, &h->M_data);
  if (rc) { delete h; return rc; }
  h->M_occ = h->M_pilot + h->M_data;
  if (h->M_occ == 0) { delete h; return fail(MIMO_ERR_SCTYPE, "no occupied subcarriers"); }
  h->occ_index.resize(h->M);
  std::vector<int8_t> sign((size_t)N * h->nac * h->M);
  for (uint32_t i = 0, j = 0; i < h->M; i++) h->occ_index[i] = (h->p[i] != MIMO_SC_NULL) ? (int32_t)j++ : -1;
  for (uint32_t t = 0; t < N; t++)
    for (uint32_t c = 0; c < h->nac; c++)
      for (uint32_t i = 0; i < h->M; i++) {
        const size_t o = ((size_t)t * h->nac + c) * h->M + i;
        sign[o] = (h->p[i] == MIMO_SC_NULL) ? 0 : ((cfg->s1_bits[o] & 1) ? 1 : -1);
      }
  h->det = cfg->detector;
  h->noise_var = cfg->noise_var;
  h->keep_bias = cfg->keep_identity_bias ? 1 : 0;
  h->siso_tx = cfg->siso_tx; h->siso_rx = cfg->siso_rx;
  h->thr = cfg->plateau_threshold;
  h->cfo = cfg->cfo_correct != 0;
  h->qam = make_qam(q);
  h->acb = (uint64_t)h->SL * (h->nac * N + 4);     // framing.cc:284
  h->txl = (uint64_t)h->pid * h->SL;               // framing.cc:285
  h->win_len = h->acb + h->txl;
  h->dn = 1.0f / sqrtf((float)h->M_occ);           // framing.cc:330
  h->ls_scale = h->dn / (float)h->nac;             // framing.cc:821
  h->nv_norm = (h->nac >= 2) ? ((double)h->dn * (double)h->dn /
                                ((double)h->M_occ * N * N * (h->nac - 1)))
                             : 0.0;
  // search transform. Fused search + LS (search_ls_kernel): two slots per transform,
  // F >= 2 SL + M - 1, up to 16384. Otherwise F >= SL + M - 1 lags+taps, capped at 8192 (then
  // several lag chunks per slot) and a separate LS pass.
  uint32_t F = 1;
  while (F < 2 * h->SL + h->M - 1 || F < 2 * h->M) F <<= 1;
  h->search_ls = F <= 16384 && search_ls_supported(ilog2(F), ilog2(h->M));
  if (!h->search_ls) {
    F = 1;
    while (F < h->SL + h->M - 1) F <<= 1;
    if (F > 8192) F = 8192;
    if (F < 2 * h->M) F = 2 * h->M;
  }
  h->F = F; h->log2F = ilog2(F);
  h->lagc = F - h->M + 1;
  h->n_lagc = (h->SL + h->lagc - 1) / h->lagc;
  h->n_slots = N * h->nac + 1;
  if (hip_stream) {
    h->stream = (hipStream_t)hip_stream;
  } else {
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
      delete h;
      return fail(MIMO_ERR_HIP, "hipStreamCreate failed");
    }
    h->own_stream = true;
  }
  {
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        ncu > 0)
      h->n_cu = (uint32_t)ncu;
  }
  rc = get_twiddles(&h->tw);
  if (!rc) rc = build_codes(h->codes, h->M, N, h->nac, h->p.data(), cfg->s0_bits, cfg->s1_bits,
                            h->log2F, true, h->stream);
  if (rc) { mimo_rx_destroy(h); return rc; }
  uint32_t m_s0 = 0;
  for (uint32_t i = 0; i < h->M; i += 2) if (h->p[i] != MIMO_SC_NULL) m_s0++;
  std::vector<float> vs(h->n_slots);
  const double FF = (double)F * (double)F, MM = (double)h->M * (double)h->M;
  vs[0] = (float)((double)m_s0 / (MM * FF));
  for (uint32_t sl = 1; sl < h->n_slots; sl++) vs[sl] = (float)(1.0 / ((double)h->M * FF));
  if (h->M >= 512) {   // ls_window_kernel: thread lt's 8 subcarriers lt + (M/8) e adjacent
    const uint32_t T = h->M / 8;
    std::vector<int8_t> sw(sign.size());
    for (size_t row = 0; row < (size_t)N * h->nac; row++)
      for (uint32_t lt = 0; lt < T; lt++)
        for (uint32_t e = 0; e < 8; e++) sw[row * h->M + 8 * lt + e] = sign[row * h->M + lt + T * e];
    if (h->s1sign_w.ensure(sw.size()) != hipSuccess ||
        hipMemcpy(h->s1sign_w.p, sw.data(), sw.size(), hipMemcpyHostToDevice) != hipSuccess) {
      mimo_rx_destroy(h);
      return fail(MIMO_ERR_HIP, "table upload failed");
    }
  }
  if (h->vscale.ensure(h->n_slots) != hipSuccess || h->s1sign.ensure(sign.size()) != hipSuccess ||
      h->occ.ensure(h->M) != hipSuccess ||
      hipMemcpy(h->vscale.p, vs.data(), sizeof(float) * vs.size(), hipMemcpyHostToDevice) !=
          hipSuccess ||
      hipMemcpy(h->s1sign.p, sign.data(), sign.size(), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(h->occ.p, h->occ_index.data(), sizeof(int32_t) * h->M, hipMemcpyHostToDevice) !=
          hipSuccess) {
    mimo_rx_destroy(h);
    return fail(MIMO_ERR_HIP, "table upload failed");
  }
  *out = h;
  return MIMO_OK;
}

int mimo_rx_destroy(mimo_rx *h) {
  if (!h) return MIMO_OK;
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  close_debug_files(h);
  for (auto &e : h->timer.ev) {
    (void)hipEventDestroy(e.second.first);
    (void)hipEventDestroy(e.second.second);
  }
  for (auto &g : h->graphs)
    if (g.exec) (void)hipGraphExecDestroy(g.exec);
  if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
  return MIMO_OK;
}

int mimo_rx_set_callback(mimo_rx *h, mimo_rx_symbol_cb cb, void *user) {
  if (!h) return fail(MIMO_ERR_ARG, "null handle");
  h->cb = cb;
  h->user = user;
  return MIMO_OK;
}

// A captured batch graph bakes every host scalar of the launch arguments (siso indices,
// detector, noise variance, threshold) into its kernel nodes: any setter of such a scalar
// drops the graph so the next batch is launched (and later re-captured) with the new value.
static void drop_graph(mimo_rx *h, mimo_rx::GraphEntry &g) {
  if (g.exec) {   // a replay may still be in flight on its stream
    (void)hipStreamSynchronize(g.stream ? g.stream : h->stream);
    (void)hipGraphExecDestroy(g.exec);
  }
  g = mimo_rx::GraphEntry{};
}

static void invalidate_graph(mimo_rx *h) {
  for (auto &g : h->graphs) drop_graph(h, g);
}

int mimo_rx_set_siso(mimo_rx *h, uint32_t tx, uint32_t rx) {
  if (!h || tx >= h->N || rx >= h->N) return fail(MIMO_ERR_ARG, "siso index out of range");
  if (tx != h->siso_tx || rx != h->siso_rx) invalidate_graph(h);
  h->siso_tx = tx;
  h->siso_rx = rx;
  return MIMO_OK;
}

// ---------------- streaming framesync::execute ----------------
static int grow_capture(mimo_rx *h, uint64_t need) {
  if (need <= h->cap_len && h->capbuf.p) return MIMO_OK;
  // 1.5x growth in 16 K steps (the streaming capture is trimmed while seeking, so its size
  // follows what is held plus one piece, not the stream length)
  uint64_t nc = std::max<uint64_t>(need, h->cap_len + h->cap_len / 2);
  nc = std::max<uint64_t>((nc + 16383) / 16384 * 16384, 1 << 16);
  float2 *np = nullptr;
  HIPCHK(hipMalloc(&np, sizeof(float2) * nc * h->N));
  if (h->capbuf.p && h->total) {
    HIPCHK(hipMemcpy2DAsync(np, sizeof(float2) * nc, h->capbuf.p, sizeof(float2) * h->cap_len,
                            sizeof(float2) * h->total, h->N, hipMemcpyDeviceToDevice, h->stream));
  }
  HIPCHK(hipStreamSynchronize(h->stream));
  h->capbuf.release();
  h->capbuf.p = np;
  h->capbuf.n = nc * h->N;
  h->cap_len = nc;
  return MIMO_OK;
}

// DEBUG_LOG: the search metric of every lag as the reference's corr_<rx>_<ac>.dat files, one
// float per window index over [0, ACB - M): S0's lags at [0, SL) (corr_<rx>_0), access code
// ac's at SL (ac + 1) + [0, SL) (framing.cc:716-737), zeros elsewhere
static int write_corr_logs(mimo_rx *h) {
  const size_t per = (size_t)h->n_slots * h->SL;
  std::vector<float> tr((size_t)h->N * per);
  HIPCHK(hipMemcpy(tr.data(), h->dbg_corr.p, sizeof(float) * tr.size(), hipMemcpyDeviceToHost));
  const size_t len = h->acb - h->M;
  std::vector<float> out(len);
  for (uint32_t ch = 0; ch < h->N; ch++)
    for (uint32_t slot = 0; slot < h->n_slots; slot++) {
      std::fill(out.begin(), out.end(), 0.0f);
      const size_t at = (size_t)h->SL * slot;
      for (uint32_t i = 0; i < h->SL && at + i < len; i++) out[at + i] = tr[ch * per + (size_t)slot * h->SL + i];
      const std::string fn = h->dbg_dir + "/corr_" + std::to_string(ch + 1) + "_" +
                             std::to_string(slot) + ".dat";
      FILE *fp = fopen(fn.c_str(), "wb");
      if (!fp) return fail(MIMO_ERR_ARG, "cannot open " + fn);
      const size_t w = fwrite(out.data(), sizeof(float), len, fp);
      fclose(fp);
      if (w != len) return fail(MIMO_ERR_ARG, "short write " + fn);
    }
  return MIMO_OK;
}

static int finish_estimate(mimo_rx *h) {
  // channel estimate + replay decode of the complete window; callbacks per OFDM symbol
  const float2 *iq = h->capbuf.p;
  // the window is complete: the device frame record says so (the plateau kernel saw it
  // incomplete when the trigger fired)
  h->sinfo.status = MIMO_FRAME_OK;
  HIPCHK(hipMemcpyAsync(h->info.p, &h->sinfo, sizeof(FrameInfo), hipMemcpyHostToDevice,
                        h->stream));
  if (!h->dbg_dir.empty()) {
    HIPCHK(h->dbg_corr.ensure((size_t)h->N * h->n_slots * h->SL));
    HIPCHK(hipMemsetAsync(h->dbg_corr.p, 0, sizeof(float) * h->N * h->n_slots * h->SL, h->stream));
    h->cur_corr_trace = h->dbg_corr.p;
  }
  int rc = run_estimate(h, iq, h->cap_len, 1, h->total, h->stream);
  h->cur_corr_trace = nullptr;
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(&h->sinfo, h->info.p, sizeof(FrameInfo), hipMemcpyDeviceToHost,
                        h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  if (!h->dbg_dir.empty() && (rc = write_corr_logs(h))) return rc;
  const uint32_t n_sym = h->sinfo.n_sym;
  const size_t per = (size_t)h->N * h->M_occ;
  if (n_sym) {
    HIPCHK(h->symbuf.ensure(per * n_sym));
    h->cur_layout = MIMO_LAYOUT_STREAM_MAJOR;        // symbuf is [N][n_sym][M_occ]
    rc = run_decode(h, iq, h->cap_len, 1, h->total, n_sym, h->symbuf.p, nullptr, 0, nullptr, 0,
                    0, h->stream);
    if (rc) return rc;
    h->symhost.resize(per * n_sym);
    HIPCHK(hipMemcpyAsync(h->symhost.data(), h->symbuf.p, sizeof(float2) * per * n_sym,
                          hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
  } else {
    h->symhost.clear();
  }
  h->have_est = true;
  h->last_frames = 1;
  h->last_max_out = n_sym;
  if (h->cb) {
    std::vector<const float *> ptr(h->N);
    for (uint32_t s = 0; s < n_sym; s++) {
      for (uint32_t t = 0; t < h->N; t++)
        ptr[t] = reinterpret_cast<const float *>(h->symhost.data() +
                                                 ((size_t)t * n_sym + s) * h->M_occ);
      h->cb(ptr.data(), h->N, h->M_occ, h->user);
    }
  }
  return MIMO_OK;
}

// Bounded streaming memory. The reference holds a window ring of ACB + TX samples
// (framing.cc:387-388, 639-651) and constant-size S&C filter state, so an unsynchronised stream
// costs it nothing. Here the device capture keeps, while seeking, only what a later trigger can
// still reach: the S&C history of the next chunk's work item (its halo and M samples of
// filter history) and, in front of it, room for a plateau run and the window's leading SL.
// Samples before a drop point D (a multiple of the chunk length, so the chunk grid stays
// aligned) are dropped only when every antenna has a proven metric zero (y <= threshold in
// the oracle's fp32, certified in fp64 with the decision band) in [D + SL + M, next item): no
// plateau run then reaches back past it, so every run start, sync index and window start of
// a later trigger lie inside the kept samples. A run that never ends (pathological input)
// postpones the drop and the capture grows, as before.
__global__ void trim_probe_kernel(const float2 *x, uint64_t stride, uint32_t M, int64_t lo,
                                  int64_t hi, double thr, double band, uint32_t *ok) {
  const uint32_t s = blockIdx.x, lane = threadIdx.x;
  const float2 *r = x + (uint64_t)s * stride;
  const int64_t span = hi - lo;
  bool zero = false;
  if (span > 0) {
    const int64_t q = hi - 1 - (span * (int64_t)lane) / 64;   // 64 positions spread over [lo, hi)
    double pr = 0.0, pi = 0.0, z = 0.0;
    const int64_t h = M / 2;
    for (int64_t k = q - (int64_t)M + 1; k <= q; k++) {
      const float2 v = r[k];
      z += (double)v.x * v.x + (double)v.y * v.y;
      if (k > q - h) {
        const float2 d = r[k - h];
        pr += (double)d.x * v.x + (double)d.y * v.y;
        pi += (double)d.x * v.y - (double)d.y * v.x;
      }
    }
    const double R = 0.5 * z;
    // the fp64 metric clears the threshold by more than the fp32 error band: the oracle's y
    // is not above the threshold either
    // an all-zero window (R = 0, so P = 0: an idle radio or zero padding) is the oracle's 0/0,
    // which compares false: not above the threshold either
    zero = R == 0.0 || pr * pr + pi * pi < (thr - band) * R * R;
  }
  const unsigned long long b = __ballot(zero);
  if (lane == 0) ok[s] = b ? 1u : 0u;
}

static int maybe_trim(mimo_rx *h) {
  const uint64_t K = sc_chunk_len(h->cp);
  const uint64_t H = kScSpan - K;                     // halo of an S&C item
  const uint64_t c_lo = h->total / K;                 // the next S&C starts at this chunk
  const uint64_t need = H + 2 * (uint64_t)h->SL + 2 * (uint64_t)h->M + K;
  if (c_lo * K < need + K) return MIMO_OK;            // nothing to drop yet
  const uint64_t D = (c_lo * K - need) / K * K;
  // high-water mark: only once the droppable prefix reaches half a window (pieces are half a
  // window too), so a probe and its host round trip come once per half window of stream, not
  // once per S&C chunk, and the capture stays within about a window plus the S&C reach
  if (D < std::max<uint64_t>(K, h->win_len / 2)) return MIMO_OK;
  const int64_t lo = (int64_t)(D + h->SL + h->M), hi = (int64_t)(c_lo * K - H);
  if (hi - lo < (int64_t)K / 2) return MIMO_OK;
  // the probe's span moves only when the S&C reaches a new chunk: a caller feeding small pieces
  // pays one probe (and its host round trip) per chunk of stream, not one per call. (The stream
  // position of that chunk, not its capture-relative index: a trim re-bases the capture.)
  const uint64_t c_abs = h->origin + c_lo * K;
  if (c_abs == h->trim_clo) return MIMO_OK;
  h->trim_clo = c_abs;
  HIPCHK(h->probe.ensure(h->N));
  hipLaunchKernelGGL(trim_probe_kernel, dim3(h->N), dim3(64), 0, h->stream, h->capbuf.p,
                     h->cap_len, h->M, lo, hi, h->thr, sc_band(h->M), h->probe.p);
  HIPCHK(hipGetLastError());
  std::vector<uint32_t> ok(h->N);
  HIPCHK(hipMemcpyAsync(ok.data(), h->probe.p, sizeof(uint32_t) * h->N, hipMemcpyDeviceToHost,
                        h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  for (uint32_t a = 0; a < h->N; a++)
    if (!ok[a]) return MIMO_OK;                       // a run may reach back: keep everything
  // move [D, total) to the front in pieces of D samples (each piece's source is read before
  // any later piece writes over it: copies on one stream run in order; one piece when D >= keep)
  const uint64_t keep = h->total - D;
  for (uint64_t o = 0; o < keep; o += D) {
    const uint64_t m = std::min<uint64_t>(D, keep - o);
    HIPCHK(hipMemcpy2DAsync(h->capbuf.p + o, sizeof(float2) * h->cap_len,
                            h->capbuf.p + D + o, sizeof(float2) * h->cap_len,
                            sizeof(float2) * m, h->N, hipMemcpyDeviceToDevice, h->stream));
  }
  h->origin += D;
  h->total = keep;
  return MIMO_OK;
}

// At the trigger: nothing before the window start (base) is read again -- the S&C is done and
// the search, LS and decode read [base, base + ACB + TX) -- so the capture is re-based there
// into a buffer sized for the window (positions of the frame record shift with it).
static int rebase_to_window(mimo_rx *h, uint64_t piece) {
  const int64_t D = h->sinfo.base;
  if (D <= 0) return MIMO_OK;
  const uint64_t keep = h->total - (uint64_t)D;
  uint64_t nc = std::max<uint64_t>(keep, h->win_len + piece + 64);
  nc = (nc + 16383) / 16384 * 16384;
  float2 *np = nullptr;
  HIPCHK(hipMalloc(&np, sizeof(float2) * nc * h->N));
  if (keep)
    HIPCHK(hipMemcpy2DAsync(np, sizeof(float2) * nc, h->capbuf.p + D, sizeof(float2) * h->cap_len,
                            sizeof(float2) * keep, h->N, hipMemcpyDeviceToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  h->capbuf.release();
  h->capbuf.p = np;
  h->capbuf.n = nc * h->N;
  h->cap_len = nc;
  h->origin += (uint64_t)D;
  h->total = keep;
  FrameInfo &I = h->sinfo;   // (unsigned fields wrap consistently: getters add origin back)
  I.base -= D;
  I.trigger -= (uint64_t)D;
  I.sync_index -= (uint64_t)D;
  for (uint32_t a = 0; a < h->N; a++) {
    I.plateau_start[a] -= (uint64_t)D;
    I.plateau_end[a] -= (uint64_t)D;
  }
  return MIMO_OK;
}

// one piece of an execute call (at most a window's worth of samples)
static int execute_piece(mimo_rx *h, const float *const *iq, uint64_t off, uint64_t n,
                         uint64_t call_end, uint64_t piece) {
  if (h->state == MIMO_STATE_SEEK_PLATEAU && h->total) {
    int rc = maybe_trim(h);
    if (rc) return rc;
  }
  const uint64_t old_total = h->total;
  int rc = grow_capture(h, old_total + n);
  if (rc) return rc;
  for (uint32_t s = 0; s < h->N; s++)
    HIPCHK(hipMemcpyAsync(h->capbuf.p + (size_t)s * h->cap_len + old_total,
                          reinterpret_cast<const float2 *>(iq[s]) + off, sizeof(float2) * n,
                          hipMemcpyHostToDevice, h->stream));
  h->total = old_total + n;
  if (h->state == MIMO_STATE_SEEK_PLATEAU) {
    const uint64_t K = sc_chunk_len(h->cp);
    rc = ensure_workspace(h, 1, (h->total + K - 1) / K, 0);
    if (rc) return rc;
    if (old_total == 0 && h->origin == 0)
      HIPCHK(hipMemsetAsync(h->trig.p, 0xFF, sizeof(unsigned long long), h->stream));
    // re-run the partially filled chunk; earlier chunks are final (y[n] uses x[<=n] only)
    rc = run_sync(h, h->capbuf.p, h->cap_len, 1, h->total, old_total / K, false, h->stream);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(&h->sinfo, h->info.p, sizeof(FrameInfo), hipMemcpyDeviceToHost,
                          h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    if (!h->dbg_fsc.empty()) {
      // DEBUG_LOG: y of every sample this piece processed while seeking, through the trigger
      const uint64_t hi = h->sinfo.status == MIMO_FRAME_NO_SYNC ? h->total : h->sinfo.trigger + 1;
      if (hi > old_total) {
        const uint64_t cnt = hi - old_total;
        HIPCHK(h->dbg_y.ensure(cnt * h->N));
        launch_sc_trace(h->capbuf.p, h->cap_len, h->N, h->M, (int64_t)old_total, (int64_t)hi,
                        h->dbg_y.p, h->stream);
        HIPCHK(hipGetLastError());
        std::vector<float> y(cnt * h->N);
        HIPCHK(hipMemcpyAsync(y.data(), h->dbg_y.p, sizeof(float) * y.size(),
                              hipMemcpyDeviceToHost, h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
        for (uint32_t a = 0; a < h->N; a++)
          if (fwrite(y.data() + (size_t)a * cnt, sizeof(float), cnt, h->dbg_fsc[a]) != cnt)
            return fail(MIMO_ERR_ARG, "short write of an f_sc debug file");
      }
    }
    if (h->sinfo.status == MIMO_FRAME_NO_SYNC) {
      h->nsp = h->origin + h->total;
      return MIMO_OK;
    }
    h->have_sync = true;
    h->state = MIMO_STATE_SAVE_ACCESS_CODES;
    rc = rebase_to_window(h, piece);
    if (rc) return rc;
  }
  // SAVE_ACCESS_CODES (framing.cc:639-651): estimate_channel runs at window sample n_e =
  // base + ACB + TX; a call that continues past it consumes one more sample in STATE_MIMO
  // (framing.cc:494-503)
  const uint64_t n_e = (uint64_t)h->sinfo.base + h->win_len;   // capture-relative
  if (n_e < h->total) {
    h->nsp = h->origin + n_e + ((h->origin + n_e + 1 < call_end) ? 2 : 1);
    rc = finish_estimate(h);
    if (rc) return rc;
    h->state = MIMO_STATE_MIMO;
  } else {
    h->nsp = h->origin + h->total;
  }
  return MIMO_OK;
}

int mimo_rx_execute(mimo_rx *h, const float *const *iq, uint32_t n_ant, uint64_t n,
                    int32_t *state_out) {
  if (!h || (!iq && n)) return fail(MIMO_ERR_ARG, "null argument");
  if (n_ant != h->N) return fail(MIMO_ERR_ARG, "n_ant must equal num_streams");
  if (h->state == MIMO_STATE_MIMO) {   // framing.cc:494-503: consume one sample and break
    if (n) h->nsp += 1;
    if (state_out) *state_out = h->state;
    return MIMO_OK;
  }
  // long calls are taken a window at a time, so the capture stays bounded whatever the
  // caller's chunking (results are those of one call: the S&C is chunk-exact)
  const uint64_t call_end = h->origin + h->total + n;
  const uint64_t piece = std::max<uint64_t>(h->win_len / 2, 2 * sc_chunk_len(h->cp));
  for (uint64_t off = 0; off < n && h->state != MIMO_STATE_MIMO; off += piece) {
    const int rc = execute_piece(h, iq, off, std::min<uint64_t>(piece, n - off), call_end, piece);
    if (rc) return rc;
  }
  if (state_out) *state_out = h->state;
  return MIMO_OK;
}

int mimo_rx_reset(mimo_rx *h) {
  // framing.cc:461-464 only rewinds the state; here the receiver re-arms on a fresh capture
  // (documented deviation: the reference keeps stale S&C filter history and accumulates
  // sync_index across resets).
  if (!h) return fail(MIMO_ERR_ARG, "null handle");
  HIPCHK(hipStreamSynchronize(h->stream));
  h->state = MIMO_STATE_SEEK_PLATEAU;
  h->total = 0;
  h->origin = 0;
  h->trim_clo = ~0ull;
  h->nsp = 0;
  h->have_sync = false;
  h->have_est = false;
  return MIMO_OK;
}

int mimo_rx_get_state(const mimo_rx *h, int32_t *st) {
  if (!h || !st) return fail(MIMO_ERR_ARG, "null argument");
  *st = h->state;
  return MIMO_OK;
}

int mimo_rx_get_sync_index(const mimo_rx *h, uint64_t *out) {
  if (!h || !out) return fail(MIMO_ERR_ARG, "null argument");
  *out = h->have_sync ? h->origin + h->sinfo.sync_index : 0;
  return MIMO_OK;
}

int mimo_rx_get_num_samples_processed(const mimo_rx *h, uint64_t *out) {
  if (!h || !out) return fail(MIMO_ERR_ARG, "null argument");
  *out = h->nsp;
  return MIMO_OK;
}

int mimo_rx_get_plateau(const mimo_rx *h, uint32_t s, uint64_t *start, uint64_t *end) {
  if (!h || s >= h->N) return fail(MIMO_ERR_ARG, "bad stream");
  if (start) *start = h->have_sync ? h->origin + h->sinfo.plateau_start[s] : 0;
  if (end) *end = h->have_sync ? h->origin + h->sinfo.plateau_end[s] : 0;
  return MIMO_OK;
}

int mimo_rx_get_m_occ(const mimo_rx *h, uint32_t *m) {
  if (!h || !m) return fail(MIMO_ERR_ARG, "null argument");
  *m = h->M_occ;
  return MIMO_OK;
}

int mimo_rx_get_G(mimo_rx *h, float *G) {
  if (!h || !G) return fail(MIMO_ERR_ARG, "null argument");
  const size_t n = (size_t)h->M * h->N * h->N;
  if (!h->have_est) {   // framing.cc:302-319 identity on occupied carriers
    std::memset(G, 0, sizeof(float2) * n);
    for (uint32_t k = 0; k < h->M; k++)
      if (h->p[k] != MIMO_SC_NULL)
        for (uint32_t r = 0; r < h->N; r++) G[2 * ((k * h->N + r) * h->N + r)] = 1.0f;
    return MIMO_OK;
  }
  HIPCHK(hipMemcpy(G, h->G.p, sizeof(float2) * n, hipMemcpyDeviceToHost));
  return MIMO_OK;
}

static int copy_W(mimo_rx *h, uint32_t f, float *W) {
  const size_t n = (size_t)h->M * h->N * h->N;
  std::vector<float2> tmp(n);
  HIPCHK(hipMemcpy(tmp.data(), h->W.p + (size_t)f * n, sizeof(float2) * n,
                   hipMemcpyDeviceToHost));
  float2 *o = reinterpret_cast<float2 *>(W);
  for (uint32_t t = 0; t < h->N; t++)
    for (uint32_t r = 0; r < h->N; r++)
      for (uint32_t k = 0; k < h->M; k++)
        o[((size_t)k * h->N + t) * h->N + r] = tmp[((size_t)t * h->N + r) * h->M + k];
  return MIMO_OK;
}

int mimo_rx_get_W(mimo_rx *h, float *W) {
  if (!h || !W) return fail(MIMO_ERR_ARG, "null argument");
  if (!h->have_est) return mimo_rx_get_G(h, W);  // W also starts as identity
  return copy_W(h, 0, W);
}

int mimo_rx_get_gain(mimo_rx *h, float *gain) {
  if (!h || !gain) return fail(MIMO_ERR_ARG, "null argument");
  if (!h->have_est) {
    for (uint32_t j = 0; j < h->M_occ; j++) gain[j] = 1.0f;
    return MIMO_OK;
  }
  std::vector<float> tmp(h->M);
  HIPCHK(hipMemcpy(tmp.data(), h->gain.p, sizeof(float) * h->M, hipMemcpyDeviceToHost));
  for (uint32_t k = 0; k < h->M; k++)
    if (h->occ_index[k] >= 0) gain[h->occ_index[k]] = tmp[k];
  return MIMO_OK;
}

int mimo_rx_get_noise_var(mimo_rx *h, float *out) {
  if (!h || !out) return fail(MIMO_ERR_ARG, "null argument");
  *out = h->have_est ? h->sinfo.noise_var : h->noise_var;
  return MIMO_OK;
}

static int copy_corr(mimo_rx *h, uint32_t F, uint32_t *corr, uint32_t *s0) {
  std::vector<unsigned long long> k((size_t)F * h->N * h->n_slots);
  HIPCHK(hipMemcpy(k.data(), h->keys.p, sizeof(unsigned long long) * k.size(),
                   hipMemcpyDeviceToHost));
  auto idx = [](unsigned long long v) -> uint32_t {
    return v ? (0xFFFFFFFFu - (uint32_t)(v & 0xFFFFFFFFull)) : 0u;
  };
  for (uint32_t f = 0; f < F; f++)
    for (uint32_t r = 0; r < h->N; r++) {
      const unsigned long long *kk = k.data() + ((size_t)f * h->N + r) * h->n_slots;
      if (s0) s0[f * h->N + r] = idx(kk[0]);
      if (corr)
        for (uint32_t ac = 0; ac + 1 < h->n_slots; ac++)
          corr[((size_t)f * h->N + r) * (h->n_slots - 1) + ac] = idx(kk[1 + ac]);
    }
  return MIMO_OK;
}

int mimo_rx_get_corr(mimo_rx *h, uint32_t *corr, uint32_t *s0) {
  if (!h) return fail(MIMO_ERR_ARG, "null handle");
  if (!h->have_est) {
    if (corr) std::memset(corr, 0, sizeof(uint32_t) * h->N * (h->n_slots - 1));
    if (s0) std::memset(s0, 0, sizeof(uint32_t) * h->N);
    return MIMO_OK;
  }
  return copy_corr(h, 1, corr, s0);
}

// ---------------- batched device frames ----------------
static uint32_t batch_fpc(const mimo_batch *b) {
  return b->frames_per_capture > 1 ? b->frames_per_capture : 1u;
}

// The opt-in CFO folds into the loads (no scratch passes) where the fused search + LS (wave
// form) and the streaming decode's CPE variant run: fc32 input (read in place or widened),
// reference indices from HBM, both or neither output. Elsewhere the scratch passes remain.
static bool cfo_folds(const mimo_rx *h, const mimo_batch *b, bool widened) {
  if (!h->cfo || !h->search_ls) return false;
  if (b->sample_format == MIMO_SAMPLE_SC16 && !widened) return false;
  if (b->ref_mode != 1 || (!b->d_out_sym) != (!b->d_out_idx)) return false;
  DecodeArgs probe{};
  probe.N = h->N; probe.detector = h->det;
  probe.all_occ = (h->M_occ == h->M) ? 1 : 0;
  probe.n_caps = b->n_frames; probe.n_refs = b->n_frames * batch_fpc(b); probe.qam = h->qam;
  probe.ref_mode = b->ref_mode; probe.ref_idx = reinterpret_cast<const uint8_t *>(b->d_ref_idx);
  probe.stride = b->stride; probe.max_out = b->max_out_syms; probe.M_occ = h->M_occ;
  probe.out_sym = reinterpret_cast<float2 *>(b->d_out_sym);
  probe.out_idx = reinterpret_cast<uint8_t *>(b->d_out_idx);
  return decode_stream_accepts(probe, h->log2M, b->n_frames * batch_fpc(b));
}

static int run_batch(mimo_rx *h, const mimo_batch *b, hipStream_t s) {
  const float2 *iq = reinterpret_cast<const float2 *>(b->d_iq);
  const uint32_t fpc = batch_fpc(b), slots = b->n_frames * fpc;
  h->cur_sc16 = 0;
  h->cur_scale = 1.0f;
  h->cur_layout = b->out_layout;
  if (b->sample_format == MIMO_SAMPLE_SC16) {
    // sc16 wire input: read in place by S&C, the fused search + LS and the streaming decode
    // where the configuration takes them; otherwise widened once into an internal fc32 batch
    DecodeArgs probe{};
    probe.N = h->N; probe.detector = h->det;
    probe.all_occ = (h->M_occ == h->M) ? 1 : 0;
    probe.n_caps = b->n_frames; probe.n_refs = slots; probe.qam = h->qam;
    probe.ref_mode = b->ref_mode; probe.ref_idx = reinterpret_cast<const uint8_t *>(b->d_ref_idx);
    probe.stride = b->stride; probe.max_out = b->max_out_syms; probe.M_occ = h->M_occ;
    probe.out_sym = reinterpret_cast<float2 *>(b->d_out_sym);
    probe.out_idx = reinterpret_cast<uint8_t *>(b->d_out_idx);
    probe.sc16 = 1;
    const bool fused = sc_screen_ok(h->M) && h->search_ls && !h->cfo &&
                       (decode_stream_accepts(probe, h->log2M, slots) ||
                        decode_split_accepts(probe, h->log2M));
    if (fused) {
      h->cur_sc16 = 1;
      h->cur_scale = b->sc16_scale;
    } else if (b->stages != MIMO_STAGES_DECODE) {
      const size_t need = (size_t)b->n_frames * h->N * b->stride;
      if (h->wide.ensure(need) != hipSuccess) return fail(MIMO_ERR_NOMEM, "sc16 widening buffer");
      hipEvent_t e = h->timer.begin(s);
      const bool ok = launch_sc16_to_fc32(b->d_iq, b->stride, h->wide.p, b->stride,
                                          b->n_frames * h->N, b->frame_len, b->sc16_scale, s);
      h->timer.end(0, e, s);     // timed with the S&C stage (one extra launch)
      if (!ok) return fail(MIMO_ERR_ARG, "sc16 widening: bad geometry");
      iq = h->wide.p;
    } else {
      iq = h->wide.p;            // (widened by this batch's front half)
    }
  } else if (b->sample_format != MIMO_SAMPLE_FC32) {
    return fail(MIMO_ERR_ARG, "mimo_batch.sample_format must be MIMO_SAMPLE_FC32 or _SC16");
  }
  const bool front = b->stages != MIMO_STAGES_DECODE, decode = b->stages != MIMO_STAGES_FRONT;
  if (!front) {   // the decode half of a batch whose front half this handle ran last
    const int rc = run_decode(h, iq, b->stride, slots, b->frame_len, b->max_out_syms,
                              reinterpret_cast<float2 *>(b->d_out_sym),
                              reinterpret_cast<uint8_t *>(b->d_out_idx), b->ref_mode,
                              reinterpret_cast<const uint8_t *>(b->d_ref_idx), b->ref_seed,
                              b->frame_id0, s, b->n_frames, nullptr);
    h->cur_sc16 = 0;
    h->cur_scale = 1.0f;
    h->cur_layout = 0;
    return rc;
  }
  int rc = run_sync(h, iq, b->stride, b->n_frames, b->frame_len, 0, true, s, fpc,
                    fpc > 1 ? b->d_ref_starts : nullptr, b->ref_stride, true);
  CfoBatchArgs ca{};
  const bool fold = cfo_folds(h, b, iq != reinterpret_cast<const float2 *>(b->d_iq));
  if (!rc && fold) {
    // opt-in CFO, folded: estimates only (stage 1 here, stage 2 after the search); the
    // search + LS loads and the decode derotate by them, no scratch capture
    if (h->cfo_eps.ensure(cfo_batch_part_doubles(slots)) != hipSuccess)
      return fail(MIMO_ERR_NOMEM, "cfo estimate allocation failed");
    ca.iq = iq; ca.out = nullptr; ca.stride = b->stride; ca.frame_len = b->frame_len;
    ca.len = h->win_len + 64; ca.win = h->win_len; ca.N = h->N; ca.M = h->M; ca.cp = h->cp; ca.SL = h->SL;
    ca.n_codes = h->N * h->nac; ca.n_data = h->pid + 2; ca.info = h->info.p;
    ca.part = h->cfo_eps.p;
    ca.fold = 1;
    launch_cfo_batch(ca, slots, 1, s);
  } else if (!rc && h->cfo) {
    // opt-in CFO, stage 1: coarse estimate per synced frame at its trigger, window derotated
    // into a scratch capture that search, LS, weights and decode read (S&C ran on the raw
    // samples: |P| and R do not depend on a frequency offset)
    const size_t need = (size_t)b->n_frames * h->N * b->stride;
    if (h->cfo_iq.ensure(need) != hipSuccess ||
        h->cfo_eps.ensure(cfo_batch_part_doubles(slots)) != hipSuccess)
      return fail(MIMO_ERR_NOMEM, "cfo scratch allocation failed");
    ca.iq = iq; ca.out = h->cfo_iq.p; ca.stride = b->stride; ca.frame_len = b->frame_len;
    ca.len = h->win_len + 64; ca.win = h->win_len; ca.N = h->N; ca.M = h->M; ca.cp = h->cp; ca.SL = h->SL;
    ca.n_codes = h->N * h->nac; ca.n_data = h->pid + 2; ca.info = h->info.p;
    ca.part = h->cfo_eps.p;
    launch_cfo_batch(ca, slots, 1, s);
    iq = h->cfo_iq.p;
  }
  if (!rc) rc = run_estimate(h, iq, b->stride, slots, b->frame_len, s, true,
                             h->cfo ? &ca : nullptr);
  if (!rc && h->cfo && !fold && h->search_ls)   // stage 2's data-region derotation
    launch_cfo_batch_rot2(ca, slots, s);
  if (!rc && decode)
    rc = run_decode(h, iq, b->stride, slots, b->frame_len, b->max_out_syms,
                    reinterpret_cast<float2 *>(b->d_out_sym),
                    reinterpret_cast<uint8_t *>(b->d_out_idx), b->ref_mode,
                    reinterpret_cast<const uint8_t *>(b->d_ref_idx), b->ref_seed, b->frame_id0,
                    s, b->n_frames, fold ? ca.part : nullptr);
  h->cur_sc16 = 0;
  h->cur_scale = 1.0f;
  h->cur_layout = 0;
  return rc;
}

// The whole batch (14 launches and memsets) is captured into a HIP graph once a call repeats
// the previous call's arguments, and replayed from then on: the grid shapes depend only on
// the configuration and F (S&C items and hot items are pulled from device-side queues), so
// the graph stays valid. Not used while stage timing or a diagnostic counter is on.
// every device pointer a captured batch bakes into its kernels' arguments
static std::array<const void *, 27> ws_signature(const mimo_rx *h) {
  return {h->trig.p, h->keys.p, h->rec.p, h->info.p, h->G.p, h->W.p, h->gain.p, h->nvp.p,
          h->evm_part.p, h->evm_out.p, h->n_exact.p, h->queue.p, h->hot.p, h->lspart.p,
          h->tw, h->codes.codespec.p, h->scr_flag.p, h->scr_min.p, h->scr_max.p, h->nrec.p,
          h->cand.p, h->certfail.p, h->lsq.p, h->cfo_iq.p, h->cfo_eps.p, h->wide.p,
          h->spec.p};
}

static bool same_batch(const mimo_batch &x, const mimo_batch &y) {
  return x.d_iq == y.d_iq && x.stride == y.stride && x.frame_len == y.frame_len &&
         x.n_frames == y.n_frames && x.max_out_syms == y.max_out_syms &&
         x.d_out_sym == y.d_out_sym && x.d_out_idx == y.d_out_idx && x.ref_mode == y.ref_mode &&
         x.d_ref_idx == y.d_ref_idx && x.ref_seed == y.ref_seed && x.frame_id0 == y.frame_id0 &&
         batch_fpc(&x) == batch_fpc(&y) && x.d_ref_starts == y.d_ref_starts &&
         x.ref_stride == y.ref_stride && x.sample_format == y.sample_format &&
         x.sc16_scale == y.sc16_scale && x.out_layout == y.out_layout && x.stages == y.stages;
}

int mimo_rx_process_batch(mimo_rx *h, const mimo_batch *b, void *hip_stream) {
  if (!h || !b || !b->d_iq) return fail(MIMO_ERR_ARG, "null argument");
  if (b->n_frames == 0) return MIMO_OK;
  if (b->stride < b->frame_len) return fail(MIMO_ERR_ARG, "stride < frame_len");
  if (b->ref_mode == 1 && !b->d_ref_idx) return fail(MIMO_ERR_ARG, "ref_mode 1 needs d_ref_idx");
  if (b->out_layout != MIMO_LAYOUT_STREAM_MAJOR && b->out_layout != MIMO_LAYOUT_SYMBOL_MAJOR)
    return fail(MIMO_ERR_ARG, "mimo_batch.out_layout must be MIMO_LAYOUT_STREAM_MAJOR or _SYMBOL_MAJOR");
  if (batch_fpc(b) > 64)
    return fail(MIMO_ERR_ARG, "frames_per_capture must be at most 64");
  if (b->stages > MIMO_STAGES_DECODE) return fail(MIMO_ERR_ARG, "mimo_batch.stages must be 0, 1 or 2");
  if (b->stages != MIMO_STAGES_ALL && h->cfo)
    return fail(MIMO_ERR_UNSUPPORTED, "split stages with cfo_correct");
  // the unfolded CFO stages derotate each frame's window into one scratch capture per
  // capture: back-to-back frames' windows overlap there, so that combination is refused (the
  // folded form has no scratch)
  if (h->cfo && batch_fpc(b) > 1 && !cfo_folds(h, b, b->sample_format == MIMO_SAMPLE_SC16))
    return fail(MIMO_ERR_UNSUPPORTED, "cfo_correct with frames_per_capture > 1 needs the folded "
                                      "CFO path (fc32 C2/C3-type geometry, ref_mode 1)");
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : h->stream;
  static const bool no_graph = [] {
    const char *e = getenv("RMIMO_NO_GRAPH");
    const char *p1 = getenv("RMIMO_SC_PROF");
    const char *p2 = getenv("RMIMO_DEC_PROF");
    return (e && e[0] == '1') || (p1 && p1[0] == '1') || (p2 && p2[0] == '1');
  }();
  // the cache entry of this batch: same arguments, stream and workspace pointers
  const auto sig = ws_signature(h);
  mimo_rx::GraphEntry *hit = nullptr;
  for (auto &g : h->graphs)
    if (g.used && same_batch(g.key, *b) && g.stream == s && g.sig == sig) hit = &g;
  int rc = MIMO_OK;
  if (no_graph || h->timer.on) {
    rc = run_batch(h, b, s);
  } else if (hit && hit->exec) {
    hit->used = ++h->graph_tick;
    HIPCHK(hipGraphLaunch(hit->exec, s));
  } else if (hit) {
    // second identical call: workspace and one-time kernel attributes are settled; capture
    hit->used = ++h->graph_tick;
    hipGraph_t g = nullptr;
    HIPCHK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
    rc = run_batch(h, b, s);
    const hipError_t ec = hipStreamEndCapture(s, &g);
    if (!rc && ec == hipSuccess && g) {
      hipGraphExec_t ex = nullptr;
      const bool inst = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0) == hipSuccess;
      (void)hipGraphDestroy(g);
      if (inst && hit->sig == ws_signature(h)) {
        hit->exec = ex;
        HIPCHK(hipGraphLaunch(hit->exec, s));
      } else {
        if (inst) (void)hipGraphExecDestroy(ex);
        *hit = mimo_rx::GraphEntry{};
        rc = run_batch(h, b, s);
      }
    } else {
      if (g) (void)hipGraphDestroy(g);
      (void)hipGetLastError();
      *hit = mimo_rx::GraphEntry{};
      if (!rc) rc = run_batch(h, b, s);   // capture failed: run directly
    }
  } else {
    rc = run_batch(h, b, s);
    // a workspace reallocation makes every earlier capture stale
    const auto sig2 = ws_signature(h);
    for (auto &g : h->graphs)
      if (g.used && g.sig != sig2) drop_graph(h, g);
    if (rc == MIMO_OK) {
      mimo_rx::GraphEntry *slot = &h->graphs[0];   // an empty or the least recently used slot
      for (auto &g : h->graphs)
        if (g.used < slot->used) slot = &g;
      drop_graph(h, *slot);
      slot->key = *b;
      slot->stream = s;
      slot->sig = sig2;
      slot->used = ++h->graph_tick;
    }
  }
  if (rc) return rc;
  h->last_frames = b->n_frames * batch_fpc(b);
  h->last_max_out = b->max_out_syms;
  return MIMO_OK;
}

int mimo_rx_batch_results(mimo_rx *h, mimo_frame_result *out, uint32_t F) {
  if (!h || !out) return fail(MIMO_ERR_ARG, "null argument");
  if (F > h->last_frames) return fail(MIMO_ERR_ARG, "more frames than the last batch");
  std::vector<FrameInfo> inf(F);
  std::vector<double> ev((size_t)F * h->N * 3);
  HIPCHK(hipStreamSynchronize(h->stream));
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(inf.data(), h->info.p, sizeof(FrameInfo) * F, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(ev.data(), h->evm_out.p, sizeof(double) * ev.size(), hipMemcpyDeviceToHost));
  for (uint32_t f = 0; f < F; f++) {
    mimo_frame_result &r = out[f];
    std::memset(&r, 0, sizeof(r));
    const FrameInfo &I = inf[f];
    const bool synced = I.status == MIMO_FRAME_OK || I.status == MIMO_FRAME_INCOMPLETE;
    const uint64_t o = I.origin;   // positions as the framesync started at origin reports them
    r.status = I.status;
    r.n_sym = (I.status == 0) ? I.n_sym : 0;
    r.trigger = synced ? I.trigger - o : I.trigger;
    r.sync_index = synced ? I.sync_index - o : 0;
    r.num_samples_processed = I.nsp;
    r.noise_var = I.noise_var;
    r.cfo_eps = h->cfo ? I.cfo_eps : 0.0f;
    r.origin = o;
    r.capture = I.cap;
    r.ref_frame = I.ref;
    for (uint32_t s = 0; s < h->N; s++) {
      r.plateau_start[s] = synced ? I.plateau_start[s] - o : 0;
      r.plateau_end[s] = synced ? I.plateau_end[s] - o : 0;
      if (inf[f].status == 0) {
        r.evm_num[s] = ev[((size_t)f * h->N + s) * 3 + 0];
        r.evm_den[s] = ev[((size_t)f * h->N + s) * 3 + 1];
        r.errors[s] = (uint64_t)ev[((size_t)f * h->N + s) * 3 + 2];
      }
    }
  }
  return MIMO_OK;
}

int mimo_rx_batch_corr(mimo_rx *h, uint32_t *corr, uint32_t *s0, uint32_t F) {
  if (!h) return fail(MIMO_ERR_ARG, "null handle");
  if (F > h->last_frames) return fail(MIMO_ERR_ARG, "more frames than the last batch");
  HIPCHK(hipDeviceSynchronize());
  return copy_corr(h, F, corr, s0);
}

int mimo_rx_batch_G(mimo_rx *h, float *G, uint32_t F) {
  if (!h || !G) return fail(MIMO_ERR_ARG, "null argument");
  if (F > h->last_frames) return fail(MIMO_ERR_ARG, "more frames than the last batch");
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(G, h->G.p, sizeof(float2) * (size_t)F * h->M * h->N * h->N,
                   hipMemcpyDeviceToHost));
  return MIMO_OK;
}

int mimo_rx_batch_W(mimo_rx *h, float *W, uint32_t F) {
  if (!h || !W) return fail(MIMO_ERR_ARG, "null argument");
  if (F > h->last_frames) return fail(MIMO_ERR_ARG, "more frames than the last batch");
  HIPCHK(hipDeviceSynchronize());
  for (uint32_t f = 0; f < F; f++) {
    int rc = copy_W(h, f, W + (size_t)f * h->M * h->N * h->N * 2);
    if (rc) return rc;
  }
  return MIMO_OK;
}

int mimo_rx_set_grid_cus(mimo_rx *h, uint32_t n_cu) {
  if (!h) return fail(MIMO_ERR_ARG, "null handle");
  int dev = 0, ncu = 0;
  if (n_cu == 0 && hipGetDevice(&dev) == hipSuccess &&
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && ncu > 0)
    n_cu = (uint32_t)ncu;
  if (n_cu == 0) return fail(MIMO_ERR_ARG, "no CU count");
  h->n_cu = n_cu;
  return MIMO_OK;
}

int mimo_rx_set_timing(mimo_rx *h, int enable) {
  if (!h) return fail(MIMO_ERR_ARG, "null handle");
  h->timer.on = enable != 0;
  return MIMO_OK;
}

int mimo_rx_set_debug_log(mimo_rx *h, const char *dir) {
  if (!h) return fail(MIMO_ERR_ARG, "null handle");
  close_debug_files(h);
  h->dbg_dir.clear();
  if (!dir || !dir[0]) return MIMO_OK;
  h->dbg_dir = dir;
  for (uint32_t a = 0; a < h->N; a++) {   // framing.cc:390-402: f_sc_<k>.dat, k from 1
    const std::string fn = h->dbg_dir + "/f_sc_" + std::to_string(a + 1) + ".dat";
    FILE *f = fopen(fn.c_str(), "wb");
    if (!f) {
      close_debug_files(h);
      h->dbg_dir.clear();
      return fail(MIMO_ERR_ARG, "cannot open " + fn);
    }
    h->dbg_fsc.push_back(f);
  }
  return MIMO_OK;
}

int mimo_rx_get_stream_capacity(const mimo_rx *h, uint64_t *samples, uint64_t *held) {
  if (!h) return fail(MIMO_ERR_ARG, "null handle");
  if (samples) *samples = h->capbuf.p ? h->cap_len : 0;
  if (held) *held = h->total;
  return MIMO_OK;
}

int mimo_rx_get_decode_path(const mimo_rx *h, int32_t *path) {
  if (!h || !path) return fail(MIMO_ERR_ARG, "null argument");
  *path = h->last_decode_path;
  return MIMO_OK;
}

int mimo_rx_get_cfo_mode(const mimo_rx *h, int32_t *mode) {
  if (!h || !mode) return fail(MIMO_ERR_ARG, "null argument");
  *mode = h->last_cfo_mode;
  return MIMO_OK;
}

int mimo_rx_get_sc_exact_count(mimo_rx *h, uint64_t *out) {
  if (!h || !out) return fail(MIMO_ERR_ARG, "null argument");
  *out = 0;
  if (!h->n_exact.p) return MIMO_OK;
  unsigned long long v = 0;
  HIPCHK(hipStreamSynchronize(h->stream));
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(&v, h->n_exact.p, sizeof(v), hipMemcpyDeviceToHost));
  HIPCHK(hipMemset(h->n_exact.p, 0, sizeof(v)));
  *out = v;
  return MIMO_OK;
}

int mimo_rx_get_stage_times(mimo_rx *h, double *ms, uint32_t *launches) {
  if (!h) return fail(MIMO_ERR_ARG, "null handle");
  for (int i = 0; i < MIMO_NUM_STAGES; i++) {
    if (ms) ms[i] = 0.0;
    if (launches) launches[i] = 0;
  }
  for (auto &e : h->timer.ev) {
    HIPCHK(hipEventSynchronize(e.second.second));
    float t = 0.0f;
    HIPCHK(hipEventElapsedTime(&t, e.second.first, e.second.second));
    if (ms) ms[e.first] += t;
    if (launches) launches[e.first] += 1;
    (void)hipEventDestroy(e.second.first);
    (void)hipEventDestroy(e.second.second);
  }
  h->timer.ev.clear();
  return MIMO_OK;
}

// ---------------- transmitter ----------------
int mimo_tx_create(uint32_t M, uint32_t cp, uint32_t N, uint32_t nac, const uint8_t *p,
                   const uint8_t *s0_bits, const uint8_t *s1_bits, mimo_tx **out) {
  if (!p || !s0_bits || !s1_bits || !out) return fail(MIMO_ERR_ARG, "null argument");
  const int l2 = ilog2(M);
  if (l2 < 6 || l2 > 12) return fail(MIMO_ERR_UNSUPPORTED, "M must be a power of two in [64, 4096]");
  if (N == 0 || N > MIMO_MAX_STREAMS || cp == 0 || cp > M / 2 || nac == 0)
    return fail(MIMO_ERR_ARG, "bad framegen parameters");
  uint32_t n0, n1, n2;
  int rc = validate_sctype(p, M, &n0, &n1, &n2);
  if (rc) return rc;
  mimo_tx *h = new mimo_tx();
  h->M = M; h->cp = cp; h->SL = M + cp; h->N = N; h->nac = nac; h->M_occ = n1 + n2;
  h->log2M = l2;
  h->dn = 1.0f / sqrtf((float)h->M_occ);   // framing.cc:115
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    return fail(MIMO_ERR_HIP, "hipStreamCreate failed");
  }
  rc = get_twiddles(&h->tw);
  if (!rc) rc = build_codes(h->codes, M, N, nac, p, s0_bits, s1_bits, l2 + 1, false, h->stream);
  if (rc) { mimo_tx_destroy(h); return rc; }
  const uint32_t n_slots = N * nac + 1;
  std::vector<float2> all((size_t)n_slots * M);
  std::vector<int32_t> occ;
  for (uint32_t i = 0; i < M; i++) if (p[i] != MIMO_SC_NULL) occ.push_back((int32_t)i);
  if (hipMemcpy(all.data(), h->codes.code_time.p, sizeof(float2) * all.size(),
                hipMemcpyDeviceToHost) != hipSuccess ||
      h->occ_list.ensure(occ.size()) != hipSuccess ||
      hipMemcpy(h->occ_list.p, occ.data(), sizeof(int32_t) * occ.size(),
                hipMemcpyHostToDevice) != hipSuccess) {
    mimo_tx_destroy(h);
    return fail(MIMO_ERR_HIP, "framegen table upload failed");
  }
  h->s0.assign(all.begin(), all.begin() + M);
  // regroup slot-major (slot = 1 + code*N + t) into per-stream [t][code*M + i]
  h->s1.resize((size_t)N * nac * M);
  for (uint32_t c = 0; c < nac; c++)
    for (uint32_t t = 0; t < N; t++)
      std::memcpy(h->s1.data() + ((size_t)t * nac + c) * M,
                  all.data() + (size_t)(1 + c * N + t) * M, sizeof(float2) * M);
  *out = h;
  return MIMO_OK;
}

int mimo_tx_destroy(mimo_tx *h) {
  if (!h) return MIMO_OK;
  if (h->stream) {
    (void)hipStreamSynchronize(h->stream);
    (void)hipStreamDestroy(h->stream);
  }
  delete h;
  return MIMO_OK;
}

int mimo_tx_get_codes(mimo_tx *h, float *s0, float *s1) {
  if (!h) return fail(MIMO_ERR_ARG, "null handle");
  if (s0) std::memcpy(s0, h->s0.data(), sizeof(float2) * h->s0.size());
  if (s1) std::memcpy(s1, h->s1.data(), sizeof(float2) * h->s1.size());
  return MIMO_OK;
}

int mimo_tx_write_sync_words(mimo_tx *h, float *const *tx, uint32_t *n_written) {
  // framing.cc:169-208: S0 (CP + body) on stream 0, then nac x N TDMA slots of S1
  if (!h || !tx) return fail(MIMO_ERR_ARG, "null argument");
  const uint32_t M = h->M, cp = h->cp, total = (h->nac * h->N + 1) * h->SL;
  for (uint32_t s = 0; s < h->N; s++) std::memset(tx[s], 0, sizeof(float2) * total);
  uint32_t idx = 0;
  auto put = [&](uint32_t s, const float2 *code) {
    std::memcpy(reinterpret_cast<float2 *>(tx[s]) + idx, code + M - cp, sizeof(float2) * cp);
    idx += cp;
    std::memcpy(reinterpret_cast<float2 *>(tx[s]) + idx, code, sizeof(float2) * M);
    idx += M;
  };
  put(0, h->s0.data());
  for (uint32_t ac = 0; ac < h->nac; ac++)
    for (uint32_t s = 0; s < h->N; s++) put(s, h->s1.data() + ((size_t)s * h->nac + ac) * M);
  if (n_written) *n_written = idx;
  return MIMO_OK;
}

int mimo_tx_assemble_mimo_packet(mimo_tx *h, float *const *tx, const float *const *in,
                                 uint32_t *n_written) {
  if (!h || !tx || !in) return fail(MIMO_ERR_ARG, "null argument");
  const size_t per = h->M_occ;
  HIPCHK(h->din.ensure(per * h->N));
  HIPCHK(h->dout.ensure((size_t)h->SL * h->N));
  for (uint32_t t = 0; t < h->N; t++)
    HIPCHK(hipMemcpyAsync(h->din.p + t * per, in[t], sizeof(float2) * per, hipMemcpyHostToDevice,
                          h->stream));
  TxSymArgs a{};
  a.N = h->N; a.M = h->M; a.cp = h->cp; a.M_occ = h->M_occ; a.dn = h->dn; a.gain = 1.0f;
  a.occ_list = h->occ_list.p; a.in = h->din.p; a.n_sym = 1; a.out = h->dout.p; a.tw = h->tw;
  a.qam = make_qam(4);
  launch_tx_symbols(a, h->log2M, 1, h->stream);
  HIPCHK(hipGetLastError());
  for (uint32_t t = 0; t < h->N; t++)
    HIPCHK(hipMemcpyAsync(tx[t], h->dout.p + (size_t)t * h->SL, sizeof(float2) * h->SL,
                          hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  if (n_written) *n_written = h->SL;
  return MIMO_OK;
}

// ---------------- synthetic captures ----------------
static uint64_t synth_offset(const mimo_synth_config *c, uint64_t frame_id) {
  const uint64_t SL = c->M + c->cp_len;
  if (c->offset >= 0) return (uint64_t)c->offset;
  // ref_hash5(seed, DOM_OFFSET, frame, 0, 0) % SL on the host (same mixer as the kernels)
  auto mix = [](uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  };
  uint64_t hh = mix(c->seed ^ ((uint64_t)DOM_OFFSET * 0xD6E8FEB86659FD93ull));
  hh = mix(hh ^ frame_id);
  hh = mix(hh ^ 0ull);
  hh = mix(hh ^ 0ull);
  return hh % SL;
}

int mimo_synth_frame_len(const mimo_synth_config *c, uint64_t frame_id, uint64_t *len) {
  if (!c || !len) return fail(MIMO_ERR_ARG, "null argument");
  const uint64_t SL = c->M + c->cp_len;
  *len = SL * (2ull * c->num_streams * c->num_access_codes + 2 + c->pid + c->tail_syms) +
         synth_offset(c, frame_id);
  return MIMO_OK;
}

int mimo_synth_frames(const mimo_synth_config *c, uint64_t frame_id0, uint32_t n_frames,
                      void *d_out, uint64_t stride, uint64_t frame_len, void *d_tx_idx,
                      void *d_H, void *hip_stream) {
  if (!c || !d_out || !c->p || !c->s0_bits || !c->s1_bits)
    return fail(MIMO_ERR_ARG, "null argument");
  const int l2 = ilog2(c->M);
  if (l2 < 6 || l2 > 12) return fail(MIMO_ERR_UNSUPPORTED, "M must be a power of two in [64, 4096]");
  const uint32_t N = c->num_streams;
  if (N == 0 || N > MIMO_MAX_STREAMS) return fail(MIMO_ERR_ARG, "bad num_streams");
  if (stride < frame_len) return fail(MIMO_ERR_ARG, "stride < frame_len");
  uint32_t n0, n1, n2;
  int rc = validate_sctype(c->p, c->M, &n0, &n1, &n2);
  if (rc) return rc;
  const uint32_t M_occ = n1 + n2, SL = c->M + c->cp_len;
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : nullptr;
  Codes codes;
  rc = build_codes(codes, c->M, N, c->num_access_codes, c->p, c->s0_bits, c->s1_bits, l2 + 1,
                   false, s);
  if (rc) return rc;
  float2 *tw = nullptr;
  rc = get_twiddles(&tw);
  if (rc) return rc;
  std::vector<int32_t> occ;
  for (uint32_t i = 0; i < c->M; i++) if (c->p[i] != MIMO_SC_NULL) occ.push_back((int32_t)i);
  DevBuf<int32_t> docc;
  HIPCHK(docc.ensure(occ.size()));
  HIPCHK(hipMemcpy(docc.p, occ.data(), sizeof(int32_t) * occ.size(), hipMemcpyHostToDevice));
  // frames in groups so the TX scratch stays bounded (~1 GiB)
  const uint64_t per_frame = (uint64_t)N * std::max<uint32_t>(c->pid, 1) * SL;
  uint32_t group = (uint32_t)std::max<uint64_t>(1, (128ull << 20) / per_frame);
  group = std::min(group, n_frames);
  DevBuf<float2> scratch;
  HIPCHK(scratch.ensure(per_frame * group));
  const Qam qam = make_qam(c->qam_order);
  const float nstd = (float)std::sqrt(0.0625 * std::pow(10.0, -(double)c->snr_db / 10.0));
  for (uint32_t f0 = 0; f0 < n_frames; f0 += group) {
    const uint32_t nf = std::min(group, n_frames - f0);
    if (c->pid) {
      TxSymArgs a{};
      a.N = N; a.M = c->M; a.cp = c->cp_len; a.M_occ = M_occ;
      a.dn = 1.0f / sqrtf((float)M_occ); a.gain = 0.25f;
      a.occ_list = docc.p; a.in = nullptr; a.n_sym = c->pid; a.seed = c->seed;
      a.frame_id0 = frame_id0 + f0; a.qam = qam;
      a.tx_idx = d_tx_idx ? reinterpret_cast<uint8_t *>(d_tx_idx) + (size_t)f0 * N * c->pid * M_occ
                          : nullptr;
      a.out = scratch.p; a.tw = tw;
      launch_tx_symbols(a, l2, nf, s);
    }
    MixArgs m{};
    m.N = N; m.M = c->M; m.cp = c->cp_len; m.SL = SL; m.nac = c->num_access_codes;
    m.pid = c->pid; m.seed = c->seed; m.frame_id0 = frame_id0 + f0; m.offset = c->offset;
    m.identity = c->identity_channel; m.nstd = nstd; m.code_time = codes.code_time.p;
    m.tx_data = scratch.p;
    m.out = reinterpret_cast<float2 *>(d_out) + (size_t)f0 * N * stride;
    m.stride = stride; m.frame_len = frame_len;
    m.H_out = d_H ? reinterpret_cast<float2 *>(d_H) + (size_t)f0 * N * N : nullptr;
    launch_mix(m, nf, s);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));
  }
  return MIMO_OK;
}

// ---------------- helpers ----------------
int mimo_sctype_default(uint8_t *p, uint32_t M) {   // framing.cc:949-954
  if (!p) return fail(MIMO_ERR_ARG, "null argument");
  for (uint32_t i = 0; i < M; i++) p[i] = MIMO_SC_DATA;
  return MIMO_OK;
}

int mimo_sctype_liquid(uint8_t *p, uint32_t M) {    // framing.cc:956-997
  if (!p) return fail(MIMO_ERR_ARG, "null argument");
  const uint32_t M2 = M / 2;
  uint32_t G = std::max<uint32_t>(M / 10, 2);
  const uint32_t P = (M > 34) ? 8 : 4, P2 = P / 2;
  for (uint32_t i = 0; i < M; i++) p[i] = MIMO_SC_NULL;
  for (uint32_t i = 1; i + G < M2; i++) {
    const uint8_t v = (((i + P2) % P) == 0) ? MIMO_SC_PILOT : MIMO_SC_DATA;
    p[i] = v;
    p[M - i] = v;
  }
  return MIMO_OK;
}

int mimo_sctype_validate(const uint8_t *p, uint32_t M, uint32_t *a, uint32_t *b, uint32_t *c) {
  if (!p || !a || !b || !c) return fail(MIMO_ERR_ARG, "null argument");
  return validate_sctype(p, M, a, b, c);
}

int mimo_msequence_draw_bits(uint32_t m, uint32_t g, uint32_t a, uint32_t count, uint8_t *out) {
  // liquid msequence_create / msequence_generate_symbol(ms,1)
  if (!out || m < 2 || m > 31) return fail(MIMO_ERR_ARG, "bad msequence parameters");
  uint32_t gg = g >> 1, v = 0;
  for (uint32_t i = 0; i < m; i++) { v = (v << 1) | (a & 1u); a >>= 1; }
  const uint32_t n = (1u << m) - 1u;
  for (uint32_t i = 0; i < count; i++) {
    const uint32_t b = (uint32_t)__builtin_parity(v & gg);
    v = ((v << 1) | b) & n;
    out[i] = (uint8_t)b;
  }
  return MIMO_OK;
}

float mimo_invert2(float *W, const float *G) {   // framing.cc:1344-1367 on host data
  const float2 *g = reinterpret_cast<const float2 *>(G);
  float2 *w = reinterpret_cast<float2 *>(W);
  auto mul = [](float2 a, float2 b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
  };
  const float2 p0 = mul(g[0], g[3]), p1 = mul(g[1], g[2]);
  const float2 det = make_float2(p0.x - p1.x, p0.y - p1.y);
  const float2 di = make_float2(det.x, -det.y), ndi = make_float2(-det.x, det.y);
  w[0] = mul(di, g[3]);
  w[3] = mul(di, g[0]);
  w[2] = mul(ndi, g[2]);
  w[1] = mul(ndi, g[1]);
  return 1.0f / (det.x * det.x + det.y * det.y);
}

int mimo_dev_alloc(void **ptr, size_t bytes) {
  if (!ptr) return fail(MIMO_ERR_ARG, "null argument");
  HIPCHK(hipMalloc(ptr, bytes));
  return MIMO_OK;
}
int mimo_dev_free(void *ptr) {
  HIPCHK(hipFree(ptr));
  return MIMO_OK;
}
int mimo_memcpy_h2d(void *dst, const void *src, size_t bytes, void *s) {
  HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)s));
  HIPCHK(hipStreamSynchronize((hipStream_t)s));
  return MIMO_OK;
}
int mimo_memcpy_d2h(void *dst, const void *src, size_t bytes, void *s) {
  HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)s));
  HIPCHK(hipStreamSynchronize((hipStream_t)s));
  return MIMO_OK;
}
int mimo_memcpy_d2d(void *dst, const void *src, size_t bytes, void *s) {
  HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)s));
  HIPCHK(hipStreamSynchronize((hipStream_t)s));
  return MIMO_OK;
}
int mimo_memset_d(void *dst, int value, size_t bytes, void *s) {
  HIPCHK(hipMemsetAsync(dst, value, bytes, (hipStream_t)s));
  return MIMO_OK;
}
int mimo_ingest_sc16(const void *src, uint64_t src_stride, void *dst, uint64_t dst_stride,
                     uint32_t n_arrays, uint64_t n, float scale, void *s) {
  if (n == 0 || n_arrays == 0) return MIMO_OK;
  if (!src || !dst) return fail(MIMO_ERR_ARG, "mimo_ingest_sc16: null buffer");
  if (n_arrays > 1 && (src_stride < n || dst_stride < n))
    return fail(MIMO_ERR_ARG, "mimo_ingest_sc16: stride shorter than a row");
  if (!launch_sc16_to_fc32(src, src_stride, dst, dst_stride, n_arrays, n, scale,
                           (hipStream_t)s))
    return fail(MIMO_ERR_ARG, "mimo_ingest_sc16: too many rows or samples for one launch");
  HIPCHK(hipGetLastError());
  return MIMO_OK;
}
int mimo_cfo_estimate(const void *x, uint64_t stride, uint32_t n_ant, uint64_t start,
                      uint32_t M, double *eps, void *s) {
  if (!x || !eps || n_ant == 0) return fail(MIMO_ERR_ARG, "mimo_cfo_estimate: null argument");
  if (M < 2 || (M & 1)) return fail(MIMO_ERR_ARG, "mimo_cfo_estimate: M must be even");
  if (n_ant > 1 && stride < start + M)
    return fail(MIMO_ERR_ARG, "mimo_cfo_estimate: window runs past the row stride");
  double *d = nullptr;
  HIPCHK(hipMalloc(&d, sizeof(double) * 2 * n_ant));
  std::vector<double> h(2 * n_ant);
  const hipStream_t st = (hipStream_t)s;
  bool ok = launch_cfo_corr(x, stride, n_ant, start, M / 2, d, st);
  hipError_t e = ok ? hipGetLastError() : hipSuccess;
  if (ok && e == hipSuccess) e = hipMemcpyAsync(h.data(), d, sizeof(double) * 2 * n_ant,
                                                hipMemcpyDeviceToHost, st);
  if (ok && e == hipSuccess) e = hipStreamSynchronize(st);
  (void)hipFree(d);
  if (!ok) return fail(MIMO_ERR_ARG, "mimo_cfo_estimate: too many antenna rows");
  if (e != hipSuccess) return fail(MIMO_ERR_HIP, std::string("mimo_cfo_estimate: ") +
                                                     hipGetErrorString(e));
  double re = 0.0, im = 0.0;
  for (uint32_t r = 0; r < n_ant; ++r) {
    eps[r] = std::atan2(h[2 * r + 1], h[2 * r]) / M_PI;
    re += h[2 * r];
    im += h[2 * r + 1];
  }
  eps[n_ant] = std::atan2(im, re) / M_PI;
  return MIMO_OK;
}
int mimo_cfo_derotate(void *x, uint64_t stride, uint32_t n_ant, uint64_t n, int64_t n0,
                      double eps, uint32_t M, void *s) {
  if (n == 0 || n_ant == 0) return MIMO_OK;
  if (!x || M == 0) return fail(MIMO_ERR_ARG, "mimo_cfo_derotate: null buffer or M");
  if (n_ant > 1 && stride < n) return fail(MIMO_ERR_ARG, "mimo_cfo_derotate: stride < n");
  if (!launch_cfo_derotate(x, stride, n_ant, n, n0, eps / M, (hipStream_t)s))
    return fail(MIMO_ERR_ARG, "mimo_cfo_derotate: too many rows or samples for one launch");
  HIPCHK(hipGetLastError());
  return MIMO_OK;
}
int mimo_stream_sync(void *s) {
  HIPCHK(hipStreamSynchronize((hipStream_t)s));
  return MIMO_OK;
}
int mimo_device_count(int *n) {
  if (!n) return fail(MIMO_ERR_ARG, "null argument");
  HIPCHK(hipGetDeviceCount(n));
  return MIMO_OK;
}

}  // extern "C"

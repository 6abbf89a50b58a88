/*
 * include/framing.h -- drop-in replacement for /root/reference/mimo/framing.h.
 *
 * Same names and signatures: rx_beamforming::framegen (framing.h:42-103),
 * rx_beamforming::framesync (framing.h:105-213), mimo_callback (:30-31),
 * framesync_states_t (:34-39) and the free functions (:226-280). The classes are thin
 * inline wrappers over the C-ABI in mimo_rx.h, so config.h's compile-time constants
 * (PID_MAX, PLATEAU_THREASHOLD, SISO, SISO_TX/RX) are read in the caller's translation unit
 * exactly as the reference reads them. Link with -lrub_mimo_amd instead of
 * -lfftw3f -lvolk (and -lliquid becomes optional). See INTEGRATION.md.
 *
 * Error behaviour mirrors the reference where the reference has one: an invalid subcarrier
 * type or an empty S0 allocation prints and exit(1)s (framing.cc:1020-1022, 1093-1096); GPU
 * failures (which the reference cannot have) print mimo_last_error() and exit(1) too.
 */
#ifndef FRAMING_H
#define FRAMING_H

#include <complex>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mimo_rx.h"

#if __has_include(<gnuradio/gr_complex.h>)
#include <gnuradio/gr_complex.h>
#else
typedef std::complex<float> gr_complex;
#endif

#if __has_include(<liquid/liquid.h>) && !defined(RUB_MIMO_AMD_NO_LIQUID)
#include <liquid/liquid.h>
#else
#include "liquid_shim.h"
#endif

#if __has_include("config.h") && !defined(RUB_MIMO_AMD_NO_CONFIG_H)
#include "config.h"
#endif
#ifndef PID_MAX
#define PID_MAX 1000
#endif
#ifndef PLATEAU_THREASHOLD
#define PLATEAU_THREASHOLD 0.95
#endif
#ifndef SISO
#define SISO false
#endif

// callback, framing.h:30-31
typedef void *(*mimo_callback)(std::vector<gr_complex *>, unsigned int occupied_carriers);

// receiver state, framing.h:34-39
typedef enum {
  STATE_SEEK_PLATEAU = 0,
  STATE_SAVE_ACCESS_CODES,
  STATE_WAIT,
  STATE_MIMO
} framesync_states_t;

// ------------------------------------------------------------------ free functions
void ofdmframe_init_default_sctype(unsigned char *_p, unsigned int _M);
void ofdmframe_validate_sctype(const unsigned char *_p, unsigned int _M, unsigned int *_M_null,
                               unsigned int *_M_pilot, unsigned int *_M_data);
void ofdmframe_print_sctype(const unsigned char *_p, unsigned int _M);
void ofdmframe_init_S0(const unsigned char *_p, unsigned int _M, std::complex<float> *_S0,
                       std::complex<float> *_s0, msequence ms);
void ofdmframe_init_S1(const unsigned char *_p, unsigned int _M, unsigned int _num_access_codes,
                       std::complex<float> *_S1, std::complex<float> *_s1, msequence ms);
gr_complex liquid_cexpjf(float theta);
float cabsf(gr_complex z);
float cargf(gr_complex z);
float fabsf(float x);
gr_complex conjf(gr_complex z);
float invert(std::vector<std::vector<gr_complex> > &W,
             std::vector<std::vector<gr_complex> > const &G);


namespace rx_beamforming {

namespace detail {
inline void die(const char *where) {
  std::fprintf(stderr, "***** %s failed: %s\n", where, mimo_last_error());
  std::exit(1);
}
inline std::vector<unsigned char> draw(msequence ms, size_t count) {
  std::vector<unsigned char> b(count);
  for (size_t i = 0; i < count; i++) b[i] = (unsigned char)(msequence_generate_symbol(ms, 1) & 0x01);
  return b;
}
// the constructors consume the caller's generators exactly as ofdmframe_init_S0/S1 do
// (one draw per subcarrier index, framing.cc:1073-1075, 1236-1240)
inline std::vector<unsigned char> draw_s1(std::vector<msequence> const &ms, unsigned int N,
                                          unsigned int nac, unsigned int M) {
  std::vector<unsigned char> out;
  out.reserve((size_t)N * nac * M);
  for (unsigned int i = 0; i < N; i++) {
    std::vector<unsigned char> b = draw(ms[i], (size_t)nac * M);
    out.insert(out.end(), b.begin(), b.end());
  }
  return out;
}
}  // namespace detail

class framegen {
 private:
  mimo_tx *h_ = nullptr;
  unsigned int M, cp_len;
  [[maybe_unused]] unsigned int symbol_len;   // the reference's member (M + cp_len)
  unsigned int num_streams, num_access_codes;
  std::vector<unsigned char> p;
  unsigned int M_null = 0, M_pilot = 0, M_data = 0;

 public:
  framegen(unsigned int _M, unsigned int _cp_len, unsigned int _num_streams,
           unsigned int _num_access_codes, unsigned char *const &_p, msequence const &_ms_S0,
           std::vector<msequence> const &_ms_S1)
      : M(_M), cp_len(_cp_len), symbol_len(_M + _cp_len), num_streams(_num_streams),
        num_access_codes(_num_access_codes), p(_p, _p + _M) {
    if (mimo_sctype_validate(p.data(), M, &M_null, &M_pilot, &M_data) != MIMO_OK) {
      std::fprintf(stderr, "error: ofdmframe_validate_sctype(), invalid subcarrier type\n");
      std::exit(1);
    }
    std::vector<unsigned char> b0 = detail::draw(_ms_S0, M);   // framegen: S0 first (:110)
    std::vector<unsigned char> b1 = detail::draw_s1(_ms_S1, num_streams, num_access_codes, M);
    if (mimo_tx_create(M, cp_len, num_streams, num_access_codes, p.data(), b0.data(), b1.data(),
                       &h_) != MIMO_OK)
      detail::die("framegen");
  }
  ~framegen() { mimo_tx_destroy(h_); }
  framegen(const framegen &) = delete;
  framegen &operator=(const framegen &) = delete;

  void print() {
    std::printf("ofdmframegen:\n");
    std::printf("    num subcarriers     :   %-u\n", M);
    std::printf("      - NULL            :   %-u\n", M_null);
    std::printf("      - pilot           :   %-u\n", M_pilot);
    std::printf("      - data            :   %-u\n", M_data);
    std::printf("    cyclic prefix len   :   %-u\n", cp_len);
    std::printf("    ");
    ::ofdmframe_print_sctype(p.data(), M);
  }

  unsigned int write_sync_words(std::vector<std::complex<float> *> tx_buff) {
    if (tx_buff.size() != num_streams) detail::die("write_sync_words: tx_buff.size()");
    std::vector<float *> t(num_streams);
    for (unsigned int i = 0; i < num_streams; i++) t[i] = reinterpret_cast<float *>(tx_buff[i]);
    uint32_t n = 0;
    if (mimo_tx_write_sync_words(h_, t.data(), &n) != MIMO_OK) detail::die("write_sync_words");
    return n;
  }

  unsigned int assemble_mimo_packet(std::vector<gr_complex *> tx_buff,
                                    std::vector<gr_complex *> in_buff) {
    if (tx_buff.size() != num_streams || in_buff.size() != num_streams)
      detail::die("assemble_mimo_packet: buffer count");
    std::vector<float *> t(num_streams);
    std::vector<const float *> in(num_streams);
    for (unsigned int i = 0; i < num_streams; i++) {
      t[i] = reinterpret_cast<float *>(tx_buff[i]);
      in[i] = reinterpret_cast<const float *>(in_buff[i]);
    }
    uint32_t n = 0;
    if (mimo_tx_assemble_mimo_packet(h_, t.data(), in.data(), &n) != MIMO_OK)
      detail::die("assemble_mimo_packet");
    return n;
  }

  unsigned int get_num_streams() { return num_streams; }
};

class framesync {
 private:
  mimo_rx *h_ = nullptr;
  unsigned int M, cp_len;
  [[maybe_unused]] unsigned int symbol_len;   // the reference's member (M + cp_len)
  unsigned int num_streams, num_access_codes;
  std::vector<unsigned char> p;
  unsigned int M_null = 0, M_pilot = 0, M_data = 0, M_occupied = 0;
  mimo_callback callback;
  std::vector<gr_complex *> cbv;

  static void bridge(const float *const *eq, uint32_t n, uint32_t m_occ, void *user) {
    framesync *self = static_cast<framesync *>(user);
    for (uint32_t i = 0; i < n; i++)
      self->cbv[i] = reinterpret_cast<gr_complex *>(const_cast<float *>(eq[i]));
    if (self->callback) self->callback(self->cbv, m_occ);   // framing.cc:587
  }

 public:
  framesync(unsigned int _M, unsigned int _cp_len, unsigned int _num_streams,
            unsigned int _num_access_codes, unsigned char *const &_p, msequence const &_ms_S0,
            std::vector<msequence> const &_ms_S1, mimo_callback _callback)
      : M(_M), cp_len(_cp_len), symbol_len(_M + _cp_len), num_streams(_num_streams),
        num_access_codes(_num_access_codes), p(_p, _p + _M), callback(_callback),
        cbv(_num_streams, nullptr) {
    if (mimo_sctype_validate(p.data(), M, &M_null, &M_pilot, &M_data) != MIMO_OK) {
      std::fprintf(stderr, "error: ofdmframe_validate_sctype(), invalid subcarrier type\n");
      std::exit(1);
    }
    M_occupied = M_pilot + M_data;
    // framesync: S1 per stream first (:374-379), then S0 (:411-415)
    std::vector<unsigned char> b1 = detail::draw_s1(_ms_S1, num_streams, num_access_codes, M);
    std::vector<unsigned char> b0 = detail::draw(_ms_S0, M);
    mimo_rx_config c{};
    c.M = M;
    c.cp_len = cp_len;
    c.num_streams = num_streams;
    c.num_access_codes = num_access_codes;
    c.pid_max = PID_MAX;
    c.p = p.data();
    c.s0_bits = b0.data();
    c.s1_bits = b1.data();
    // INVERT_CHANNEL (config.h:102): the reference's 2x2 adjugate; NxN ZF beyond 2 streams
    c.detector = SISO ? MIMO_DET_SISO : (num_streams == 2 ? MIMO_DET_ZF2 : MIMO_DET_ZF);
    c.noise_var = -1.0f;
    c.keep_identity_bias = 1;
#if defined(SISO_TX) && defined(SISO_RX)
    c.siso_tx = SISO ? SISO_TX : 0;
    c.siso_rx = SISO ? SISO_RX : 0;
#endif
    c.plateau_threshold = PLATEAU_THREASHOLD;
    c.qam_order = 4;
    if (mimo_rx_create(&c, nullptr, &h_) != MIMO_OK) detail::die("framesync");
    mimo_rx_set_callback(h_, &framesync::bridge, this);
    // DEBUG_LOG (config.h:84-86 writes /tmp/f_sc_*, /tmp/corr_*): off unless the environment
    // names a directory, RMIMO_DEBUG_LOG=/tmp for the reference's behaviour
    if (const char *d = std::getenv("RMIMO_DEBUG_LOG"))
      if (d[0] && mimo_rx_set_debug_log(h_, d) != MIMO_OK) detail::die("framesync debug log");
  }
  ~framesync() { mimo_rx_destroy(h_); }
  framesync(const framesync &) = delete;
  framesync &operator=(const framesync &) = delete;

  void print() {
    std::printf("ofdmframegen:\n");
    std::printf("    num subcarriers     :   %-u\n", M);
    std::printf("      - NULL            :   %-u\n", M_null);
    std::printf("      - pilot           :   %-u\n", M_pilot);
    std::printf("      - data            :   %-u\n", M_data);
    std::printf("    cyclic prefix len   :   %-u\n", cp_len);
    std::printf("    ");
    ::ofdmframe_print_sctype(p.data(), M);
  }

  unsigned long int get_sync_index() {
    uint64_t v = 0;
    mimo_rx_get_sync_index(h_, &v);
    return (unsigned long int)v;
  }

  std::vector<std::vector<std::vector<gr_complex> > > get_G() {
    std::vector<gr_complex> flat((size_t)M * num_streams * num_streams);
    if (mimo_rx_get_G(h_, reinterpret_cast<float *>(flat.data())) != MIMO_OK) detail::die("get_G");
    std::vector<std::vector<std::vector<gr_complex> > > G(
        M, std::vector<std::vector<gr_complex> >(num_streams,
                                                 std::vector<gr_complex>(num_streams)));
    for (unsigned int sc = 0; sc < M; sc++)
      for (unsigned int r = 0; r < num_streams; r++)
        for (unsigned int t = 0; t < num_streams; t++)
          G[sc][r][t] = flat[((size_t)sc * num_streams + r) * num_streams + t];
    return G;
  }

  unsigned long long int get_num_samples_processed() {
    uint64_t v = 0;
    mimo_rx_get_num_samples_processed(h_, &v);
    return (unsigned long long int)v;
  }

  framesync_states_t execute(std::vector<gr_complex *> const &in_buff, unsigned int num_samples) {
    std::vector<const float *> in(num_streams);
    for (unsigned int i = 0; i < num_streams; i++)
      in[i] = reinterpret_cast<const float *>(in_buff[i]);
    int32_t st = 0;
    if (mimo_rx_execute(h_, in.data(), num_streams, num_samples, &st) != MIMO_OK)
      detail::die("framesync::execute");
    return (framesync_states_t)st;
  }

  unsigned long int get_plateau_start(unsigned int stream) {
    uint64_t s = 0, e = 0;
    if (mimo_rx_get_plateau(h_, stream, &s, &e) != MIMO_OK) detail::die("get_plateau_start");
    return (unsigned long int)s;
  }

  unsigned long int get_plateau_end(unsigned int stream) {
    uint64_t s = 0, e = 0;
    if (mimo_rx_get_plateau(h_, stream, &s, &e) != MIMO_OK) detail::die("get_plateau_end");
    return (unsigned long int)e;
  }

  void reset() { mimo_rx_reset(h_); }
  // estimation runs inside execute() once the access-code window is complete (framing.cc:649)
  void estimate_channel() {}
  void compute_receive_beamformer() {}   // empty in the reference (framing.cc:898-900)
  void set_siso_tx(unsigned int _tx) {
    siso_tx_ = _tx;
    mimo_rx_set_siso(h_, siso_tx_, siso_rx_);
  }
  void set_siso_rx(unsigned int _rx) {
    siso_rx_ = _rx;
    mimo_rx_set_siso(h_, siso_tx_, siso_rx_);
  }

 private:
  unsigned int siso_tx_ = 0, siso_rx_ = 0;
};

}  // namespace rx_beamforming

namespace tx_beamforming {}

#endif  // FRAMING_H

// rub_mimo_amd/csrc/framing_facade.cpp -- out-of-line pieces of include/framing.h: the
// reference's free functions (framing.cc:26-76, 949-1342, 1344-1367), its constellation
// tables, and the liquid msequence shim used when liquid-dsp is absent.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define RUB_MIMO_AMD_NO_LIQUID 1
#define RUB_MIMO_AMD_NO_CONFIG_H 1
#include "../../include/framing.h"

// ---------------------------------------------------------------- liquid msequence shim
struct rmimo_msequence_s {
  unsigned int m, g, a, n, v, b;
};

extern "C" {

msequence rmimo_msequence_create(unsigned int m, unsigned int g, unsigned int a) {
  if (m < 2 || m > 31) {
    std::fprintf(stderr, "error: msequence_create(), m out of range\n");
    std::exit(1);
  }
  msequence ms = new rmimo_msequence_s();
  ms->m = m;
  ms->g = g >> 1;
  ms->a = 0;
  for (unsigned int i = 0; i < m; i++) {  // initial state bit-reversed, 0001 -> 1000
    ms->a <<= 1;
    ms->a |= (a & 1u);
    a >>= 1;
  }
  ms->n = (1u << m) - 1u;
  ms->v = ms->a;
  ms->b = 0;
  return ms;
}

msequence rmimo_msequence_create_default(unsigned int m) {
  // defaults for the degrees the reference uses (config.h:70-75 / liquid's table)
  static const unsigned int g[32] = {0, 0, 0x7, 0xb, 0x13, 0x25, 0x43, 0x89, 0x11d, 0x211,
                                     0x409, 0x805, 0x1053, 0x201b, 0x402b, 0x8003};
  if (m < 2 || m > 15) {
    std::fprintf(stderr, "error: msequence_create_default(), m out of range\n");
    std::exit(1);
  }
  return rmimo_msequence_create(m, g[m], 1);
}

void rmimo_msequence_destroy(msequence ms) { delete ms; }

unsigned int rmimo_msequence_advance(msequence ms) {
  ms->b = (unsigned int)__builtin_parity(ms->v & ms->g);
  ms->v = ((ms->v << 1) | ms->b) & ms->n;
  return ms->b;
}

unsigned int rmimo_msequence_generate_symbol(msequence ms, unsigned int bps) {
  unsigned int s = 0;
  for (unsigned int i = 0; i < bps; i++) {
    s <<= 1;
    s |= rmimo_msequence_advance(ms);
  }
  return s;
}

void rmimo_msequence_reset(msequence ms) { ms->v = ms->a; }
unsigned int rmimo_msequence_get_length(msequence ms) { return ms->n; }
unsigned int rmimo_msequence_get_state(msequence ms) { return ms->v; }

}  // extern "C"

// ---------------------------------------------------------------- reference globals
static float sqrt2_ = std::sqrt(2.0f);
gr_complex BPSK_CONSTELLATION[] = {gr_complex(-1.0f, 0.0f), gr_complex(1.0f, 0.0f)};
gr_complex QPSK_CONSTELLATION[] = {gr_complex(sqrt2_, sqrt2_), gr_complex(-sqrt2_, sqrt2_),
                                   gr_complex(-sqrt2_, -sqrt2_), gr_complex(sqrt2_, -sqrt2_)};

gr_complex liquid_cexpjf(float theta) { return std::polar(1.0f, theta); }
float cabsf(gr_complex z) { return std::abs(z); }
float cargf(gr_complex z) { return std::arg(z); }
gr_complex conjf(gr_complex z) { return std::conj(z); }

void ofdmframe_init_default_sctype(unsigned char *_p, unsigned int _M) {
  mimo_sctype_default(_p, _M);   // USE_ALL_CARRIERS (framing.cc:949-954)
}

void ofdmframe_validate_sctype(const unsigned char *_p, unsigned int _M, unsigned int *_M_null,
                               unsigned int *_M_pilot, unsigned int *_M_data) {
  if (mimo_sctype_validate(_p, _M, _M_null, _M_pilot, _M_data) != MIMO_OK) {
    std::fprintf(stderr, "error: ofdmframe_validate_sctype(), invalid subcarrier type\n");
    std::exit(1);
  }
}

void ofdmframe_print_sctype(const unsigned char *_p, unsigned int _M) {
  std::printf("[");
  for (unsigned int i = 0; i < _M; i++) {
    unsigned int k = (i + _M / 2) % _M;
    switch (_p[k]) {
      case OFDMFRAME_SCTYPE_NULL: std::printf("."); break;
      case OFDMFRAME_SCTYPE_PILOT: std::printf("|"); break;
      case OFDMFRAME_SCTYPE_DATA: std::printf("+"); break;
      default:
        std::fprintf(stderr, "error: ofdmframe_print_default_sctype(), invalid subcarrier type\n");
        std::exit(1);
    }
  }
  std::printf("]\n");
}

// S0/S1 through the GPU transmitter tables (framing.cc:1054-1111, 1214-1262)
void ofdmframe_init_S0(const unsigned char *_p, unsigned int _M, std::complex<float> *_S0,
                       std::complex<float> *_s0, msequence ms) {
  std::vector<unsigned char> b0(_M), b1(_M, 0);
  unsigned int M_S0 = 0;
  for (unsigned int i = 0; i < _M; i++) {
    b0[i] = (unsigned char)(msequence_generate_symbol(ms, 1) & 0x01);
    if (_p[i] == OFDMFRAME_SCTYPE_NULL || (i % 2) != 0) {
      _S0[i] = 0.0f;
    } else {
      _S0[i] = b0[i] ? 1.0f : -1.0f;
      M_S0++;
    }
  }
  if (M_S0 == 0) {
    std::fprintf(stderr, "error: ofdmframe_init_S0(), no subcarriers enabled; check allocation\n");
    std::exit(1);
  }
  mimo_tx *h = nullptr;
  if (mimo_tx_create(_M, 1, 1, 1, _p, b0.data(), b1.data(), &h) != MIMO_OK ||
      mimo_tx_get_codes(h, reinterpret_cast<float *>(_s0), nullptr) != MIMO_OK) {
    std::fprintf(stderr, "ofdmframe_init_S0: %s\n", mimo_last_error());
    std::exit(1);
  }
  mimo_tx_destroy(h);
}

void ofdmframe_init_S1(const unsigned char *_p, unsigned int _M, unsigned int _num_access_codes,
                       std::complex<float> *_S1, std::complex<float> *_s1, msequence ms) {
  std::vector<unsigned char> b0(_M, 0), b1((size_t)_M * _num_access_codes);
  for (unsigned int j = 0; j < _num_access_codes; j++)
    for (unsigned int i = 0; i < _M; i++) {
      const size_t o = (size_t)j * _M + i;
      b1[o] = (unsigned char)(msequence_generate_symbol(ms, 1) & 0x01);
      _S1[o] = (_p[i] == OFDMFRAME_SCTYPE_NULL) ? gr_complex(0.0f, 0.0f)
                                                : BPSK_CONSTELLATION[b1[o]];
    }
  std::vector<unsigned char> pp(_p, _p + _M);
  bool any_even = false;
  for (unsigned int i = 0; i < _M; i += 2) any_even |= (pp[i] != OFDMFRAME_SCTYPE_NULL);
  if (!any_even) pp[0] = OFDMFRAME_SCTYPE_DATA;   // S0 table is unused here
  mimo_tx *h = nullptr;
  if (mimo_tx_create(_M, 1, 1, _num_access_codes, pp.data(), b0.data(), b1.data(), &h) !=
          MIMO_OK ||
      mimo_tx_get_codes(h, nullptr, reinterpret_cast<float *>(_s1)) != MIMO_OK) {
    std::fprintf(stderr, "ofdmframe_init_S1: %s\n", mimo_last_error());
    std::exit(1);
  }
  mimo_tx_destroy(h);
}

float invert(std::vector<std::vector<gr_complex> > &W,
             std::vector<std::vector<gr_complex> > const &G) {
  // framing.cc:1344-1367, currently only for 2 x 2
  if (G.size() != 2 || W.size() != 2 || G[0].size() != 2 || G[1].size() != 2 ||
      W[0].size() != 2 || W[1].size() != 2) {
    std::fprintf(stderr, "invert: only 2 x 2 supported\n");
    std::abort();
  }
  gr_complex g[4] = {G[0][0], G[0][1], G[1][0], G[1][1]}, w[4];
  const float gain = mimo_invert2(reinterpret_cast<float *>(w), reinterpret_cast<float *>(g));
  W[0][0] = w[0];
  W[0][1] = w[1];
  W[1][0] = w[2];
  W[1][1] = w[3];
  return gain;
}

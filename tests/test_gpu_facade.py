"""The C++ drop-in boundary run for real on the GPU: a mimo/main.cc-style caller compiled with
g++ against include/framing.h (the reference's framing.h surface) and -lrub_mimo_amd.

The caller does what main.cc does (/root/reference/mimo/main.cc:1268-1315, 905-922):
liquid msequences, ofdmframe_init_default_sctype / validate, framegen, msequence_reset,
framesync with a callback, msequence_destroy, then one fs.execute(rx_buffer, n) over the
capture read back from per-channel raw files (the /tmp/rx<ch>.dat handoff). The test checks
get_sync_index, get_num_samples_processed, the plateau, the PID+2 callbacks and every
callback's symbols against the committed oracle fixture, plus framegen's sync words."""
import os
import subprocess

import numpy as np
import pytest

from oracle import ref
from rub_mimo_amd import _lib

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")

CALLER = r'''
#include "framing.h"
#include <cstdio>
#include <cstring>
#include <vector>

static FILE *sym_fp = NULL;
static unsigned int n_callbacks = 0;

// mimo_callback (framing.h:30-31): one call per decoded symbol, vectors valid during the call
void *callback(std::vector<gr_complex *> x, unsigned int occupied_carriers) {
  for (size_t i = 0; i < x.size(); i++)
    fwrite(x[i], sizeof(gr_complex), occupied_carriers, sym_fp);
  n_callbacks++;
  return NULL;
}

int main(int argc, char **argv) {
  if (argc != 5) return 2;
  const char *dir = argv[1];
  unsigned long n = strtoul(argv[2], NULL, 10);
  unsigned int M = FFT_SIZE, cp_len = CP_LEN, num_streams = NUM_STREAMS;
  unsigned char *p = (unsigned char *)malloc(M);
  ofdmframe_init_default_sctype(p, M);
  unsigned int M_null, M_pilot, M_data;
  ofdmframe_validate_sctype(p, M, &M_null, &M_pilot, &M_data);

  msequence ms_S0 = msequence_create(LFSR_SMALL_LENGTH, LFSR_SMALL_0_GEN_POLY, 1);
  std::vector<msequence> ms_S1(num_streams);
  ms_S1[0] = msequence_create(LFSR_LARGE_LENGTH, LFSR_LARGE_0_GEN_POLY, 1);
  ms_S1[1] = msequence_create(LFSR_LARGE_LENGTH, LFSR_LARGE_1_GEN_POLY, 1);

  rx_beamforming::framegen fg(M, cp_len, num_streams, NUM_ACCESS_CODES, p, ms_S0, ms_S1);
  msequence_reset(ms_S0);
  msequence_reset(ms_S1[0]);
  msequence_reset(ms_S1[1]);
  rx_beamforming::framesync fs(M, cp_len, num_streams, NUM_ACCESS_CODES, p, ms_S0, ms_S1,
                               callback);
  msequence_destroy(ms_S0);
  msequence_destroy(ms_S1[0]);
  msequence_destroy(ms_S1[1]);

  // framegen: the sync words of every tx stream (framing.cc:169-208)
  unsigned int sw_len = (NUM_ACCESS_CODES * num_streams + 1) * (M + cp_len);
  std::vector<gr_complex *> tx_buff(num_streams);
  for (unsigned int s = 0; s < num_streams; s++)
    tx_buff[s] = (gr_complex *)calloc(sw_len, sizeof(gr_complex));
  unsigned int n_sw = fg.write_sync_words(tx_buff);
  char path[512];
  snprintf(path, sizeof(path), "%s/tx_sync.dat", dir);
  FILE *tf = fopen(path, "wb");
  for (unsigned int s = 0; s < num_streams; s++) fwrite(tx_buff[s], sizeof(gr_complex), n_sw, tf);
  fclose(tf);

  // the rx worker's handoff (main.cc:905-918): read each channel's capture back, then one
  // execute over all of it (main.cc:922)
  std::vector<gr_complex *> rx_buffer(num_streams);
  for (unsigned int chan = 0; chan < num_streams; chan++) {
    snprintf(path, sizeof(path), "%s/rx%u.dat", dir, chan);
    FILE *fp = fopen(path, "rb");
    if (!fp) return 3;
    rx_buffer[chan] = (gr_complex *)malloc(sizeof(gr_complex) * n);
    if (fread(rx_buffer[chan], sizeof(gr_complex), n, fp) != n) return 4;
    fclose(fp);
  }
  sym_fp = fopen(argv[3], "wb");
  framesync_states_t st = fs.execute(rx_buffer, n);
  fclose(sym_fp);
  FILE *res = fopen(argv[4], "w");
  fprintf(res, "%d %lu %llu %u %u %lu %lu %lu %lu\n", (int)st, fs.get_sync_index(),
          fs.get_num_samples_processed(), n_callbacks, n_sw, fs.get_plateau_start(0),
          fs.get_plateau_end(0), fs.get_plateau_start(1), fs.get_plateau_end(1));
  fclose(res);
  std::vector<std::vector<std::vector<gr_complex> > > G = fs.get_G();
  printf("G[0][0][0] = %f %f\n", G[0][0][0].real(), G[0][0][0].imag());
  for (unsigned int chan = 0; chan < num_streams; chan++) {
    free(rx_buffer[chan]);
    free(tx_buff[chan]);
  }
  free(p);
  return 0;
}
'''


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible: the gpu tests need an MI355X")


def test_main_cc_style_caller_runs_framesync_on_golden_capture(tmp_path):
    g = dict(np.load(os.path.join(GOLD, "m64_2x2_zf2.npz"), allow_pickle=False))
    M, cp, N, nac, pid = (int(g[k]) for k in ("M", "cp", "N", "nac", "pid"))
    assert N == 2 and int(g["detector"]) == ref.DET_ZF2          # the facade's 2-stream detector
    assert np.array_equal(g["p"], ref.default_sctype(M))
    (tmp_path / "config.h").write_text('''
#ifndef CONFIG_H
#define CONFIG_H
#define FFT_SIZE %d
#define CP_LEN %d
#define NUM_STREAMS %d
#define LFSR_SMALL_LENGTH 12
#define LFSR_LARGE_LENGTH 13
#define LFSR_SMALL_0_GEN_POLY 010123
#define LFSR_LARGE_0_GEN_POLY 020033
#define LFSR_LARGE_1_GEN_POLY 020047
#define NUM_ACCESS_CODES %d
#define PID_MAX %d
#define PLATEAU_THREASHOLD 0.95
#define SISO false
#endif
''' % (M, cp, N, nac, pid))
    src = tmp_path / "main_like.cc"
    src.write_text(CALLER)
    exe = tmp_path / "main_like"
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-I", str(tmp_path), "-I",
                           os.path.join(ROOT, "include"), str(src), "-o", str(exe),
                           "-L", libdir, "-lrub_mimo_amd", "-Wl,-rpath," + libdir])
    rx = np.ascontiguousarray(g["rx"], np.complex64)
    for ch in range(N):
        rx[ch].tofile(tmp_path / ("rx%d.dat" % ch))
    sym_path, res_path = tmp_path / "rx_sig.dat", tmp_path / "res.txt"
    subprocess.check_call([str(exe), str(tmp_path), str(rx.shape[1]), str(sym_path),
                           str(res_path)], timeout=120)
    st, si, nsp, ncb, nsw, ps0, pe0, ps1, pe1 = (int(v) for v in res_path.read_text().split())
    assert st == ref.STATE_MIMO
    assert si == int(g["sync_index"])
    assert nsp == int(g["num_samples_processed"])
    assert [ps0, ps1] == list(g["plateau_start"]) and [pe0, pe1] == list(g["plateau_end"])
    want = g["symbols"]                                        # [PID+2][N][M_occ]
    assert ncb == want.shape[0] == pid + 2
    got = np.fromfile(sym_path, np.complex64).reshape(want.shape)
    d = np.sqrt(np.sum(np.abs(got - want) ** 2) / np.sum(np.abs(want) ** 2))
    assert d <= 1e-4, d
    # framegen sync words: S0 (with cyclic prefix) on stream 0 first (framing.cc:169-208)
    SL = M + cp
    assert nsw == (nac * N + 1) * SL
    tx = np.fromfile(tmp_path / "tx_sync.dat", np.complex64).reshape(N, nsw)
    s0b, s1b = ref.code_bits(M, N, nac, (0o20033, 0o20047))
    _, s0 = ref.init_S0(g["p"], s0b)
    assert np.abs(tx[0, cp:SL] - s0).max() < 1e-5
    assert np.array_equal(tx[0, :cp], tx[0, M:SL])
    # then S1 in TDMA: code c of stream t in slot 1 + c*N + t, zeros elsewhere on the others
    for t in range(N):
        _, s1 = ref.init_S1(g["p"], nac, s1b[t * nac * M:(t + 1) * nac * M])
        for c in range(nac):
            b = SL * (1 + c * N + t)
            assert np.abs(tx[t, b + cp:b + SL] - s1[c]).max() < 1e-5, (t, c)
            assert not np.any(tx[1 - t, b:b + SL]), (t, c)

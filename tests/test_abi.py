"""CPU-side checks of the drop-in boundary: the C-ABI library loads, exports every function
declared in include/*.h, and its host-only helpers agree with the oracle. No GPU calls."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from oracle import codes as ocodes
from oracle import ref
from rub_mimo_amd import _lib
from rub_mimo_amd import framing as fr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions(path):
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    txt = re.sub(r"//[^\n]*", "", txt)
    names = set()
    for m in re.finditer(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\(", txt):
        names.add(m.group(1))
    return names


def test_library_exports_every_c_abi_symbol():
    L = _lib.lib()
    declared = {n for n in header_functions(os.path.join(ROOT, "include", "mimo_rx.h"))
                if n.startswith("mimo_")}
    assert len(declared) >= 40
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = sorted(declared - exported)
    assert not missing, missing
    # the ctypes table covers the same set
    assert declared == set(_lib.SIGNATURES)
    for name in declared:
        assert getattr(L, name) is not None


def test_facade_symbols_exported():
    out = subprocess.check_output(["nm", "-DC", "--defined-only", _lib.LIB_PATH], text=True)
    for sym in ("ofdmframe_init_default_sctype", "ofdmframe_validate_sctype",
                "ofdmframe_print_sctype", "ofdmframe_init_S0", "ofdmframe_init_S1", "invert(",
                "rmimo_msequence_create", "rmimo_msequence_generate_symbol",
                "BPSK_CONSTELLATION", "QPSK_CONSTELLATION"):
        assert sym in out, sym


def test_library_is_gfx950():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob       # device code object for MI355X
    assert b"amdgcn-amd-amdhsa--gfx942" not in blob   # and nothing else


def test_version_string():
    assert b"gfx950" in _lib.lib().mimo_version()


def test_sctype_helpers_match_oracle():
    for M in (64, 1024, 2048):
        assert np.array_equal(fr.ofdmframe_init_default_sctype(M), ref.default_sctype(M))
        assert np.array_equal(fr.ofdmframe_init_liquid_sctype(M), ref.liquid_sctype(M))
        assert fr.ofdmframe_validate_sctype(ref.liquid_sctype(M)) == \
            ref.validate_sctype(ref.liquid_sctype(M))
    with pytest.raises(ValueError):
        fr.ofdmframe_validate_sctype(np.array([0, 1, 5], np.uint8))
    assert fr.ofdmframe_print_sctype(np.array([2, 2, 0, 1], np.uint8)) == "[.|++]"


def test_msequence_shim_matches_liquid_semantics():
    assert fr.S1_POLYS == ocodes.S1_POLYS
    for m, g in [(12, fr.LFSR_SMALL_0_GEN_POLY)] + [(13, g) for g in fr.S1_POLYS]:
        ms = fr.msequence_create(m, g, 1)
        bits = ms.draw_bits(300)
        assert np.array_equal(bits, ref.draw_bits(m, g, 1, 300))
        # the generator advanced exactly as 300 generate_symbol(1) calls would
        ms2 = fr.msequence_create(m, g, 1)
        for _ in range(300):
            ms2.generate_symbol(1)
        assert ms.v == ms2.v
        more = ms.draw_bits(17)
        assert np.array_equal(more, ref.draw_bits(m, g, 1, 317)[300:])
        fr.msequence_reset(ms)
        assert ms.v == ms.a


def test_invert2_matches_oracle():
    rng = np.random.default_rng(1)
    for _ in range(20):
        G = (rng.standard_normal((2, 2)) + 1j * rng.standard_normal((2, 2))).astype(np.complex64)
        W, g = fr.invert(G)
        Wr, gr = ref.invert2(G)
        assert np.array_equal(W, Wr) and g == gr


def test_struct_layouts(tmp_path):
    """Every ctypes mirror matches the C header field for field (offsets and sizes from a
    compiled probe of include/mimo_rx.h)."""
    structs = {"mimo_frame_result": _lib.FrameResult, "mimo_batch": _lib.Batch,
               "mimo_rx_config": _lib.RxConfig, "mimo_synth_config": _lib.SynthConfig}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "mimo_rx.h"', 'int main(void) {']
    for cname, py in structs.items():
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for fname, _ in py._fields_:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, fname, cname, fname))
    lines.append("return 0; }")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = dict(l.split() for l in subprocess.check_output([str(exe)]).decode().splitlines())
    for cname, py in structs.items():
        assert int(got[cname]) == C.sizeof(py), cname
        for fname, _ in py._fields_:
            assert int(got["%s.%s" % (cname, fname)]) == getattr(py, fname).offset, (cname, fname)


def test_error_path_without_gpu_is_loud():
    """Creating a receiver on a machine without a GPU fails with an error, never a fallback."""
    if _lib.device_count() > 0:
        pytest.skip("GPU present: covered by the gpu tests")
    from rub_mimo_amd.receiver import Receiver, RxParams
    with pytest.raises(_lib.MimoError):
        Receiver(RxParams(M=64, cp_len=16, num_streams=2, num_access_codes=4, pid_max=8))


def test_facade_header_compiles_like_main_cc(tmp_path):
    """A main.cc-style caller compiles and links against include/framing.h + the library."""
    src = tmp_path / "caller.cc"
    src.write_text(r'''
#include "framing.h"
#include <cstdio>
static unsigned calls = 0;
void *callback(std::vector<gr_complex *> x, unsigned int occ) { calls++; (void)x; (void)occ; return NULL; }
int main() {
  unsigned int M = 64, cp = 16, N = 2;
  unsigned char *p = (unsigned char *)malloc(M);
  ofdmframe_init_default_sctype(p, M);
  unsigned int a, b, c;
  ofdmframe_validate_sctype(p, M, &a, &b, &c);
  msequence ms_S0 = msequence_create(LFSR_SMALL_LENGTH, LFSR_SMALL_0_GEN_POLY, 1);
  std::vector<msequence> ms_S1(2);
  ms_S1[0] = msequence_create(LFSR_LARGE_LENGTH, LFSR_LARGE_0_GEN_POLY, 1);
  ms_S1[1] = msequence_create(LFSR_LARGE_LENGTH, LFSR_LARGE_1_GEN_POLY, 1);
  if (argc_dummy()) {
    rx_beamforming::framegen fg(M, cp, N, NUM_ACCESS_CODES, p, ms_S0, ms_S1);
    msequence_reset(ms_S0); msequence_reset(ms_S1[0]); msequence_reset(ms_S1[1]);
    rx_beamforming::framesync fs(M, cp, N, NUM_ACCESS_CODES, p, ms_S0, ms_S1, callback);
    std::vector<gr_complex *> buf(2);
    fs.execute(buf, 0);
    printf("%lu %llu\n", fs.get_sync_index(), fs.get_num_samples_processed());
  }
  std::vector<std::vector<gr_complex> > W(2, std::vector<gr_complex>(2)), G(2, std::vector<gr_complex>(2, 1.0f));
  G[0][1] = 0.5f;
  printf("%f\n", invert(W, G));
  return 0;
}
''')
    cfg = tmp_path / "config.h"
    cfg.write_text('''
#ifndef CONFIG_H
#define CONFIG_H
#define LFSR_SMALL_LENGTH 12
#define LFSR_LARGE_LENGTH 13
#define LFSR_SMALL_0_GEN_POLY 010123
#define LFSR_LARGE_0_GEN_POLY 020033
#define LFSR_LARGE_1_GEN_POLY 020047
#define NUM_ACCESS_CODES 4
#define PID_MAX 8
#define PLATEAU_THREASHOLD 0.95
#define SISO false
static inline int argc_dummy() { return 0; }
#endif
''')
    exe = tmp_path / "caller"
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-I", str(tmp_path), "-I",
                           os.path.join(ROOT, "include"), str(src), "-o", str(exe),
                           "-L", libdir, "-lrub_mimo_amd", "-Wl,-rpath," + libdir])
    out = subprocess.check_output([str(exe)], text=True)
    assert abs(float(out.split()[-1]) - 1.0 / abs(1 - 0.5) ** 2) < 1e-5


def test_ingest_sc16_argument_errors_without_gpu():
    L = _lib.lib()
    assert L.mimo_ingest_sc16(None, 0, None, 0, 0, 0, 1.0, None) == 0       # empty: no-op
    assert L.mimo_ingest_sc16(None, 8, None, 8, 2, 8, 1.0, None) == -1      # null buffers
    assert L.mimo_ingest_sc16(16, 4, 16, 8, 2, 8, 1.0, None) == -1          # rows overlap
    assert b"stride" in L.mimo_last_error()


def test_cfo_argument_errors_without_gpu():
    L = _lib.lib()
    eps = (C.c_double * 3)()
    assert L.mimo_cfo_estimate(None, 0, 2, 0, 64, eps, None) == -1          # null rows
    assert L.mimo_cfo_estimate(16, 64, 2, 0, 63, eps, None) == -1           # odd M
    assert L.mimo_cfo_estimate(16, 64, 2, 8, 64, eps, None) == -1           # window past stride
    assert b"stride" in L.mimo_last_error()
    assert L.mimo_cfo_derotate(None, 0, 0, 0, 0, 0.1, 64, None) == 0        # empty: no-op
    assert L.mimo_cfo_derotate(16, 10, 2, 20, 0, 0.1, 64, None) == -1       # stride < n


def test_capture_ring_arguments_and_no_gpu_error():
    """mimo_ring_create validates its geometry, and without a GPU (no pinned host memory)
    fails with an error instead of handing out pageable buffers."""
    from rub_mimo_amd.ring import CaptureRing
    for bad in ((0, 1024, 2), (9, 1024, 2), (4, 0, 2), (4, 1024, 0)):
        with pytest.raises(_lib.MimoError):
            CaptureRing(*bad)
    if _lib.device_count() == 0:
        with pytest.raises(_lib.MimoError):
            CaptureRing(4, 1024, 2)

"""Python mirror of the reference framing API (/root/reference/mimo/framing.h), backed by the
HIP library. Names, argument meaning and error behaviour follow the reference so tests read
like mimo/main.cc:

    p = ofdmframe_init_default_sctype(M)
    ms_S0 = msequence_create(LFSR_SMALL_LENGTH, LFSR_SMALL_0_GEN_POLY, 1)
    ms_S1 = [msequence_create(LFSR_LARGE_LENGTH, g, 1) for g in s1_polynomials(N)]
    fs = framesync(M, cp_len, N, NUM_ACCESS_CODES, p, ms_S0, ms_S1, callback)
    state = fs.execute(rx_buffer, num_samples)        # framing.cc:471-506

Invalid subcarrier types raise ValueError where the reference exit(1)s
(framing.cc:1020-1022); GPU errors raise MimoError.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, lib

# config.h constants (mimo/config.h:65-114)
NUM_SUBCARRIERS = 2048
CP_LENGTH = 152
LFSR_SMALL_LENGTH = 12
LFSR_LARGE_LENGTH = 13
LFSR_SMALL_0_GEN_POLY = 0o10123
LFSR_SMALL_1_GEN_POLY = 0o10151
LFSR_LARGE_0_GEN_POLY = 0o20033
LFSR_LARGE_1_GEN_POLY = 0o20047
PLATEAU_THREASHOLD = 0.95
PID_MAX = 1000
NUM_ACCESS_CODES = 20
NUM_STREAMS = 2
BASEBAND_GAIN = 0.25

# degree-13 generators for S1 of streams 0..7: the two of config.h:74-75, then the next
# ascending polynomials whose m-sequence has full period 8191 (tests verify the period)
S1_POLYS = (0o20033, 0o20047, 0o20065, 0o20123, 0o20145, 0o20157, 0o20213, 0o20215)

OFDMFRAME_SCTYPE_NULL, OFDMFRAME_SCTYPE_PILOT, OFDMFRAME_SCTYPE_DATA = 0, 1, 2
STATE_SEEK_PLATEAU = _lib.STATE_SEEK_PLATEAU
STATE_SAVE_ACCESS_CODES = _lib.STATE_SAVE_ACCESS_CODES
STATE_WAIT = _lib.STATE_WAIT
STATE_MIMO = _lib.STATE_MIMO
DET_ZF2, DET_ZF, DET_MMSE, DET_SISO = _lib.DET_ZF2, _lib.DET_ZF, _lib.DET_MMSE, _lib.DET_SISO


def s1_polynomials(n):
    if n > len(S1_POLYS):
        raise ValueError("at most %d streams" % len(S1_POLYS))
    return S1_POLYS[:n]


# ---------------------------------------------------------------------- liquid msequence
class msequence:
    """liquid-dsp msequence semantics (g >>= 1, bit-reversed initial state); host setup."""

    def __init__(self, m, g, a=1):
        if not 2 <= m <= 31:
            raise ValueError("msequence m out of range")
        self.m, self.g = m, g >> 1
        v = 0
        for _ in range(m):
            v = (v << 1) | (a & 1)
            a >>= 1
        self.a = v
        self.n = (1 << m) - 1
        self.v = self.a

    def advance(self):
        b = bin(self.v & self.g).count("1") & 1
        self.v = ((self.v << 1) | b) & self.n
        return b

    def generate_symbol(self, bps):
        s = 0
        for _ in range(bps):
            s = (s << 1) | self.advance()
        return s

    def draw_bits(self, count):
        """count x generate_symbol(1) & 1 through the C helper, advancing this generator
        exactly as the reference constructors advance the caller's msequence."""
        out = np.zeros(count, np.uint8)
        a, x = 0, self.v           # the helper bit-reverses its seed: pass reverse(v)
        for _ in range(self.m):
            a = (a << 1) | (x & 1)
            x >>= 1
        check(lib().mimo_msequence_draw_bits(self.m, self.g << 1, a, count, out.ctypes.data),
              "msequence draw")
        v = self.v
        for b in out[-self.m:] if count >= self.m else out:
            v = ((v << 1) | int(b)) & self.n
        self.v = v
        return out

    def reset(self):
        self.v = self.a


def msequence_create(m, g, a=1):
    return msequence(m, g, a)


def msequence_reset(ms):
    ms.reset()


def msequence_generate_symbol(ms, bps):
    return ms.generate_symbol(bps)


# ---------------------------------------------------------------------- sctype helpers
def ofdmframe_init_default_sctype(M):
    p = np.zeros(M, np.uint8)
    check(lib().mimo_sctype_default(p.ctypes.data, M), "sctype_default")
    return p


def ofdmframe_init_liquid_sctype(M):
    """The guard/pilot allocation compiled out under USE_ALL_CARRIERS (framing.cc:956-997)."""
    p = np.zeros(M, np.uint8)
    check(lib().mimo_sctype_liquid(p.ctypes.data, M), "sctype_liquid")
    return p


def ofdmframe_validate_sctype(p):
    p = np.ascontiguousarray(p, np.uint8)
    a, b, c = C.c_uint32(), C.c_uint32(), C.c_uint32()
    if lib().mimo_sctype_validate(p.ctypes.data, len(p), C.byref(a), C.byref(b), C.byref(c)):
        raise ValueError("ofdmframe_validate_sctype(), invalid subcarrier type")
    return a.value, b.value, c.value


def ofdmframe_print_sctype(p):
    M = len(p)
    ch = {0: ".", 1: "|", 2: "+"}
    return "[" + "".join(ch[int(p[(i + M // 2) % M])] for i in range(M)) + "]"


def invert(G):
    """2x2 invert of framing.cc:1344-1367: returns (W, gain) with W*gain = G^-1."""
    G = np.ascontiguousarray(G, np.complex64).reshape(4)
    if G.size != 4:
        raise ValueError("invert: currently only for 2 x 2 matrix")
    W = np.zeros(4, np.complex64)
    gain = lib().mimo_invert2(W.ctypes.data, G.ctypes.data)
    return W.reshape(2, 2), float(gain)


def _draw_codes(M, N, nac, ms_S0, ms_S1, s1_first):
    if s1_first:   # framesync ctor: S1 per stream (framing.cc:374-379) then S0 (:411-415)
        b1 = np.concatenate([ms_S1[i].draw_bits(nac * M) for i in range(N)])
        b0 = ms_S0.draw_bits(M)
    else:          # framegen ctor: S0 (framing.cc:110) then S1 per stream (:141-146)
        b0 = ms_S0.draw_bits(M)
        b1 = np.concatenate([ms_S1[i].draw_bits(nac * M) for i in range(N)])
    return b0, b1


# ---------------------------------------------------------------------- framegen
class framegen:
    """rx_beamforming::framegen (framing.h:42-103) on the GPU transmitter kernels."""

    def __init__(self, M, cp_len, num_streams, num_access_codes, p, ms_S0, ms_S1):
        self.M, self.cp_len, self.num_streams, self.num_access_codes = (
            M, cp_len, num_streams, num_access_codes)
        self.symbol_len = M + cp_len
        self.p = np.ascontiguousarray(p, np.uint8).copy()
        self.M_null, self.M_pilot, self.M_data = ofdmframe_validate_sctype(self.p)
        b0, b1 = _draw_codes(M, num_streams, num_access_codes, ms_S0, ms_S1, s1_first=False)
        h = C.c_void_p()
        check(lib().mimo_tx_create(M, cp_len, num_streams, num_access_codes, self.p.ctypes.data,
                                   b0.ctypes.data, b1.ctypes.data, C.byref(h)), "framegen")
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            lib().mimo_tx_destroy(self._h)
            self._h = None

    def get_num_streams(self):
        return self.num_streams

    def write_sync_words(self, tx_buff=None):
        """framing.cc:169-208. Returns (count, buffers[N, (nac*N+1)*SL])."""
        n = (self.num_access_codes * self.num_streams + 1) * self.symbol_len
        if tx_buff is None:
            tx_buff = np.zeros((self.num_streams, n), np.complex64)
        ptrs = (C.c_void_p * self.num_streams)(*[tx_buff[i].ctypes.data
                                                 for i in range(self.num_streams)])
        cnt = C.c_uint32()
        check(lib().mimo_tx_write_sync_words(self._h, ptrs, C.byref(cnt)), "write_sync_words")
        return cnt.value, tx_buff

    def assemble_mimo_packet(self, in_buff, tx_buff=None):
        """framing.cc:210-235: in_buff[N, M_occ] symbols -> (SL, tx_buff[N, SL])."""
        N = self.num_streams
        ins = [np.ascontiguousarray(in_buff[i], np.complex64) for i in range(N)]
        if tx_buff is None:
            tx_buff = np.zeros((N, self.symbol_len), np.complex64)
        tp = (C.c_void_p * N)(*[tx_buff[i].ctypes.data for i in range(N)])
        ip = (C.c_void_p * N)(*[x.ctypes.data for x in ins])
        cnt = C.c_uint32()
        check(lib().mimo_tx_assemble_mimo_packet(self._h, tp, ip, C.byref(cnt)),
              "assemble_mimo_packet")
        return cnt.value, tx_buff

    def codes(self):
        """Time-domain S0 [M] and S1 [N, nac, M] (ofdmframe_init_S0/S1 outputs)."""
        s0 = np.zeros(self.M, np.complex64)
        s1 = np.zeros((self.num_streams, self.num_access_codes, self.M), np.complex64)
        check(lib().mimo_tx_get_codes(self._h, s0.ctypes.data, s1.ctypes.data), "codes")
        return s0, s1

    def print(self):
        return ("ofdmframegen:\n    num subcarriers     :   %u\n      - NULL            :   %u\n"
                "      - pilot           :   %u\n      - data            :   %u\n"
                "    cyclic prefix len   :   %u\n    %s" % (
                    self.M, self.M_null, self.M_pilot, self.M_data, self.cp_len,
                    ofdmframe_print_sctype(self.p)))


# ---------------------------------------------------------------------- framesync
class framesync:
    """rx_beamforming::framesync (framing.h:105-213): streaming receiver on the GPU.

    callback(x, occupied_carriers) receives a list of N complex64 arrays (one per stream),
    valid during the call (framing.cc:587). Extra keyword arguments expose the config.h
    switches and the build's extensions (detector, MMSE noise variance, QAM order)."""

    def __init__(self, M, cp_len, num_streams, num_access_codes, p, ms_S0, ms_S1,
                 callback=None, pid_max=PID_MAX, detector=None, noise_var=-1.0,
                 keep_identity_bias=True, siso_tx=0, siso_rx=0,
                 plateau_threshold=PLATEAU_THREASHOLD, qam_order=4):
        self.M, self.cp_len, self.num_streams, self.num_access_codes = (
            M, cp_len, num_streams, num_access_codes)
        self.symbol_len = M + cp_len
        self.p = np.ascontiguousarray(p, np.uint8).copy()
        self.M_null, self.M_pilot, self.M_data = ofdmframe_validate_sctype(self.p)
        self.M_occupied = self.M_pilot + self.M_data
        if detector is None:
            detector = DET_ZF2 if num_streams == 2 else DET_ZF
        b0, b1 = _draw_codes(M, num_streams, num_access_codes, ms_S0, ms_S1, s1_first=True)
        cfg = _lib.RxConfig(M, cp_len, num_streams, num_access_codes, pid_max,
                            self.p.ctypes.data, b0.ctypes.data, b1.ctypes.data, detector,
                            noise_var, 1 if keep_identity_bias else 0, siso_tx, siso_rx,
                            plateau_threshold, qam_order)
        h = C.c_void_p()
        check(lib().mimo_rx_create(C.byref(cfg), None, C.byref(h)), "framesync")
        self._h = h
        self.callback = callback
        self._cb = _lib.SYMBOL_CB(self._bridge)
        check(lib().mimo_rx_set_callback(self._h, self._cb, None), "set_callback")

    def _bridge(self, eq, n, m_occ, user):
        if self.callback is None:
            return
        xs = [np.ctypeslib.as_array(eq[i], shape=(m_occ * 2,)).view(np.complex64)
              for i in range(n)]
        self.callback(xs, m_occ)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().mimo_rx_destroy(self._h)
            self._h = None

    def execute(self, in_buff, num_samples=None):
        bufs = [np.ascontiguousarray(b, np.complex64) for b in in_buff]
        if len(bufs) != self.num_streams:
            raise ValueError("in_buff must hold num_streams arrays")
        if num_samples is None:
            num_samples = len(bufs[0])
        ptrs = (C.c_void_p * self.num_streams)(*[b.ctypes.data for b in bufs])
        st = C.c_int32()
        check(lib().mimo_rx_execute(self._h, ptrs, self.num_streams, num_samples, C.byref(st)),
              "framesync::execute")
        return st.value

    def reset(self):
        check(lib().mimo_rx_reset(self._h), "reset")

    def set_debug_log(self, directory):
        """DEBUG_LOG (mimo/config.h:84-86): write the reference's f_sc_<k>.dat and
        corr_<k>_<ac>.dat traces into `directory` (None: off), the files mimo/apps/plot.py
        reads (mimo_rx_set_debug_log)."""
        d = None if directory is None else str(directory).encode()
        check(lib().mimo_rx_set_debug_log(self._h, d), "set_debug_log")

    def stream_capacity(self):
        """(device capture capacity, samples held) per antenna of the streaming execute
        (mimo_rx_get_stream_capacity; diagnostic)."""
        cap, held = C.c_uint64(), C.c_uint64()
        check(lib().mimo_rx_get_stream_capacity(self._h, C.byref(cap), C.byref(held)),
              "stream_capacity")
        return cap.value, held.value

    def set_siso_tx(self, tx):
        self._siso = (tx, getattr(self, "_siso", (0, 0))[1])
        check(lib().mimo_rx_set_siso(self._h, *self._siso), "set_siso_tx")

    def set_siso_rx(self, rx):
        self._siso = (getattr(self, "_siso", (0, 0))[0], rx)
        check(lib().mimo_rx_set_siso(self._h, *self._siso), "set_siso_rx")

    def estimate_channel(self):
        """Runs inside execute() once the access-code window is complete (framing.cc:649)."""

    def compute_receive_beamformer(self):
        """Empty in the reference (framing.cc:898-900)."""

    def get_state(self):
        st = C.c_int32()
        check(lib().mimo_rx_get_state(self._h, C.byref(st)), "get_state")
        return st.value

    def get_sync_index(self):
        v = C.c_uint64()
        check(lib().mimo_rx_get_sync_index(self._h, C.byref(v)), "get_sync_index")
        return v.value

    def get_num_samples_processed(self):
        v = C.c_uint64()
        check(lib().mimo_rx_get_num_samples_processed(self._h, C.byref(v)), "nsp")
        return v.value

    def get_plateau_start(self, stream):
        s, e = C.c_uint64(), C.c_uint64()
        check(lib().mimo_rx_get_plateau(self._h, stream, C.byref(s), C.byref(e)), "plateau")
        return s.value

    def get_plateau_end(self, stream):
        s, e = C.c_uint64(), C.c_uint64()
        check(lib().mimo_rx_get_plateau(self._h, stream, C.byref(s), C.byref(e)), "plateau")
        return e.value

    def get_G(self):
        G = np.zeros((self.M, self.num_streams, self.num_streams), np.complex64)
        check(lib().mimo_rx_get_G(self._h, G.ctypes.data), "get_G")
        return G

    def get_W(self):
        W = np.zeros((self.M, self.num_streams, self.num_streams), np.complex64)
        check(lib().mimo_rx_get_W(self._h, W.ctypes.data), "get_W")
        return W

    def get_gain(self):
        g = np.zeros(self.M_occupied, np.float32)
        check(lib().mimo_rx_get_gain(self._h, g.ctypes.data), "get_gain")
        return g

    def get_noise_var(self):
        v = C.c_float()
        check(lib().mimo_rx_get_noise_var(self._h, C.byref(v)), "noise_var")
        return v.value

    def get_corr(self):
        N = self.num_streams
        ci = np.zeros((N, N * self.num_access_codes), np.uint32)
        si = np.zeros(N, np.uint32)
        check(lib().mimo_rx_get_corr(self._h, ci.ctypes.data, si.ctypes.data), "get_corr")
        return ci, si

    def print(self):
        return ("ofdmframegen:\n    num subcarriers     :   %u\n      - NULL            :   %u\n"
                "      - pilot           :   %u\n      - data            :   %u\n"
                "    cyclic prefix len   :   %u\n    %s" % (
                    self.M, self.M_null, self.M_pilot, self.M_data, self.cp_len,
                    ofdmframe_print_sctype(self.p)))

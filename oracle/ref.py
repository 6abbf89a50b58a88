"""oracle/ref.py -- TEST INFRASTRUCTURE ONLY: ctypes binding of the C oracle (libmimo_ref.so).

The oracle is the CPU restatement of /root/reference/mimo/framing.cc (see mimo_ref.h).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker; the product (rub_mimo_amd) never touches it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libmimo_ref.so")
_lib = None

STATE_SEEK_PLATEAU, STATE_SAVE_ACCESS_CODES, STATE_WAIT, STATE_MIMO = 0, 1, 2, 3
DET_ZF2, DET_ZF, DET_MMSE, DET_SISO = 0, 1, 2, 3


def build():
    """Compile the oracle with its Makefile (gcc, -ffp-contract=off)."""
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = C.CDLL(_SO)
        u8p, u32p, f32p, f64p, u64p = (C.POINTER(C.c_uint8), C.POINTER(C.c_uint32),
                                       C.POINTER(C.c_float), C.POINTER(C.c_double),
                                       C.POINTER(C.c_uint64))
        vp = C.c_void_p
        sig = {
            "ref_msequence_period": (C.c_uint64, [C.c_uint32, C.c_uint32, C.c_uint32]),
            "ref_msequence_draw_bits": (None, [C.c_uint32] * 4 + [u8p]),
            "ref_init_default_sctype": (None, [u8p, C.c_uint32]),
            "ref_init_liquid_sctype": (None, [u8p, C.c_uint32]),
            "ref_validate_sctype": (C.c_int, [u8p, C.c_uint32, u32p, u32p, u32p]),
            "ref_fft": (None, [vp, C.c_uint32, C.c_int]),
            "ref_init_S0": (None, [u8p, C.c_uint32, u8p, vp, vp]),
            "ref_init_S1": (None, [u8p, C.c_uint32, C.c_uint32, u8p, vp, vp]),
            "ref_invert2": (C.c_float, [vp, vp]),
            "ref_qam_point": (_CF32, [C.c_uint32, C.c_uint32]),
            "ref_qam_demap": (C.c_uint32, [_CF32, C.c_uint32]),
            "ref_hash5": (C.c_uint64, [C.c_uint64] * 5),
            "ref_synth_frame_len": (C.c_uint64, [vp]),
            "ref_synth_frame": (C.c_uint64, [vp, u8p, u8p, u8p, vp, u8p, vp]),
            "ref_framesync_create": (vp, [vp, u8p, u8p, u8p]),
            "ref_framesync_destroy": (None, [vp]),
            "ref_framesync_execute": (C.c_int, [vp, vp, C.c_uint32]),
            "ref_framesync_reset": (None, [vp]),
            "ref_framesync_get_sync_index": (C.c_uint64, [vp]),
            "ref_framesync_get_num_samples_processed": (C.c_uint64, [vp]),
            "ref_framesync_get_plateau_start": (C.c_uint64, [vp, C.c_uint32]),
            "ref_framesync_get_plateau_end": (C.c_uint64, [vp, C.c_uint32]),
            "ref_framesync_get_state": (C.c_int, [vp]),
            "ref_framesync_get_corr": (None, [vp, u32p, f32p, u32p, f32p]),
            "ref_framesync_get_G": (None, [vp, vp]),
            "ref_framesync_get_W": (None, [vp, vp]),
            "ref_framesync_get_gain": (None, [vp, f32p]),
            "ref_framesync_get_noise_var": (C.c_float, [vp]),
            "ref_framesync_num_symbols": (C.c_uint32, [vp]),
            "ref_framesync_get_symbols": (None, [vp, vp, C.c_uint32]),
            "ref_framesync_sc_trace_len": (C.c_uint64, [vp]),
            "ref_framesync_get_sc_trace": (None, [vp, C.c_uint32, f32p]),
            "ref_framesync_M_occ": (C.c_uint32, [vp]),
            "ref_framesync_get_corr_trace": (C.c_int, [vp, f32p, f32p]),
            "ref_framesync_get_phase_times": (None, [vp, f64p]),
            "ref_framesync_get_cfo": (None, [vp, f64p]),
            "ref_framesync_skip_to_sync": (C.c_int, [vp, vp, C.c_uint64, C.c_uint64]),
            "ref_framesync_fast_forward": (C.c_int, [vp, vp, C.c_uint64]),
            "ref_sc_metric_at": (C.c_float, [vp, C.c_uint64, C.c_uint32]),
            "ref_demap_evm": (None, [vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                     u8p, u8p, f64p, f64p, u64p]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


class _CF32(C.Structure):
    _fields_ = [("re", C.c_float), ("im", C.c_float)]


class _SynthCfg(C.Structure):
    _fields_ = [("M", C.c_uint32), ("cp", C.c_uint32), ("N", C.c_uint32), ("nac", C.c_uint32),
                ("pid", C.c_uint32), ("qam", C.c_uint32), ("seed", C.c_uint64),
                ("frame", C.c_uint64), ("offset", C.c_int32), ("snr_db", C.c_float),
                ("tail_syms", C.c_uint32), ("identity_channel", C.c_int)]


class _RxCfg(C.Structure):
    _fields_ = [("M", C.c_uint32), ("cp", C.c_uint32), ("N", C.c_uint32), ("nac", C.c_uint32),
                ("pid_max", C.c_uint32), ("detector", C.c_int), ("noise_var", C.c_float),
                ("keep_identity_bias", C.c_int), ("siso_tx", C.c_uint32),
                ("siso_rx", C.c_uint32), ("threshold", C.c_double), ("trace_sc", C.c_int),
                ("trace_corr", C.c_int), ("search_mode", C.c_int), ("cfo_mode", C.c_int),
                ("qam", C.c_uint32)]


def _u8(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


def _vp(a):
    return C.c_void_p(a.ctypes.data)


# ------------------------------------------------------------------------------------
# reference configuration constants (mimo/config.h:70-75)
LFSR_SMALL_LENGTH, LFSR_LARGE_LENGTH = 12, 13
S0_POLY = 0o10123
S1_POLYS_REF = (0o20033, 0o20047)


def msequence_period(m, g, a=1):
    return int(lib().ref_msequence_period(m, g, a))


def draw_bits(m, g, a, count):
    out = np.zeros(count, np.uint8)
    lib().ref_msequence_draw_bits(m, g, a, count, _u8(out))
    return out


def default_sctype(M):
    p = np.zeros(M, np.uint8)
    lib().ref_init_default_sctype(_u8(p), M)
    return p


def liquid_sctype(M):
    p = np.zeros(M, np.uint8)
    lib().ref_init_liquid_sctype(_u8(p), M)
    return p


def validate_sctype(p):
    a, b, c = C.c_uint32(), C.c_uint32(), C.c_uint32()
    rc = lib().ref_validate_sctype(_u8(np.ascontiguousarray(p, np.uint8)), len(p),
                                   C.byref(a), C.byref(b), C.byref(c))
    if rc != 0:
        raise ValueError("invalid subcarrier type")
    return a.value, b.value, c.value


def fft(x, inverse=False):
    y = np.ascontiguousarray(x, np.complex64).copy()
    lib().ref_fft(_vp(y), len(y), 1 if inverse else 0)
    return y


def init_S0(p, bits):
    M = len(p)
    S0, s0 = np.zeros(M, np.complex64), np.zeros(M, np.complex64)
    lib().ref_init_S0(_u8(np.ascontiguousarray(p, np.uint8)), M,
                      _u8(np.ascontiguousarray(bits, np.uint8)), _vp(S0), _vp(s0))
    return S0, s0


def init_S1(p, nac, bits):
    M = len(p)
    S1, s1 = np.zeros(nac * M, np.complex64), np.zeros(nac * M, np.complex64)
    lib().ref_init_S1(_u8(np.ascontiguousarray(p, np.uint8)), M, nac,
                      _u8(np.ascontiguousarray(bits, np.uint8)), _vp(S1), _vp(s1))
    return S1.reshape(nac, M), s1.reshape(nac, M)


def invert2(G):
    G = np.ascontiguousarray(G, np.complex64).reshape(4)
    W = np.zeros(4, np.complex64)
    g = lib().ref_invert2(_vp(W), _vp(G))
    return W.reshape(2, 2), float(g)


def qam_point(index, order):
    r = lib().ref_qam_point(index, order)
    return complex(r.re, r.im)


def qam_demap(y, order):
    v = _CF32(np.float32(y.real), np.float32(y.imag))
    return int(lib().ref_qam_demap(v, order))


def hash5(seed, dom, a, b, c):
    return int(lib().ref_hash5(seed, dom, a, b, c))


def sc_metric_at(x, n, M):
    x = np.ascontiguousarray(x, np.complex64)
    return float(lib().ref_sc_metric_at(_vp(x), n, M))


def code_bits(M, N, nac, s1_polys):
    """msequence draws consumed by the framesync/framegen constructors (fresh generators)."""
    s0 = draw_bits(LFSR_SMALL_LENGTH, S0_POLY, 1, M)
    s1 = np.concatenate([draw_bits(LFSR_LARGE_LENGTH, s1_polys[t], 1, nac * M)
                         for t in range(N)])
    return s0, s1


# ------------------------------------------------------------------------------------
def synth_frame(M, cp, N, nac, pid, qam, seed, frame=0, offset=-1, snr_db=30.0,
                tail_syms=3, identity_channel=False, p=None, s1_polys=None):
    """Synthetic capture in the tx_worker layout; returns (rx[N,L], tx_idx[N,pid,Mocc], H)."""
    from oracle.codes import s1_polynomials
    if p is None:
        p = default_sctype(M)
    if s1_polys is None:
        s1_polys = s1_polynomials(N)
    s0b, s1b = code_bits(M, N, nac, s1_polys)
    cfg = _SynthCfg(M, cp, N, nac, pid, qam, seed, frame, offset, snr_db, tail_syms,
                    1 if identity_channel else 0)
    L = int(lib().ref_synth_frame_len(C.byref(cfg)))
    _, _, ndata = validate_sctype(p)
    npil = validate_sctype(p)[1]
    mocc = ndata + npil
    rx = np.zeros((N, L), np.complex64)
    ptrs = (C.c_void_p * N)(*[rx[i].ctypes.data for i in range(N)])
    tx_idx = np.zeros((N, pid, mocc), np.uint8)
    H = np.zeros((N, N), np.complex64)
    lib().ref_synth_frame(C.byref(cfg), _u8(np.ascontiguousarray(p, np.uint8)), _u8(s0b),
                          _u8(s1b), ptrs, _u8(tx_idx), _vp(H))
    return rx, tx_idx, H


class FrameSyncRef:
    """CPU restatement of rx_beamforming::framesync (framing.cc:268-944)."""

    def __init__(self, M, cp, N, nac, pid_max=1000, detector=DET_ZF2, noise_var=-1.0,
                 keep_identity_bias=True, siso_tx=0, siso_rx=0, threshold=0.95,
                 trace_sc=False, trace_corr=False, p=None, s1_polys=None, search_mode=0,
                 cfo_mode=0, qam=0):
        """search_mode 0: the reference's brute-force search (framing.cc:702-744); 1: the
        Parseval overlap-save variant (a CPU-baseline mode, labelled as such where used).
        cfo_mode (a build extension; the reference has no CFO step, framing.cc:486): 1 the CFO
        stages of the GPU's batched path, 2 the same plus the per-symbol common phase (needs
        qam, the order of the hard decision); see mimo_ref.c "Opt-in CFO"."""
        from oracle.codes import s1_polynomials
        self.M, self.cp, self.N, self.nac, self.pid_max = M, cp, N, nac, pid_max
        self.p = default_sctype(M) if p is None else np.ascontiguousarray(p, np.uint8)
        if s1_polys is None:
            s1_polys = s1_polynomials(N)
        s0b, s1b = code_bits(M, N, nac, s1_polys)
        cfg = _RxCfg(M, cp, N, nac, pid_max, detector, noise_var,
                     1 if keep_identity_bias else 0, siso_tx, siso_rx, threshold,
                     1 if trace_sc else 0, 1 if trace_corr else 0, int(search_mode),
                     int(cfo_mode), int(qam))
        self._h = lib().ref_framesync_create(C.byref(cfg), _u8(self.p), _u8(s0b), _u8(s1b))
        if not self._h:
            raise ValueError("ref_framesync_create failed")
        self.M_occ = int(lib().ref_framesync_M_occ(self._h))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().ref_framesync_destroy(self._h)
            self._h = None

    def execute(self, rx, n=None):
        rx = [np.ascontiguousarray(r, np.complex64) for r in rx]
        if n is None:
            n = len(rx[0])
        ptrs = (C.c_void_p * self.N)(*[r.ctypes.data for r in rx])
        return int(lib().ref_framesync_execute(self._h, ptrs, n))

    def reset(self):
        lib().ref_framesync_reset(self._h)

    def execute_from_sync(self, rx, trigger, sync_index):
        """CPU-baseline mode: skip the S&C scan (the plateau rule fired at `trigger`, e.g. as
        the GPU reported) and run search, LS, weights and decode on the rest of the capture.
        Same symbols as execute(rx) when trigger/sync_index are the real ones."""
        rx = [np.ascontiguousarray(r, np.complex64) for r in rx]
        ptrs = (C.c_void_p * self.N)(*[r.ctypes.data for r in rx])
        if lib().ref_framesync_skip_to_sync(self._h, ptrs, int(trigger), int(sync_index)) != 0:
            raise RuntimeError("skip_to_sync needs a fresh framesync")
        return self.execute([r[int(trigger) + 1:] for r in rx])

    def execute_from(self, rx, p0):
        """Test helper: S&C state advanced over samples [0, p0) without the per-sample dot
        products (ref_framesync_fast_forward: the metric from p0 on equals the full scan's bit
        for bit; no plateau run may be open at p0 - 1), then execute(rx[:, p0:])."""
        rx = [np.ascontiguousarray(r, np.complex64) for r in rx]
        ptrs = (C.c_void_p * self.N)(*[r.ctypes.data for r in rx])
        rc = lib().ref_framesync_fast_forward(self._h, ptrs, int(p0))
        if rc != 0:
            raise RuntimeError("fast_forward(%d) refused: %d" % (p0, rc))
        return self.execute([r[int(p0):] for r in rx])

    def cfo(self):
        """(eps0, delta) of the last estimate (cfo_mode != 0), subcarrier spacings."""
        e = np.zeros(2)
        lib().ref_framesync_get_cfo(self._h, e.ctypes.data_as(C.POINTER(C.c_double)))
        return float(e[0]), float(e[1])

    def phase_times(self):
        """Wall seconds per phase: S&C+plateau, search, LS+weights, replay decode."""
        t = np.zeros(4)
        lib().ref_framesync_get_phase_times(self._h, t.ctypes.data_as(C.POINTER(C.c_double)))
        return dict(zip(("sc", "search", "ls_weights", "decode"), t.tolist()))

    @property
    def state(self):
        return int(lib().ref_framesync_get_state(self._h))

    def get_sync_index(self):
        return int(lib().ref_framesync_get_sync_index(self._h))

    def get_num_samples_processed(self):
        return int(lib().ref_framesync_get_num_samples_processed(self._h))

    def get_plateau_start(self, s):
        return int(lib().ref_framesync_get_plateau_start(self._h, s))

    def get_plateau_end(self, s):
        return int(lib().ref_framesync_get_plateau_end(self._h, s))

    def get_corr(self):
        N, nac = self.N, self.nac
        ci = np.zeros((N, N * nac), np.uint32)
        cm = np.zeros((N, N * nac), np.float32)
        si = np.zeros(N, np.uint32)
        sm = np.zeros(N, np.float32)
        L = lib()
        L.ref_framesync_get_corr(self._h, ci.ctypes.data_as(C.POINTER(C.c_uint32)),
                                 cm.ctypes.data_as(C.POINTER(C.c_float)),
                                 si.ctypes.data_as(C.POINTER(C.c_uint32)),
                                 sm.ctypes.data_as(C.POINTER(C.c_float)))
        return ci, cm, si, sm

    def get_G(self):
        G = np.zeros((self.M, self.N, self.N), np.complex64)
        lib().ref_framesync_get_G(self._h, _vp(G))
        return G

    def get_W(self):
        W = np.zeros((self.M, self.N, self.N), np.complex64)
        lib().ref_framesync_get_W(self._h, _vp(W))
        return W

    def get_gain(self):
        g = np.zeros(self.M_occ, np.float32)
        lib().ref_framesync_get_gain(self._h, g.ctypes.data_as(C.POINTER(C.c_float)))
        return g

    def get_noise_var(self):
        return float(lib().ref_framesync_get_noise_var(self._h))

    def symbols(self):
        """All callback payloads: [n_callbacks, N, M_occ] complex64."""
        n = int(lib().ref_framesync_num_symbols(self._h))
        out = np.zeros((n, self.N, self.M_occ), np.complex64)
        if n:
            lib().ref_framesync_get_symbols(self._h, _vp(out), n)
        return out

    def corr_trace(self):
        """Search metrics by lag: (corr [N, N*nac, SL], s0 [N, SL]) (DEBUG_LOG corr files)."""
        SL = self.M + self.cp
        c = np.zeros((self.N, self.N * self.nac, SL), np.float32)
        s = np.zeros((self.N, SL), np.float32)
        rc = lib().ref_framesync_get_corr_trace(self._h, c.ctypes.data_as(C.POINTER(C.c_float)),
                                                s.ctypes.data_as(C.POINTER(C.c_float)))
        if rc != 0:
            raise RuntimeError("corr trace not recorded (trace_corr=False or no estimate yet)")
        return c, s

    def sc_trace(self, s):
        n = int(lib().ref_framesync_sc_trace_len(self._h))
        out = np.zeros(n, np.float32)
        if n:
            lib().ref_framesync_get_sc_trace(self._h, s, out.ctypes.data_as(C.POINTER(C.c_float)))
        return out


def demap_evm(sym, qam, tx_idx=None):
    """sym [n_sym, N, M_occ]; tx_idx [N, n_sym, M_occ] or None.
    Returns (rx_idx [N, n_sym, M_occ], evm_num[N], evm_den[N], errors[N])."""
    sym = np.ascontiguousarray(sym, np.complex64)
    n_sym, N, mocc = sym.shape
    rx_idx = np.zeros((N, n_sym, mocc), np.uint8)
    num, den = np.zeros(N), np.zeros(N)
    err = np.zeros(N, np.uint64)
    txp = _u8(np.ascontiguousarray(tx_idx, np.uint8)) if tx_idx is not None else None
    lib().ref_demap_evm(_vp(sym), n_sym, N, mocc, qam, txp, _u8(rx_idx),
                        num.ctypes.data_as(C.POINTER(C.c_double)),
                        den.ctypes.data_as(C.POINTER(C.c_double)),
                        err.ctypes.data_as(C.POINTER(C.c_uint64)))
    return rx_idx, num, den, err


def stream_ref(rx, M, cp, N, nac, pid_max=1000, max_frames=None, **kw):
    """Back-to-back frames in one capture, received the way a caller of the reference API
    would: a fresh framesync (framing.cc:268-436) is constructed for the samples after each
    frame, starting at origin r_{k+1} = r_k + get_num_samples_processed() (framing.cc:471-506;
    the reference's own STATE_MIMO is terminal, :494-496, and reset() keeps stale filter
    state, :461-464). Positions in each record are those that framesync reports (relative to
    its origin). Stops at the first frame that does not reach STATE_MIMO.

    Returns a list of dicts: origin, state, num_samples_processed and, once synced,
    sync_index, plateau_start/end, corr_idx, s0_idx, G, noise_var, symbols."""
    rx = np.ascontiguousarray(rx, np.complex64)
    L = rx.shape[1]
    r = 0
    out = []
    while r < L and (max_frames is None or len(out) < max_frames):
        fs = FrameSyncRef(M, cp, N, nac, pid_max=pid_max, **kw)
        st = fs.execute([row[r:] for row in rx])
        d = dict(origin=r, state=st, num_samples_processed=fs.get_num_samples_processed())
        if st != STATE_SEEK_PLATEAU:
            d.update(sync_index=fs.get_sync_index(),
                     plateau_start=[fs.get_plateau_start(s) for s in range(N)],
                     plateau_end=[fs.get_plateau_end(s) for s in range(N)])
        if st == STATE_MIMO:
            ci, _, si, _ = fs.get_corr()
            d.update(corr_idx=ci, s0_idx=si, G=fs.get_G(), noise_var=fs.get_noise_var(),
                     symbols=fs.symbols())
        out.append(d)
        if st != STATE_MIMO:
            break
        r += d["num_samples_processed"]
    return out


def stream_ref_file(path, M, cp, N, nac, pid_max, max_frames, detector, max_syms, qam,
                    tx_path=None, frame_starts=None):
    """stream_ref on a capture saved with numpy.save (worker entry for parallel checks):
    returns the records with symbols cut to max_syms and, with tx_path ([frames][N][pid][M_occ]
    transmitted indices) and frame_starts, each frame's EVM sums over those symbols."""
    rx = np.load(path, mmap_mode="r")
    recs = stream_ref(np.asarray(rx), M, cp, N, nac, pid_max=pid_max, max_frames=max_frames,
                      detector=detector)
    tx = np.load(tx_path, mmap_mode="r") if tx_path else None
    for r in recs:
        if r["state"] == STATE_MIMO:
            r["symbols"] = r["symbols"][:max_syms]
            r.pop("G", None)
            if tx is not None:
                j = int(np.searchsorted(frame_starts, r["origin"] + r["sync_index"], "right")) - 1
                _, num, den, err = demap_evm(r["symbols"], qam, np.asarray(tx[j][:, :max_syms]))
                r.update(tx_frame=j, evm_num=num, evm_den=den, errors=err)
    return recs


def frame_ref_file(path, M, cp, N, nac, pid_max, detector, qam=0, cfo_mode=0, search_mode=1,
                   max_syms=None):
    """One framesync over a capture saved with numpy.save ([N][L] complex64; worker entry for
    parallel checks): the records of the frame (state, sync index, the CFO estimates, corr
    indices, symbols cut to max_syms). search_mode 1 is the Parseval search (labelled CPU
    mode; the brute force gives the same indices up to fp32 ties)."""
    rx = np.load(path, mmap_mode="r")
    fs = FrameSyncRef(M, cp, N, nac, pid_max=pid_max, detector=detector, qam=qam,
                      cfo_mode=cfo_mode, search_mode=search_mode)
    st = fs.execute([np.asarray(r) for r in rx])
    out = dict(state=st, sync_index=fs.get_sync_index())
    if st == STATE_MIMO:
        syms = fs.symbols()
        out.update(cfo=fs.cfo(), corr_idx=fs.get_corr()[0],
                   symbols=syms if max_syms is None else syms[:max_syms])
    return out

"""Batched device-resident receiver and GPU frame synthesiser (the bench's hot path).

`Receiver.process(iq_ptr, ...)` runs the whole receive chain of include/mimo_rx.h's
mimo_rx_process_batch over n_frames captures already in HBM: Schmidl-Cox + plateau,
access-code search, LS estimate, detector weights, replay decode, demap and EVM, all HIP
kernels on one stream with no host synchronisation.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import check, lib
from .framing import LFSR_LARGE_LENGTH, LFSR_SMALL_0_GEN_POLY, LFSR_SMALL_LENGTH, msequence, \
    ofdmframe_init_default_sctype, ofdmframe_validate_sctype, s1_polynomials


@dataclass
class RxParams:
    M: int = 2048
    cp_len: int = 152
    num_streams: int = 4
    num_access_codes: int = 20
    pid_max: int = 1000
    detector: int = _lib.DET_MMSE
    noise_var: float = -1.0
    keep_identity_bias: bool = True
    siso_tx: int = 0
    siso_rx: int = 0
    plateau_threshold: float = 0.95
    qam_order: int = 64
    p: np.ndarray = field(default=None)
    cfo_correct: bool = False

    @property
    def SL(self):
        return self.M + self.cp_len

    def sctype(self):
        return ofdmframe_init_default_sctype(self.M) if self.p is None else \
            np.ascontiguousarray(self.p, np.uint8)

    def m_occ(self):
        _, a, b = ofdmframe_validate_sctype(self.sctype())
        return a + b


def code_bits(M, N, nac):
    """Fresh-generator msequence draws for S0 and the per-stream S1 codes."""
    b0 = msequence(LFSR_SMALL_LENGTH, LFSR_SMALL_0_GEN_POLY, 1).draw_bits(M)
    b1 = np.concatenate([msequence(LFSR_LARGE_LENGTH, g, 1).draw_bits(nac * M)
                         for g in s1_polynomials(N)])
    return b0, b1


def _ptr(x):
    """Device address of a torch tensor, a DeviceBuffer or an int."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if hasattr(x, "addr"):
        return x.addr
    raise TypeError("expected a device pointer")


# UHD's sc16 -> fc32 host conversion scales by 1/32767 (so +32767 maps to 1.0): the reference's
# rx worker receives fc32 produced that way from the sc16 wire (mimo/config.h:51-52,
# mimo/main.cc:837-848), so that is the default here. Callers may pass another scale.
SC16_SCALE = 1.0 / 32767.0


def ingest_sc16(src, src_stride, dst, dst_stride, n_arrays, n, scale=SC16_SCALE, stream=None):
    """Widen n_arrays rows of n sc16 wire samples (interleaved int16 I/Q, UHD's wire format,
    mimo/config.h:52) on the device into planar complex64 rows of the batch layout
    (mimo_ingest_sc16, ingest_kernels.hip). Strides are in samples."""
    check(lib().mimo_ingest_sc16(_ptr(src), src_stride, _ptr(dst), dst_stride, n_arrays, n,
                                 scale, stream), "mimo_ingest_sc16")


def cfo_estimate(iq, stride, n_ant, start, M, stream=None):
    """CFO over the S0 body at `start` (mimo_cfo_estimate): eps per antenna and combined, in
    subcarrier spacings. Absent from the reference (framing.cc:486 FIXME); opt-in."""
    eps = (C.c_double * (n_ant + 1))()
    check(lib().mimo_cfo_estimate(_ptr(iq), stride, n_ant, start, M, eps, stream),
          "mimo_cfo_estimate")
    return np.array(eps[:n_ant]), float(eps[n_ant])


def cfo_derotate(iq, stride, n_ant, n, n0, eps, M, stream=None):
    """In-place x[n] *= exp(-j 2 pi (eps/M) (n - n0)) on every antenna row (mimo_cfo_derotate)."""
    check(lib().mimo_cfo_derotate(_ptr(iq), stride, n_ant, n, n0, eps, M, stream),
          "mimo_cfo_derotate")


class Receiver:
    def __init__(self, params: RxParams, stream=None):
        self.params = params
        P = params
        p = P.sctype()
        self.p = p
        b0, b1 = code_bits(P.M, P.num_streams, P.num_access_codes)
        cfg = _lib.RxConfig(P.M, P.cp_len, P.num_streams, P.num_access_codes, P.pid_max,
                            p.ctypes.data, b0.ctypes.data, b1.ctypes.data, P.detector,
                            P.noise_var, 1 if P.keep_identity_bias else 0, P.siso_tx, P.siso_rx,
                            P.plateau_threshold, P.qam_order, 1 if P.cfo_correct else 0)
        h = C.c_void_p()
        check(lib().mimo_rx_create(C.byref(cfg), stream, C.byref(h)), "mimo_rx_create")
        self._h = h
        self.M_occ = P.m_occ()
        self._last = 0

    def __del__(self):
        if getattr(self, "_h", None):
            lib().mimo_rx_destroy(self._h)
            self._h = None

    def process(self, iq, stride, frame_len, n_frames, max_out=None, out_sym=None, out_idx=None,
                ref_mode=0, ref_idx=None, ref_seed=0, frame_id0=0, stream=None,
                frames_per_capture=1, ref_starts=None, ref_stride=0, sc16=False,
                sc16_scale=None, out_layout=0, stages=0):
        """One batch (mimo_rx_process_batch). stages: _lib.STAGES_ALL, or the front half
        (STAGES_FRONT) / decode half (STAGES_DECODE) of it (see mimo_batch.stages). frames_per_capture > 1: every capture is a
        stream of back-to-back frames, received as fresh framesyncs re-armed after each frame
        (frame slots [capture][frames_per_capture]; see include/mimo_rx.h). sc16: iq holds
        the UHD sc16 wire format (interleaved int16 I/Q), read as float(i16) * sc16_scale.
        out_layout: _lib.LAYOUT_STREAM_MAJOR (out_sym, out_idx and ref_idx frame slots are
        [N][max_out][M_occ]) or _lib.LAYOUT_SYMBOL_MAJOR ([max_out][N][M_occ])."""
        P = self.params
        b = _lib.Batch(_ptr(iq), stride, frame_len, n_frames,
                       P.pid_max if max_out is None else max_out, _ptr(out_sym), _ptr(out_idx),
                       ref_mode, _ptr(ref_idx), ref_seed, frame_id0, frames_per_capture,
                       ref_stride, _ptr(ref_starts), 1 if sc16 else 0,
                       SC16_SCALE if sc16_scale is None else sc16_scale, out_layout, stages)
        check(lib().mimo_rx_process_batch(self._h, C.byref(b), stream), "process_batch")
        self._last = n_frames * max(1, frames_per_capture)

    def receive_streams(self, iq, stride, frame_len, n_caps, frames_per_capture, max_out=None,
                        out_sym=None, out_idx=None, ref_mode=0, ref_idx=None, ref_seed=0,
                        frame_id0=0, ref_starts=None, stream=None, out_layout=0):
        """Back-to-back frames in n_caps captures (process with frames_per_capture), then
        every capture whose chain stopped at a MIMO_FRAME_RESCAN frame is resumed at that
        frame's origin as a fresh capture, into the same frame slots, until none is left.
        ref_starts: host uint64 array [n_caps][frames_per_capture] (see mimo_batch), uploaded
        here. Returns the per-slot result dicts ([capture][k] order, origins absolute)."""
        import torch
        P = self.params
        K = frames_per_capture
        mo = P.pid_max if max_out is None else max_out
        N, mocc = P.num_streams, self.M_occ
        dev_rs = None
        rs_host = None
        if ref_starts is not None:
            rs_host = np.ascontiguousarray(ref_starts, np.uint64).reshape(n_caps, K)
            dev_rs = torch.from_numpy(rs_host.view(np.int64).copy()).cuda()
        self.process(iq, stride, frame_len, n_caps, max_out=mo, out_sym=out_sym, out_idx=out_idx,
                     ref_mode=ref_mode, ref_idx=ref_idx, ref_seed=ref_seed, frame_id0=frame_id0,
                     stream=stream, frames_per_capture=K, ref_starts=dev_rs,
                     out_layout=out_layout)
        res = self.results(n_caps * K)
        base = _ptr(iq)
        slot_sym = N * mo * mocc * 8
        slot_idx = N * mo * mocc
        for c in range(n_caps):
            while True:
                ks = [k for k in range(K) if res[c * K + k]["status"] == _lib.FRAME_RESCAN]
                if not ks:
                    break
                k0 = ks[0]
                org = res[c * K + k0]["origin"]
                rem = K - k0
                rs = None
                if rs_host is not None:
                    sh = rs_host[c].astype(np.int64) - org
                    sh = np.where(rs_host[c] == np.uint64(2 ** 64 - 1), -1, np.maximum(sh, 0))
                    rs = torch.from_numpy(sh.astype(np.int64)).cuda()
                    fid0 = frame_id0 + c * K
                    refp = None if ref_idx is None else _ptr(ref_idx) + c * K * slot_idx
                else:
                    fid0 = frame_id0 + c * K + k0
                    refp = None if ref_idx is None else _ptr(ref_idx) + (c * K + k0) * slot_idx
                sl = c * K + k0
                # the resumed call runs in stream mode with at least two slots; a lone last
                # slot decodes into scratch and is copied into place
                osym = None if out_sym is None else _ptr(out_sym) + sl * slot_sym
                oidx = None if out_idx is None else _ptr(out_idx) + sl * slot_idx
                scratch = ref2 = None
                if rem == 1 and ref_mode == 1 and rs is None and refp is not None:
                    # the scratch second slot reads reference row refp + 1, one past the last
                    # capture's rows: give it a two-row copy
                    ref2 = torch.zeros(2 * slot_idx, dtype=torch.uint8, device="cuda")
                    _lib.memcpy_d2d(ref2.data_ptr(), refp, slot_idx)
                    refp = ref2.data_ptr()
                if rem == 1 and (osym or oidx):
                    scratch = torch.empty(2 * (slot_sym + slot_idx), dtype=torch.uint8,
                                          device="cuda")
                    dsym = scratch.data_ptr() if osym else None
                    didx = scratch.data_ptr() + 2 * slot_sym if oidx else None
                else:
                    dsym, didx = osym, oidx
                self.process(base + ((c * N) * stride + org) * 8, stride, frame_len - org, 1,
                             max_out=mo, out_sym=dsym, out_idx=didx, ref_mode=ref_mode,
                             ref_idx=refp, ref_seed=ref_seed, frame_id0=fid0, stream=stream,
                             frames_per_capture=max(rem, 2), ref_starts=rs,
                             ref_stride=K if rs is not None else 0, out_layout=out_layout)
                if ref2 is not None and scratch is None:
                    # ref2 is read by the asynchronous decode on `stream`: keep it alive until
                    # that work has finished, not just until it is rebound
                    torch.cuda.synchronize()
                if scratch is not None:
                    torch.cuda.synchronize()
                    if osym:
                        _lib.memcpy_d2d(osym, dsym, slot_sym)
                    if oidx:
                        _lib.memcpy_d2d(oidx, didx, slot_idx)
                sub_res = self.results(max(rem, 2))
                for k, r in enumerate(sub_res[:rem]):
                    r = dict(r)
                    r["origin"] += org
                    r["capture"] = c
                    if rs_host is not None or r["status"] == _lib.FRAME_OK:
                        r["ref_frame"] = (c * K + r["ref_frame"]) if rs_host is not None \
                            else (c * K + k0 + k)
                    res[sl + k] = r
        self._last = n_caps * K
        return res

    def results(self, n_frames=None):
        n = self._last if n_frames is None else n_frames
        arr = (_lib.FrameResult * n)()
        check(lib().mimo_rx_batch_results(self._h, arr, n), "batch_results")
        N = self.params.num_streams
        out = []
        for r in arr:
            out.append(dict(
                status=r.status, n_sym=r.n_sym, trigger=r.trigger, sync_index=r.sync_index,
                num_samples_processed=r.num_samples_processed,
                plateau_start=list(r.plateau_start)[:N], plateau_end=list(r.plateau_end)[:N],
                noise_var=r.noise_var, cfo_eps=r.cfo_eps, evm_num=np.array(r.evm_num[:N]),
                evm_den=np.array(r.evm_den[:N]), errors=np.array(r.errors[:N], np.int64),
                origin=r.origin, capture=r.capture, ref_frame=r.ref_frame))
        return out

    def corr(self, n_frames=None):
        n = self._last if n_frames is None else n_frames
        N, nac = self.params.num_streams, self.params.num_access_codes
        ci = np.zeros((n, N, N * nac), np.uint32)
        si = np.zeros((n, N), np.uint32)
        check(lib().mimo_rx_batch_corr(self._h, ci.ctypes.data, si.ctypes.data, n), "batch_corr")
        return ci, si

    def G(self, n_frames=None):
        n = self._last if n_frames is None else n_frames
        P = self.params
        G = np.zeros((n, P.M, P.num_streams, P.num_streams), np.complex64)
        check(lib().mimo_rx_batch_G(self._h, G.ctypes.data, n), "batch_G")
        return G

    def W(self, n_frames=None):
        n = self._last if n_frames is None else n_frames
        P = self.params
        W = np.zeros((n, P.M, P.num_streams, P.num_streams), np.complex64)
        check(lib().mimo_rx_batch_W(self._h, W.ctypes.data, n), "batch_W")
        return W

    def set_siso(self, tx, rx):
        """framesync::set_siso_tx/rx: the stream pair the SISO detector decodes (a change
        invalidates the captured batch graph, whose kernels carry the indices)."""
        check(lib().mimo_rx_set_siso(self._h, tx, rx), "set_siso")

    def set_timing(self, on):
        check(lib().mimo_rx_set_timing(self._h, 1 if on else 0), "set_timing")

    def sc_exact_count(self):
        v = C.c_uint64()
        check(lib().mimo_rx_get_sc_exact_count(self._h, C.byref(v)), "sc_exact_count")
        return v.value

    def decode_path(self):
        """Kernel family of the last decode launch (_lib.DECODE_STREAM / _SPLIT / _SYMBOL)."""
        v = C.c_int32()
        check(lib().mimo_rx_get_decode_path(self._h, C.byref(v)), "decode_path")
        return v.value

    def cfo_mode(self):
        """CFO stages of the last batch: 0 off, 1 estimate + derotation, 2 plus the per-symbol
        common phase (the oracle's cfo_mode for the same batch)."""
        v = C.c_int32()
        check(lib().mimo_rx_get_cfo_mode(self._h, C.byref(v)), "cfo_mode")
        return v.value

    def stage_times(self):
        ms = (C.c_double * _lib.NUM_STAGES)()
        cnt = (C.c_uint32 * _lib.NUM_STAGES)()
        check(lib().mimo_rx_get_stage_times(self._h, ms, cnt), "stage_times")
        return {n: (ms[i], cnt[i]) for i, n in enumerate(_lib.STAGE_NAMES)}


@dataclass
class SynthParams:
    M: int = 2048
    cp_len: int = 152
    num_streams: int = 4
    num_access_codes: int = 20
    pid: int = 1000
    qam_order: int = 64
    seed: int = 1
    snr_db: float = 30.0
    tail_syms: int = 3
    identity_channel: bool = False
    offset: int = -1
    p: np.ndarray = field(default=None)

    @property
    def SL(self):
        return self.M + self.cp_len

    def max_frame_len(self):
        """Uniform capture length that holds any offset u in [0, SL)."""
        SL = self.SL
        return SL * (2 * self.num_streams * self.num_access_codes + 2 + self.pid +
                     self.tail_syms) + SL


class Synthesizer:
    """GPU synthetic captures in the reference tx_worker layout (mimo_synth_frames)."""

    def __init__(self, params: SynthParams):
        self.params = params
        P = params
        self.p = ofdmframe_init_default_sctype(P.M) if P.p is None else \
            np.ascontiguousarray(P.p, np.uint8)
        self.b0, self.b1 = code_bits(P.M, P.num_streams, P.num_access_codes)
        self._cfg = _lib.SynthConfig(P.M, P.cp_len, P.num_streams, P.num_access_codes, P.pid,
                                     P.qam_order, P.seed, P.snr_db, P.tail_syms,
                                     1 if P.identity_channel else 0, P.offset,
                                     self.p.ctypes.data, self.b0.ctypes.data, self.b1.ctypes.data)

    def frame_len(self, frame_id):
        v = C.c_uint64()
        check(lib().mimo_synth_frame_len(C.byref(self._cfg), frame_id, C.byref(v)), "frame_len")
        return v.value

    def generate(self, out, stride, frame_len, n_frames, frame_id0=0, tx_idx=None, H=None,
                 stream=None):
        check(lib().mimo_synth_frames(C.byref(self._cfg), frame_id0, n_frames, _ptr(out), stride,
                                      frame_len, _ptr(tx_idx), _ptr(H), stream), "synth_frames")

    def stream_layout(self, n_streams, frames_per_stream, stream0=0):
        """Frame lengths [S][J] of streams that carry the synthesiser's frames
        (stream0+s)*J .. (stream0+s)*J+J-1 back to back, and the common capture length."""
        J = frames_per_stream
        lens = [[self.frame_len((stream0 + s) * J + j) for j in range(J)]
                for s in range(n_streams)]
        return lens, max(sum(l) for l in lens)

    def generate_streams(self, iq, L, n_streams, frames_per_stream, slots, stream0=0,
                         tx_idx=None, stream=None):
        """Back-to-back frames (BASELINE config C5's per-stream workload) into iq [S][N][L]
        (complex64, zeroed by the caller past each stream's last frame). tx_idx, if given:
        [S*slots][N][pid][M_occ] reference rows, row s*slots+j for frame j of stream s.
        Returns the host uint64 array [S][slots] of frame starts (UINT64_MAX after the last),
        the d_ref_starts of mimo_batch, and the lengths [S][J]."""
        P = self.params
        J = frames_per_stream
        lens, _ = self.stream_layout(n_streams, J, stream0)
        N = P.num_streams
        row = N * P.pid * (len(self.p) if P.p is None else
                           int(np.count_nonzero(self.p)))
        starts = np.full((n_streams, slots), np.uint64(2 ** 64 - 1), np.uint64)
        base = _ptr(iq)
        for s in range(n_streams):
            pos = 0
            for j in range(J):
                txp = None if tx_idx is None else _ptr(tx_idx) + (s * slots + j) * row
                self.generate(base + ((s * N) * L + pos) * 8, L, lens[s][j], 1,
                              frame_id0=(stream0 + s) * J + j, tx_idx=txp, stream=stream)
                starts[s, j] = pos
                pos += lens[s][j]
        return starts, lens

"""ctypes binding of librub_mimo_amd.so (include/mimo_rx.h).

The shared library is the product: every receive stage runs in its HIP kernels. There is no
CPU fallback -- if the library is missing or was built for another target, importing the
binding raises immediately.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# RMIMO_LIB selects a diagnostics build of the same library (e.g. make PROFILE=1 into another path)
LIB_PATH = os.environ.get("RMIMO_LIB") or os.path.join(_HERE, "librub_mimo_amd.so")

MIMO_OK = 0
MAX_STREAMS = 8
NUM_STAGES = 7
STAGE_NAMES = ("sc", "plateau", "search", "ls", "weights", "decode", "evm")

STATE_SEEK_PLATEAU, STATE_SAVE_ACCESS_CODES, STATE_WAIT, STATE_MIMO = 0, 1, 2, 3
DET_ZF2, DET_ZF, DET_MMSE, DET_SISO = 0, 1, 2, 3
FRAME_OK, FRAME_NO_SYNC, FRAME_INCOMPLETE, FRAME_RESCAN, FRAME_NONE = 0, 1, 2, 3, 4
DECODE_NONE, DECODE_STREAM, DECODE_SPLIT, DECODE_SYMBOL = 0, 1, 2, 3
# mimo_batch.out_layout: [F][N][max_out][M_occ] or [F][max_out][N][M_occ]
LAYOUT_STREAM_MAJOR, LAYOUT_SYMBOL_MAJOR = 0, 1
# mimo_batch.stages: the whole chain, the front half (S&C .. weights) or the decode half
STAGES_ALL, STAGES_FRONT, STAGES_DECODE = 0, 1, 2


class RxConfig(C.Structure):
    _fields_ = [("M", C.c_uint32), ("cp_len", C.c_uint32), ("num_streams", C.c_uint32),
                ("num_access_codes", C.c_uint32), ("pid_max", C.c_uint32),
                ("p", C.c_void_p), ("s0_bits", C.c_void_p), ("s1_bits", C.c_void_p),
                ("detector", C.c_int32), ("noise_var", C.c_float),
                ("keep_identity_bias", C.c_int32), ("siso_tx", C.c_uint32),
                ("siso_rx", C.c_uint32), ("plateau_threshold", C.c_double),
                ("qam_order", C.c_uint32), ("cfo_correct", C.c_int32)]


class Batch(C.Structure):
    _fields_ = [("d_iq", C.c_void_p), ("stride", C.c_uint64), ("frame_len", C.c_uint64),
                ("n_frames", C.c_uint32), ("max_out_syms", C.c_uint32),
                ("d_out_sym", C.c_void_p), ("d_out_idx", C.c_void_p), ("ref_mode", C.c_int32),
                ("d_ref_idx", C.c_void_p), ("ref_seed", C.c_uint64), ("frame_id0", C.c_uint64),
                ("frames_per_capture", C.c_uint32), ("ref_stride", C.c_uint32),
                ("d_ref_starts", C.c_void_p), ("sample_format", C.c_uint32),
                ("sc16_scale", C.c_float), ("out_layout", C.c_uint32), ("stages", C.c_uint32)]


class FrameResult(C.Structure):
    _fields_ = [("status", C.c_int32), ("n_sym", C.c_uint32), ("trigger", C.c_uint64),
                ("sync_index", C.c_uint64), ("num_samples_processed", C.c_uint64),
                ("plateau_start", C.c_uint64 * MAX_STREAMS),
                ("plateau_end", C.c_uint64 * MAX_STREAMS), ("noise_var", C.c_float),
                ("cfo_eps", C.c_float), ("evm_num", C.c_double * MAX_STREAMS),
                ("evm_den", C.c_double * MAX_STREAMS), ("errors", C.c_uint64 * MAX_STREAMS),
                ("origin", C.c_uint64), ("capture", C.c_uint32), ("ref_frame", C.c_uint32)]


class SynthConfig(C.Structure):
    _fields_ = [("M", C.c_uint32), ("cp_len", C.c_uint32), ("num_streams", C.c_uint32),
                ("num_access_codes", C.c_uint32), ("pid", C.c_uint32), ("qam_order", C.c_uint32),
                ("seed", C.c_uint64), ("snr_db", C.c_float), ("tail_syms", C.c_uint32),
                ("identity_channel", C.c_int32), ("offset", C.c_int32),
                ("p", C.c_void_p), ("s0_bits", C.c_void_p), ("s1_bits", C.c_void_p)]


_vp, _u32, _u64, _i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int32
_P = C.POINTER
SYMBOL_CB = C.CFUNCTYPE(None, _P(_P(C.c_float)), _u32, _u32, _vp)

# every symbol declared in include/mimo_rx.h, with its ctypes signature
SIGNATURES = {
    "mimo_rx_create": (C.c_int, [_P(RxConfig), _vp, _P(_vp)]),
    "mimo_rx_destroy": (C.c_int, [_vp]),
    "mimo_rx_set_callback": (C.c_int, [_vp, SYMBOL_CB, _vp]),
    "mimo_rx_execute": (C.c_int, [_vp, _P(_vp), _u32, _u64, _P(_i32)]),
    "mimo_rx_reset": (C.c_int, [_vp]),
    "mimo_rx_set_siso": (C.c_int, [_vp, _u32, _u32]),
    "mimo_rx_get_state": (C.c_int, [_vp, _P(_i32)]),
    "mimo_rx_get_sync_index": (C.c_int, [_vp, _P(_u64)]),
    "mimo_rx_get_num_samples_processed": (C.c_int, [_vp, _P(_u64)]),
    "mimo_rx_get_plateau": (C.c_int, [_vp, _u32, _P(_u64), _P(_u64)]),
    "mimo_rx_get_G": (C.c_int, [_vp, _vp]),
    "mimo_rx_get_W": (C.c_int, [_vp, _vp]),
    "mimo_rx_get_gain": (C.c_int, [_vp, _vp]),
    "mimo_rx_get_noise_var": (C.c_int, [_vp, _P(C.c_float)]),
    "mimo_rx_get_corr": (C.c_int, [_vp, _vp, _vp]),
    "mimo_rx_get_m_occ": (C.c_int, [_vp, _P(_u32)]),
    "mimo_rx_process_batch": (C.c_int, [_vp, _P(Batch), _vp]),
    "mimo_rx_batch_results": (C.c_int, [_vp, _P(FrameResult), _u32]),
    "mimo_rx_batch_corr": (C.c_int, [_vp, _vp, _vp, _u32]),
    "mimo_rx_batch_G": (C.c_int, [_vp, _vp, _u32]),
    "mimo_rx_batch_W": (C.c_int, [_vp, _vp, _u32]),
    "mimo_rx_set_timing": (C.c_int, [_vp, C.c_int]),
    "mimo_rx_get_stage_times": (C.c_int, [_vp, _P(C.c_double), _P(_u32)]),
    "mimo_rx_get_sc_exact_count": (C.c_int, [_vp, _P(_u64)]),
    "mimo_rx_get_decode_path": (C.c_int, [_vp, _P(_i32)]),
    "mimo_rx_set_grid_cus": (C.c_int, [_vp, _u32]),
    "mimo_probe_decode_pattern": (C.c_int, [_vp, _u64, _u32, _u32, _u32, _u32, _u32, _u32, _vp,
                                            _vp, _vp, C.c_int, _vp, _P(C.c_float)]),
    "mimo_rx_get_cfo_mode": (C.c_int, [_vp, _P(_i32)]),
    "mimo_rx_get_stream_capacity": (C.c_int, [_vp, _P(_u64), _P(_u64)]),
    "mimo_rx_set_debug_log": (C.c_int, [_vp, C.c_char_p]),
    "mimo_tx_create": (C.c_int, [_u32, _u32, _u32, _u32, _vp, _vp, _vp, _P(_vp)]),
    "mimo_tx_destroy": (C.c_int, [_vp]),
    "mimo_tx_write_sync_words": (C.c_int, [_vp, _P(_vp), _P(_u32)]),
    "mimo_tx_assemble_mimo_packet": (C.c_int, [_vp, _P(_vp), _P(_vp), _P(_u32)]),
    "mimo_tx_get_codes": (C.c_int, [_vp, _vp, _vp]),
    "mimo_synth_frame_len": (C.c_int, [_P(SynthConfig), _u64, _P(_u64)]),
    "mimo_synth_frames": (C.c_int, [_P(SynthConfig), _u64, _u32, _vp, _u64, _u64, _vp, _vp, _vp]),
    "mimo_sctype_default": (C.c_int, [_vp, _u32]),
    "mimo_sctype_liquid": (C.c_int, [_vp, _u32]),
    "mimo_sctype_validate": (C.c_int, [_vp, _u32, _P(_u32), _P(_u32), _P(_u32)]),
    "mimo_msequence_draw_bits": (C.c_int, [_u32, _u32, _u32, _u32, _vp]),
    "mimo_invert2": (C.c_float, [_vp, _vp]),
    "mimo_dev_alloc": (C.c_int, [_P(_vp), C.c_size_t]),
    "mimo_dev_free": (C.c_int, [_vp]),
    "mimo_memcpy_h2d": (C.c_int, [_vp, _vp, C.c_size_t, _vp]),
    "mimo_memcpy_d2h": (C.c_int, [_vp, _vp, C.c_size_t, _vp]),
    "mimo_memcpy_d2d": (C.c_int, [_vp, _vp, C.c_size_t, _vp]),
    "mimo_memset_d": (C.c_int, [_vp, C.c_int, C.c_size_t, _vp]),
    "mimo_cfo_estimate": (C.c_int, [_vp, _u64, _u32, _u64, _u32, _P(C.c_double), _vp]),
    "mimo_cfo_derotate": (C.c_int, [_vp, _u64, _u32, _u64, C.c_int64, C.c_double, _u32, _vp]),
    "mimo_ingest_sc16": (C.c_int, [_vp, _u64, _vp, _u64, _u32, _u64, C.c_float, _vp]),
    "mimo_ring_create": (C.c_int, [_u32, _u32, _u32, _P(_vp)]),
    "mimo_ring_destroy": (C.c_int, [_vp]),
    "mimo_ring_bind": (C.c_int, [_vp, _vp, _u64, _u64]),
    "mimo_ring_bind_after": (C.c_int, [_vp, _vp, _u64, _u64, _vp]),
    "mimo_ring_acquire": (C.c_int, [_vp, _P(_vp), _P(_u32)]),
    "mimo_ring_commit": (C.c_int, [_vp, _u32]),
    "mimo_ring_publish": (C.c_int, [_vp, _vp, _P(_u64)]),
    "mimo_stream_sync": (C.c_int, [_vp]),
    "mimo_device_count": (C.c_int, [_P(C.c_int)]),
    "mimo_last_error": (C.c_char_p, []),
    "mimo_version": (C.c_char_p, []),
}

_lib = None


class MimoError(RuntimeError):
    pass


def lib():
    """Load the HIP library (raises if it has not been built: no silent fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MimoError(
                "librub_mimo_amd.so is not built (expected %s); run "
                "`make -C rub_mimo_amd/csrc -j8` or __graft_entry__.build()" % LIB_PATH)
        L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc, what=""):
    if rc != MIMO_OK:
        msg = lib().mimo_last_error().decode(errors="replace")
        raise MimoError("%s failed (%d): %s" % (what, rc, msg))
    return rc


def memcpy_d2d(dst, src, nbytes, stream=None):
    check(lib().mimo_memcpy_d2d(dst, src, nbytes, stream), "d2d")


def device_count():
    n = C.c_int(0)
    rc = lib().mimo_device_count(C.byref(n))
    return n.value if rc == MIMO_OK else 0


class DeviceBuffer:
    """Plain HIP device allocation (tests and tools that do not use torch)."""

    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        self.ptr = C.c_void_p()
        check(lib().mimo_dev_alloc(C.byref(self.ptr), max(self.nbytes, 1)), "mimo_dev_alloc")

    @property
    def addr(self):
        return self.ptr.value

    def upload(self, arr):
        import numpy as np
        a = np.ascontiguousarray(arr)
        assert a.nbytes <= self.nbytes
        check(lib().mimo_memcpy_h2d(self.ptr, C.c_void_p(a.ctypes.data), a.nbytes, None), "h2d")

    def download(self, dtype, count):
        import numpy as np
        out = np.empty(count, dtype)
        assert out.nbytes <= self.nbytes
        check(lib().mimo_memcpy_d2h(C.c_void_p(out.ctypes.data), self.ptr, out.nbytes, None), "d2h")
        return out

    def zero(self):
        check(lib().mimo_memset_d(self.ptr, 0, self.nbytes, None), "memset")
        check(lib().mimo_stream_sync(None), "sync")

    def free(self):
        if self.ptr is not None and self.ptr.value:
            lib().mimo_dev_free(self.ptr)
        self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

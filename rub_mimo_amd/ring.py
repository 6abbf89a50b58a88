"""rub_mimo_amd/ring.py -- Python mirror of the pinned-host capture ring (mimo_ring_* in
include/mimo_rx.h, csrc/ring.cpp).

It stands where the reference's rx worker keeps its malloc'd rx_buffer and /tmp file round
trip (mimo/main.cc:842-848, 872-898, 906-918): a producer (the recv loop) writes UHD sc16 wire
samples into pinned chunks, each commit is uploaded asynchronously into the bound device
capture, and the consumer's stream waits for the uploads on the device before
Receiver.process(..., sc16=True) reads the capture in place.

    ring = CaptureRing(n_ant=4, chunk_samples=1 << 16)
    ring.bind(capture)                  # torch int16 [n_ant][stride][2] on the GPU
    rows = ring.acquire()               # per antenna: numpy int16 [chunk][2], pinned memory
    n = recv(rows, ...)                 # the recv loop writes each channel's samples
    ring.commit(n)
    n_written = ring.publish(stream)    # stream now waits for every committed upload
"""
import ctypes as C

import numpy as np

from ._lib import check, lib


class CaptureRing:
    """n_chunks pinned chunks of chunk_samples sc16 samples per antenna (see module doc).
    One producer thread calls acquire/commit; bind/publish may run on another."""

    def __init__(self, n_ant, chunk_samples, n_chunks=4):
        self.n_ant, self.chunk, self.n_chunks = n_ant, chunk_samples, n_chunks
        h = C.c_void_p()
        check(lib().mimo_ring_create(n_ant, chunk_samples, n_chunks, C.byref(h)), "mimo_ring_create")
        self._h = h
        self._rows = (C.c_void_p * n_ant)()

    def close(self):
        if self._h:
            check(lib().mimo_ring_destroy(self._h), "mimo_ring_destroy")
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def bind(self, capture, stride=None, capacity=None, after_stream=None):
        """Target of the following commits: a device sc16 capture. `capture` is a torch int16
        tensor [n_ant][stride][2] (or a raw device pointer with stride/capacity given).
        after_stream (a hipStream_t handle, e.g. torch.cuda.current_stream().cuda_stream):
        the uploads into this capture wait for the work enqueued there so far (a batch still
        reading the capture); without it the caller synchronises before rebinding."""
        if hasattr(capture, "data_ptr"):
            ptr = capture.data_ptr()
            if stride is None:
                stride = capture.shape[-2]
        else:
            ptr = int(capture)
        if capacity is None:
            capacity = stride
        if after_stream is not None:
            check(lib().mimo_ring_bind_after(self._h, C.c_void_p(ptr), stride, capacity,
                                             C.c_void_p(after_stream)), "mimo_ring_bind_after")
        else:
            check(lib().mimo_ring_bind(self._h, C.c_void_p(ptr), stride, capacity),
                  "mimo_ring_bind")

    def acquire(self):
        """The next chunk: one numpy int16 view [chunk_samples][2] of pinned memory per
        antenna (waits for that chunk's previous upload)."""
        n = C.c_uint32()
        check(lib().mimo_ring_acquire(self._h, self._rows, C.byref(n)), "mimo_ring_acquire")
        return [np.ctypeslib.as_array(C.cast(self._rows[a], C.POINTER(C.c_int16)),
                                      shape=(n.value, 2)) for a in range(self.n_ant)]

    def commit(self, n):
        check(lib().mimo_ring_commit(self._h, n), "mimo_ring_commit")

    def publish(self, stream=None):
        """Make `stream` (a HIP stream handle, None = the default stream) wait for every
        committed upload; returns the bound capture's samples per antenna so far."""
        n = C.c_uint64()
        check(lib().mimo_ring_publish(self._h, stream, C.byref(n)), "mimo_ring_publish")
        return n.value

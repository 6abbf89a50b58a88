"""The reference's /tmp capture and result files, so its Qt GUI and plot tool drop in.

Formats (all raw, no header, little-endian, one file per channel, channels numbered from 1):
- ``rx<ch>.dat``      complex64 capture, appended chunk by chunk by the rx worker
                      (mimo/main.cc:829-833 open, :881-887 fwrite per recv), re-read whole
                      before framesync (mimo/main.cc:905-918);
- ``tx_sig<ch>.dat``  complex64 transmitted constellation points (mimo/main.cc:1257-1258);
- ``tx_data<ch>.dat`` uint32 transmitted symbol indices (mimo/main.cc:1255-1256);
- ``rx_sig<ch>.dat``  complex64 equalised symbols (mimo/main.cc:1409-1416);
- ``rx_data<ch>.dat`` uint32 hard decisions (mimo/main.cc:1411-1414).
Readers: Interface/mainwindow.cpp:217-230 and mimo/apps/plot.py:27-40 (which reads the index
files as int32; the bytes are the same for indices < 2^31).

This is host I/O around the device path, not compute: the equalised symbols and indices come
from the library's decode kernels (Receiver.process out_sym/out_idx, or framesync callbacks).
The library writes uint8 indices; they are widened to the reference's uint32 here.
"""
import os

import numpy as np

LOG_DIR = "/tmp/"          # mimo/config.h LOG_DIR


def _path(log_dir, stem, ch):
    return os.path.join(log_dir, f"{stem}{ch + 1}.dat")


def rx_capture_paths(num_channels, log_dir=LOG_DIR):
    return [_path(log_dir, "rx", c) for c in range(num_channels)]


class CaptureWriter:
    """rx_worker's per-channel capture files (mimo/main.cc:829-887): opened "wb" once, then each
    recv's ``num_samples_read`` samples per channel appended with one fwrite each."""

    def __init__(self, num_channels, log_dir=LOG_DIR):
        self.num_channels = num_channels
        self._fp = [open(p, "wb") for p in rx_capture_paths(num_channels, log_dir)]
        self.num_accumulated_samples = 0

    def write(self, rx_buffer, num_samples_read=None):
        if len(rx_buffer) != self.num_channels:
            raise ValueError("rx_buffer must hold one array per channel")
        bufs = [np.ascontiguousarray(b, np.complex64) for b in rx_buffer]
        n = len(bufs[0]) if num_samples_read is None else int(num_samples_read)
        for fp, b in zip(self._fp, bufs):
            if len(b) < n:
                raise ValueError("channel buffer shorter than num_samples_read")
            fp.write(b[:n].tobytes())
        self.num_accumulated_samples += n
        return n

    def close(self):
        for fp in self._fp:
            fp.close()
        self._fp = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def read_rx_capture(num_channels, log_dir=LOG_DIR, mmap=True):
    """Re-read the whole capture (mimo/main.cc:905-918). Returns one complex64 array per channel
    (memory-mapped by default: a C3 capture is ~20 MB per antenna, a long one far more). Every
    channel must hold the same sample count, as the reference asserts (:913-917)."""
    out = []
    for p in rx_capture_paths(num_channels, log_dir):
        size = os.path.getsize(p)
        if size % 8:
            raise ValueError(f"{p}: {size} bytes is not a whole number of complex64 samples")
        if size == 0:
            out.append(np.zeros(0, np.complex64))
        elif mmap:
            out.append(np.memmap(p, dtype="<c8", mode="r"))
        else:
            out.append(np.fromfile(p, dtype="<c8"))
    lens = {len(a) for a in out}
    if len(lens) > 1:
        raise ValueError(f"channels hold different sample counts: {sorted(lens)}")
    return out


def _write_all(stem_sig, stem_data, sig, data, log_dir):
    if len(sig) != len(data):
        raise ValueError("sig and data must hold the same number of channels")
    paths = []
    for ch, (s, d) in enumerate(zip(sig, data)):
        s = np.ascontiguousarray(s, np.complex64).reshape(-1)
        d = np.asarray(d).reshape(-1)
        if d.dtype.kind not in "ui" or (d.size and d.min() < 0):
            raise ValueError("symbol indices must be non-negative integers")
        if len(s) != len(d):
            raise ValueError(f"channel {ch + 1}: {len(s)} symbols but {len(d)} indices")
        ps, pd = _path(log_dir, stem_sig, ch), _path(log_dir, stem_data, ch)
        s.astype("<c8", copy=False).tofile(ps)
        d.astype("<u4").tofile(pd)
        paths += [ps, pd]
    return paths


def write_tx_logs(tx_sig, tx_data, log_dir=LOG_DIR):
    """tx_sig<ch>.dat / tx_data<ch>.dat (mimo/main.cc:1250-1259)."""
    return _write_all("tx_sig", "tx_data", tx_sig, tx_data, log_dir)


def write_rx_logs(rx_sig, rx_data, log_dir=LOG_DIR):
    """rx_sig<ch>.dat / rx_data<ch>.dat (mimo/main.cc:1409-1419). ``rx_data`` may be the
    library's uint8 indices; they are widened to uint32."""
    return _write_all("rx_sig", "rx_data", rx_sig, rx_data, log_dir)


def read_logs(num_channels, log_dir=LOG_DIR):
    """What plot.py reads back (mimo/apps/plot.py:27-40): per channel tx_sig, rx_sig
    (complex64) and tx_data, rx_data (int32)."""
    def rd(stem, ch, dt):
        return np.fromfile(_path(log_dir, stem, ch), dtype=dt)
    return {stem: [rd(stem, c, dt) for c in range(num_channels)]
            for stem, dt in (("tx_sig", "<c8"), ("rx_sig", "<c8"),
                             ("tx_data", "<i4"), ("rx_data", "<i4"))}

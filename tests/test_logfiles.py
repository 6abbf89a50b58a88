"""The /tmp capture and result files (rub_mimo_amd/logfiles.py) against the reference's byte
layout: raw little-endian complex64 / uint32, channel numbers from 1 (mimo/main.cc:829-833,
881-887, 905-918, 1250-1259, 1409-1419; readers mimo/apps/plot.py:27-40). CPU only."""
import os
import struct

import numpy as np
import pytest

from rub_mimo_amd import logfiles as lf


def test_capture_append_chunks_then_reread(tmp_path):
    rng = np.random.default_rng(1)
    N, n = 4, 5000
    x = (rng.standard_normal((N, n)) + 1j * rng.standard_normal((N, n))).astype(np.complex64)
    with lf.CaptureWriter(N, str(tmp_path)) as w:
        pos = 0
        while pos < n:                         # ragged recv sizes, last one short
            c = int(rng.integers(1, 900))
            buf = [np.concatenate([r[pos:pos + c], np.zeros(7, np.complex64)]) for r in x]
            pos += w.write(buf, min(c, n - pos))
        assert w.num_accumulated_samples == n
    assert sorted(os.listdir(tmp_path)) == [f"rx{c}.dat" for c in range(1, N + 1)]
    for mm in (True, False):
        back = lf.read_rx_capture(N, str(tmp_path), mmap=mm)
        assert all(np.array_equal(b, r) for b, r in zip(back, x))
    # raw interleaved fp32 I/Q, little endian, no header
    raw = open(tmp_path / "rx1.dat", "rb").read(8)
    assert struct.unpack("<ff", raw) == (float(x[0, 0].real), float(x[0, 0].imag))


def test_capture_unequal_channels_and_partial_sample_rejected(tmp_path):
    np.zeros(10, np.complex64).tofile(tmp_path / "rx1.dat")
    np.zeros(11, np.complex64).tofile(tmp_path / "rx2.dat")
    with pytest.raises(ValueError, match="different sample counts"):
        lf.read_rx_capture(2, str(tmp_path))
    open(tmp_path / "rx2.dat", "wb").write(b"\0" * 84)
    with pytest.raises(ValueError, match="whole number"):
        lf.read_rx_capture(2, str(tmp_path))


def test_empty_capture(tmp_path):
    with lf.CaptureWriter(2, str(tmp_path)):
        pass
    back = lf.read_rx_capture(2, str(tmp_path))
    assert [len(b) for b in back] == [0, 0]


def test_result_logs_roundtrip_and_layout(tmp_path):
    rng = np.random.default_rng(2)
    N, n = 2, 3000
    sig = (rng.standard_normal((N, n)) + 1j * rng.standard_normal((N, n))).astype(np.complex64)
    idx8 = rng.integers(0, 256, (N, n), dtype=np.uint8)      # library's uint8 indices
    tx_idx = rng.integers(0, 64, (N, n)).astype(np.uint32)
    lf.write_tx_logs(sig, tx_idx, str(tmp_path))
    lf.write_rx_logs(sig[::-1], idx8, str(tmp_path))
    assert os.path.getsize(tmp_path / "rx_data1.dat") == 4 * n     # widened to uint32
    assert os.path.getsize(tmp_path / "rx_sig2.dat") == 8 * n
    d = lf.read_logs(N, str(tmp_path))
    for c in range(N):
        assert np.array_equal(d["tx_sig"][c], sig[c])
        assert np.array_equal(d["rx_sig"][c], sig[N - 1 - c])
        assert np.array_equal(d["tx_data"][c], tx_idx[c].astype(np.int32))
        assert np.array_equal(d["rx_data"][c], idx8[c].astype(np.int32))
    assert struct.unpack("<I", open(tmp_path / "rx_data1.dat", "rb").read(4))[0] == idx8[0, 0]


def test_result_logs_reject_mismatch(tmp_path):
    with pytest.raises(ValueError, match="symbols but"):
        lf.write_rx_logs([np.zeros(4, np.complex64)], [np.zeros(3, np.uint8)], str(tmp_path))
    with pytest.raises(ValueError, match="non-negative"):
        lf.write_rx_logs([np.zeros(2, np.complex64)], [np.array([0, -1])], str(tmp_path))
    with pytest.raises(ValueError, match="same number of channels"):
        lf.write_tx_logs([np.zeros(2, np.complex64)] * 2, [np.zeros(2, np.uint32)], str(tmp_path))

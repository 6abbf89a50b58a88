"""GPU parity tests: the HIP pipeline (through the C-ABI) against the CPU oracle and the
committed golden fixtures. Integer/index results (plateau, sync index, samples processed,
corr indices, demapped indices away from decision boundaries) must be bit-exact; equalised
symbols must agree to an error-vector ratio <= 1e-4 (north_star: EVM delta <= 1e-4)."""
import glob
import os

import numpy as np
import pytest

from oracle import codes, ref
from rub_mimo_amd import _lib
from rub_mimo_amd import framing as fr
from rub_mimo_amd.receiver import Receiver, RxParams, Synthesizer, SynthParams

pytestmark = pytest.mark.gpu

GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "m[0-9]*.npz")))
GOLDEN = [g for g in GOLDEN if "_stream" not in os.path.basename(g)]
STREAMS = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "m*_stream*.npz")))
SYM_TOL = 1e-4        # sqrt(sum|y_gpu - y_cpu|^2 / sum|y_cpu|^2)
EVM_DB_TOL = 1e-3


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible: the gpu tests need an MI355X")


def load(path):
    return dict(np.load(path, allow_pickle=False))


def evm_delta(a, b):
    a = np.asarray(a, np.complex128)
    b = np.asarray(b, np.complex128)
    return float(np.sqrt(np.sum(np.abs(a - b) ** 2) / max(np.sum(np.abs(b) ** 2), 1e-300)))


def new_codes(N):
    ms0 = fr.msequence_create(fr.LFSR_SMALL_LENGTH, fr.LFSR_SMALL_0_GEN_POLY, 1)
    ms1 = [fr.msequence_create(fr.LFSR_LARGE_LENGTH, g, 1) for g in fr.s1_polynomials(N)]
    return ms0, ms1


def gpu_framesync(g, qam=4):
    N = int(g["N"])
    ms0, ms1 = new_codes(N)
    got = []
    fs = fr.framesync(int(g["M"]), int(g["cp"]), N, int(g["nac"]), g["p"], ms0, ms1,
                      callback=lambda xs, m: got.append(np.stack([x.copy() for x in xs])),
                      pid_max=int(g["pid"]), detector=int(g["detector"]),
                      keep_identity_bias=bool(g["keep_identity_bias"]),
                      siso_tx=int(g["siso_tx"]), siso_rx=int(g["siso_rx"]), qam_order=qam)
    return fs, got


def assert_sync_equal(fs_gpu, g):
    N = int(g["N"])
    assert fs_gpu.get_sync_index() == int(g["sync_index"])
    assert fs_gpu.get_num_samples_processed() == int(g["num_samples_processed"])
    assert [fs_gpu.get_plateau_start(s) for s in range(N)] == list(g["plateau_start"])
    assert [fs_gpu.get_plateau_end(s) for s in range(N)] == list(g["plateau_end"])


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_streaming_framesync_matches_golden(path):
    g = load(path)
    fs, got = gpu_framesync(g)
    st = fs.execute(list(g["rx"]))
    assert st == fr.STATE_MIMO
    assert_sync_equal(fs, g)
    ci, si = fs.get_corr()
    assert np.array_equal(ci, g["corr_idx"]) and np.array_equal(si, g["s0_idx"])
    G = fs.get_G()
    assert np.abs(G - g["G"]).max() <= 1e-4 * np.abs(g["G"]).max()
    syms = np.stack(got)
    assert syms.shape == g["symbols"].shape          # PID+2 callbacks (framing.cc:857-868)
    assert evm_delta(syms, g["symbols"]) <= SYM_TOL
    if int(g["detector"]) == ref.DET_ZF2:
        gn = fs.get_gain()
        assert np.allclose(gn, g["gain"], rtol=1e-3)
    if int(g["detector"]) == ref.DET_MMSE:
        assert abs(fs.get_noise_var() - float(g["noise_var"])) <= 1e-4 * float(g["noise_var"])
    if int(g["detector"]) in (ref.DET_ZF2, ref.DET_ZF, ref.DET_MMSE):
        W = fs.get_W()
        assert np.abs(W - g["W"]).max() <= 1e-4 * np.abs(g["W"]).max()


@pytest.mark.parametrize("path", GOLDEN[:3], ids=[os.path.basename(p) for p in GOLDEN[:3]])
def test_chunked_execute_equals_one_shot(path):
    g = load(path)
    rx = g["rx"]
    fs, got = gpu_framesync(g)
    pos = 0
    rng = np.random.default_rng(5)
    while pos < rx.shape[1]:
        c = int(rng.integers(1, 3000))
        fs.execute([r[pos:pos + c] for r in rx], min(c, rx.shape[1] - pos))
        pos += c
    assert_sync_equal(fs, g)
    assert evm_delta(np.stack(got), g["symbols"]) <= SYM_TOL


def test_batch_then_reset_then_chunked_execute_on_one_handle():
    """One handle runs a batch of 8 captures (its S&C records grow to F = 8 rows), then
    reset(), then the chunked streaming execute: the streaming path keeps only frame 0's
    records across record growth (engine.cpp ensure_workspace), so its results still equal
    the golden fixture."""
    import ctypes as C
    g = load([p for p in GOLDEN if "m64_2x2_zf2" in p][0])
    rx = g["rx"]
    fs, got = gpu_framesync(g)
    F = 8
    buf, L = _upload_batch([rx] * F)
    b = _lib.Batch(buf.addr, L, rx.shape[1], F, int(g["pid"]), None, None, 0, None, 0, 0, 1,
                   0, None, 0, 1.0)
    _lib.check(_lib.lib().mimo_rx_process_batch(fs._h, C.byref(b), None), "process_batch")
    res = (_lib.FrameResult * F)()
    _lib.check(_lib.lib().mimo_rx_batch_results(fs._h, res, F), "batch_results")
    assert all(r.status == _lib.FRAME_OK and r.sync_index == int(g["sync_index"]) for r in res)
    fs.reset()
    got.clear()
    pos = 0
    rng = np.random.default_rng(11)
    while pos < rx.shape[1]:
        c = int(rng.integers(1, 2500))
        fs.execute([r[pos:pos + c] for r in rx], min(c, rx.shape[1] - pos))
        pos += c
    assert_sync_equal(fs, g)
    assert evm_delta(np.stack(got), g["symbols"]) <= SYM_TOL


@pytest.mark.parametrize("lead_kind", ["noise", "zeros"])
def test_streaming_execute_memory_is_bounded_by_the_window(lead_kind):
    """A live stream that stays unsynchronised for a long time: a lead of more than 20
    reference windows (ACB + TX, framing.cc:387-388) before a frame, fed to the streaming
    execute in random chunks. The device capture stays within 2x the window (the reference
    holds one window ring; here only what a later trigger can reach is kept while seeking),
    and sync, plateau, samples processed and symbols equal the oracle's on the whole stream.
    The lead is noise, or exact zeros (an idle radio: every S&C window is the oracle's 0/0,
    which compares false, so those positions are proven zeros too)."""
    M, cp, N, nac, pid, qam = 1024, 76, 2, 4, 40, 16
    SL = M + cp
    win = SL * (nac * N + 4) + pid * SL                   # ACB + TX
    rx, txo, _ = ref.synth_frame(M, cp, N, nac, pid, qam, seed=5, frame=0, offset=-1,
                                 snr_db=25.0)
    rng = np.random.default_rng(17)
    lead_len = 21 * win
    nstd = np.sqrt(0.0625 * 10 ** (-25.0 / 10) / 2)
    lead = (rng.standard_normal((N, lead_len)) + 1j * rng.standard_normal((N, lead_len))) * nstd
    if lead_kind == "zeros":
        lead[:] = 0
    stream = np.concatenate([lead.astype(np.complex64), rx], axis=1)
    o = ref.FrameSyncRef(M, cp, N, nac, pid_max=pid, detector=_lib.DET_ZF2)
    assert o.execute(stream) == ref.STATE_MIMO
    got = []
    ms0, ms1 = new_codes(N)
    fs = fr.framesync(M, cp, N, nac, fr.ofdmframe_init_default_sctype(M), ms0, ms1,
                      callback=lambda xs, m: got.append(np.stack([x.copy() for x in xs])),
                      pid_max=pid, detector=_lib.DET_ZF2, qam_order=qam)
    pos, peak = 0, 0
    while pos < stream.shape[1]:
        c = int(rng.integers(1, 40000))
        fs.execute([r[pos:pos + c] for r in stream], min(c, stream.shape[1] - pos))
        pos += c
        peak = max(peak, fs.stream_capacity()[0])
    assert peak <= 2 * win, (peak, win)
    assert fs.get_sync_index() == o.get_sync_index()
    assert fs.get_num_samples_processed() == o.get_num_samples_processed()
    assert [fs.get_plateau_start(s) for s in range(N)] == [o.get_plateau_start(s)
                                                          for s in range(N)]
    assert evm_delta(np.stack(got)[:pid], o.symbols()[:pid]) <= SYM_TOL


@pytest.mark.parametrize("M", [64, 1024])
def test_debug_log_traces_match_oracle(tmp_path, M):
    """DEBUG_LOG (mimo/config.h:84-86): the streaming execute writes the reference's traces,
    the files mimo/apps/plot.py opens -- f_sc_<k>.dat (y of every sample processed while
    seeking, through the trigger: the oracle's trace bit for bit) and corr_<k>_<ac>.dat
    (every lag's search metric at window index SL (ac + 1) + lag, ACB - M floats: the oracle's
    brute-force metric to fp32 FFT rounding). M = 64 runs the LDS search kernel, M = 1024 the
    wave-local one; the capture is fed in ragged chunks."""
    if M == 64:
        g = load([p for p in GOLDEN if "m64_2x2_zf2" in p][0])
        cp, N, nac, pid = (int(g[k]) for k in ("cp", "N", "nac", "pid"))
        rx = g["rx"]
        det = _lib.DET_ZF2
    else:
        cp, N, nac, pid, det = 76, 2, 4, 20, _lib.DET_ZF2
        rx, _, _ = ref.synth_frame(M, cp, N, nac, pid, 16, seed=5, frame=0, offset=-1,
                                   snr_db=25.0)
    o = ref.FrameSyncRef(M, cp, N, nac, pid_max=pid, detector=det, trace_sc=True,
                         trace_corr=True)
    assert o.execute(rx) == ref.STATE_MIMO
    ms0, ms1 = new_codes(N)
    fs = fr.framesync(M, cp, N, nac, fr.ofdmframe_init_default_sctype(M), ms0, ms1,
                      pid_max=pid, detector=det, qam_order=16)
    fs.set_debug_log(tmp_path)
    pos = 0
    rng = np.random.default_rng(3)
    while pos < rx.shape[1]:
        c = int(rng.integers(1, 5000))
        fs.execute([r[pos:pos + c] for r in rx], min(c, rx.shape[1] - pos))
        pos += c
    assert fs.get_sync_index() == o.get_sync_index()
    fs.set_debug_log(None)                       # closes the f_sc files
    SL = M + cp
    acb = SL * (nac * N + 4)
    for k in range(N):
        y = np.fromfile(tmp_path / f"f_sc_{k + 1}.dat", np.float32)
        yo = o.sc_trace(k)
        assert len(y) == len(yo) == max(fs.get_plateau_end(s) for s in range(N)) + 1
        assert np.array_equal(y.view(np.uint32), yo.view(np.uint32))
    ctr, s0tr = o.corr_trace()                   # [N][N nac][SL], [N][SL]
    for k in range(N):
        for ac in range(N * nac + 1):
            c = np.fromfile(tmp_path / f"corr_{k + 1}_{ac}.dat", np.float32)
            assert len(c) == acb - M
            want = s0tr[k] if ac == 0 else ctr[k, ac - 1]
            seg = c[SL * ac:SL * ac + SL]
            assert np.count_nonzero(np.delete(c, np.arange(SL * ac, SL * ac + SL))) == 0
            assert np.allclose(seg, want, rtol=2e-3, atol=2e-4 * want.max()), (k, ac)


def test_incomplete_then_complete_and_mimo_semantics():
    g = load([p for p in GOLDEN if "m64_2x2_zf2" in p][0])
    M, cp, N, nac, pid = (int(g[k]) for k in ("M", "cp", "N", "nac", "pid"))
    SL = M + cp
    n_e = int(g["sync_index"]) - SL + SL * (nac * N + 4) + pid * SL
    fs, got = gpu_framesync(g)
    rx = g["rx"]
    assert fs.execute(list(rx[:, :n_e])) == fr.STATE_SAVE_ACCESS_CODES
    assert fs.get_num_samples_processed() == n_e and not got
    assert fs.execute(list(rx[:, n_e:n_e + 1])) == fr.STATE_MIMO
    assert fs.get_num_samples_processed() == n_e + 1
    fs.execute(list(rx[:, n_e + 1:]))
    assert fs.get_num_samples_processed() == n_e + 2
    assert len(got) == pid + 2


def _upload_batch(frames, pad=0):
    """frames: list of [N, L_i] arrays -> DeviceBuffer [F][N][stride]."""
    N = frames[0].shape[0]
    L = max(f.shape[1] for f in frames) + pad
    host = np.zeros((len(frames), N, L), np.complex64)
    for i, f in enumerate(frames):
        host[i, :, :f.shape[1]] = f
    buf = _lib.DeviceBuffer(host.nbytes)
    buf.upload(host)
    return buf, L


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_batch_path_matches_golden(path):
    g = load(path)
    M, cp, N, nac, pid, qam = (int(g[k]) for k in ("M", "cp", "N", "nac", "pid", "qam"))
    P = RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                 detector=int(g["detector"]), keep_identity_bias=bool(g["keep_identity_bias"]),
                 siso_tx=int(g["siso_tx"]), siso_rx=int(g["siso_rx"]), qam_order=qam, p=g["p"])
    rxo = Receiver(P)
    F = 3
    buf, L = _upload_batch([g["rx"]] * F)
    mocc = rxo.M_occ
    out = _lib.DeviceBuffer(F * N * pid * mocc * 8)
    idx = _lib.DeviceBuffer(F * N * pid * mocc)
    ref_idx = np.broadcast_to(g["tx_idx"], (F,) + g["tx_idx"].shape).copy()
    rbuf = _lib.DeviceBuffer(ref_idx.nbytes)
    rbuf.upload(ref_idx)
    rxo.process(buf, L, g["rx"].shape[1], F, max_out=pid, out_sym=out, out_idx=idx, ref_mode=1,
                ref_idx=rbuf)
    res = rxo.results()
    ci, si = rxo.corr()
    syms = out.download(np.complex64, F * N * pid * mocc).reshape(F, N, pid, mocc)
    rid = idx.download(np.uint8, F * N * pid * mocc).reshape(F, N, pid, mocc)
    for f in range(F):
        r = res[f]
        assert r["status"] == _lib.FRAME_OK
        assert r["sync_index"] == int(g["sync_index"])
        assert r["num_samples_processed"] == int(g["num_samples_processed"])
        assert r["plateau_start"] == list(g["plateau_start"])
        assert r["n_sym"] == pid + 2
        assert np.array_equal(ci[f], g["corr_idx"]) and np.array_equal(si[f], g["s0_idx"])
        ours = syms[f].transpose(1, 0, 2)            # -> [sym][t][j] like the callbacks
        assert evm_delta(ours, g["symbols"][:pid]) <= SYM_TOL
        # demap parity: identical indices except where the oracle sits on a boundary
        ref_idx_o, num, den, err = ref.demap_evm(g["symbols"][:pid], qam, g["tx_idx"])
        mism = rid[f] != ref_idx_o
        if mism.any():
            y = g["symbols"][:pid].transpose(1, 0, 2)[mism]
            L_ = int(np.sqrt(qam))
            s = np.sqrt(2 * (L_ * L_ - 1) / 3.0)
            v = np.concatenate([(y.real * s + L_) / 2, (y.imag * s + L_) / 2])
            assert np.min(np.abs(v - np.round(v))) < 1e-3
        assert np.array_equal(r["errors"], err.astype(np.int64)) or mism.any()
        if np.all(den > 0):
            edb_gpu = 10 * np.log10(r["evm_num"] / r["evm_den"])
            edb_ref = 10 * np.log10(num / den)
            assert np.abs(edb_gpu - edb_ref).max() <= EVM_DB_TOL


def test_batch_frames_are_independent():
    gs = [load(p) for p in GOLDEN if "m64_2x2" in p and "liquid" not in p and "siso" not in p]
    g = gs[0]
    M, cp, N, nac, pid = (int(g[k]) for k in ("M", "cp", "N", "nac", "pid"))
    frames = [ref.synth_frame(M, cp, N, nac, pid, 16, seed=11, frame=f, offset=-1,
                              snr_db=30.0)[0] for f in range(6)]
    # frame 4 is pure noise (no sync); frame 5 is truncated before the window completes
    frames[4] = (np.random.default_rng(0).standard_normal(frames[4].shape) * 0.01).astype(
        np.complex64)
    P = RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                 detector=_lib.DET_ZF2, qam_order=16)
    rxo = Receiver(P)
    Lmin = min(f.shape[1] for f in frames)
    oracle = []
    for i, f in enumerate(frames):
        o = ref.FrameSyncRef(M, cp, N, nac, pid_max=pid)
        o.execute(f[:, :Lmin])
        oracle.append(o)
    buf, L = _upload_batch([f[:, :Lmin] for f in frames])
    rxo.process(buf, L, Lmin, len(frames), max_out=pid)
    res = rxo.results()
    for i, o in enumerate(oracle):
        r = res[i]
        st = o.state
        if st == ref.STATE_SEEK_PLATEAU:
            assert r["status"] == _lib.FRAME_NO_SYNC
        elif st == ref.STATE_SAVE_ACCESS_CODES:
            assert r["status"] == _lib.FRAME_INCOMPLETE
            assert r["sync_index"] == o.get_sync_index()
        else:
            assert r["status"] == _lib.FRAME_OK
            assert r["sync_index"] == o.get_sync_index()
        assert r["num_samples_processed"] == o.get_num_samples_processed()
    assert res[4]["status"] == _lib.FRAME_NO_SYNC


def test_set_siso_after_graph_capture_decodes_the_new_pair():
    """mimo_rx_set_siso between identical batch calls: the captured graph (whose decode
    arguments carry the SISO indices) must not be replayed; the third call equals a receiver
    created with the new pair."""
    import torch
    from rub_mimo_amd.receiver import Synthesizer, SynthParams
    M, cp, N, nac, pid, F = 256, 19, 2, 4, 16, 2
    sp = SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid,
                     qam_order=16, seed=9, snr_db=30.0)
    syn = Synthesizer(sp)
    L = sp.max_frame_len()
    iq = torch.empty((F, N, L), dtype=torch.complex64, device="cuda")
    syn.generate(iq, L, L, F, frame_id0=0)

    def run(rx):
        sym = torch.zeros((F, N, pid, M), dtype=torch.complex64, device="cuda")
        rx.process(iq, L, L, F, max_out=pid, out_sym=sym, ref_mode=2, ref_seed=9)
        torch.cuda.synchronize()
        return sym.cpu(), [float(np.sum(r["evm_num"])) for r in rx.results()]

    base = dict(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                detector=_lib.DET_SISO, qam_order=16)
    rx = Receiver(RxParams(**base, siso_tx=0, siso_rx=0))
    first = run(rx)
    run(rx)                            # captured into a graph
    rx.set_siso(1, 1)
    got = run(rx)
    want = run(Receiver(RxParams(**base, siso_tx=1, siso_rx=1)))
    assert torch.equal(got[0], want[0]) and got[1] == want[1]
    assert not torch.equal(got[0], first[0])


def test_repeated_batch_graph_replay_is_identical():
    """A repeated process() call is captured into a HIP graph and replayed (engine.cpp); its
    results, symbols and indices must equal the direct launches bit for bit, and a changed
    argument must fall back to direct launches."""
    import torch
    from rub_mimo_amd.receiver import Synthesizer, SynthParams
    M, cp, N, nac, pid, F = 256, 19, 4, 4, 24, 3
    sp = SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid,
                     qam_order=16, seed=5, snr_db=30.0)
    syn = Synthesizer(sp)
    L = sp.max_frame_len()
    dev = torch.device("cuda", 0)
    iq = torch.empty((F, N, L), dtype=torch.complex64, device=dev)
    syn.generate(iq, L, L, F, frame_id0=0)
    rx = Receiver(RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                           detector=_lib.DET_MMSE, qam_order=16))
    sym = torch.zeros((F, N, pid, M), dtype=torch.complex64, device=dev)
    idx = torch.zeros((F, N, pid, M), dtype=torch.uint8, device=dev)
    outs = []
    for it in range(4):   # direct, capture, replay, replay
        sym.zero_()
        idx.zero_()
        rx.process(iq, L, L, F, max_out=pid, out_sym=sym, out_idx=idx, ref_mode=2, ref_seed=5)
        torch.cuda.synchronize()
        res = rx.results()
        outs.append((sym.clone(), idx.clone(), [(r["status"], r["sync_index"],
                                                 float(np.sum(r["evm_num"]))) for r in res]))
    for o in outs[1:]:
        assert torch.equal(o[0], outs[0][0]) and torch.equal(o[1], outs[0][1])
        assert o[2] == outs[0][2]
    # a different frame count must not replay the captured batch
    rx.process(iq, L, L, F - 1, max_out=pid, out_sym=sym, out_idx=idx, ref_mode=2, ref_seed=5)
    torch.cuda.synchronize()
    res2 = rx.results(F - 1)
    assert [(r["status"], r["sync_index"]) for r in res2] == [t[:2] for t in outs[0][2][:F - 1]]


def test_alternating_capture_buffers_replay_their_own_graphs():
    """Double-buffered ingest alternates two capture buffers: each batch key keeps its own
    captured graph (a small cache in engine.cpp), and every replay equals the direct launch
    of the same buffer."""
    import torch
    M, cp, N, nac, pid, F = 256, 19, 4, 4, 24, 2
    sp = SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid,
                     qam_order=16, seed=15, snr_db=30.0)
    syn = Synthesizer(sp)
    L = sp.max_frame_len()
    bufs = [torch.empty((F, N, L), dtype=torch.complex64, device="cuda") for _ in range(2)]
    syn.generate(bufs[0], L, L, F, frame_id0=0)
    syn.generate(bufs[1], L, L, F, frame_id0=F)
    rx = Receiver(RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                           detector=_lib.DET_MMSE, qam_order=16))
    sym = torch.zeros((F, N, pid, M), dtype=torch.complex64, device="cuda")
    seen = {0: [], 1: []}
    for it in range(8):             # direct, direct, capture, capture, replays
        k = it % 2
        sym.zero_()
        rx.process(bufs[k], L, L, F, max_out=pid, out_sym=sym, ref_mode=0)
        torch.cuda.synchronize()
        seen[k].append((sym.clone(), [(r["status"], r["sync_index"]) for r in rx.results()]))
    for k in (0, 1):
        for o in seen[k][1:]:
            assert torch.equal(o[0], seen[k][0][0]) and o[1] == seen[k][0][1]
    assert not torch.equal(seen[0][0][0], seen[1][0][0])


def test_gpu_synth_matches_oracle_synth():
    M, cp, N, nac, pid, qam = 128, 16, 4, 3, 5, 64
    S = Synthesizer(SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid,
                                qam_order=qam, seed=7, snr_db=25.0))
    F = 2
    L = max(S.frame_len(f) for f in range(F))
    out = _lib.DeviceBuffer(F * N * L * 8)
    tx = _lib.DeviceBuffer(F * N * pid * M)
    Hb = _lib.DeviceBuffer(F * N * N * 8)
    S.generate(out, L, L, F, frame_id0=0, tx_idx=tx, H=Hb)
    got = out.download(np.complex64, F * N * L).reshape(F, N, L)
    txi = tx.download(np.uint8, F * N * pid * M).reshape(F, N, pid, M)
    H = Hb.download(np.complex64, F * N * N).reshape(F, N, N)
    for f in range(F):
        rx, txo, Ho = ref.synth_frame(M, cp, N, nac, pid, qam, seed=7, frame=f, offset=-1,
                                      snr_db=25.0)
        assert S.frame_len(f) == rx.shape[1]
        assert np.array_equal(txi[f], txo)
        assert np.abs(H[f] - Ho).max() < 1e-5
        d = got[f, :, :rx.shape[1]] - rx
        assert np.sqrt(np.mean(np.abs(d) ** 2)) < 1e-5 * np.sqrt(np.mean(np.abs(rx) ** 2)) + 1e-7


def test_framegen_matches_oracle_tx():
    M, cp, N, nac = 64, 16, 2, 4
    p = fr.ofdmframe_init_default_sctype(M)
    ms0, ms1 = new_codes(N)
    fg = fr.framegen(M, cp, N, nac, p, ms0, ms1)
    n, sw = fg.write_sync_words()
    assert n == (nac * N + 1) * (M + cp)
    s0b, s1b = ref.code_bits(M, N, nac, codes.s1_polynomials(N))
    S0, s0 = ref.init_S0(p, s0b)
    gs0, gs1 = fg.codes()
    assert np.abs(gs0 - s0).max() < 1e-6
    rng = np.random.default_rng(2)
    syms = (rng.standard_normal((N, M)) + 1j * rng.standard_normal((N, M))).astype(np.complex64)
    cnt, tx = fg.assemble_mimo_packet(syms)
    assert cnt == M + cp
    for t in range(N):
        y = ref.fft(syms[t], inverse=True) / np.float32(np.sqrt(M))
        assert np.abs(tx[t, cp:] - y).max() < 1e-5
        assert np.array_equal(tx[t, :cp], tx[t, M:])      # cyclic prefix


def _c_frame_parity(M, cp, N, nac, pid, qam, det, snr, seed, bias=True, max_delta=SYM_TOL,
                    search_mode=0, path=None, out_idx=False, ff_margin=None):
    S = Synthesizer(SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid,
                                qam_order=qam, seed=seed, snr_db=snr))
    L = S.frame_len(0)
    out = _lib.DeviceBuffer(N * L * 8)
    tx = _lib.DeviceBuffer(N * pid * M)
    S.generate(out, L, L, 1, tx_idx=tx)
    rx = out.download(np.complex64, N * L).reshape(N, L)
    txi = tx.download(np.uint8, N * pid * M).reshape(N, pid, M)
    P = RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                 detector=det, keep_identity_bias=bias, qam_order=qam)
    rxo = Receiver(P)
    osym = _lib.DeviceBuffer(N * pid * M * 8)
    oidx = _lib.DeviceBuffer(N * pid * M) if out_idx else None
    rxo.process(out, L, L, 1, max_out=pid, out_sym=osym, out_idx=oidx, ref_mode=2,
                ref_seed=seed, frame_id0=0)
    r = rxo.results()[0]
    if path is not None:                 # the decode kernel family this geometry must take
        assert rxo.decode_path() == path, (rxo.decode_path(), path)
    ci, si = rxo.corr()
    o = ref.FrameSyncRef(M, cp, N, nac, pid_max=pid, detector=det, keep_identity_bias=bias,
                         trace_corr=True, search_mode=search_mode)
    if ff_margin is None:
        assert o.execute(rx) == ref.STATE_MIMO
    else:
        # full-size frames: the oracle's S&C histories advanced without the dot products to
        # ff_margin samples before the frame's S0 symbol (the metric from there on is the full
        # scan's bit for bit, ref_framesync_fast_forward; the oracle refuses a start inside a
        # plateau run), then its own plateau rule, search, LS and decode. The start comes from
        # the synthesiser's frame layout (synth_kernels.hip mix_kernel: SL (N nac + 1) + u
        # samples of noise, then S0), not from what the GPU reported, and the GPU's plateau
        # starts must lie near that S0
        SL = M + cp
        u = L - SL * (2 * N * nac + 2 + pid + 3)          # SynthParams.tail_syms = 3
        assert 0 <= u < SL
        s0_at = SL * (N * nac + 1) + u
        assert all(s0_at - SL <= ps <= s0_at + 2 * SL for ps in r["plateau_start"][:N]), \
            (r["plateau_start"][:N], s0_at)
        p0 = s0_at - ff_margin
        assert p0 > 0
        assert o.execute_from(rx, p0) == ref.STATE_MIMO
    assert r["status"] == _lib.FRAME_OK
    assert r["sync_index"] == o.get_sync_index()
    assert r["plateau_start"] == [o.get_plateau_start(s) for s in range(N)]
    assert r["num_samples_processed"] == o.get_num_samples_processed()
    oci, _, osi, _ = o.get_corr()
    ctr, _ = o.corr_trace()
    # corr indices bit-exact wherever the oracle's peak is unambiguous (first max wins;
    # a deep-faded link has no peak in the reference either, see test_oracle)
    SL = M + cp
    for rr in range(N):
        for ac in range(N * nac):
            tr = np.sort(ctr[rr, ac])
            if tr[-1] > (1 + 1e-3) * tr[-2]:
                assert ci[0, rr, ac] == oci[rr, ac], (rr, ac)
    syms_o = o.symbols()[:pid]
    ours = osym.download(np.complex64, N * pid * M).reshape(N, pid, M).transpose(1, 0, 2)
    d = evm_delta(ours, syms_o)
    assert d <= max_delta, d
    dec_o, num, den, err = ref.demap_evm(syms_o, qam, txi)
    edb_gpu = 10 * np.log10(r["evm_num"] / r["evm_den"])
    edb_ref = 10 * np.log10(num / den)
    assert np.abs(edb_gpu - edb_ref).max() <= EVM_DB_TOL, (edb_gpu, edb_ref)
    if out_idx:
        # hard decisions equal the oracle's except where its symbol sits within 1e-3 of a
        # decision boundary; the symbol-error counts likewise
        got = oidx.download(np.uint8, N * pid * M).reshape(N, pid, M)
        mism = got != dec_o
        if mism.any():
            y = syms_o.transpose(1, 0, 2)[mism]
            Lq = int(np.sqrt(qam))
            sc = np.sqrt(2 * (Lq * Lq - 1) / 3.0)
            v = np.concatenate([(y.real * sc + Lq) / 2, (y.imag * sc + Lq) / 2])
            assert np.min(np.abs(v - np.round(v))) < 1e-3
        assert np.abs(r["errors"] - err.astype(np.int64)).max() <= int(mism.sum())
    return d, edb_gpu


def test_c2_2x2_zf_1024_16qam():
    d, e = _c_frame_parity(1024, 76, 2, 20, 200, 16, _lib.DET_ZF2, 25.0, seed=21)
    assert np.all(e < -15)


def test_c2_2x2_zf_1024_16qam_full_frame():
    """BASELINE config C2 at full size (PID 1000, the streaming decode's 2x2 form)."""
    d, e = _c_frame_parity(1024, 76, 2, 20, 1000, 16, _lib.DET_ZF2, 25.0, seed=22)
    assert np.all(e < -15)


def test_block_search_form_matches_oracle():
    """The wave-local search_ls_wave_kernel is the default for F >= 1024; the block-exchange
    search_ls_kernel stays behind RMIMO_SEARCH_FORM=block (read once per process, so a child
    interpreter runs the same C2/C3 parity cases with it)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r); sys.path.insert(0, %r)\n"
            "import test_gpu as t\nfrom rub_mimo_amd import _lib\n"
            "t._c_frame_parity(1024, 76, 2, 20, 200, 16, _lib.DET_ZF2, 25.0, seed=21)\n"
            "t._c_frame_parity(2048, 152, 4, 20, 60, 64, _lib.DET_MMSE, 30.0, seed=31,"
            " path=_lib.DECODE_STREAM, out_idx=True)\nprint('block-search parity ok')\n"
            % (root, os.path.join(root, "tests")))
    env = dict(os.environ, RMIMO_SEARCH_FORM="block")
    out = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, timeout=100,
                         capture_output=True, text=True)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    assert "block-search parity ok" in out.stdout


def _ls_batch_outputs(M, cp, N, nac, pid, qam, det, seed, n_frames):
    """One batch of n_frames synthetic frames through the default receive path: G, W, the
    frames' noise variances and EVM sums and the decoded symbols (raw bytes for bitwise
    comparisons)."""
    S = Synthesizer(SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid,
                                qam_order=qam, seed=seed, snr_db=30.0))
    L = max(S.frame_len(i) for i in range(n_frames))
    out = _lib.DeviceBuffer(n_frames * N * L * 8)
    S.generate(out, L, L, n_frames)
    P = RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                 detector=det, keep_identity_bias=True, qam_order=qam)
    rxo = Receiver(P)
    osym = _lib.DeviceBuffer(n_frames * N * pid * M * 8)
    osym.zero()                          # (frames that do not sync write no symbols)
    rxo.process(out, L, L, n_frames, max_out=pid, out_sym=osym, ref_mode=2, ref_seed=seed)
    res = rxo.results()
    # frames that did not sync leave G, W and their symbols unwritten: compared as zeros
    ok = np.array([r["status"] == _lib.FRAME_OK for r in res])
    nv = np.array([r["noise_var"] for r in res], np.float64)
    ev = np.array([[r["evm_num"], r["evm_den"]] for r in res], np.float64)
    G, W = rxo.G(), rxo.W()
    G[~ok] = 0
    W[~ok] = 0
    y = osym.download(np.complex64, n_frames * N * pid * M).reshape(n_frames, -1)
    y[~ok] = 0
    return G, W, nv, ev, y


def test_ls_window_equals_fused_terms():
    """The default LS (ls_window_kernel: each (frame, rx, tx) workgroup transforms its access-code
    windows at the search's keys and sums X/S1 in code order, no terms in HBM) against the fused
    form (RMIMO_LS_FORM=terms, read once per process: a child interpreter; the search stores
    every code's X/S1 and ls_combine_q_kernel sums them): G, W, the noise variances, EVM sums and
    symbols agree to fp32 rounding at M = 512, 1024 (C2), 2048 (C3) and 4096 (C4): the codes are
    summed in the same order in fp64 with the same residual-variance reduction tree, and the
    transforms are the same plan, but hipcc contracts a few of the butterflies' products into
    FMAs differently in the two kernels (1-ulp differences in some terms, measured). Each form
    is deterministic on its own (the batch = single-frame and replay tests)."""
    import subprocess
    import sys
    import tempfile
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cases = [(1024, 76, 2, 20, 24, 16, _lib.DET_ZF2, 51, 5),
             (2048, 152, 4, 20, 12, 64, _lib.DET_MMSE, 52, 6),
             (512, 40, 4, 6, 12, 16, _lib.DET_MMSE, 53, 4),
             (4096, 304, 8, 2, 66, 256, _lib.DET_MMSE, 54, 2)]
    with tempfile.TemporaryDirectory() as td:
        code = ("import sys; sys.path.insert(0, %r); sys.path.insert(0, %r)\n"
                "import numpy as np, test_gpu as t\n"
                "for i, c in enumerate(%r):\n"
                "    G, W, nv, ev, y = t._ls_batch_outputs(*c)\n"
                "    np.savez(%r + '/c%%d.npz' %% i, G=G, W=W, nv=nv, ev=ev, y=y)\n"
                "print('terms ok')\n" % (root, os.path.join(root, "tests"), cases, td))
        env = dict(os.environ, RMIMO_LS_FORM="terms")
        out = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, timeout=150,
                             capture_output=True, text=True)
        assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
        for i, c in enumerate(cases):
            G, W, nv, ev, y = _ls_batch_outputs(*c)
            o = np.load(os.path.join(td, "c%d.npz" % i))
            assert np.abs(G).max() > 0
            assert np.abs(G - o["G"]).max() <= 2e-6 * np.abs(o["G"]).max(), c
            assert np.abs(W - o["W"]).max() <= 1e-5 * np.abs(o["W"]).max(), c
            assert np.allclose(nv, o["nv"], rtol=1e-5, atol=0), c
            assert np.allclose(ev, o["ev"], rtol=1e-5, atol=0), c
            assert evm_delta(y, o["y"]) <= 1e-5, c



_CFO_GEOMS = {"c3": (2048, 152, 4, 20, 24, 64, _lib.DET_MMSE, 4),
              "c2": (1024, 76, 2, 20, 24, 16, _lib.DET_ZF2, 4),
              "c4": (4096, 304, 8, 2, 24, 256, _lib.DET_MMSE, 2)}


def _cfo_ls_outputs(mode, seed=813, eps=0.3, geom="c3"):
    """A batch (C3 geometry by default: 4 captures, 24 data symbols) rotated by eps subcarrier
    spacings through the opt-in CFO path ("fold": reference indices from HBM, the derotating
    loads; "scratch": ref_mode 2, the stage-1 scratch capture): G, W, noise variances, EVM sums
    and the frames' CFO estimates."""
    import torch
    from rub_mimo_amd.receiver import cfo_derotate
    M, cp, N, nac, pid, qam, det, F = _CFO_GEOMS[geom]
    sp = SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid,
                     qam_order=qam, seed=seed, snr_db=30.0)
    S = Synthesizer(sp)
    L = sp.max_frame_len()
    iq = torch.empty((F, N, L), dtype=torch.complex64, device="cuda")
    tx = torch.empty((F, N, pid, M), dtype=torch.uint8, device="cuda")
    S.generate(iq, L, L, F, tx_idx=tx)
    cfo_derotate(iq, L, F * N, L, 0, -eps, M)
    rxo = Receiver(RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                            detector=det, qam_order=qam, cfo_correct=True))
    if mode == "fold":
        rxo.process(iq, L, L, F, max_out=pid, ref_mode=1, ref_idx=tx)
    else:
        rxo.process(iq, L, L, F, max_out=pid, ref_mode=2, ref_seed=seed, frame_id0=0)
    torch.cuda.synchronize()
    res = rxo.results()
    ok = np.array([r["status"] == _lib.FRAME_OK for r in res])
    nv = np.array([r["noise_var"] for r in res], np.float64)
    ev = np.array([[r["evm_num"], r["evm_den"]] for r in res], np.float64)
    ce = np.array([r["cfo_eps"] for r in res], np.float64)
    G, W = rxo.G(), rxo.W()
    G[~ok] = 0
    W[~ok] = 0
    return G, W, nv, ev, ce, ok


@pytest.mark.parametrize("mode,geom", [("fold", "c3"), ("scratch", "c3"), ("scratch", "c2"),
                                       ("scratch", "c4")])
def test_ls_window_with_cfo_equals_fused_terms(mode, geom):
    """With the opt-in CFO the default LS is ls_window_kernel too: the folded form's stage-1
    derotation of the window and the stage-2 residual's rotation of the code's term (a constant
    per window) are applied as one phasor sequence to the window's samples before the transform.
    Against the fused-terms form (RMIMO_LS_FORM=terms in a child: the search's derotated terms,
    rotated in fp64 and summed by ls_combine_q_kernel): G, W, noise variances and EVM sums to
    fp32 rounding, the CFO estimates (recorded by the LS kernel of either form) equal; at C3,
    C2 (M = 1024, 2x2 ZF) and C4 (M = 4096, 8x8, two access codes per stream)."""
    import subprocess
    import sys
    import tempfile
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with tempfile.TemporaryDirectory() as td:
        code = ("import sys; sys.path.insert(0, %r); sys.path.insert(0, %r)\n"
                "import numpy as np, test_gpu as t\n"
                "G, W, nv, ev, ce, ok = t._cfo_ls_outputs(%r, geom=%r)\n"
                "np.savez(%r + '/o.npz', G=G, W=W, nv=nv, ev=ev, ce=ce, ok=ok)\n"
                "print('terms ok')\n" % (root, os.path.join(root, "tests"), mode, geom, td))
        env = dict(os.environ, RMIMO_LS_FORM="terms")
        out = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, timeout=150,
                             capture_output=True, text=True)
        assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
        G, W, nv, ev, ce, ok = _cfo_ls_outputs(mode, geom=geom)
        o = np.load(os.path.join(td, "o.npz"))
    assert ok.sum() >= 1 and np.array_equal(ok, o["ok"])
    assert np.array_equal(ce, o["ce"]) and np.all(np.abs(ce[ok] - 0.3) < (2e-5 if geom == "c3" else 1e-3))
    assert np.abs(G - o["G"]).max() <= 2e-6 * np.abs(o["G"]).max()
    assert np.abs(W - o["W"]).max() <= 1e-5 * np.abs(o["W"]).max()
    assert np.allclose(nv, o["nv"], rtol=1e-5, atol=0)
    assert np.allclose(ev, o["ev"], rtol=1e-5, atol=0)

def _sctype(M, kind):
    """None (the default allocation), "liquid" (guard bands and pilots) or "all" (every
    subcarrier a data carrier)."""
    if kind == "liquid":
        return fr.ofdmframe_init_liquid_sctype(M)
    if kind == "all":
        return np.full(M, 2, np.uint8)
    return None


def _layout_batch(M, cp, N, nac, pid, qam, det, seed, n_frames, layout, path, sct=None):
    """n_frames synthetic frames decoded with out_layout = layout and reference indices
    (ref_mode 1) in that layout; returns the outputs as stream-major host arrays and the
    frames' result records."""
    p = _sctype(M, sct)
    S = Synthesizer(SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid,
                                qam_order=qam, seed=seed, snr_db=30.0, p=p))
    L = max(S.frame_len(i) for i in range(n_frames))
    rx = Receiver(RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                           detector=det, keep_identity_bias=True, qam_order=qam, p=p))
    mocc = rx.M_occ
    out = _lib.DeviceBuffer(n_frames * N * L * 8)
    tx = _lib.DeviceBuffer(n_frames * N * pid * mocc)
    S.generate(out, L, L, n_frames, tx_idx=tx)
    txi = tx.download(np.uint8, n_frames * N * pid * mocc).reshape(n_frames, N, pid, mocc)
    ref = _lib.DeviceBuffer(txi.nbytes)
    sym_major = layout == _lib.LAYOUT_SYMBOL_MAJOR
    ref.upload(np.ascontiguousarray(txi.transpose(0, 2, 1, 3) if sym_major else txi))
    osym = _lib.DeviceBuffer(n_frames * N * pid * mocc * 8)
    oidx = _lib.DeviceBuffer(n_frames * N * pid * mocc)
    rx.process(out, L, L, n_frames, max_out=pid, out_sym=osym, out_idx=oidx, ref_mode=1,
               ref_idx=ref, out_layout=layout)
    res = rx.results()                   # (synchronises the receiver's stream)
    assert rx.decode_path() == path, (rx.decode_path(), path)
    shape = (n_frames, pid, N, mocc) if sym_major else (n_frames, N, pid, mocc)
    y = osym.download(np.complex64, n_frames * N * pid * mocc).reshape(shape)
    d = oidx.download(np.uint8, n_frames * N * pid * mocc).reshape(shape)
    if sym_major:
        y, d = y.transpose(0, 2, 1, 3), d.transpose(0, 2, 1, 3)
    return np.ascontiguousarray(y), np.ascontiguousarray(d), res


@pytest.mark.parametrize("case", [
    (1024, 76, 2, 20, 24, 16, _lib.DET_ZF2, 61, 3, _lib.DECODE_STREAM),
    (2048, 152, 4, 20, 12, 64, _lib.DET_MMSE, 62, 3, _lib.DECODE_STREAM),
    (4096, 304, 8, 2, 66, 256, _lib.DET_MMSE, 63, 2, _lib.DECODE_SPLIT),
    (4096, 304, 8, 2, 12, 256, _lib.DET_MMSE, 64, 2, _lib.DECODE_SYMBOL),
    (64, 16, 2, 4, 10, 4, _lib.DET_ZF2, 65, 3, _lib.DECODE_SYMBOL),
    (2048, 152, 4, 20, 12, 64, _lib.DET_MMSE, 66, 2, _lib.DECODE_SYMBOL, "liquid"),
    (256, 32, 2, 4, 10, 4, _lib.DET_ZF2, 67, 3, _lib.DECODE_SYMBOL, "all"),
], ids=["c2_stream", "c3_stream", "c4_split", "c4_symbol", "m64_guard_symbol",
        "c3_guard_reg", "m256_allocc_persistent"])
def test_symbol_major_layout_equals_stream_major(case):
    """mimo_batch.out_layout = SYMBOL_MAJOR ([F][max_out][N][M_occ], reference rows likewise)
    writes exactly the stream-major outputs, transposed, on every decode path (streaming,
    8x8 split, per-symbol incl. a guard-band geometry); results (EVM sums, symbol errors) are
    bitwise the same. The per-symbol family is reached by three kernels, each by geometry
    (decode_kernels.hip decode_launch_na): decode_kernel (8x8, and M = 64 with guard bands),
    decode_reg_kernel (4x4 at M = 2048 with the liquid guard/pilot allocation, which the
    streaming decode refuses: it needs every subcarrier occupied) and decode_persistent_kernel
    (2x2 at M = 256, every subcarrier occupied)."""
    *geo, path = case[:10]
    sct = case[10] if len(case) > 10 else None
    pid = geo[4]
    y0, d0, r0 = _layout_batch(*geo, _lib.LAYOUT_STREAM_MAJOR, path, sct)
    y1, d1, r1 = _layout_batch(*geo, _lib.LAYOUT_SYMBOL_MAJOR, path, sct)
    assert any(r["status"] == _lib.FRAME_OK for r in r0)
    for f, (a, b) in enumerate(zip(r0, r1)):
        assert a["status"] == b["status"]
        if a["status"] != _lib.FRAME_OK:
            continue                      # (a frame without sync writes no outputs)
        n = min(a["n_sym"], pid)
        assert np.array_equal(y0[f, :, :n].view(np.uint32), y1[f, :, :n].view(np.uint32)), f
        assert np.array_equal(d0[f, :, :n], d1[f, :, :n]), f
        assert a["evm_num"].tobytes() == b["evm_num"].tobytes()
        assert a["evm_den"].tobytes() == b["evm_den"].tobytes()
        assert np.array_equal(a["errors"], b["errors"])


def test_c3_4x4_mmse_2048_64qam_full_frame():
    """BASELINE config C3 at full size (PID 1000): the oracle needs ~20 s of CPU."""
    d, e = _c_frame_parity(2048, 152, 4, 20, 1000, 64, _lib.DET_MMSE, 30.0, seed=31,
                           path=_lib.DECODE_STREAM, out_idx=True)
    assert np.median(e) < -20


def test_c4_8x8_mmse_4096_256qam_reduced_codes():
    """C4 geometry with 2 access codes so the brute-force oracle stays within ~30 s. PID 12 is
    below M/64, so this takes the per-symbol decode_kernel<12, 8>."""
    _c_frame_parity(4096, 304, 8, 2, 12, 256, _lib.DET_MMSE, 35.0, seed=41, bias=False,
                    path=_lib.DECODE_SYMBOL)


def test_c4_split_decode_matches_oracle():
    """The production C4 decode: with max_out >= M/64 the 8x8 frame takes the split form
    (spectra_persist_kernel<12> writes every symbol's spectra, apply_split2_kernel<8> applies
    W, demaps and sums EVM; decode_stream.hip). PID 66 against the brute-force oracle with 2
    access codes: symbols within the EVM tolerance, indices, errors and EVM-dB."""
    _c_frame_parity(4096, 304, 8, 2, 66, 256, _lib.DET_MMSE, 35.0, seed=48, bias=False,
                    path=_lib.DECODE_SPLIT, out_idx=True)


def test_c4_batch_equals_single_frames():
    """The production C4 decode on a batch equals one-frame batches bit for bit."""
    _c4_batch_equals_single_frames(_lib.DECODE_SPLIT)


def _c4_batch_equals_single_frames(path):
    """A C4 decode on a batch: its workgroups' symbol ranges straddle frames (3 frames x PID
    67), yet each frame's symbols and indices equal a one-frame batch bit for bit; the indices
    are the hard decisions of the symbols and the EVM / symbol-error sums equal a float64
    recount (ref_mode 1)."""
    import torch
    M, cp, N, nac, pid, qam, F = 4096, 304, 8, 2, 67, 256, 3
    sp = SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid,
                     qam_order=qam, seed=58, snr_db=35.0)
    syn = Synthesizer(sp)
    L = sp.max_frame_len()
    iq = torch.empty((F, N, L), dtype=torch.complex64, device="cuda")
    tx = torch.empty((F, N, pid, M), dtype=torch.uint8, device="cuda")
    syn.generate(iq, L, L, F, frame_id0=0, tx_idx=tx)
    P = RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                 detector=_lib.DET_MMSE, qam_order=qam, keep_identity_bias=False)
    rx = Receiver(P)
    sym = torch.zeros((F, N, pid, M), dtype=torch.complex64, device="cuda")
    idx = torch.zeros((F, N, pid, M), dtype=torch.uint8, device="cuda")
    rx.process(iq, L, L, F, max_out=pid, out_sym=sym, out_idx=idx, ref_mode=1, ref_idx=tx)
    torch.cuda.synchronize()
    assert rx.decode_path() == path
    res = rx.results(F)
    ok = [f for f in range(F) if res[f]["status"] == _lib.FRAME_OK]
    assert len(ok) >= 1, [r["status"] for r in res]
    for f in ok:
        s1 = torch.zeros((1, N, pid, M), dtype=torch.complex64, device="cuda")
        i1 = torch.zeros((1, N, pid, M), dtype=torch.uint8, device="cuda")
        r1 = Receiver(P)
        r1.process(iq[f:f + 1], L, L, 1, max_out=pid, out_sym=s1, out_idx=i1, ref_mode=1,
                   ref_idx=tx[f:f + 1])
        torch.cuda.synchronize()
        assert torch.equal(s1[0], sym[f]) and torch.equal(i1[0], idx[f]), f
        ys = sym[f].cpu().numpy()
        dec, num, den, err = ref.demap_evm(ys.transpose(1, 0, 2), qam, tx[f].cpu().numpy())
        assert np.array_equal(dec, idx[f].cpu().numpy()), f
        r = res[f]
        assert np.array_equal(r["errors"], err.astype(np.int64)), (r["errors"], err)
        assert np.allclose(r["evm_num"], num, rtol=1e-4), (r["evm_num"], num)
        assert np.allclose(r["evm_den"], den, rtol=1e-5), (r["evm_den"], den)


@pytest.mark.parametrize("det", [_lib.DET_ZF, _lib.DET_MMSE])
def test_split_decode_m512_matches_oracle(det):
    """spectra_kernel<9> + apply_split_kernel<8>: 8x8 at M = 512 with PID >= M/64."""
    _c_frame_parity(512, 38, 8, 2, 21, 64, det, 35.0, seed=91 + det, bias=False,
                    path=_lib.DECODE_SPLIT, out_idx=True)


def _late_frames_capture(F=4, offs_frac=(0.02, 0.30, 0.55, 0.80), noise_only=()):
    """Noisy captures of five frame lengths with one frame each at the given fraction of the
    capture (past the S&C's first phase from 0.30 on); captures in noise_only hold no frame."""
    import torch
    M, cp, N, nac, pid, qam = 1024, 76, 2, 4, 40, 16
    sp = SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid,
                     qam_order=qam, seed=21, snr_db=25.0)
    S = Synthesizer(sp)
    Lf = sp.max_frame_len()
    frames = torch.zeros((F, N, Lf), dtype=torch.complex64, device="cuda")
    tx = torch.empty((F, N, pid, M), dtype=torch.uint8, device="cuda")
    S.generate(frames, Lf, Lf, F, tx_idx=tx)
    L = 5 * Lf
    rng = np.random.default_rng(7)
    noise = (rng.standard_normal((F, N, L)) + 1j * rng.standard_normal((F, N, L))) * 1e-3
    cap = torch.from_numpy(noise.astype(np.complex64)).cuda()
    offs = [int(offs_frac[f % len(offs_frac)] * L) for f in range(F)]
    for f in range(F):
        if f not in noise_only:
            cap[f, :, offs[f]:offs[f] + Lf] += frames[f]
    geom = (M, cp, N, nac, pid, qam)
    return geom, cap, tx, L, offs


def _late_frames_run(F=7, calls=3):
    """Batch receive of _late_frames_capture(F) (capture 5 noise only), repeated `calls` times
    on one receiver (the second call is captured into a graph, the third replays it); returns
    every call's symbols and per-frame results."""
    import torch
    (M, cp, N, nac, pid, qam), cap, tx, L, offs = _late_frames_capture(F, noise_only=(5,))
    rxo = Receiver(RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                            detector=_lib.DET_ZF2, qam_order=qam))
    out = []
    sym = torch.empty((F, N, pid, M), dtype=torch.complex64, device="cuda")   # one buffer:
    for _ in range(calls):                                                    # graph replays
        sym.zero_()
        torch.cuda.synchronize()
        rxo.process(cap, L, L, F, max_out=pid, out_sym=sym, ref_mode=1, ref_idx=tx)
        torch.cuda.synchronize()
        res = rxo.results(F)
        keys = ("status", "trigger", "sync_index", "num_samples_processed", "plateau_start",
                "noise_var", "evm_num", "evm_den", "errors")
        out.append((sym.cpu().numpy(), [{k: np.asarray(r[k]) for k in keys} for r in res]))
    return out


def _same_runs(a, b):
    assert np.array_equal(a[0], b[0])
    for f, (ra, rb) in enumerate(zip(a[1], b[1])):
        for k in ra:
            assert np.array_equal(ra[k], rb[k]), (f, k, ra[k], rb[k])


def test_two_phase_screen_finds_late_frames():
    """The S&C screen runs in two phases (every capture's chunks through a leading frame's S0, then the
    rest for captures with no trigger yet). Frames placed past the first phase -- at 30%, 55%
    and 80% of a noisy capture -- sync exactly as the oracle does on the whole capture, beside
    one early frame; symbols within the EVM tolerance."""
    import torch
    F = 4
    (M, cp, N, nac, pid, qam), cap, tx, L, offs = _late_frames_capture(F)
    rxo = Receiver(RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                            detector=_lib.DET_ZF2, qam_order=qam))
    sym = torch.zeros((F, N, pid, M), dtype=torch.complex64, device="cuda")
    rxo.process(cap, L, L, F, max_out=pid, out_sym=sym, ref_mode=1, ref_idx=tx)
    torch.cuda.synchronize()
    res = rxo.results(F)
    host = cap.cpu().numpy()
    synced = late = 0
    for f in range(F):
        o = ref.FrameSyncRef(M, cp, N, nac, pid_max=pid, detector=_lib.DET_ZF2)
        st = o.execute(host[f])
        r = res[f]
        if st != ref.STATE_MIMO:
            assert r["status"] != _lib.FRAME_OK, f
            continue
        synced += 1
        assert r["status"] == _lib.FRAME_OK, f
        assert r["sync_index"] == o.get_sync_index(), (f, r["sync_index"], o.get_sync_index())
        assert r["num_samples_processed"] == o.get_num_samples_processed(), f
        assert r["plateau_start"][:N] == [o.get_plateau_start(s) for s in range(N)], f
        assert r["sync_index"] >= offs[f], f
        ours = sym[f].cpu().numpy().transpose(1, 0, 2)
        assert evm_delta(ours, o.symbols()[:pid]) <= SYM_TOL, f
        late += 1 if f > 0 else 0
    assert synced >= 2 and late >= 1


def test_two_phase_screen_equals_one_pass():
    """Early, late and frame-less captures in one batch: the two-phase S&C (engine.cpp
    run_sync) returns what one pass over every chunk returns (RMIMO_SC_PHASES=1, read once per
    process: a child interpreter), bit for bit, on every call -- direct launches, the captured
    graph and its replay. A capture without a frame reports zeros in the fields the estimation
    stages fill in (the first call of a process whose device memory held other data: those
    fields used to keep the slot's previous contents)."""
    import subprocess
    import sys
    import tempfile
    runs = _late_frames_run()
    for r in runs[1:]:
        _same_runs(runs[0], r)
    res = runs[0][1]
    st = [int(r["status"]) for r in res]
    assert st[5] == _lib.FRAME_NO_SYNC
    assert float(res[5]["noise_var"]) == 0.0 and not np.any(res[5]["plateau_start"])
    assert sum(1 for f in (1, 2, 3, 4) if st[f] == _lib.FRAME_OK) >= 2, st
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with tempfile.TemporaryDirectory() as td:
        dst = os.path.join(td, "one_pass.npz")
        code = ("import sys; sys.path.insert(0, %r); sys.path.insert(0, %r)\n"
                "import numpy as np, test_gpu as t\n"
                "sym, res = t._late_frames_run(calls=1)[0]\n"
                "flat = {'sym': sym}\n"
                "for f, r in enumerate(res):\n"
                "    for k, v in r.items(): flat['%%d_%%s' %% (f, k)] = v\n"
                "np.savez(%r, **flat)\nprint('one pass ok')\n"
                % (root, os.path.join(root, "tests"), dst))
        env = dict(os.environ, RMIMO_SC_PHASES="1")
        out = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, timeout=100,
                             capture_output=True, text=True)
        assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
        z = np.load(dst)
        one = (z["sym"], [{k: z["%d_%s" % (f, k)] for k in r} for f, r in enumerate(res)])
    _same_runs(runs[0], one)


def test_captures_starting_at_the_frame_origin():
    """The S&C screen proves positions n < M/2 of a batch capture outright (every lagged sample
    of P[n] precedes the capture, i.e. the framesync's empty delay line: P = 0, y = 0 or 0/0).
    Captures cut so that the frame's S0 begins at or just after sample 0, or preceded by M
    exact zeros (0/0 windows), sync exactly as the oracle does on the same samples."""
    M, cp, N, nac, pid, qam = 1024, 76, 2, 4, 40, 16
    SL = M + cp
    S = Synthesizer(SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid,
                                qam_order=qam, seed=23, snr_db=25.0))
    L0 = S.frame_len(0)
    out = _lib.DeviceBuffer(N * L0 * 8)
    S.generate(out, L0, L0, 1)
    full = out.download(np.complex64, N * L0).reshape(N, L0)
    o = ref.FrameSyncRef(M, cp, N, nac, pid_max=pid, detector=_lib.DET_ZF2)
    assert o.execute(full) == ref.STATE_MIMO
    s0 = min(o.get_plateau_start(s) for s in range(N)) - M   # about where S0's body begins
    caps = []
    for cut in (s0 - cp, s0, s0 + M // 4):                   # S0 at / just before sample 0
        caps.append(np.ascontiguousarray(full[:, max(cut, 0):]))
    caps.append(np.concatenate([np.zeros((N, M), np.complex64), caps[0]], axis=1))
    L = max(c.shape[1] for c in caps)
    F = len(caps)
    host = np.zeros((F, N, L), np.complex64)
    for f, c in enumerate(caps):
        host[f, :, :c.shape[1]] = c
    buf = _lib.DeviceBuffer(host.nbytes)
    buf.upload(host)
    rxo = Receiver(RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                            detector=_lib.DET_ZF2, qam_order=qam))
    rxo.process(buf, L, L, F, max_out=pid)
    res = rxo.results(F)
    for f in range(F):
        of = ref.FrameSyncRef(M, cp, N, nac, pid_max=pid, detector=_lib.DET_ZF2)
        st = of.execute(host[f])
        r = res[f]
        assert (r["status"] == _lib.FRAME_OK) == (st == ref.STATE_MIMO), f
        if st == ref.STATE_MIMO:
            assert r["sync_index"] == of.get_sync_index(), (f, r["sync_index"], of.get_sync_index())
            assert r["plateau_start"][:N] == [of.get_plateau_start(s) for s in range(N)], f
            assert r["num_samples_processed"] == of.get_num_samples_processed(), f


def test_c4_full_codes_against_parseval_oracle():
    """C4 with all 20 access codes per stream (160 codes, 8 rx) on a reduced PID. The oracle
    runs its Parseval search variant (search_mode 1: one overlap-save correlation per (rx,
    code), pinned to the brute force by test_parseval_search_variant_matches_brute_force);
    the brute force itself would be ~1.4 TFLOP per frame. Sync bit-exact, corr indices exact
    wherever the peak is unambiguous, symbols within the EVM tolerance."""
    _c_frame_parity(4096, 304, 8, 20, 12, 256, _lib.DET_MMSE, 35.0, seed=43, bias=False,
                    search_mode=1)


def test_c4_full_frame_split_decode_against_parseval_oracle():
    """BASELINE config C4 at full size: 8x8 MMSE, M 4096, 256-QAM, all 20 access codes per
    stream, PID 1000, through the production split decode (path asserted). The oracle runs the
    Parseval search variant (search_mode 1, pinned to the brute force by test_oracle) and
    starts its S&C scan two symbols before the frame's S0 symbol, placed by the synthesiser's
    layout, not by the GPU (test_oracle::
    test_fast_forward_equals_full_run; the full scan of the 700k-sample prefix on 8 antennas
    is ~75 s of CPU, and test_c4_full_codes_against_parseval_oracle runs it on the same frame
    layout). Sync, plateau starts and samples processed bit-exact, corr indices exact where
    the peak is unambiguous, all 1000 symbols within the EVM tolerance, indices and
    symbol-error counts up to boundary decisions, EVM-dB within 1e-3 dB."""
    d, e = _c_frame_parity(4096, 304, 8, 20, 1000, 256, _lib.DET_MMSE, 35.0, seed=44, bias=False,
                           search_mode=1, path=_lib.DECODE_SPLIT, out_idx=True,
                           ff_margin=2 * (4096 + 304))
    assert np.median(e) < -20


@pytest.mark.parametrize("det", [_lib.DET_ZF, _lib.DET_MMSE])
def test_row_solve_8x8_matches_oracle(det):
    """8 streams take the 8-lane row solve (weights_row_kernel): reduced 8x8 frames checked
    against the oracle's Gauss-Jordan, symbols within the EVM tolerance."""
    _c_frame_parity(256, 32, 8, 2, 12, 16, det, 35.0, seed=68 + det, path=_lib.DECODE_SYMBOL)


def test_c4_batched_full_size_properties():
    """C4 at full size, batched: every frame syncs, PID+2 symbols, finite EVM."""
    M, cp, N, nac, pid, qam, F = 4096, 304, 8, 20, 1000, 256, 2
    S = Synthesizer(SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid,
                                qam_order=qam, seed=51, snr_db=35.0))
    L = S.params.max_frame_len()
    out = _lib.DeviceBuffer(F * N * L * 8)
    S.generate(out, L, L, F)
    rxo = Receiver(RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                            detector=_lib.DET_MMSE, qam_order=qam))
    rxo.process(out, L, L, F, ref_mode=2, ref_seed=51)
    for r in rxo.results():
        assert r["status"] == _lib.FRAME_OK and r["n_sym"] == pid + 2
        assert np.all(np.isfinite(r["evm_num"])) and np.all(r["evm_den"] > 0)
    ci, _ = rxo.corr()
    SL = M + cp
    good = (np.diff(ci.astype(np.int64), axis=2) == SL).mean()
    assert good > 0.9


def test_stream_decode_batch_equals_single_frames():
    """decode_stream_kernel (C3 geometry, decode_stream.hip): in a batch the persistent
    workgroups' symbol ranges straddle frames (PID 331 is prime to every range length), yet
    symbols and indices equal one-frame-per-call runs bit for bit; the indices are the hard
    decisions of the symbols and the per-frame EVM / symbol-error sums equal a float64
    recount from the outputs (ref_mode 1: transmitted indices read from HBM)."""
    import torch
    from rub_mimo_amd.receiver import Synthesizer, SynthParams
    M, cp, N, nac, pid, qam, F = 2048, 152, 4, 20, 331, 64, 4
    sp = SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid,
                     qam_order=qam, seed=77, snr_db=30.0)
    syn = Synthesizer(sp)
    L = sp.max_frame_len()
    dev = torch.device("cuda", 0)
    iq = torch.empty((F, N, L), dtype=torch.complex64, device=dev)
    tx = torch.empty((F, N, pid, M), dtype=torch.uint8, device=dev)
    syn.generate(iq, L, L, F, frame_id0=0, tx_idx=tx)
    P = RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                 detector=_lib.DET_MMSE, qam_order=qam)
    rx = Receiver(P)
    sym = torch.zeros((F, N, pid, M), dtype=torch.complex64, device=dev)
    idx = torch.zeros((F, N, pid, M), dtype=torch.uint8, device=dev)
    rx.process(iq, L, L, F, max_out=pid, out_sym=sym, out_idx=idx, ref_mode=1, ref_idx=tx)
    torch.cuda.synchronize()
    res = rx.results(F)
    ok = [f for f in range(F) if res[f]["status"] == _lib.FRAME_OK]
    assert len(ok) >= 2, [r["status"] for r in res]
    for f in ok:
        s1 = torch.zeros((1, N, pid, M), dtype=torch.complex64, device=dev)
        i1 = torch.zeros((1, N, pid, M), dtype=torch.uint8, device=dev)
        r1 = Receiver(P)
        r1.process(iq[f:f + 1], L, L, 1, max_out=pid, out_sym=s1, out_idx=i1, ref_mode=1,
                   ref_idx=tx[f:f + 1])
        torch.cuda.synchronize()
        assert torch.equal(s1[0], sym[f]) and torch.equal(i1[0], idx[f]), f
        ys = sym[f].cpu().numpy()
        dec, num, den, err = ref.demap_evm(ys.transpose(1, 0, 2), qam, tx[f].cpu().numpy())
        assert np.array_equal(dec, idx[f].cpu().numpy()), f
        r = res[f]
        assert np.array_equal(r["errors"], err.astype(np.int64)), (r["errors"], err)
        assert np.allclose(r["evm_num"], num, rtol=1e-4), (r["evm_num"], num)
        assert np.allclose(r["evm_den"], den, rtol=1e-5), (r["evm_den"], den)


def test_capture_files_replay_matches_golden(tmp_path):
    """main.cc's file round trip (rx worker appends rx<ch>.dat, main re-reads it and runs
    framesync, results land in rx_sig<ch>.dat), with the capture memory-mapped from disk."""
    from rub_mimo_amd import logfiles as lf
    g = load(GOLDEN[0])
    N = int(g["N"])
    with lf.CaptureWriter(N, str(tmp_path)) as w:
        for pos in range(0, g["rx"].shape[1], 4096):
            w.write([r[pos:pos + 4096] for r in g["rx"]])
    cap = lf.read_rx_capture(N, str(tmp_path))
    fs, got = gpu_framesync(g)
    assert fs.execute(cap) == fr.STATE_MIMO
    assert_sync_equal(fs, g)
    syms = np.stack(got)                               # [callbacks][N][M_occ]
    rx_sig = [syms[:, t, :].reshape(-1) for t in range(N)]
    lf.write_rx_logs(rx_sig, [np.zeros(len(s), np.uint32) for s in rx_sig], str(tmp_path))
    back = [np.fromfile(tmp_path / f"rx_sig{t + 1}.dat", np.complex64) for t in range(N)]
    assert evm_delta(np.stack(back), np.stack([g["symbols"][:, t, :].reshape(-1)
                                               for t in range(N)])) <= SYM_TOL


@pytest.mark.parametrize("rows,n,src_stride,dst_stride,off", [
    (4, 100003, 100004, 100008, 0),     # vector path with a ragged tail
    (3, 4099, 4101, 4099, 0),           # odd, unequal strides: scalar path
    (5, 4099, 4099, 4099, 0),           # odd equal strides: per-row aligned head + vectors
    (4, 2, 1027, 1027, 0),              # rows shorter than their head
    (6, 9, 9, 9, 0),
    (2, 1024, 1024, 1024, 1),           # misaligned source: scalar path
    (1, 0, 0, 0, 0),                    # empty
])
def test_ingest_sc16_bit_exact(rows, n, src_stride, dst_stride, off):
    import torch
    from rub_mimo_amd.receiver import SC16_SCALE, ingest_sc16
    rng = np.random.default_rng(rows * 7 + n)
    src = rng.integers(-32768, 32768, (rows * max(src_stride, 1) + off) * 2, dtype=np.int16)
    if n >= 2:
        src[off * 2: off * 2 + 4] = [-32768, 32767, 0, -1]   # full-scale ends
    d_src = torch.from_numpy(src).cuda()
    d_dst = torch.full((rows * max(dst_stride, 1) * 2 + 64,), 7.0, dtype=torch.float32,
                       device="cuda")
    ingest_sc16(d_src.data_ptr() + off * 4, src_stride, d_dst, dst_stride, rows, n,
                stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    out = d_dst.cpu().numpy()
    for r in range(rows):
        s = src[(off + r * src_stride) * 2:(off + r * src_stride + n) * 2]
        want = s.astype(np.float32) * np.float32(SC16_SCALE)
        got = out[r * dst_stride * 2:(r * dst_stride + n) * 2]
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
        gap_end = min((r + 1) * dst_stride, rows * dst_stride) * 2
        assert np.all(out[(r * dst_stride + n) * 2:gap_end] == 7.0)   # no writes past a row
    assert np.all(out[rows * max(dst_stride, 1) * 2:] == 7.0)


@pytest.mark.parametrize("M,eps_true", [(2048, 0.0), (2048, 0.3137), (1024, -0.71), (64, 0.05)])
def test_cfo_estimate_and_derotate(M, eps_true):
    """Opt-in CFO (absent from the reference): a period-M/2 preamble rotated by eps subcarrier
    spacings is estimated to 1e-6 (noise-free) against numpy fp64, and derotation restores the
    samples to fp32 rounding. Parity unpinned against the reference (it has no CFO)."""
    import torch
    from rub_mimo_amd.receiver import cfo_derotate, cfo_estimate
    rng = np.random.default_rng(M)
    N, start, n = 3, 1000, 1000 + 3 * M
    stride = n + 64
    half = (rng.standard_normal((N, M // 2)) + 1j * rng.standard_normal((N, M // 2)))
    x = (rng.standard_normal((N, n)) + 1j * rng.standard_normal((N, n))) * 0.1
    x[:, start:start + M] = np.concatenate([half, half], axis=1)
    rot = np.exp(2j * np.pi * eps_true / M * (np.arange(n) - 17))
    xr = (x * rot).astype(np.complex64)
    buf = np.zeros((N, stride), np.complex64)
    buf[:, :n] = xr
    d = torch.from_numpy(buf.view(np.float32)).cuda()
    s = torch.cuda.current_stream().cuda_stream
    per, comb = cfo_estimate(d, stride, N, start, M, stream=s)
    xd = xr.astype(np.complex128)
    P = np.sum(np.conj(xd[:, start:start + M // 2]) * xd[:, start + M // 2:start + M], axis=1)
    assert np.allclose(per, np.angle(P) / np.pi, atol=1e-9, rtol=0)
    assert abs(comb - np.angle(P.sum()) / np.pi) < 1e-9
    assert abs(comb - eps_true) < 1e-5
    cfo_derotate(d, stride, N, n, 17, comb, M, stream=s)
    torch.cuda.synchronize()
    back = d.cpu().numpy().view(np.complex64)
    assert np.abs(back[:, :n] - x).max() < 1e-4 * np.abs(x).max()
    assert np.all(back[:, n:] == 0)                                   # nothing past n


@pytest.mark.parametrize("eps_true,mode", [(0.3, "fold"), (-0.62, "fold"), (0.3, "scratch")])
def test_cfo_batch_corrects_rotated_c3_frames(eps_true, mode):
    """Opt-in CFO on the batched path (mimo_rx_config.cfo_correct; the reference has a FIXME at
    framing.cc:486 and no CFO step, so parity is unpinned). C3 captures rotated by eps_true
    subcarrier spacings:
    - sync exactly as the unrotated ones do, and the per-frame estimate (S0 coarse + data prefix
      fine) is within 2e-5 of eps_true;
    - decode with EVM within 0.1 dB of the unrotated frames through the same receiver (the
      correction is invariant to the offset);
    - against the unrotated frames with no correction at all (the reference's path) within
      0.5 dB for every frame: the estimator's own variance (prefix correlation, std ~3e-6
      subcarrier spacings at 30 dB) would cost the cleanest (-32 dB) frames ~2.4 dB of drift
      over 1000 symbols; the decode's per-symbol common phase (each symbol's own decisions,
      cfo_mode 2) removes it;
    - without the correction the rotated frames collapse (> 10 dB worse).
    mode "fold" (reference indices from HBM): the search + LS loads and the streaming decode
    derotate in place; "scratch" (ref_mode 2): the estimate-and-derotate scratch passes."""
    import torch
    from rub_mimo_amd.receiver import cfo_derotate
    M, cp, N, nac, pid, qam, F = 2048, 152, 4, 20, 1000, 64, 4
    sp = SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid,
                     qam_order=qam, seed=812, snr_db=30.0)
    S = Synthesizer(sp)
    L = sp.max_frame_len()
    iq = torch.empty((F, N, L), dtype=torch.complex64, device="cuda")
    tx = torch.empty((F, N, pid, M), dtype=torch.uint8, device="cuda")
    S.generate(iq, L, L, F, tx_idx=tx)

    def run(x, cfo):
        rxo = Receiver(RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac,
                                pid_max=pid, detector=_lib.DET_MMSE, qam_order=qam,
                                cfo_correct=cfo))
        if mode == "fold":
            rxo.process(x, L, L, F, max_out=pid, ref_mode=1, ref_idx=tx)
        else:
            rxo.process(x, L, L, F, max_out=pid, ref_mode=2, ref_seed=812, frame_id0=0)
        return rxo.results()

    def evm(r):
        return 10 * np.log10(np.sum(r["evm_num"]) / np.sum(r["evm_den"]))

    plain = run(iq, False)
    clean = run(iq, True)
    rot = iq.clone()
    cfo_derotate(rot, L, F * N, L, 0, -eps_true, M)          # applies a CFO of +eps_true
    corr = run(rot, True)
    raw = run(rot, False)
    torch.cuda.synchronize()
    ok = [f for f in range(F) if plain[f]["status"] == _lib.FRAME_OK]
    assert len(ok) >= 2
    for f in range(F):
        assert corr[f]["status"] == plain[f]["status"], f
        assert corr[f]["sync_index"] == plain[f]["sync_index"], f
    for f in ok:
        e0, e1, e2, e3 = evm(plain[f]), evm(corr[f]), evm(raw[f]), evm(clean[f])
        assert abs(corr[f]["cfo_eps"] - eps_true) < 2e-5, (f, corr[f]["cfo_eps"])
        assert abs(clean[f]["cfo_eps"]) < 2e-5, (f, clean[f]["cfo_eps"])
        assert abs(e1 - e3) <= 0.1, (f, e3, e1)
        # (the scratch mode's ref_mode-2 decode has no per-symbol common phase: the
        # estimator's residual drift costs the cleanest frames ~2.4 dB there)
        assert e3 - e0 <= (0.5 if mode == "fold" else 3.0), (f, e0, e3)
        print("cfo frame %d: plain %.3f dB, corrected %.3f dB, raw %.3f dB" % (f, e0, e3, e2))
        assert e2 > e0 + 10.0, (f, e0, e2)


def _oracle_frames(tmp_path, caps, M, cp, N, nac, pid, qam, cfo_mode):
    """oracle/mimo_ref.c framesync (cfo_mode) over each capture [N][L], in parallel processes"""
    from concurrent.futures import ProcessPoolExecutor
    import multiprocessing as mp
    paths = []
    for i, c in enumerate(caps):
        pth = tmp_path / ("cap%d.npy" % i)
        np.save(pth, c)
        paths.append(str(pth))
    with ProcessPoolExecutor(max_workers=min(8, len(paths)),
                             mp_context=mp.get_context("spawn")) as ex:
        futs = [ex.submit(ref.frame_ref_file, pth, M, cp, N, nac, pid, ref.DET_MMSE, qam,
                          cfo_mode, 1, pid) for pth in paths]
        return [f.result() for f in futs]


@pytest.mark.timeout(600)
def test_cfo_folded_matches_oracle_and_is_frame_deterministic(tmp_path):
    """Opt-in CFO (a build extension: the reference's framing.cc:486 is a FIXME) on the folded
    path (fused search + LS loads and the streaming decode derotate; per-symbol common phase),
    against its restatement in oracle/mimo_ref.c (cfo_mode 2, cross-checked by the numpy model
    in test_oracle.py): C3 frames rotated by eps = 0.3 and -0.62 subcarrier spacings give the
    oracle's sync index, its estimate eps0 + delta to 1e-6, and its equalised symbols to EVM
    delta 1e-4 (all 1000 data symbols). And the decode is a function of the frame: each frame
    received alone gives bit-identical symbols and indices to the batch, whose persistent
    workgroups' symbol ranges start mid-frame."""
    import torch
    from rub_mimo_amd.receiver import cfo_derotate
    M, cp, N, nac, pid, qam, F = 2048, 152, 4, 20, 1000, 64, 4
    sp = SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid,
                     qam_order=qam, seed=812, snr_db=30.0)
    S = Synthesizer(sp)
    L = sp.max_frame_len()
    iq = torch.empty((F, N, L), dtype=torch.complex64, device="cuda")
    tx = torch.empty((F, N, pid, M), dtype=torch.uint8, device="cuda")
    S.generate(iq, L, L, F, tx_idx=tx)
    P = RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                 detector=_lib.DET_MMSE, qam_order=qam, cfo_correct=True)
    for eps in (0.3, -0.62):
        rot = iq.clone()
        cfo_derotate(rot, L, F * N, L, 0, -eps, M)              # a CFO of +eps
        rxo = Receiver(P)
        sym = torch.zeros((F, N, pid, M), dtype=torch.complex64, device="cuda")
        idx = torch.zeros((F, N, pid, M), dtype=torch.uint8, device="cuda")
        rxo.process(rot, L, L, F, max_out=pid, out_sym=sym, out_idx=idx, ref_mode=1, ref_idx=tx)
        torch.cuda.synchronize()
        assert rxo.decode_path() == _lib.DECODE_STREAM and rxo.cfo_mode() == 2
        res = rxo.results(F)
        orc = _oracle_frames(tmp_path, list(rot.cpu().numpy()), M, cp, N, nac, pid, qam, 2)
        ok = 0
        for f in range(F):
            o, r = orc[f], res[f]
            assert (r["status"] == _lib.FRAME_OK) == (o["state"] == ref.STATE_MIMO), f
            if r["status"] != _lib.FRAME_OK:
                continue
            ok += 1
            assert r["sync_index"] == o["sync_index"], f
            e0, d = o["cfo"]
            assert abs(r["cfo_eps"] - (e0 + d)) <= 1e-6, (f, r["cfo_eps"], e0, d)
            assert abs(e0 + d - eps) < 2e-5, (f, e0, d)
            got = sym[f].cpu().numpy().transpose(1, 0, 2)
            assert evm_delta(got, o["symbols"]) <= SYM_TOL, f
            _, num, den, _ = ref.demap_evm(o["symbols"], qam, tx[f].cpu().numpy())
            e_gpu = 10 * np.log10(r["evm_num"] / r["evm_den"])
            assert np.abs(e_gpu - 10 * np.log10(num / den)).max() <= EVM_DB_TOL, f
            # the same frame alone: bit-identical
            r1 = Receiver(P)
            s1 = torch.zeros((1, N, pid, M), dtype=torch.complex64, device="cuda")
            i1 = torch.zeros((1, N, pid, M), dtype=torch.uint8, device="cuda")
            r1.process(rot[f:f + 1], L, L, 1, max_out=pid, out_sym=s1, out_idx=i1, ref_mode=1,
                       ref_idx=tx[f:f + 1])
            torch.cuda.synchronize()
            assert torch.equal(s1[0], sym[f]) and torch.equal(i1[0], idx[f]), f
            assert r1.results(1)[0]["cfo_eps"] == r["cfo_eps"], f
        assert ok >= 2
    # the unfolded (scratch) path -- EVM reference from the seed (ref_mode 2), so no CPE
    # variant: estimate + scratch derotation, the oracle's cfo_mode 1
    rxo = Receiver(P)
    sym = torch.zeros((F, N, pid, M), dtype=torch.complex64, device="cuda")
    idx = torch.zeros((F, N, pid, M), dtype=torch.uint8, device="cuda")
    rxo.process(rot, L, L, F, max_out=pid, out_sym=sym, out_idx=idx, ref_mode=2, ref_seed=812,
                frame_id0=0)
    torch.cuda.synchronize()
    assert rxo.cfo_mode() == 1
    res = rxo.results(F)
    orc = _oracle_frames(tmp_path, list(rot.cpu().numpy()), M, cp, N, nac, pid, qam, 1)
    for f in range(F):
        if res[f]["status"] != _lib.FRAME_OK:
            continue
        e0, d = orc[f]["cfo"]
        assert abs(res[f]["cfo_eps"] - (e0 + d)) <= 1e-6, f
        got = sym[f].cpu().numpy().transpose(1, 0, 2)
        assert evm_delta(got, orc[f]["symbols"]) <= SYM_TOL, f


def test_cfo_with_back_to_back_frames_is_refused_unfolded():
    """The unfolded CFO stages derotate each frame's window into a per-capture scratch, where
    back-to-back frames' windows would overlap: frames_per_capture > 1 is refused loudly
    outside the folded path (here M = 256: no fused search + streaming decode)."""
    import torch
    M, cp, N, nac, pid = 256, 19, 2, 4, 16
    rxo = Receiver(RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                            detector=_lib.DET_ZF2, qam_order=16, cfo_correct=True))
    L = 40 * (M + cp)
    iq = torch.zeros((1, N, L), dtype=torch.complex64, device="cuda")
    with pytest.raises(_lib.MimoError, match="frames_per_capture"):
        rxo.process(iq, L, L, 1, max_out=pid, frames_per_capture=2)


def test_cfo_folded_on_back_to_back_frames():
    """Folded CFO (no scratch) on streams of back-to-back C3 frames with tight gaps: the
    captures rotated by eps sync and re-arm exactly as the unrotated ones (S&C is
    offset-invariant), every decoded frame's estimate is within 2e-5 of eps, and its EVM is
    within 0.5 dB of the unrotated frame decoded without correction."""
    import torch
    from rub_mimo_amd.receiver import cfo_derotate
    M, cp, N, nac, pid, qam = 2048, 152, 4, 20, 200, 64
    eps = 0.27
    sp = SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid,
                     qam_order=qam, seed=611, snr_db=30.0)
    S = Synthesizer(sp)
    F, J, K = 2, 3, 4
    lens, L = S.stream_layout(F, J)
    iq = torch.zeros((F, N, L), dtype=torch.complex64, device="cuda")
    tx = torch.zeros((F * K, N, pid, M), dtype=torch.uint8, device="cuda")
    starts, _ = S.generate_streams(iq, L, F, J, K, tx_idx=tx)
    rs = torch.from_numpy(starts.view(np.int64).copy()).cuda()
    rot = iq.clone()
    cfo_derotate(rot, L, F * N, L, 0, -eps, M)              # a CFO of +eps

    def run(x, cfo):
        rxo = Receiver(RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac,
                                pid_max=pid, detector=_lib.DET_MMSE, qam_order=qam,
                                cfo_correct=cfo))
        rxo.process(x, L, L, F, max_out=pid, ref_mode=1, ref_idx=tx, frames_per_capture=K,
                    ref_starts=rs)
        torch.cuda.synchronize()
        return rxo.results(F * K)

    plain, corr = run(iq, False), run(rot, True)
    ok = 0
    for a_, b_ in zip(plain, corr):
        assert a_["status"] == b_["status"] and a_["sync_index"] == b_["sync_index"]
        assert a_["origin"] == b_["origin"]
        if a_["status"] != _lib.FRAME_OK:
            continue
        ok += 1
        assert abs(b_["cfo_eps"] - eps) < 2e-5, b_["cfo_eps"]
        e0 = 10 * np.log10(np.sum(a_["evm_num"]) / np.sum(a_["evm_den"]))
        e1 = 10 * np.log10(np.sum(b_["evm_num"]) / np.sum(b_["evm_den"]))
        assert e1 - e0 <= 0.5, (e0, e1)
    assert ok >= 2


def _sc16_capture(iq, amax):
    """Quantise complex64 captures [F][N][L] to the sc16 wire format (int16 I/Q) at full scale
    amax, as a radio's ADC path would; returns the int16 tensor [F][N][L][2] and the scale."""
    import torch
    q = torch.view_as_real(iq) * (32767.0 / amax)
    return q.round_().clamp_(-32768, 32767).to(torch.int16).contiguous(), amax / 32767.0


@pytest.mark.parametrize("geom", ["c3", "c3_streams", "c2", "m512", "m512x8"])
def test_sc16_batch_equals_widened_batch(geom):
    """mimo_batch.sample_format = SC16 (UHD wire samples read in place by the S&C, fused search
    + LS, streaming decode and 8x8 split decode kernels; other geometries widen internally)
    gives bit-identical results to widening with mimo_ingest_sc16 first and running the
    complex64 path: sync, corr indices, symbols, indices and EVM sums."""
    import torch
    from rub_mimo_amd.receiver import ingest_sc16
    if geom == "c2":
        M, cp, N, nac, pid, qam, det, F, K = 1024, 76, 2, 20, 200, 16, _lib.DET_ZF2, 4, 1
    elif geom == "m512":
        M, cp, N, nac, pid, qam, det, F, K = 512, 38, 2, 8, 100, 16, _lib.DET_ZF2, 4, 1
    elif geom == "m512x8":     # 8x8 split decode (spectra_kernel<9> reads the wire samples)
        M, cp, N, nac, pid, qam, det, F, K = 512, 38, 8, 4, 40, 64, _lib.DET_MMSE, 5, 1
    else:
        M, cp, N, nac, pid, qam, det, F, K = 2048, 152, 4, 20, 300, 64, _lib.DET_MMSE, 4, 1
    sp = SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid,
                     qam_order=qam, seed=404, snr_db=30.0)
    S = Synthesizer(sp)
    if geom == "c3_streams":
        J, K = 2, 3
        lens, L = S.stream_layout(F, J)
        iq = torch.zeros((F, N, L), dtype=torch.complex64, device="cuda")
        tx = torch.zeros((F * K, N, pid, M), dtype=torch.uint8, device="cuda")
        starts, _ = S.generate_streams(iq, L, F, J, K, tx_idx=tx)
        rs = torch.from_numpy(starts.view(np.int64).copy()).cuda()
    else:
        L = sp.max_frame_len()
        iq = torch.empty((F, N, L), dtype=torch.complex64, device="cuda")
        tx = torch.empty((F, N, pid, M), dtype=torch.uint8, device="cuda")
        S.generate(iq, L, L, F, tx_idx=tx)
        rs = None
    wire, scale = _sc16_capture(iq, float(torch.view_as_real(iq).abs().max()) * 1.01)
    wide = torch.empty_like(iq)
    ingest_sc16(wire, L, wide, L, F * N, L, scale)
    outs = []
    for src, sc16 in ((wide, False), (wire, True)):
        rxo = Receiver(RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac,
                                pid_max=pid, detector=det, qam_order=qam))
        sym = torch.zeros((F * K, N, pid, M), dtype=torch.complex64, device="cuda")
        idx = torch.zeros((F * K, N, pid, M), dtype=torch.uint8, device="cuda")
        rxo.set_timing(True)
        rxo.process(src, L, L, F, max_out=pid, out_sym=sym, out_idx=idx, ref_mode=1,
                    ref_idx=tx, frames_per_capture=K, ref_starts=rs, sc16=sc16,
                    sc16_scale=scale)
        torch.cuda.synchronize()
        launches = rxo.stage_times()[_lib.STAGE_NAMES[0]][1]
        outs.append((rxo.results(F * K), rxo.corr(F * K)[0], sym.cpu(), idx.cpu(),
                     rxo.G(F * K), rxo.W(F * K), launches))
    (ra, ca, sa, ia, ga, wa, na), (rb, cb, sb, ib, gb, wb, nb) = outs
    # C2/C3 geometries read the wire samples in place; M = 512 (no streaming decode) widens
    # them first, one extra launch timed with the S&C stage
    assert nb == na + (1 if geom == "m512" else 0), (geom, na, nb)
    ok = [i for i, r in enumerate(ra) if r["status"] == _lib.FRAME_OK]
    assert len(ok) >= 1
    assert torch.equal(ia, ib)
    assert torch.equal(sa, sb), (sa - sb).abs().max()
    for x, y in zip(ra, rb):
        for k in ("status", "sync_index", "trigger", "num_samples_processed", "n_sym", "origin"):
            assert x[k] == y[k], (k, x[k], y[k])
    for i in ok:       # per-frame outputs exist for frames that reach the detector
        assert np.array_equal(ca[i], cb[i])
        assert np.array_equal(ga[i], gb[i]) and np.array_equal(wa[i], wb[i]), i
        assert np.array_equal(ra[i]["evm_num"], rb[i]["evm_num"]), i
        assert np.array_equal(ra[i]["errors"], rb[i]["errors"]), i


def test_capture_ring_feeds_sc16_batch():
    """The pinned-host capture ring (mimo_ring_*): a producer thread writes sc16
    wire captures in ragged recv-sized chunks, the uploads land byte-exact in the bound device
    captures, and the batch received from them equals the batch received from the same wire
    samples made resident directly. Misuse (capacity overrun, double acquire) is an error."""
    import threading
    import torch
    from rub_mimo_amd.ring import CaptureRing
    M, cp, N, nac, pid, qam, F = 2048, 152, 4, 20, 60, 64, 2
    sp = SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid,
                     qam_order=qam, seed=77, snr_db=30.0)
    S = Synthesizer(sp)
    L = sp.max_frame_len()
    iq = torch.empty((F, N, L), dtype=torch.complex64, device="cuda")
    tx = torch.empty((F, N, pid, M), dtype=torch.uint8, device="cuda")
    S.generate(iq, L, L, F, tx_idx=tx)
    wire, scale = _sc16_capture(iq, float(torch.view_as_real(iq).abs().max()) * 1.01)
    host = wire.cpu().numpy()
    cap = torch.zeros_like(wire)
    ring = CaptureRing(N, chunk_samples=50000, n_chunks=3)
    rng = np.random.default_rng(5)
    errors = []

    def producer():
        try:
            for f in range(F):
                ring.bind(cap[f], L, L)
                pos = 0
                while pos < L:
                    rows = ring.acquire()
                    n = int(min(L - pos, rng.integers(1, ring.chunk + 1)))
                    for a in range(N):
                        rows[a][:n] = host[f, a, pos:pos + n]
                    ring.commit(n)
                    pos += n
        except Exception as e:      # surfaced by the main thread
            errors.append(e)

    th = threading.Thread(target=producer)
    th.start()
    th.join(timeout=120)
    assert not th.is_alive() and not errors, errors
    stream = torch.cuda.current_stream().cuda_stream
    assert ring.publish(stream) == L
    torch.cuda.synchronize()
    assert torch.equal(cap, wire)
    # overrun and protocol errors are loud
    rows = ring.acquire()
    with pytest.raises(_lib.MimoError):
        ring.acquire()
    with pytest.raises(_lib.MimoError):
        ring.commit(1)              # the bound capture is full
    ring.bind(cap[0], L, 10)
    ring.commit(10)
    ring.close()
    outs = []
    for src in (wire, cap):
        rxo = Receiver(RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac,
                                pid_max=pid, detector=_lib.DET_MMSE, qam_order=qam))
        sym = torch.zeros((F, N, pid, M), dtype=torch.complex64, device="cuda")
        idx = torch.zeros((F, N, pid, M), dtype=torch.uint8, device="cuda")
        if src is cap:
            cap.copy_(wire)           # the ring's last test commit overwrote 10 samples
        rxo.process(src, L, L, F, max_out=pid, out_sym=sym, out_idx=idx, ref_mode=1,
                    ref_idx=tx, sc16=True, sc16_scale=scale)
        torch.cuda.synchronize()
        outs.append((rxo.results(F), sym.cpu(), idx.cpu()))
    (ra, sa, ia), (rb, sb, ib) = outs
    assert sum(r["status"] == _lib.FRAME_OK for r in ra) >= 1
    for x, y in zip(ra, rb):
        assert x["status"] == y["status"] and x["sync_index"] == y["sync_index"]
    assert torch.equal(sa, sb) and torch.equal(ia, ib)


def test_split_stages_equal_whole_batch():
    """mimo_batch.stages: the front half (S&C .. weights) then the decode half of a batch, on two
    different streams ordered by an event, write bitwise the outputs and results of the whole
    chain in one call (C3 geometry, symbol-major, reference rows; fc32 and sc16 read in place);
    a decode half on the other handle of a pair leaves each handle's own batch intact."""
    import torch
    M, cp, N, nac, pid, qam, F = 2048, 152, 4, 20, 12, 64, 3
    S = Synthesizer(SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid,
                                qam_order=qam, seed=71, snr_db=30.0))
    L = max(S.frame_len(i) for i in range(F))
    iq = torch.empty((F, N, L), dtype=torch.complex64, device="cuda")
    tx = torch.empty((F, N, pid, M), dtype=torch.uint8, device="cuda")
    S.generate(iq, L, L, F, tx_idx=tx)
    ref_rows = tx.transpose(1, 2).contiguous()
    scale = float(torch.view_as_real(iq).abs().max()) * 1.01 / 32767.0
    w16 = (torch.view_as_real(iq) / scale).round_().clamp_(-32768, 32767).to(torch.int16)
    P = RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                 detector=_lib.DET_MMSE, qam_order=qam)

    def run(src, sc16, split):
        rxs = [Receiver(P), Receiver(P)]
        outs = []
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        for h, rx in enumerate(rxs):
            y = torch.zeros((F, pid, N, M), dtype=torch.complex64, device="cuda")
            d = torch.zeros((F, pid, N, M), dtype=torch.uint8, device="cuda")
            kw = dict(max_out=pid, out_sym=y, out_idx=d, ref_mode=1, ref_idx=ref_rows, sc16=sc16,
                      sc16_scale=scale, out_layout=_lib.LAYOUT_SYMBOL_MAJOR)
            if split:
                rx.process(src, L, L, F, stream=s1.cuda_stream, stages=_lib.STAGES_FRONT, **kw)
                ev = torch.cuda.Event()
                ev.record(s1)
                s2.wait_event(ev)
                rx.process(src, L, L, F, stream=s2.cuda_stream, stages=_lib.STAGES_DECODE, **kw)
            else:
                rx.process(src, L, L, F, **kw)
            outs.append((y, d))
        torch.cuda.synchronize()
        return [(y.cpu(), d.cpu(), rx.results(F)) for (y, d), rx in zip(outs, rxs)]

    for src, sc16 in ((iq, False), (w16, True)):
        whole = run(src, sc16, False)
        split = run(src, sc16, True)
        for (y0, d0, r0), (y1, d1, r1) in zip(whole, split):
            assert any(r["status"] == _lib.FRAME_OK for r in r0)
            assert torch.equal(y0.view(torch.int32), y1.view(torch.int32))
            assert torch.equal(d0, d1)
            for a, b in zip(r0, r1):
                assert a["status"] == b["status"] and a["sync_index"] == b["sync_index"]
                assert a["evm_num"].tobytes() == b["evm_num"].tobytes()
                assert np.array_equal(a["errors"], b["errors"])

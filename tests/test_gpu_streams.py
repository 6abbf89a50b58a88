"""GPU parity tests of back-to-back frames in one capture (BASELINE config C5's per-stream
workload, SURVEY 8f-4 "streaming re-arm after STATE_MIMO").

The oracle is a caller of the reference API: after each frame a fresh framesync
(framing.cc:268-436) takes the samples from r_{k+1} = r_k + get_num_samples_processed()
(oracle/ref.py stream_ref). The GPU receives every frame of every capture in one batch
(mimo_batch.frames_per_capture) and must report, per frame, the same origin, sync index,
plateau starts/ends and samples processed bit for bit, and symbols within EVM delta 1e-4."""
import glob
import os
from concurrent.futures import ProcessPoolExecutor
import multiprocessing as mp

import numpy as np
import pytest

from oracle import ref
from rub_mimo_amd import _lib
from rub_mimo_amd.receiver import Receiver, RxParams, Synthesizer, SynthParams

pytestmark = pytest.mark.gpu

STREAMS = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "m*_stream*.npz")))
SYM_TOL = 1e-4
EVM_DB_TOL = 1e-3
NONE64 = np.uint64(2 ** 64 - 1)


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible: the gpu tests need an MI355X")


def evm_delta(a, b):
    a = np.asarray(a, np.complex128)
    b = np.asarray(b, np.complex128)
    return float(np.sqrt(np.sum(np.abs(a - b) ** 2) / max(np.sum(np.abs(b) ** 2), 1e-300)))


def ref_rows(tx_frames, K, n_caps=1):
    """Transmitted indices [frames][N][pid][M_occ] -> the [n_caps*K] reference rows."""
    import torch
    t = np.zeros((n_caps * K,) + tx_frames.shape[1:], np.uint8)
    t[:len(tx_frames)] = tx_frames
    return torch.from_numpy(t).cuda()


def starts_row(starts, K):
    s = np.full(K, NONE64, np.uint64)
    s[:len(starts)] = starts
    return s


def _golden_receiver(g):
    M, cp, N, nac, pid, qam = (int(g[k]) for k in ("M", "cp", "N", "nac", "pid", "qam"))
    return Receiver(RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                             detector=int(g["detector"]), qam_order=qam, p=g["p"]))


def _check_frame(r, g, k, N):
    assert r["status"] == _lib.FRAME_OK, (k, r["status"])
    assert r["origin"] == int(g["origin"][k]), k
    assert r["sync_index"] == int(g["sync_index"][k]), k
    assert r["plateau_start"] == list(g["plateau_start"][k]), k
    assert r["plateau_end"] == list(g["plateau_end"][k]), k
    assert r["num_samples_processed"] == int(g["num_samples_processed"][k]), k
    assert r["n_sym"] == g["symbols"].shape[1], k          # PID+2 callbacks per frame


@pytest.mark.parametrize("path", STREAMS, ids=[os.path.basename(p) for p in STREAMS])
def test_stream_matches_golden(path):
    import torch
    g = dict(np.load(path, allow_pickle=False))
    M, N, nac, pid, qam = (int(g[k]) for k in ("M", "N", "nac", "pid", "qam"))
    n_ok = int(g["n_ok"])
    K = n_ok + 1
    rx = torch.from_numpy(np.ascontiguousarray(g["rx"])).cuda().unsqueeze(0)
    L = rx.shape[2]
    rxo = _golden_receiver(g)
    mocc = rxo.M_occ
    sym = torch.zeros((K, N, pid, mocc), dtype=torch.complex64, device="cuda")
    idx = torch.zeros((K, N, pid, mocc), dtype=torch.uint8, device="cuda")
    refi = ref_rows(g["tx_idx"], K)
    rs = starts_row(g["frame_starts"], K)
    rs_dev = torch.from_numpy(rs.view(np.int64).copy()).cuda()
    rxo.process(rx, L, L, 1, max_out=pid, out_sym=sym, out_idx=idx, ref_mode=1, ref_idx=refi,
                frames_per_capture=K, ref_starts=rs_dev)
    direct = rxo.results(K)
    rescan = [k for k in range(K) if direct[k]["status"] == _lib.FRAME_RESCAN]
    if "rescan" in os.path.basename(path):
        # frame 2's S0 follows frame 1's window end within one symbol: its fresh framesync
        # window reaches before the re-arm point, so the walk hands it back for a resume
        assert rescan == [2] and direct[2]["origin"] == int(g["origin"][2])
        assert all(direct[k]["status"] == _lib.FRAME_NONE for k in range(3, K))
    else:
        assert not rescan
        ci, si = rxo.corr(K)
        for k in range(n_ok):
            assert np.array_equal(ci[k], g["corr_idx"][k]), k
    res = rxo.receive_streams(rx, L, L, 1, K, max_out=pid, out_sym=sym, out_idx=idx,
                              ref_mode=1, ref_idx=refi, ref_starts=rs)
    torch.cuda.synchronize()
    for k in range(n_ok):
        r = res[k]
        _check_frame(r, g, k, N)
        assert r["ref_frame"] == int(g["tx_frame"][k]), k
        want = g["symbols"][k][:pid]                          # [pid][N][M_occ]
        got = sym[k].cpu().numpy().transpose(1, 0, 2)
        assert evm_delta(got, want) <= SYM_TOL, k
        _, num, den, err = ref.demap_evm(want, qam, g["tx_idx"][int(g["tx_frame"][k])])
        e_gpu = 10 * np.log10(r["evm_num"] / r["evm_den"])
        e_ref = 10 * np.log10(num / den)
        assert np.abs(e_gpu - e_ref).max() <= EVM_DB_TOL, (k, e_gpu, e_ref)
    tail = res[n_ok]
    want_tail = {ref.STATE_SEEK_PLATEAU: _lib.FRAME_NO_SYNC,
                 ref.STATE_SAVE_ACCESS_CODES: _lib.FRAME_INCOMPLETE}[int(g["tail_state"])]
    assert tail["status"] == want_tail and tail["origin"] == int(g["tail_origin"])
    assert tail["num_samples_processed"] == int(g["tail_nsp"])


def test_stream_graph_replay_is_identical():
    """A repeated stream batch is captured into a HIP graph and replayed: same results."""
    import torch
    g = dict(np.load([p for p in STREAMS if "rescan" not in p][0], allow_pickle=False))
    K = int(g["n_ok"]) + 1
    rx = torch.from_numpy(np.ascontiguousarray(g["rx"])).cuda().unsqueeze(0)
    L = rx.shape[2]
    rxo = _golden_receiver(g)
    N, pid = int(g["N"]), int(g["pid"])
    sym = torch.zeros((K, N, pid, rxo.M_occ), dtype=torch.complex64, device="cuda")
    outs = []
    for _ in range(4):      # direct, direct + capture, replay, replay
        sym.zero_()
        rxo.process(rx, L, L, 1, max_out=pid, out_sym=sym, frames_per_capture=K)
        torch.cuda.synchronize()
        outs.append((rxo.results(K), sym.clone()))
    for res, s in outs[1:]:
        assert [r["sync_index"] for r in res] == [r["sync_index"] for r in outs[0][0]]
        assert [r["origin"] for r in res] == [r["origin"] for r in outs[0][0]]
        assert torch.equal(s, outs[0][1])


def synth_streams(S, J, K, seed, M=2048, cp=152, N=4, nac=20, pid=1000, qam=64, snr=30.0):
    """S captures, each the GPU synthesiser's frames s*J .. s*J+J-1 back to back. Returns
    (iq [S][N][L] tensor, L, tx [S*K][N][pid][M] reference rows, starts [S][K] uint64)."""
    import torch
    syn = Synthesizer(SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid,
                                  qam_order=qam, seed=seed, snr_db=snr))
    lens = [[syn.frame_len(s * J + j) for j in range(J)] for s in range(S)]
    L = max(sum(l) for l in lens)
    iq = torch.zeros((S, N, L), dtype=torch.complex64, device="cuda")
    tx = torch.zeros((S * K, N, pid, M), dtype=torch.uint8, device="cuda")
    starts = np.full((S, K), NONE64, np.uint64)
    for s in range(S):
        pos = 0
        for j in range(J):
            ptr = iq.data_ptr() + ((s * N) * L + pos) * 8
            syn.generate(ptr, L, lens[s][j], 1, frame_id0=s * J + j,
                         tx_idx=tx.data_ptr() + (s * K + j) * N * pid * M)
            starts[s, j] = pos
            pos += lens[s][j]
    torch.cuda.synchronize()
    return iq, L, tx, starts


@pytest.mark.timeout(600)
def test_c5_streams_8x3_c3_frames_match_oracle(tmp_path):
    """C5's per-stream workload at C3 geometry: 8 captures of 3 back-to-back frames, one batch
    on the GPU, each capture checked against the oracle's stream driver (8 CPU processes).
    Every decoded frame is compared at its full PID (1000 data symbols, framing.cc:853-868),
    as the C5 bench line decodes them."""
    import torch
    S, J, K, M, cp, N, nac, pid, qam = 8, 3, 4, 2048, 152, 4, 20, 1000, 64
    MAXS = pid
    iq, L, tx, starts = synth_streams(S, J, K, seed=901)
    rxo = Receiver(RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                            detector=_lib.DET_MMSE, qam_order=qam))
    sym = torch.zeros((S * K, N, MAXS, M), dtype=torch.complex64, device="cuda")
    res = rxo.receive_streams(iq, L, L, S, K, max_out=MAXS, out_sym=sym, ref_mode=1,
                              ref_idx=tx[:, :, :MAXS].contiguous(), ref_starts=starts)
    torch.cuda.synchronize()
    host = iq.cpu().numpy()
    txh = tx.cpu().numpy()
    jobs = []
    for s in range(S):
        p = tmp_path / ("s%d.npy" % s)
        np.save(p, host[s])
        tp = tmp_path / ("t%d.npy" % s)
        np.save(tp, txh[s * K:(s + 1) * K])
        jobs.append((str(p), str(tp), starts[s][:J].astype(np.int64)))
    del host, txh
    with ProcessPoolExecutor(max_workers=8, mp_context=mp.get_context("spawn")) as ex:
        futs = [ex.submit(ref.stream_ref_file, p, M, cp, N, nac, pid, K, ref.DET_MMSE, MAXS, qam,
                          tp, st) for p, tp, st in jobs]
        orc = [f.result() for f in futs]
    n_frames = 0
    for s in range(S):
        ok = [r for r in orc[s] if r["state"] == ref.STATE_MIMO]
        got = [res[s * K + k] for k in range(K) if res[s * K + k]["status"] == _lib.FRAME_OK]
        assert len(got) == len(ok), (s, [r["status"] for r in res[s * K:(s + 1) * K]])
        for k, (r, o) in enumerate(zip(got, ok)):
            assert r["origin"] == o["origin"], (s, k)
            assert r["sync_index"] == o["sync_index"], (s, k)
            assert r["plateau_start"] == list(o["plateau_start"]), (s, k)
            assert r["num_samples_processed"] == o["num_samples_processed"], (s, k)
            assert r["ref_frame"] == s * K + o["tx_frame"], (s, k)
            slot = [q for q in range(K) if res[s * K + q] is r][0]
            ours = sym[s * K + slot].cpu().numpy().transpose(1, 0, 2)
            assert evm_delta(ours, o["symbols"]) <= SYM_TOL, (s, k)
            e_gpu = 10 * np.log10(r["evm_num"] / r["evm_den"])
            e_ref = 10 * np.log10(o["evm_num"] / o["evm_den"])
            assert np.abs(e_gpu - e_ref).max() <= EVM_DB_TOL, (s, k, e_gpu, e_ref)
            n_frames += 1
    assert n_frames >= S * J // 2, n_frames


def test_streams_symbol_major_layout_equals_stream_major():
    """Back-to-back streams (frames_per_capture > 1, the C5 path) with mimo_batch.out_layout =
    SYMBOL_MAJOR: every frame slot's outputs are the stream-major ones transposed, bit for bit,
    and the per-slot results (origins, EVM sums, errors against the transposed reference rows)
    are identical. Also an out-of-range layout is refused."""
    import torch
    S, J, K, pid = 3, 2, 3, 40
    iq, L, tx, starts = synth_streams(S, J, K, seed=907, pid=pid)
    M, N = 2048, 4
    outs = []
    for layout in (_lib.LAYOUT_STREAM_MAJOR, _lib.LAYOUT_SYMBOL_MAJOR):
        rxo = Receiver(RxParams(M=M, cp_len=152, num_streams=N, num_access_codes=20,
                                pid_max=pid, detector=_lib.DET_MMSE, qam_order=64))
        sm = layout == _lib.LAYOUT_SYMBOL_MAJOR
        shape = (S * K, pid, N, M) if sm else (S * K, N, pid, M)
        sym = torch.zeros(shape, dtype=torch.complex64, device="cuda")
        idx = torch.zeros(shape, dtype=torch.uint8, device="cuda")
        refr = (tx.transpose(1, 2) if sm else tx).contiguous()
        res = rxo.receive_streams(iq, L, L, S, K, max_out=pid, out_sym=sym, out_idx=idx,
                                  ref_mode=1, ref_idx=refr, ref_starts=starts, out_layout=layout)
        torch.cuda.synchronize()
        if sm:
            sym, idx = sym.transpose(1, 2), idx.transpose(1, 2)
        outs.append((res, sym.contiguous().cpu().numpy(), idx.contiguous().cpu().numpy()))
    (r0, y0, d0), (r1, y1, d1) = outs
    assert sum(r["status"] == _lib.FRAME_OK for r in r0) >= S
    for q, (a, b) in enumerate(zip(r0, r1)):
        assert (a["status"], a["origin"], a["sync_index"]) == (b["status"], b["origin"], b["sync_index"])
        if a["status"] != _lib.FRAME_OK:
            continue
        n = min(a["n_sym"], pid)
        assert np.array_equal(y0[q, :, :n].view(np.uint32), y1[q, :, :n].view(np.uint32)), q
        assert np.array_equal(d0[q, :, :n], d1[q, :, :n]), q
        assert a["evm_num"].tobytes() == b["evm_num"].tobytes()
        assert np.array_equal(a["errors"], b["errors"])
    rxo = Receiver(RxParams(M=M, cp_len=152, num_streams=N, num_access_codes=20, pid_max=pid,
                            detector=_lib.DET_MMSE, qam_order=64))
    with pytest.raises(_lib.MimoError):
        rxo.process(iq, L, L, 1, max_out=pid, out_layout=2)

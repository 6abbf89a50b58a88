"""Generate the committed golden fixtures (tests/golden/*.npz).

No reference fixtures exist (the reference ships no tests and cannot be built here), so the
fixtures are produced by the C oracle (oracle/mimo_ref.c) and accepted only after the
independent numpy model (oracle/numpy_model.py) reproduces them:
  sync index / plateau / corr indices / samples processed bit-exact,
  G within 1e-6, equalised symbols within 1e-5 relative.
Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import codes, numpy_model as nm, ref  # noqa: E402

CASES = [
    # name, M, cp, N, nac, pid, qam, detector, seed, sctype, snr, bias
    ("m64_2x2_zf2", 64, 16, 2, 4, 8, 16, "zf2", 1, "all", 30.0, True),
    ("m64_1x1_zf", 64, 16, 1, 4, 8, 4, "zf", 2, "all", 20.0, True),
    ("m128_4x4_mmse", 128, 16, 4, 6, 6, 64, "mmse", 3, "all", 30.0, True),
    ("m64_2x2_liquid_zf", 64, 16, 2, 4, 8, 16, "zf", 4, "liquid", 30.0, False),
    ("m64_2x2_siso", 64, 16, 2, 4, 8, 4, "siso", 5, "all", 30.0, True),
    ("m256_8x8_mmse", 256, 32, 8, 3, 4, 256, "mmse", 6, "all", 35.0, False),
]
DETS = {"zf2": ref.DET_ZF2, "zf": ref.DET_ZF, "mmse": ref.DET_MMSE, "siso": ref.DET_SISO}


def make_case(name, M, cp, N, nac, pid, qam, det, seed, sct, snr, bias):
    p = ref.default_sctype(M) if sct == "all" else ref.liquid_sctype(M)
    rx, tx_idx, H = ref.synth_frame(M, cp, N, nac, pid, qam, seed=seed, frame=0, offset=-1,
                                    snr_db=snr, p=p)
    siso = dict(siso_tx=1, siso_rx=1) if det == "siso" else {}
    fs = ref.FrameSyncRef(M, cp, N, nac, pid_max=pid, detector=DETS[det],
                          keep_identity_bias=bias, trace_sc=True, p=p, **siso)
    state = fs.execute(rx)
    assert state == ref.STATE_MIMO, name
    ci, cm, si, sm = fs.get_corr()
    syms = fs.symbols()
    rec = dict(
        M=M, cp=cp, N=N, nac=nac, pid=pid, qam=qam, detector=DETS[det], seed=seed,
        keep_identity_bias=int(bias), p=p, rx=rx, tx_idx=tx_idx, H=H,
        sync_index=fs.get_sync_index(), num_samples_processed=fs.get_num_samples_processed(),
        plateau_start=np.array([fs.get_plateau_start(s) for s in range(N)], np.int64),
        plateau_end=np.array([fs.get_plateau_end(s) for s in range(N)], np.int64),
        corr_idx=ci, corr_max=cm, s0_idx=si, G=fs.get_G(), W=fs.get_W(), gain=fs.get_gain(),
        noise_var=np.float32(fs.get_noise_var()), symbols=syms,
        y0=fs.sc_trace(0), siso_tx=1 if det == "siso" else 0,
        siso_rx=1 if det == "siso" else 0)
    rx_idx, num, den, err = ref.demap_evm(syms[:pid], qam, tx_idx)
    rec.update(rx_idx=rx_idx, evm_num=num, evm_den=den, errors=err.astype(np.int64))
    # independent cross-check before accepting the fixture
    if det != "siso":
        s0b, s1b = ref.code_bits(M, N, nac, codes.s1_polynomials(N))
        out = nm.receive(rx, M, cp, N, nac, pid, s0b, s1b, p=p, detector=det,
                         keep_identity_bias=bias)
        assert out["sync_index"] == rec["sync_index"], name
        assert list(out["plateau_start"]) == list(rec["plateau_start"]), name
        assert out["num_samples_processed"] == rec["num_samples_processed"], name
        assert (out["corr_idx"] == ci).all(), name
        assert (out["s0_idx"] == si).all(), name
        assert np.abs(out["G"] - rec["G"]).max() < 1e-6, name
        scale = np.abs(out["symbols"]).max()
        assert np.abs(out["symbols"] - syms).max() / scale < 1e-5, name
    return rec


STREAM_CASES = [
    # name, M, cp, N, nac, pid, qam, detector, seed, frames, snr, lead_cut (frame -> samples
    # removed from its lead: a frame whose S0 follows the previous window end too closely)
    ("m64_2x2_stream", 64, 16, 2, 4, 8, 16, "zf2", 11, 4, 30.0, {}),
    ("m64_2x2_stream_rescan", 64, 16, 2, 4, 8, 16, "zf2", 11, 3, 30.0, {2: 735}),
]


def make_stream_case(name, M, cp, N, nac, pid, qam, det, seed, frames, snr, lead_cut):
    """Back-to-back frames in one capture (frames 0..frames-1 of the synthesiser, optionally
    with part of a frame's lead removed), received by the oracle's fresh-framesync-per-frame
    stream driver (oracle/ref.py stream_ref) and accepted after the numpy model's own
    stream driver agrees frame by frame."""
    p = ref.default_sctype(M)
    parts, txs, starts = [], [], []
    pos = 0
    for f in range(frames):
        rx, tx_idx, _ = ref.synth_frame(M, cp, N, nac, pid, qam, seed=seed, frame=f, offset=-1,
                                        snr_db=snr, p=p)
        cut = lead_cut.get(f, 0)
        rx = rx[:, cut:]
        starts.append(pos)
        pos += rx.shape[1]
        parts.append(rx)
        txs.append(tx_idx)
    rx = np.concatenate(parts, axis=1)
    recs = ref.stream_ref(rx, M, cp, N, nac, pid_max=pid, detector=DETS[det], p=p)
    ok = [r for r in recs if r["state"] == ref.STATE_MIMO]
    assert len(ok) >= 2, (name, len(ok))
    s0b, s1b = ref.code_bits(M, N, nac, codes.s1_polynomials(N))
    nmo = nm.receive_stream(rx, M, cp, N, nac, pid, s0b, s1b, p=p, detector=det)
    assert len(nmo) == len(ok), name
    for r, (org, d) in zip(ok, nmo):
        assert r["origin"] == org and r["sync_index"] == d["sync_index"], name
        assert list(r["plateau_start"]) == list(d["plateau_start"]), name
        assert r["num_samples_processed"] == d["num_samples_processed"], name
        assert (r["corr_idx"] == d["corr_idx"]).all(), name
        scale = np.abs(d["symbols"]).max()
        assert np.abs(d["symbols"] - r["symbols"]).max() / scale < 1e-5, name
    K = len(ok)
    # transmitted frame of each decoded frame (sync index inside that frame's span)
    fidx = np.array([int(np.searchsorted(starts, r["origin"] + r["sync_index"], "right")) - 1
                     for r in ok], np.int64)
    return dict(
        M=M, cp=cp, N=N, nac=nac, pid=pid, qam=qam, detector=DETS[det], seed=seed, p=p, rx=rx,
        frame_starts=np.array(starts, np.uint64), tx_idx=np.stack(txs),
        n_ok=K, origin=np.array([r["origin"] for r in ok], np.int64),
        sync_index=np.array([r["sync_index"] for r in ok], np.int64),
        plateau_start=np.array([r["plateau_start"] for r in ok], np.int64),
        plateau_end=np.array([r["plateau_end"] for r in ok], np.int64),
        num_samples_processed=np.array([r["num_samples_processed"] for r in ok], np.int64),
        corr_idx=np.stack([r["corr_idx"] for r in ok]), symbols=np.stack([r["symbols"] for r in ok]),
        tx_frame=fidx, tail_state=recs[-1]["state"], tail_origin=recs[-1]["origin"],
        tail_nsp=recs[-1]["num_samples_processed"])


def main():
    for case in STREAM_CASES:
        rec = make_stream_case(*case)
        path = os.path.join(HERE, case[0] + ".npz")
        np.savez_compressed(path, **rec)
        print("wrote", path, os.path.getsize(path), "bytes; frames", rec["n_ok"], "origins",
              list(rec["origin"]), "syncs", list(rec["sync_index"]), "tx frames",
              list(rec["tx_frame"]))
    if len(sys.argv) > 1 and sys.argv[1] == "streams":
        return
    for case in CASES:
        rec = make_case(*case)
        path = os.path.join(HERE, case[0] + ".npz")
        np.savez_compressed(path, **rec)
        print("wrote", path, os.path.getsize(path), "bytes; sync", rec["sync_index"],
              "EVM dB", np.round(10 * np.log10(rec["evm_num"] / rec["evm_den"]), 2))
    bits = {("s0_%o" % codes.S0_POLY): ref.draw_bits(12, codes.S0_POLY, 1, 256)}
    for g in codes.S1_POLYS:
        bits["s1_%o" % g] = ref.draw_bits(13, g, 1, 256)
    for g in codes.S1_POLYS[:2]:
        assert (nm.msequence_bits(13, g, 1, 256) == bits["s1_%o" % g]).all()
    np.savez_compressed(os.path.join(HERE, "msequence_bits.npz"), **bits)
    print("wrote msequence_bits.npz")


if __name__ == "__main__":
    main()

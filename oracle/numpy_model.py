"""oracle/numpy_model.py -- TEST INFRASTRUCTURE ONLY: an independent numpy model of the
reference receive path, used to cross-check the C oracle (oracle/mimo_ref.c) and to
produce the committed fixtures in tests/golden/.

Written separately from the C restatement (float64 numpy FFTs, vectorised cumulative-sum
Schmidl-Cox metric, sliding-window brute-force search), so agreement between the two is
evidence that both follow the reference logic:
  framing.cc:591-637  Schmidl-Cox metric + plateau rule
  framing.cc:639-651  access-code window [sync_index - SL, sync_index - SL + ACB + TX)
  framing.cc:702-744  access-code search (first maximum, strict >, initial 0)
  framing.cc:801-831  LS estimate with identity start, 2x2 invert
  framing.cc:535-589  replay decode from corr_indices[N-1][last] + M
and, with cfo=True, the opt-in CFO stages (a build extension: the reference has no CFO step,
framing.cc:486) as oracle/mimo_ref.c restates them ("Opt-in CFO"), here in float64 numpy.
"""
from __future__ import annotations

import numpy as np


def msequence_bits(m, g, a, count):
    """liquid msequence (g >>= 1, bit-reversed initial state), one bit per draw."""
    g >>= 1
    v = 0
    for _ in range(m):
        v = (v << 1) | (a & 1)
        a >>= 1
    n = (1 << m) - 1
    out = np.zeros(count, np.uint8)
    for i in range(count):
        b = bin(v & g).count("1") & 1
        v = ((v << 1) | b) & n
        out[i] = b
    return out


def init_S0(p, bits):
    M = len(p)
    S0 = np.zeros(M, np.complex128)
    occ = (p != 0)
    even = (np.arange(M) % 2) == 0
    sel = occ & even
    S0[sel] = np.where(bits[sel] & 1, 1.0, -1.0)
    m_s0 = int(sel.sum())
    s0 = np.fft.ifft(S0) * M * np.sqrt(1.0 / m_s0)
    return S0, s0


def init_S1(p, nac, bits):
    M = len(p)
    S1 = np.zeros((nac, M), np.complex128)
    b = bits.reshape(nac, M)
    S1[:, p != 0] = np.where(b[:, p != 0] & 1, 1.0, -1.0)
    s1 = np.fft.ifft(S1, axis=1) * M * np.sqrt(1.0 / M)
    return S1, s1


def sc_metric(x, M):
    """y[n] = |sum_{M/2} conj(x[k-M/2]) x[k]|^2 / (0.5 sum_M |x|^2)^2 in float64."""
    x = x.astype(np.complex128)
    L = len(x)
    M2 = M // 2
    xd = np.concatenate([np.zeros(M2, np.complex128), x[:-M2]]) if L > M2 else np.zeros(L)
    pv = np.conj(xd) * x
    z = (x.real ** 2 + x.imag ** 2)
    cp_ = np.concatenate([[0.0], np.cumsum(pv)])
    cz = np.concatenate([[0.0], np.cumsum(z)])
    n = np.arange(L)
    P = cp_[n + 1] - cp_[np.maximum(n + 1 - M2, 0)]
    R = 0.5 * (cz[n + 1] - cz[np.maximum(n + 1 - M, 0)])
    with np.errstate(divide="ignore", invalid="ignore"):
        y = np.abs(P) ** 2 / R ** 2
    return y


def plateau_trigger(ys, cp, thr=0.95):
    """Reference plateau rule (framing.cc:601-623) on per-antenna metric traces.
    Returns (trigger n, [starts], sync_index) or None."""
    N = len(ys)
    L = min(len(y) for y in ys)
    b = np.stack([np.nan_to_num(y[:L], nan=0.0) > thr for y in ys])
    # run start of the current run at each sample (index of last False + 1)
    starts = np.zeros((N, L), np.int64)
    ok = np.zeros((N, L), bool)
    for s in range(N):
        idx = np.arange(L)
        last_false = np.where(~b[s], idx, -1)
        last_false = np.maximum.accumulate(last_false)
        starts[s] = last_false + 1
        ok[s] = b[s] & (idx - starts[s] > cp)
    allok = ok.all(axis=0)
    hits = np.nonzero(allok)[0]
    if len(hits) == 0:
        return None
    n = int(hits[0])
    st = [int(starts[s, n]) for s in range(N)]
    return n, st, sum(st) // N


def qam_decision_point(y, order):
    """Square QAM hard decision (as mimo_ref.c ref_qam_demap): each dimension's level
    floor((v sqrt(2(L^2-1)/3) + L) / 2) clamped to [0, L-1], point (2m - (L-1)) / that scale."""
    L = int(round(np.sqrt(order)))
    s = np.sqrt(2.0 * (L * L - 1) / 3.0)

    def lev(v):
        return np.clip(np.floor((v * s + L) * 0.5), 0, L - 1)
    return ((2 * lev(y.real) - (L - 1)) + 1j * (2 * lev(y.imag) - (L - 1))) / s


def receive(rx, M, cp, N, nac, pid_max, s0_bits, s1_bits, p=None, detector="zf2",
            noise_var=None, keep_identity_bias=True, thr=0.95, cfo=False, qam=None):
    """Full frame receive. Returns a dict, or None if no sync / incomplete capture.
    cfo=True: the opt-in CFO stages (eps0 from the S&C window at the trigger, search and LS on
    the window turned by eps0, delta from the data prefixes, LS terms turned by delta at their
    window centres, decode of the window turned by eps0 + delta) and, with qam, the per-symbol
    common phase from the decisions of every stream at the even occupied indices with bit 9
    clear."""
    if p is None:
        p = np.full(M, 2, np.uint8)
    SL = M + cp
    occ = np.nonzero(p != 0)[0]
    mocc = len(occ)
    dn = 1.0 / np.sqrt(mocc)
    S0, _ = init_S0(p, s0_bits)
    S1 = []
    for t in range(N):
        S1t, _ = init_S1(p, nac, s1_bits[t * nac * M:(t + 1) * nac * M])
        S1.append(S1t)
    ys = [sc_metric(rx[s], M) for s in range(N)]
    trig = plateau_trigger(ys, cp, thr)
    if trig is None:
        return None
    n_trig, starts, sync = trig
    acb = SL * (nac * N + 4)
    txl = pid_max * SL
    win_len = acb + txl
    base = sync - SL
    n_e = base + win_len              # sample at which estimate_channel runs
    if n_e >= rx.shape[1]:
        return None
    win = np.zeros((N, win_len), np.complex128)
    lo = max(0, base)
    win[:, lo - base:] = rx[:, lo:base + win_len]
    raw = win
    eps0 = delta = 0.0
    jj = np.arange(win_len)
    if cfo:
        t0 = n_trig - base - M + 1
        a = win[:, t0:t0 + M // 2]
        b = win[:, t0 + M // 2:t0 + M]
        eps0 = float(np.angle(np.sum(np.conj(a) * b)) / np.pi)
        win = raw * np.exp(-2j * np.pi * eps0 * jj / M)[None, :]
    nacN = nac * N
    corr_idx = np.zeros((N, nacN), np.int64)
    s0_idx = np.zeros(N, np.int64)
    MM = float(M * M)
    for r in range(N):
        w0 = np.lib.stride_tricks.sliding_window_view(win[r, :SL + M - 1], M)
        X = np.fft.fft(w0, axis=1)
        v = np.abs(X @ np.conj(S0)) ** 2 / MM
        s0_idx[r] = int(np.argmax(v)) if v.max() > 0 else 0
        for code in range(nac):
            for t in range(N):
                ac = code * N + t
                off = SL * (ac + 1)
                wv = np.lib.stride_tricks.sliding_window_view(win[r, off:off + SL + M - 1], M)
                X = np.fft.fft(wv, axis=1)
                cv = np.abs(X @ np.conj(S1[t][code])) ** 2 / MM
                corr_idx[r, ac] = (int(np.argmax(cv)) + off) if cv.max() > 0 else 0
    G = np.zeros((M, N, N), np.complex128)
    if keep_identity_bias:
        for r in range(N):
            G[occ, r, r] = 1.0
    if cfo:
        i0 = corr_idx[N - 1, nacN - 1] + M
        ks = []
        for s in range(pid_max + 2):
            k = i0 + s * SL + 4 + np.arange(max(cp - 8, 0))
            ks.append(k[k + M < win_len])
        k = np.concatenate(ks)
        P1 = np.sum(np.conj(raw[:, k]) * raw[:, k + M]) * np.exp(-2j * np.pi * eps0)
        delta = float(np.angle(P1) / (2 * np.pi))
    per_code = np.zeros((nac, M, N, N), np.complex128)
    for code in range(nac):
        for r in range(N):
            for t in range(N):
                i0 = corr_idx[r, code * N + t]
                X = np.fft.fft(win[r, i0:i0 + M])
                per_code[code, occ, r, t] = X[occ] / S1[t][code][occ]
                if cfo:
                    per_code[code, occ, r, t] *= np.exp(-2j * np.pi * delta * (i0 + M / 2) / M)
    G[occ] += per_code[:, occ].sum(axis=0)
    G[occ] *= dn / nac
    v = per_code[:, occ]
    var_sum = (np.abs(v) ** 2).sum(axis=0) - np.abs(v.sum(axis=0)) ** 2 / nac
    nv_est = float(var_sum.sum() * dn * dn / (mocc * N * N * (nac - 1))) if nac > 1 else 0.0
    s2 = nv_est if noise_var is None else noise_var
    W = np.zeros((M, N, N), np.complex128)
    gain = np.ones(mocc)
    for j, sc in enumerate(occ):
        g = G[sc]
        if detector == "zf2":
            det = g[0, 0] * g[1, 1] - g[0, 1] * g[1, 0]
            di = np.conj(det)
            W[sc] = np.array([[di * g[1, 1], -di * g[0, 1]], [-di * g[1, 0], di * g[0, 0]]])
            gain[j] = 1.0 / abs(det) ** 2
        elif detector == "zf":
            W[sc] = np.linalg.inv(g)
        elif detector == "mmse":
            W[sc] = np.linalg.solve(g.conj().T @ g + s2 * np.eye(N), g.conj().T)
        else:
            raise ValueError(detector)
    i0 = corr_idx[N - 1, nacN - 1] + M
    nsym = (win_len - i0) // SL
    syms = np.zeros((nsym, N, mocc), np.complex128)
    if cfo:
        win = raw * np.exp(-2j * np.pi * (eps0 + delta) * jj / M)[None, :]
    for s in range(nsym):
        st = i0 + s * SL + cp
        X = np.fft.fft(win[:, st:st + M], axis=1) * dn
        Y = np.einsum("ktr,rk->tk", W[occ], X[:, occ])
        syms[s] = Y * gain[None, :]
        if cfo and qam:
            j = np.arange(syms[s].shape[1])
            ev = syms[s][:, ((j & 1) == 0) & (((j >> 9) & 1) == 0)]   # every stream; j even, bit 9 clear
            c = np.sum(np.conj(qam_decision_point(ev, qam)) * ev)
            if c != 0:
                syms[s] *= np.conj(c) / abs(c)
    return dict(trigger=n_trig, plateau_start=starts, plateau_end=[n_trig] * N,
                cfo_eps0=eps0, cfo_delta=delta,
                sync_index=sync, base=base, corr_idx=corr_idx, s0_idx=s0_idx, G=G, W=W,
                gain=gain, noise_var=nv_est, symbols=syms, y=ys,
                num_samples_processed=n_e + 2 if n_e + 1 < rx.shape[1] else n_e + 1)


def receive_stream(rx, M, cp, N, nac, pid_max, s0_bits, s1_bits, max_frames=None, **kw):
    """Back-to-back frames: `receive` on the samples after each frame, from origin
    r_{k+1} = r_k + num_samples_processed (a fresh framesync per frame; see oracle/ref.py
    stream_ref). Returns [(origin, receive() dict)] for the frames that complete."""
    L = rx.shape[1]
    r = 0
    out = []
    while r < L and (max_frames is None or len(out) < max_frames):
        d = receive(rx[:, r:], M, cp, N, nac, pid_max, s0_bits, s1_bits, **kw)
        if d is None:
            break
        out.append((r, d))
        r += d["num_samples_processed"]
    return out

"""tools/cfo_diag2.py -- opt-in CFO decode diagnostics (GPU box): EVM of the folded CFO decode
with every output kind and with none, and per-symbol phase / gain of its outputs against the
uncorrected decode of the same (unrotated) frames."""
import sys
import numpy as np
import torch
sys.path.insert(0, '.')
from rub_mimo_amd import _lib
from rub_mimo_amd.receiver import Receiver, RxParams, Synthesizer, SynthParams

F = int(sys.argv[1]) if len(sys.argv) > 1 else 2
M, cp, N, nac, pid, qam = 2048, 152, 4, 20, 1000, 64
sp = SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid, qam_order=qam,
                 seed=812, snr_db=30.0)
S = Synthesizer(sp)
L = sp.max_frame_len()
iq = torch.empty((F, N, L), dtype=torch.complex64, device="cuda")
tx = torch.empty((F, N, pid, M), dtype=torch.uint8, device="cuda")
S.generate(iq, L, L, F, tx_idx=tx)


def run(cfo, outs, x=None):
    x = iq if x is None else x
    r = Receiver(RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                          detector=_lib.DET_MMSE, qam_order=qam, cfo_correct=cfo))
    mo = r.M_occ
    sym = torch.zeros((F, N, pid, mo), dtype=torch.complex64, device="cuda") if outs else None
    idx = torch.zeros((F, N, pid, mo), dtype=torch.uint8, device="cuda") if outs else None
    r.process(x, L, L, F, max_out=pid, out_sym=sym, out_idx=idx, ref_mode=1, ref_idx=tx)
    torch.cuda.synchronize()
    return r, r.results(), (sym.cpu().numpy() if outs else None)


def e(res):
    return 10 * np.log10(np.sum(res["evm_num"]) / np.sum(res["evm_den"])) if res["status"] == 0 else None


rp, plain, ps = run(False, True)
rc3, c3, cs = run(True, True)
rc0, c0, _ = run(True, False)
from rub_mimo_amd.receiver import cfo_derotate
rot = iq.clone()
cfo_derotate(rot, L, F * N, L, 0, -0.3, M)
torch.cuda.synchronize()
rr, cr, rs = run(True, True, rot)
print("result keys", sorted(plain[0].keys()))
print("paths", rp.decode_path(), rc3.decode_path(), rc0.decode_path(), "cfo_mode", rc3.cfo_mode(), rc0.cfo_mode())
for f in range(F):
    print("frame", f, "status", plain[f]["status"], "eps", c3[f]["cfo_eps"], c0[f]["cfo_eps"],
          "evm plain/cfo-outs/cfo-none", e(plain[f]), e(c3[f]), e(c0[f]))
    if plain[f]["status"] != 0:
        continue
    for s in list(range(6)) + [100, 500, 999]:
        a, b = ps[f, :, s], cs[f, :, s]
        z = np.sum(np.conj(a) * b)
        print("  sym", s, "phase %.4f" % np.angle(z), "gain %.4f" % (np.sum(np.abs(b) ** 2) / max(np.sum(np.abs(a) ** 2), 1e-30)),
              "per-stream phase", ["%.3f" % np.angle(np.sum(np.conj(a[t]) * b[t])) for t in range(N)],
              "nan", int(np.isnan(b).sum()))

for f in range(F):
    print("rotated frame", f, "eps", cr[f]["cfo_eps"], "evm", e(cr[f]), "sync", cr[f]["sync_index"], plain[f]["sync_index"])
    if plain[f]["status"] != 0:
        continue
    for s_ in list(range(6)) + [100, 500, 999]:
        a, b = ps[f, :, s_], rs[f, :, s_]
        z = np.sum(np.conj(a) * b)
        print("  sym", s_, "phase %.4f" % np.angle(z), "gain %.4f" % (np.sum(np.abs(b) ** 2) / max(np.sum(np.abs(a) ** 2), 1e-30)),
              "corr %.4f" % (abs(z) / np.sqrt(np.sum(np.abs(a) ** 2) * np.sum(np.abs(b) ** 2))),
              "per-stream phase", ["%.3f" % np.angle(np.sum(np.conj(a[t]) * b[t])) for t in range(N)])
    # subcarrier-dependent phase: slope over k of symbol 0
    a, b = ps[f, 0, 0], rs[f, 0, 0]
    ph = np.angle(np.conj(a) * b)
    print("  sym0 stream0 phase at k=0,256,512,..:", ["%.3f" % ph[k] for k in range(0, len(ph), 256)])

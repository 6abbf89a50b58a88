"""tools/cfo_diag.py -- per-frame opt-in CFO diagnostics (GPU box): estimates, EVM with and
without the correction, and whether the search's corr indices moved."""
import sys
import numpy as np
import torch
sys.path.insert(0, '.')
from rub_mimo_amd import _lib
from rub_mimo_amd.receiver import Receiver, RxParams, Synthesizer, SynthParams, cfo_derotate

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 1234
F = int(sys.argv[2]) if len(sys.argv) > 2 else 8
M, cp, N, nac, pid, qam = 2048, 152, 4, 20, 1000, 64
sp = SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid, qam_order=qam,
                 seed=seed, snr_db=30.0)
S = Synthesizer(sp)
L = sp.max_frame_len()
iq = torch.empty((F, N, L), dtype=torch.complex64, device="cuda")
tx = torch.empty((F, N, pid, M), dtype=torch.uint8, device="cuda")
S.generate(iq, L, L, F, tx_idx=tx)


def run(x, cfo):
    r = Receiver(RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                          detector=_lib.DET_MMSE, qam_order=qam, cfo_correct=cfo))
    r.process(x, L, L, F, max_out=pid, ref_mode=1, ref_idx=tx)
    return r.results(), r.corr(F)[0]


p0, c0 = run(iq, False)
b, cb = run(iq, True)
rot = iq.clone()
cfo_derotate(rot, L, F * N, L, 0, -0.3, M)
c, cc = run(rot, True)


def e(r):
    return 10 * np.log10(np.sum(r["evm_num"]) / np.sum(r["evm_den"])) if r["status"] == 0 else None


for f in range(F):
    moved_b = int(np.sum(c0[f] != cb[f]))
    moved_c = int(np.sum(c0[f] != cc[f]))
    print(f, p0[f]["status"], "eps", b[f]["cfo_eps"], c[f]["cfo_eps"], "evm plain/clean/rot",
          e(p0[f]), e(b[f]), e(c[f]), "corr moved", moved_b, moved_c)

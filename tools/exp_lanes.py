"""tools/exp_lanes.py -- experiment: split a C3 batch over L receiver handles on L HIP streams
(each replays its own captured graph) and time a step against the one-handle batch.

usage: python tools/exp_lanes.py [--frames 8] [--lanes 1 2 4] [--steps 20]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--lanes", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from rub_mimo_amd import _lib
    from rub_mimo_amd.receiver import Receiver, RxParams, Synthesizer, SynthParams
    M, cp, N, nac, pid, F = 2048, 152, 4, 20, 1000, a.frames
    sp = SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid, qam_order=64,
                     seed=1234, snr_db=30.0)
    syn = Synthesizer(sp)
    L = sp.max_frame_len()
    iq = torch.empty((F, N, L), dtype=torch.complex64, device="cuda")
    tx = torch.empty((F, N, pid, M), dtype=torch.uint8, device="cuda")
    syn.generate(iq, L, L, F, tx_idx=tx)
    out_sym = torch.empty((F, N, pid, M), dtype=torch.complex64, device="cuda")
    out_idx = torch.empty((F, N, pid, M), dtype=torch.uint8, device="cuda")
    main_s = torch.cuda.current_stream()
    res = {}
    for nl in a.lanes:
        per = F // nl
        streams = [main_s] + [torch.cuda.Stream() for _ in range(nl - 1)]
        rxs = [Receiver(RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac,
                                 pid_max=pid, detector=_lib.DET_MMSE, qam_order=64),
                        stream=s.cuda_stream) for s in streams]

        def step():
            for s in streams[1:]:
                s.wait_stream(main_s)
            for i, (rx, s) in enumerate(zip(rxs, streams)):
                f0 = i * per
                rx.process(iq[f0:f0 + per], L, L, per, max_out=pid, out_sym=out_sym[f0:f0 + per],
                           out_idx=out_idx[f0:f0 + per], ref_mode=1, ref_idx=tx[f0:f0 + per],
                           stream=s.cuda_stream)
            for s in streams[1:]:
                main_s.wait_stream(s)

        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        ok = sum(1 for rx in rxs for r in rx.results(per) if r["status"] == _lib.FRAME_OK)
        res[nl] = {"ms_per_step": dt * 1e3, "frames_ok": ok}
        print(nl, res[nl], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

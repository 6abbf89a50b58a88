"""tools/exp_cumask.py -- can space-sharing the chip between batches beat the serial step?

VERDICT r05 item 4: batch i's decode on D CUs beside batch i+1's front stages (S&C, search,
LS, weights) on the other 256 - D. Whatever the pipelining, an overlapped step cannot be shorter
than max(decode on D CUs, front stages on 256 - D CUs), each measured alone. This runs the C3 x 64
bench batch through receivers whose HIP streams are CU-masked to D CUs
(hipExtStreamCreateWithCUMask: a contiguous range of mask bits lands D/8 CUs on each XCD) with
the persistent decode grid sized to D (mimo_rx_set_grid_cus), and records every stage's event
time per D, the serial step on the whole chip, and that lower bound for every split D.

    python tools/exp_cumask.py [--out gpurun_out/cumask.json] [--steps 5]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "cumask.json"))
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--cus", default="256,224,192,160,128,96,64,32")
    args = ap.parse_args()
    import numpy as np
    import torch
    from rub_mimo_amd import _lib
    from rub_mimo_amd.receiver import Receiver, RxParams, Synthesizer, SynthParams

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    # the HIP runtime already in the process (torch's and the library's): dlopen of the path
    # it was loaded from returns that instance, never a second runtime
    torch.zeros(1, device=dev)
    _lib.lib()
    path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64.so" in ln)
    hip = ctypes.CDLL(path)
    hip.hipExtStreamCreateWithCUMask.restype = ctypes.c_int
    hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                                 ctypes.POINTER(ctypes.c_uint32)]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count

    M, cp, N, nac, pid, F = 2048, 152, 4, 20, 1000, args.frames
    sp = SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid, qam_order=64,
                     seed=1, snr_db=30.0)
    syn = Synthesizer(sp)
    L = sp.max_frame_len()
    iq = torch.empty((F, N, L), dtype=torch.complex64, device=dev)
    tx = torch.empty((F, N, pid, M), dtype=torch.uint8, device=dev)
    syn.generate(iq, L, L, F, tx_idx=tx)
    ref = tx.transpose(1, 2).contiguous()
    out_sym = torch.empty((F, pid, N, M), dtype=torch.complex64, device=dev)
    out_idx = torch.empty((F, pid, N, M), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    rows = []
    for D in [int(x) for x in args.cus.split(",")]:
        words = (n_cu + 31) // 32
        mask = (ctypes.c_uint32 * words)()
        for c in range(min(D, n_cu)):
            mask[c // 32] |= 1 << (c % 32)
        s = ctypes.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), words, mask)
        if rc != 0:
            raise SystemExit("hipExtStreamCreateWithCUMask failed: %d" % rc)
        rx = Receiver(RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                               detector=_lib.DET_MMSE, qam_order=64), stream=s.value)
        _lib.check(_lib.lib().mimo_rx_set_grid_cus(rx._h, D), "set_grid_cus")

        def step():
            rx.process(iq, L, L, F, max_out=pid, out_sym=out_sym, out_idx=out_idx, ref_mode=1,
                       ref_idx=ref, stream=s.value, out_layout=_lib.LAYOUT_SYMBOL_MAJOR)
        for _ in range(2):
            step()
        hip.hipStreamSynchronize(s)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        hip.hipStreamSynchronize(s)
        wall = (time.perf_counter() - t0) / args.steps * 1e3
        rx.stage_times()
        rx.set_timing(True)
        for _ in range(args.steps):
            step()
        hip.hipStreamSynchronize(s)
        rx.set_timing(False)
        st = {k: v[0] / args.steps for k, v in rx.stage_times().items()}
        ok = sum(1 for r in rx.results(F) if r["status"] == _lib.FRAME_OK)
        front = sum(v for k, v in st.items() if k not in ("decode", "evm"))
        row = {"cus": D, "step_ms": wall, "stages_ms": st, "front_ms": front,
               "decode_ms": st.get("decode", 0.0) + st.get("evm", 0.0), "frames_ok": ok}
        rows.append(row)
        print(json.dumps(row), flush=True)
        del rx
        hip.hipStreamDestroy(s)
    full = next(r for r in rows if r["cus"] >= n_cu)
    by = {r["cus"]: r for r in rows}
    bounds = []
    for r in rows:
        D = r["cus"]
        if D >= n_cu or (n_cu - D) not in by:
            continue
        lb = max(r["decode_ms"], by[n_cu - D]["front_ms"])
        bounds.append({"decode_cus": D, "front_cus": n_cu - D, "decode_ms": r["decode_ms"],
                       "front_ms": by[n_cu - D]["front_ms"], "overlapped_step_lower_bound_ms": lb,
                       "serial_step_ms": full["step_ms"]})
    res = {"workload": "C3 x %d captures, fc32 resident, symbol-major, ref_mode 1" % F,
           "n_cu": n_cu, "rows": rows, "split_bounds": bounds,
           "note": "an overlapped step (decode of batch i on D CUs beside the front stages of "
                   "batch i+1 on the rest) is at least max(decode on D, front on 256 - D), each "
                   "measured alone on a CU-masked stream"}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(res, fh, indent=1)
    for b in bounds:
        print("decode %3d CUs %.3f ms | front %3d CUs %.3f ms | bound %.3f vs serial %.3f" % (
            b["decode_cus"], b["decode_ms"], b["front_cus"], b["front_ms"],
            b["overlapped_step_lower_bound_ms"], b["serial_step_ms"]))


if __name__ == "__main__":
    main()

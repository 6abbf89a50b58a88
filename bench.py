"""bench.py -- complex IQ samples/s through the 4x4 MMSE receive path (BASELINE.json metric),
config C3: 2048-pt FFT, cp 152, 4x4, 20 access codes, 1000 data symbols, 64-QAM, synthetic
flat Rayleigh channel at 30 dB SNR.

One step = one pass of the whole receive chain (Schmidl-Cox + plateau, access-code search,
LS estimate, MMSE weights, replay decode, demap, EVM) over a batch of --frames synthetic
captures already resident in HBM. Symbol errors and EVM are counted against the transmitted
QAM indices read from HBM (--ref-mode 1), as main.cc compares with its tx_data file
(main.cc:1394-1411). Repeated steps replay a captured HIP graph of the batch; per-stage
times come from a separate pass with event timing (direct launches). With --gpus N (torchrun, one rank per GPU) every rank
receives its own independent frames (weak scaling, no data-path collective); timing is the
max over ranks between barriers.

Prints one JSON line (rank 0) with the roofline of the dominant kernel (decode) and the CPU
oracle baseline measured on this host.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=8, help="captures per step per GPU")
    ap.add_argument("--M", type=int, default=2048)
    ap.add_argument("--cp", type=int, default=152)
    ap.add_argument("--streams", type=int, default=4)
    ap.add_argument("--nac", type=int, default=20)
    ap.add_argument("--pid", type=int, default=1000)
    ap.add_argument("--qam", type=int, default=64)
    ap.add_argument("--snr", type=float, default=30.0)
    ap.add_argument("--detector", default="mmse", choices=["zf2", "zf", "mmse"])
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--cpu-baseline", type=int, default=1, help="0 to skip the oracle timing")
    ap.add_argument("--ref-mode", type=int, default=1,
                    help="EVM reference: 0 decided symbols, 1 transmitted indices from HBM, "
                         "2 transmitted indices regenerated from the seed")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "decode_pmc.json"))
    return ap.parse_args()


def decode_kernel_name(M, N, args):
    """The decode kernel launch_decode picks for this configuration (decode_stream.hip /
    decode_kernels.hip dispatch rules; all-carrier allocation, 16-byte aligned buffers)."""
    lg = M.bit_length() - 1
    stream_ok = (os.environ.get("RMIMO_DECODE_STREAM", "1") != "0" and args.detector != "siso"
                 and args.frames <= 256 and args.qam <= 256
                 and (N, lg) in ((4, 11), (4, 10), (2, 12), (2, 11)))
    if stream_ok:
        return "decode_stream_kernel<%d,%d>" % (lg, N)
    if 512 <= M <= 4096 and N in (2, 4):
        return "decode_reg_kernel<%d,%d>" % (lg, N)
    return "decode_persistent_kernel"


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from rub_mimo_amd import _lib
    from rub_mimo_amd.receiver import Receiver, RxParams, Synthesizer, SynthParams

    det = {"zf2": _lib.DET_ZF2, "zf": _lib.DET_ZF, "mmse": _lib.DET_MMSE}[args.detector]
    M, cp, N, nac, pid, F = args.M, args.cp, args.streams, args.nac, args.pid, args.frames
    SL = M + cp
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    # ---- synthetic captures, generated on this GPU (outside the timed region)
    from rub_mimo_amd.shard import frame_ids, reduce_stats
    frame_id0, _ = frame_ids(rank, F)
    sp = SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid,
                     qam_order=args.qam, seed=args.seed, snr_db=args.snr)
    syn = Synthesizer(sp)
    L = sp.max_frame_len()
    iq = torch.empty((F, N, L), dtype=torch.complex64, device=dev)
    m_occ_s = M   # all-carrier allocation (framing.cc:949-954)
    tx_idx = torch.empty((F, N, pid, m_occ_s), dtype=torch.uint8, device=dev)
    syn.generate(iq, L, L, F, frame_id0=frame_id0, tx_idx=tx_idx, stream=sh)
    true_len = sum(syn.frame_len(frame_id0 + f) for f in range(F))   # samples per antenna

    rx = Receiver(RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                           detector=det, qam_order=args.qam), stream=sh)
    m_occ = rx.M_occ
    out_sym = torch.empty((F, N, pid, m_occ), dtype=torch.complex64, device=dev)
    out_idx = torch.empty((F, N, pid, m_occ), dtype=torch.uint8, device=dev)

    def step():
        rx.process(iq, L, L, F, max_out=pid, out_sym=out_sym, out_idx=out_idx,
                   ref_mode=args.ref_mode, ref_idx=tx_idx if args.ref_mode == 1 else None,
                   ref_seed=args.seed, frame_id0=frame_id0, stream=sh)

    for _ in range(max(args.warmup, 2)):   # the second identical call captures the HIP graph
        step()
    torch.cuda.synchronize(dev)
    rx.stage_times()  # drop warmup events
    n_exact0 = rx.sc_exact_count()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    n_exact = rx.sc_exact_count()
    # per-stage HIP-event times (roofline numerator/denominator) from a separate pass over the
    # same workload: event timing runs the launches directly instead of the captured graph
    n_stage = max(1, min(args.steps, 5))
    rx.set_timing(True)
    for _ in range(n_stage):
        step()
    torch.cuda.synchronize(dev)
    rx.set_timing(False)
    stages = rx.stage_times()
    res = rx.results(F)
    ok = sum(1 for r in res if r["status"] == _lib.FRAME_OK)
    evm_num = sum(float(np.sum(r["evm_num"])) for r in res)
    evm_den = sum(float(np.sum(r["evm_den"])) for r in res)
    errors = sum(int(np.sum(r["errors"])) for r in res)

    samples_local = float(N) * true_len * args.steps
    # symbols decoded per step (frames that sync; the others are scanned, not decoded)
    n_dec = sum(min(int(r["n_sym"]), pid) for r in res if r["status"] == _lib.FRAME_OK)
    tot, elapsed = reduce_stats(dict(samples=samples_local, frames_ok=ok, symbols=n_dec,
                                     evm_num=evm_num, evm_den=evm_den, errors=errors), elapsed,
                                dist if world > 1 else None, device=dev)
    samples_total, ok, n_dec_all, evm_num, evm_den, errors = (
        tot[k] for k in ("samples", "frames_ok", "symbols", "evm_num", "evm_den", "errors"))

    # ---- roofline of the dominant kernel: decode (HBM bound)
    dec_ms, dec_n = stages["decode"]
    dec_avg_s = dec_ms / max(dec_n, 1) / 1e3
    # per decoded symbol: N bodies read, N x M_occ complex64 + uint8 written (+ the uint8
    # transmitted index read when the EVM reference comes from HBM)
    per_sym = N * M * 8 + N * m_occ * 9 + (N * m_occ if args.ref_mode == 1 else 0)
    dec_bytes = n_dec * per_sym
    achieved = dec_bytes / dec_avg_s / 1e9 if dec_avg_s > 0 else 0.0
    traffic = None
    if os.path.exists(args.pmc_json):
        try:
            pm = json.load(open(args.pmc_json))
            cfgm = pm.get("config", {})
            if ((cfgm.get("M"), cfgm.get("streams"), cfgm.get("frames"), cfgm.get("pid"),
                    cfgm.get("ref_mode")) == (M, N, F, pid, args.ref_mode)
                    and pm.get("kernel") == decode_kernel_name(M, N, args).split("<")[0]):
                traffic = pm.get("decode_hbm_bytes_per_launch")
        except Exception:
            traffic = None

    # ---- CPU baseline: the C oracle (faithful brute-force search, 1 core) on the first frame
    # of this rank's batch that syncs, plus the EVM-dB delta of the GPU vs the oracle on it
    cpu = None
    evm_delta = None
    if rank == 0 and world == 1 and args.cpu_baseline:
        from oracle import ref
        fsel = next((f for f, r in enumerate(res) if r["status"] == _lib.FRAME_OK), None)
        if fsel is not None:
            L0 = syn.frame_len(frame_id0 + fsel)
            host = iq[fsel, :, :L0].cpu().numpy()
            o = ref.FrameSyncRef(M, cp, N, nac, pid_max=pid, detector=det)
            c0 = time.perf_counter()
            o.execute(host)
            c1 = time.perf_counter()
            cpu = {"value": N * L0 / (c1 - c0), "unit": "complex samples/s", "cores": 1,
                   "kind": "port",
                   "sample": "frame %d of the batch (first that syncs): %d samples x %d "
                             "antennas through oracle/mimo_ref.c framesync (Schmidl-Cox direct "
                             "sums, brute-force search as framing.cc:702-744, MMSE, decode), "
                             "gcc -O3, 1 thread, %.1f s" % (fsel, L0, N, c1 - c0)}
            sym = o.symbols()[:pid]
            if len(sym):
                _, en, ed, _ = ref.demap_evm(sym, args.qam, tx_idx[fsel, :, :len(sym)].cpu().numpy())
                r = res[fsel]
                evm_cpu = 10 * np.log10(float(np.sum(en)) / float(np.sum(ed)))
                evm_gpu = 10 * np.log10(float(np.sum(r["evm_num"])) / float(np.sum(r["evm_den"])))
                evm_delta = {"frame": fsel, "gpu_db": evm_gpu, "cpu_db": evm_cpu,
                             "delta_db": evm_gpu - evm_cpu,
                             "sync_index_equal": int(o.get_sync_index()) == int(r["sync_index"])}

    value = samples_total / elapsed
    ms_step = elapsed / args.steps * 1e3
    bytes_alg = samples_total * 8 + args.steps * n_dec_all * N * m_occ * 9
    line = {
        "metric": "complex IQ samples/s through 4x4 MMSE detect; EVM-dB delta vs CPU ref",
        "value": value,
        "unit": "complex samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32 (complex64; fp64 weight solve)",
        "data": "synthetic (GPU tx_worker-layout frames, flat Rayleigh 4x4, AWGN %.0f dB)"
                % args.snr,
        "config": {"workload": "C3: 4x4 MMSE, 2048-pt FFT, cp 152, 64-QAM, 20 access codes, "
                               "1000 data symbols/frame",
                   "M": M, "cp": cp, "streams": N, "access_codes": nac, "pid": pid,
                   "qam": args.qam, "detector": args.detector, "frames_per_step_per_gpu": F,
                   "parallelism": "frames sharded across %d GPU(s), no collective" % world},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": decode_kernel_name(M, N, args),
                     "bytes_per_launch": dec_bytes,
                     "symbols_per_launch": n_dec, "bytes_per_symbol": per_sym,
                     "avg_launch_ms": dec_avg_s * 1e3},
        "cpu_baseline": cpu,
        "evm_db_delta_vs_cpu": evm_delta,
        "pipeline_hbm_gbs": bytes_alg / elapsed / 1e9,
        "stages_ms_per_step": {k: v[0] / n_stage for k, v in stages.items()},
        "frames_ok": int(ok), "frames": int(F * world),
        "sc_exact_recomputes_per_step": n_exact / max(args.steps, 1),
        "evm_db": 10 * np.log10(evm_num / evm_den) if evm_den > 0 else None,
        "symbol_errors_last_step": int(errors),
    }
    if rank == 0:
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

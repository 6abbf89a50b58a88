"""bench.py -- complex IQ samples/s through the N x N MMSE receive path (BASELINE.json metric).

Default workload C3 (BASELINE.json configs[2], the config the metric is quoted on): 2048-pt
FFT, cp 152, 4x4, 20 access codes, 1000 data symbols, 64-QAM, synthetic flat Rayleigh channel
at 30 dB SNR, 64 captures per step per GPU. --workload c2 / c4 / c5 run the other GPU configs.

One step = one pass of the whole receive chain (Schmidl-Cox + plateau, access-code search, LS
estimate, detector weights, replay decode, demap, EVM) over a batch of synthetic captures
already resident in HBM. Symbol errors and EVM are counted against the transmitted QAM indices
read from HBM (--ref-mode 1), as main.cc compares with its tx_data file (main.cc:1394-1411).
Repeated steps replay a captured HIP graph of the batch; per-stage times come from a separate
pass with event timing (direct launches).

`value` counts the samples of the frames that reach the detector (status OK) per second;
captures that never sync are scanned (S&C) but not detected and only count toward the
secondary `scan_rate_all_captures`.

Multi-GPU: one process per GPU. `python bench.py --gpus N` with N > 1 starts its N rank
processes itself (fresh children, before any GPU call in the parent) unless it already runs
under torchrun (WORLD_SIZE set, which must equal --gpus). Every rank receives its own frames
(weak scaling, no data-path collective). With N > 1 a second, bounded leg measures the rank-0
ingest path: rank 0 holds every rank's captures at the sc16 wire format and scatters them over
RCCL point-to-point (double-buffered against the receive; rub_mimo_amd/shard.py), reported
under `rank0_scatter`; `--ingest scatter` makes that the timed mode.

Prints one JSON line (rank 0) with the roofline of the dominant kernel (decode) and the CPU
oracle baseline measured on this host (1 core and the box's core share).
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
C5_STREAMS = 8          # BASELINE configs[4]: 8 independent 20 MS/s streams

WORKLOADS = {
    "c2": dict(M=1024, cp=152 // 2, streams=2, nac=20, pid=1000, qam=16, snr=25.0,
               detector="zf2", frames=32, fps=1,
               desc="C2: 2x2 ZF (reference adjugate), 1024-pt FFT, cp 76, 16-QAM, 20 access "
                    "codes, 1000 data symbols/frame (synthetic stand-in for recorded USRP IQ)"),
    "c3": dict(M=2048, cp=152, streams=4, nac=20, pid=1000, qam=64, snr=30.0, detector="mmse",
               frames=64, fps=1,
               desc="C3: 4x4 MMSE, 2048-pt FFT, cp 152, 64-QAM, 20 access codes, "
                    "1000 data symbols/frame"),
    "c4": dict(M=4096, cp=304, streams=8, nac=20, pid=1000, qam=256, snr=35.0, detector="mmse",
               frames=8, fps=1,
               desc="C4: 8x8 MMSE, 4096-pt FFT, cp 304, 256-QAM, 20 access codes, 1000 data "
                    "symbols/frame, batched frames"),
    "c5": dict(M=2048, cp=152, streams=4, nac=20, pid=1000, qam=64, snr=30.0, detector="mmse",
               frames=C5_STREAMS, fps=4,
               desc="C5: 4x4 MMSE, 8 independent 20 MS/s IQ streams of back-to-back C3 frames "
                    "(re-armed per frame), streams sharded across GPUs"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--frames", type=int, default=None,
                    help="captures per step per GPU (c5: streams in the whole job)")
    ap.add_argument("--frames-per-stream", type=int, default=None, help="c5: frames per stream")
    for k, t in (("M", int), ("cp", int), ("streams", int), ("nac", int), ("pid", int),
                 ("qam", int), ("snr", float)):
        ap.add_argument("--" + k, type=t, default=None)
    ap.add_argument("--detector", default=None, choices=["zf2", "zf", "mmse"])
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--ingest", default="resident", choices=["resident", "scatter"],
                    help="resident: each rank's captures already in its HBM (headline); "
                         "scatter: rank 0 scatters sc16 wire captures every step (timed)")
    ap.add_argument("--scatter-steps", type=int, default=5,
                    help="steps of the secondary rank-0 scatter leg when N > 1 (0: skip)")
    ap.add_argument("--cfo", type=float, default=0.0,
                    help="apply this carrier-frequency offset (subcarrier spacings) to the "
                         "synthetic captures and turn on the receiver's opt-in CFO correction")
    ap.add_argument("--sample-format", default="fc32", choices=["fc32", "sc16"],
                    help="resident capture format: fc32 (complex64, the reference's framesync "
                         "input) or sc16 (UHD wire samples read in place, 4 B/sample)")
    ap.add_argument("--sc16-steps", type=int, default=None,
                    help="steps of the secondary sc16-resident leg of an fc32 run (0: skip; "
                         "default: --steps)")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="0 to skip the oracle timing")
    ap.add_argument("--h2d", type=int, default=1,
                    help="0 to skip the separately reported pinned-host -> HBM copy timing")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the multi-core CPU baseline (0: the box's core share)")
    ap.add_argument("--out-layout", default="symbol", choices=["symbol", "stream"],
                    help="output (and reference-index) layout per frame slot: symbol-major "
                         "[pid][N][M_occ] (the reference callback's per-symbol order) or "
                         "stream-major [N][pid][M_occ]; the same bytes either way")
    ap.add_argument("--ref-mode", type=int, default=1,
                    help="EVM reference: 0 decided symbols, 1 transmitted indices from HBM, "
                         "2 transmitted indices regenerated from the seed")
    ap.add_argument("--pmc-json", default=None)
    ap.add_argument("--pipeline", type=int, default=0,
                    help="D > 0: two receivers alternate batches, batch i's decode on D CUs "
                         "beside batch i+1's front stages (S&C .. weights) on the other CUs "
                         "(CU-masked HIP streams, mimo_batch.stages); 0: one serial stream")
    a = ap.parse_args()
    w = WORKLOADS[a.workload]
    for k in ("M", "cp", "streams", "nac", "pid", "qam", "snr", "detector", "frames"):
        if getattr(a, k) is None:
            setattr(a, k, w[k])
    if a.frames_per_stream is None:
        a.frames_per_stream = w["fps"]
    if a.pmc_json is None:
        a.pmc_json = os.path.join(ROOT, "profiles", "decode_pmc_%s.json" % a.workload)
    return a


def spawn_ranks(args):
    """bench.py --gpus N outside torchrun: start N fresh rank processes (this parent never
    touches the GPU) and exit with the first non-zero status."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable] + sys.argv, env=env))
    rc = 0
    for p in procs:
        c = p.wait()
        if c != 0 and rc == 0:
            rc = c
    return rc


def cu_masked_stream(lo, hi):
    """A HIP stream whose kernels run on CUs [lo, hi) only (hi None: the device's count):
    hipExtStreamCreateWithCUMask from the HIP runtime already loaded in this process (a
    contiguous range of mask bits spreads evenly over the XCDs). Returns the raw handle."""
    import torch
    path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64.so" in ln)
    hip = ctypes.CDLL(path)
    n = torch.cuda.get_device_properties(0).multi_processor_count
    hi = n if hi is None else hi
    words = (n + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for c in range(lo, hi):
        mask[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                                 ctypes.POINTER(ctypes.c_uint32)]
    if hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), words, mask) != 0:
        raise SystemExit("hipExtStreamCreateWithCUMask failed")
    return s.value


def decode_kernel_name(M, N, args, path=None):
    """The decode kernel family launch_decode ran (mimo_rx_get_decode_path), named as rocprof
    shows it; for the per-symbol family the dispatch rules of decode_kernels.hip pick it."""
    lg = M.bit_length() - 1
    if path == 1:
        return "decode_stream_kernel<%d,%d>" % (lg, N)
    if path == 2:   # (the persistent spectra form for M >= 2048 and the 128-subcarrier apply)
        return ("spectra_persist_kernel<%d>|apply_split2_kernel<8>" % lg if lg >= 11 else
                "spectra_kernel<%d>|apply_split2_kernel<8>" % lg)
    stream_ok = (args.detector != "siso" and args.qam <= 256 and (N, lg) in ((4, 11), (4, 10), (2, 12), (2, 11), (2, 10)))
    if stream_ok:
        return "decode_stream_kernel<%d,%d>" % (lg, N)
    if 512 <= M <= 4096 and N in (2, 4):
        return "decode_reg_kernel<%d,%d>" % (lg, N)
    if M < 512 and N in (2, 4):
        return "decode_persistent_kernel"
    if N == 8 and 512 <= M <= 4096 and args.detector != "siso" and args.pid >= M // 64:
        return "spectra_kernel<%d>|apply_split_kernel<8>" % lg
    return "decode_kernel<%d,%d>" % (lg, N)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def core_share():
    """CPU threads this process may use: the affinity set, capped at the box's share of 16
    per GPU (nproc on the GPU box shows the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_baseline(args, det, frames, c4_mode):
    """The C oracle (oracle/mimo_ref.c, gcc -O2 as mimo/makefile:9) on frames of this rank's
    batch. frames: list of (rx [N][L] complex64 host, trigger, sync_index) of frames that
    synced on the GPU. Mode 1: one frame, 1 thread. Mode 2: independent frames, one per thread,
    core_share() threads. C4 (c4_mode): S&C skipped from the GPU's trigger and the Parseval
    search variant (the faithful brute force costs ~1.4 TFLOP per frame), plus the decode
    stage alone."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import ref
    M, cp, N, nac, pid = args.M, args.cp, args.streams, args.nac, args.pid

    def run_one(item):
        rx, trig, si = item
        o = ref.FrameSyncRef(M, cp, N, nac, pid_max=pid, detector=det,
                             search_mode=1 if c4_mode else 0)
        t0 = time.perf_counter()
        if c4_mode:
            o.execute_from_sync(rx, trig, si)
        else:
            o.execute(rx)
        t1 = time.perf_counter()
        return o, t1 - t0

    rx0 = frames[0][0]
    o, dt1 = run_one(frames[0])
    n1 = N * rx0.shape[1]
    ph = o.phase_times()
    T = args.cpu_threads or core_share()
    items = [frames[i % len(frames)] for i in range(T)]
    with ThreadPoolExecutor(max_workers=T) as ex:
        t0 = time.perf_counter()
        outs = list(ex.map(run_one, items))
        wall = time.perf_counter() - t0
    nT = sum(N * it[0].shape[1] for it in items)
    kind = ("S&C skipped (GPU trigger), Parseval search variant, LS, MMSE weights, decode"
            if c4_mode else "Schmidl-Cox direct sums, brute-force search as "
                            "framing.cc:702-744, %s weights, decode" % args.detector)
    res = {
        "value": n1 / dt1, "unit": "complex samples/s", "cores": 1, "kind": "port",
        "sample": "1 frame (%d samples x %d antennas) of the GPU batch through oracle/mimo_ref.c "
                  "framesync (%s), gcc -O2 (mimo/makefile:9), 1 thread, %.1f s"
                  % (rx0.shape[1], N, kind, dt1),
        "cpu_model": cpu_model(),
        "phase_s_1core": ph,
        "nproc": {"value": nT / wall, "cores": T, "frames": T, "wall_s": wall,
                  "sample": "%d independent frames (cycling over %d distinct synced frames of "
                            "the batch), one per thread, %d threads" % (T, len(frames), T)},
    }
    if c4_mode:
        n_sym = o.symbols().shape[0]
        res["decode_stage"] = {
            "value": N * (M + cp) * n_sym / max(ph["decode"], 1e-12),
            "unit": "complex samples/s", "cores": 1,
            "sample": "%d symbols x %d antennas of replay decode (FFT, %dx%d apply, gain) "
                      "given W, %.2f s" % (n_sym, N, N, N, ph["decode"])}
    return res, o


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    world = int(world_env or "1")
    if world != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world), file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from rub_mimo_amd import _lib
    from rub_mimo_amd.receiver import Receiver, RxParams, Synthesizer, SynthParams, ingest_sc16
    from rub_mimo_amd.shard import ScatterPipeline, frame_ids, reduce_stats, split_streams

    det = {"zf2": _lib.DET_ZF2, "zf": _lib.DET_ZF, "mmse": _lib.DET_MMSE}[args.detector]
    M, cp, N, nac, pid = args.M, args.cp, args.streams, args.nac, args.pid
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    c5 = args.workload == "c5"

    # ---- synthetic captures, generated on this GPU (outside the timed region)
    sp = SynthParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid=pid,
                     qam_order=args.qam, seed=args.seed, snr_db=args.snr)
    syn = Synthesizer(sp)
    m_occ_s = M   # all-carrier allocation (framing.cc:949-954)
    if c5:
        if args.frames % world:
            raise SystemExit("c5: %d streams do not split evenly over %d ranks"
                             % (args.frames, world))
        s0, s1 = split_streams(args.frames, world, rank)
        F = s1 - s0
        J = args.frames_per_stream
        K = J + 1                   # one slot past the last frame (the stream's tail)
        _, L = syn.stream_layout(args.frames, J)       # one capture length for every rank
        iq = torch.zeros((F, N, L), dtype=torch.complex64, device=dev)
        tx_idx = torch.empty((F * K, N, pid, m_occ_s), dtype=torch.uint8, device=dev)
        starts, lens = syn.generate_streams(iq, L, F, J, K, stream0=s0, tx_idx=tx_idx, stream=sh)
        ref_starts = torch.from_numpy(starts.view(np.int64).copy()).to(dev)
        frame_id0 = s0 * J
        slot_len = [[lens[f][j] if j < J else 0 for j in range(K)] for f in range(F)]
    else:
        frame_id0, F = frame_ids(rank, args.frames)
        K = 1
        L = sp.max_frame_len()
        iq = torch.empty((F, N, L), dtype=torch.complex64, device=dev)
        tx_idx = torch.empty((F, N, pid, m_occ_s), dtype=torch.uint8, device=dev)
        syn.generate(iq, L, L, F, frame_id0=frame_id0, tx_idx=tx_idx, stream=sh)
        ref_starts = None
        slot_len = [[syn.frame_len(frame_id0 + f)] for f in range(F)]
    all_len = sum(sum(r) for r in slot_len)          # transmitted samples per antenna
    if args.cfo:
        from rub_mimo_amd.receiver import cfo_derotate
        cfo_derotate(iq, L, F * N, L, 0, -args.cfo, M, stream=sh)   # a CFO of +args.cfo
    sc16 = args.sample_format == "sc16"
    # sc16 full scale: the job's peak |I|, |Q| with 1 % headroom, as a receive gain would set it
    amax = torch.view_as_real(iq).abs().max().reshape(1).float()
    if world > 1:
        dist.all_reduce(amax, op=dist.ReduceOp.MAX)
    wscale = float(amax.item()) * 1.01 / 32767.0
    src = iq
    if sc16:
        # resident wire captures [F][N][L][2] int16; iq becomes their widened copy, which the
        # CPU baseline reads
        src = (torch.view_as_real(iq) / wscale).round_().clamp_(-32768, 32767).to(torch.int16)
        ingest_sc16(src, L, iq, L, F * N, L, wscale, stream=sh)
    in_bytes = 4 if sc16 else 8             # HBM bytes per input sample

    rx = Receiver(RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac, pid_max=pid,
                           detector=det, qam_order=args.qam, cfo_correct=args.cfo != 0.0),
                  stream=sh)
    m_occ = rx.M_occ
    sym_major = args.out_layout == "symbol"
    layout = _lib.LAYOUT_SYMBOL_MAJOR if sym_major else _lib.LAYOUT_STREAM_MAJOR
    oshape = (F * K, pid, N, m_occ) if sym_major else (F * K, N, pid, m_occ)
    out_sym = torch.empty(oshape, dtype=torch.complex64, device=dev)
    out_idx = torch.empty(oshape, dtype=torch.uint8, device=dev)
    # the reference rows in the output layout (tx_idx itself stays stream-major for the CPU check)
    ref_rows = tx_idx.transpose(1, 2).contiguous() if sym_major else tx_idx

    def step(x=None, wire_in=sc16):
        rx.process(src if x is None else x, L, L, F, max_out=pid, out_sym=out_sym,
                   out_idx=out_idx, ref_mode=args.ref_mode,
                   ref_idx=ref_rows if args.ref_mode == 1 else None, ref_seed=args.seed,
                   frame_id0=frame_id0, stream=sh, frames_per_capture=K, ref_starts=ref_starts,
                   sc16=wire_in, sc16_scale=wscale, out_layout=layout)

    # ---- rank-0 sc16 ingest (used by --ingest scatter and the secondary scatter leg)
    wire = None

    def make_wire():
        """Rank 0: every rank's captures at the sc16 wire format [world][F][N][L][2] int16
        (the same synthetic frames quantised as UHD's sc16 converter would carry them)."""
        if rank != 0:
            return None
        w = torch.empty((world, F, N, L, 2), dtype=torch.int16, device=dev)
        tmp = torch.empty_like(iq)
        for r in range(world):
            if c5:
                a, b = split_streams(args.frames, world, r)
                tmp.zero_()
                syn.generate_streams(tmp, L, b - a, args.frames_per_stream, K, stream0=a,
                                     stream=sh)
            else:
                syn.generate(tmp, L, L, F, frame_id0=r * F, stream=sh)
            v = torch.view_as_real(tmp) / wscale
            w[r].copy_(v.round_().clamp_(-32768, 32767).to(torch.int16))
        del tmp
        return w

    def scatter_loop(pipe, n):
        """n steps of: wait for this rank's wire batch, receive it (read in place with
        --sample-format sc16, else widened by mimo_ingest_sc16 into the complex64 batch first);
        batch i+1's scatter overlaps batch i's receive."""
        scale = wscale
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        pipe.start()
        for _ in range(n):
            w = pipe.next()
            if sc16:
                step(w, True)
            else:
                ingest_sc16(w.data_ptr(), L, iq.data_ptr(), L, F * N, L, scale, stream=sh)
                step(iq, False)
        pipe.drain()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        return time.perf_counter() - t0

    timed_scatter = args.ingest == "scatter"
    pipe_info = None
    if args.pipeline and (timed_scatter or args.cfo or c5):
        raise SystemExit("--pipeline: resident one-frame-per-capture batches without --cfo only")
    if args.pipeline:
        # ---- pipelined: handle h = i % 2 runs batch i's front half on stream sF (the CUs
        # [D, n_cu)) and its decode half on stream sD (CUs [0, D)); batch i's decode runs
        # beside batch i+1's front half. Events order: front(i) -> decode(i) (the handle's
        # workspace), decode(i - 2) -> front(i) (the same handle's workspace reused)
        D = args.pipeline
        n_cu_dev = torch.cuda.get_device_properties(dev).multi_processor_count
        if not 0 < D < n_cu_dev or D % 8:
            raise SystemExit("--pipeline: D must be a multiple of 8 in (0, %d)" % n_cu_dev)
        sF_raw, sD_raw = cu_masked_stream(D, None), cu_masked_stream(0, D)
        sF = torch.cuda.ExternalStream(sF_raw, device=dev)
        sD = torch.cuda.ExternalStream(sD_raw, device=dev)
        hs = []
        for _ in range(2):
            r_ = Receiver(RxParams(M=M, cp_len=cp, num_streams=N, num_access_codes=nac,
                                   pid_max=pid, detector=det, qam_order=args.qam), stream=sF_raw)
            _lib.check(_lib.lib().mimo_rx_set_grid_cus(r_._h, D), "set_grid_cus")
            hs.append(r_)
        evF = [torch.cuda.Event(), torch.cuda.Event()]
        evD = [torch.cuda.Event(), torch.cuda.Event()]

        def pstep(i):
            h = i & 1
            if i >= 2:
                sF.wait_event(evD[h])
            kw = dict(max_out=pid, out_sym=out_sym, out_idx=out_idx, ref_mode=args.ref_mode,
                      ref_idx=ref_rows if args.ref_mode == 1 else None, ref_seed=args.seed,
                      frame_id0=frame_id0, sc16=sc16, sc16_scale=wscale, out_layout=layout)
            hs[h].process(src, L, L, F, stream=sF_raw, stages=_lib.STAGES_FRONT, **kw)
            evF[h].record(sF)
            sD.wait_event(evF[h])
            hs[h].process(src, L, L, F, stream=sD_raw, stages=_lib.STAGES_DECODE, **kw)
            evD[h].record(sD)

        torch.cuda.synchronize(dev)
        for i in range(max(args.warmup, 2) * 2):   # every (handle, half) captured and replayed
            pstep(i)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(args.steps):
            pstep(i + 2 * max(args.warmup, 2))
        torch.cuda.synchronize(dev)
        elapsed = time.perf_counter() - t0
        # the serial step of the same batch on the whole chip, for the line
        for _ in range(2):
            step()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize(dev)
        pipe_info = {"decode_cus": D, "front_cus": n_cu_dev - D,
                     "serial_ms_per_step": (time.perf_counter() - t1) / args.steps * 1e3,
                     "note": "batch i's decode (mimo_batch.stages = DECODE) on D CUs beside "
                             "batch i+1's S&C, search, LS and weights (stages = FRONT) on the "
                             "others; two handles alternate batches; serial_ms_per_step is the "
                             "whole chain on the whole chip, one stream"}
        hs[0].results(F * K)
        del hs
    elif timed_scatter:
        wire = make_wire()
        pipe = ScatterPipeline(dist if world > 1 else None, wire, (F, N, L, 2), torch.int16, dev,
                               rank, world)
        scatter_loop(pipe, max(args.warmup, 2))
        torch.cuda.synchronize(dev)
        rx.stage_times()
        rx.sc_exact_count()
        elapsed = scatter_loop(pipe, args.steps)
    else:
        for _ in range(max(args.warmup, 2)):   # the second identical call captures the HIP graph
            step()
        torch.cuda.synchronize(dev)
        rx.stage_times()  # drop warmup events
        rx.sc_exact_count()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
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
    res = rx.results(F * K)
    ok_slots = [i for i, r in enumerate(res) if r["status"] == _lib.FRAME_OK]
    ok = len(ok_slots)
    rescans = sum(1 for r in res if r["status"] == _lib.FRAME_RESCAN)
    evm_num = sum(float(np.sum(res[i]["evm_num"])) for i in ok_slots)
    evm_den = sum(float(np.sum(res[i]["evm_den"])) for i in ok_slots)
    errors = sum(int(np.sum(res[i]["errors"])) for i in ok_slots)

    def ok_len(i, rr=None):
        """Transmitted length of the frame decoded in slot i (its reference row)."""
        r = (res if rr is None else rr)[i]
        if not c5:
            return slot_len[i][0]
        c = i // K
        j = int(r["ref_frame"]) - c * K
        return slot_len[c][j] if 0 <= j < K else 0

    detected_len = sum(ok_len(i) for i in ok_slots)
    samples_local = float(N) * detected_len * args.steps
    scanned_local = float(N) * all_len * args.steps
    n_dec = sum(min(int(res[i]["n_sym"]), pid) for i in ok_slots)
    tot, elapsed = reduce_stats(dict(samples=samples_local, frames_ok=ok, symbols=n_dec,
                                     evm_num=evm_num, evm_den=evm_den, errors=errors), elapsed,
                                dist if world > 1 else None, device=dev)
    samples_total, ok_all, n_dec_all, evm_num, evm_den, errors = (
        tot[k] for k in ("samples", "frames_ok", "symbols", "evm_num", "evm_den", "errors"))
    scanned_total, _ = reduce_stats(dict(samples=scanned_local, frames_ok=0, symbols=0,
                                         evm_num=0, evm_den=0, errors=0), elapsed,
                                    dist if world > 1 else None, device=dev)
    scanned_total = scanned_total["samples"]

    # ---- secondary leg (fc32 headline): the same captures resident as sc16 wire samples,
    # read in place (C3-type geometries) or widened internally; its own EVM (quantised input)
    sc16_info = None
    n16 = args.steps if args.sc16_steps is None else args.sc16_steps
    if not sc16 and not timed_scatter and n16 > 0 and not args.cfo:
        w16 = (torch.view_as_real(iq) / wscale).round_().clamp_(-32768, 32767).to(torch.int16)
        for _ in range(2):
            step(w16, True)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(n16):
            step(w16, True)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        t16 = time.perf_counter() - t0
        r16 = rx.results(F * K)
        ok16 = [i for i, r in enumerate(r16) if r["status"] == _lib.FRAME_OK]
        tot16, t16 = reduce_stats(dict(
            samples=float(N) * sum(ok_len(i, r16) for i in ok16) * n16, frames_ok=len(ok16),
            symbols=0, evm_num=sum(float(np.sum(r16[i]["evm_num"])) for i in ok16),
            evm_den=sum(float(np.sum(r16[i]["evm_den"])) for i in ok16), errors=0), t16,
            dist if world > 1 else None, device=dev)
        sc16_info = {
            "value": tot16["samples"] / t16, "ms_per_step": t16 / n16 * 1e3, "steps": n16,
            "frames_ok": int(tot16["frames_ok"]),
            "evm_db": (10 * np.log10(tot16["evm_num"] / tot16["evm_den"])
                       if tot16["evm_den"] > 0 else None),
            "sc16_scale": wscale,
            "note": "the same captures quantised to UHD sc16 wire samples (4 B/sample) at the "
                    "job's peak, resident in HBM and read in place by the S&C, search + LS and "
                    "streaming decode kernels (mimo_batch.sample_format = MIMO_SAMPLE_SC16)"}
        del w16

    # ---- secondary leg (N > 1, resident headline): rank-0 sc16 scatter, bounded
    scatter_info = None
    if world > 1 and not timed_scatter and args.scatter_steps > 0:
        wire = make_wire()
        pipe = ScatterPipeline(dist, wire, (F, N, L, 2), torch.int16, dev, rank, world)
        scatter_loop(pipe, 1)
        t_sc = scatter_loop(pipe, args.scatter_steps)
        t_sc = reduce_stats(dict(samples=0, frames_ok=0, symbols=0, evm_num=0, evm_den=0,
                                 errors=0), t_sc, dist, device=dev)[1]
        wire_bytes = (world - 1) * F * N * L * 4 * args.scatter_steps
        scatter_info = {
            "value": samples_total / args.steps * args.scatter_steps / t_sc,
            "ms_per_step": t_sc / args.scatter_steps * 1e3, "steps": args.scatter_steps,
            "wire": "sc16 (4 B/sample), " + ("read in place on each rank" if sc16 else
                                              "mimo_ingest_sc16 widening on each rank"),
            "rank0_out_gbs": wire_bytes / t_sc / 1e9,
            "note": "rank 0 sends every peer its captures each step over RCCL P2P (xGMI), "
                    "double-buffered against the receive; value counts detected-frame samples"}
        del wire

    # ---- roofline of the dominant kernel: decode (HBM bound)
    dec_ms, dec_n = stages["decode"]
    dec_avg_s = dec_ms / max(dec_n, 1) / 1e3
    # per decoded symbol: N bodies read, N x M_occ complex64 + uint8 written (+ the uint8
    # transmitted index read when the EVM reference comes from HBM)
    kname = decode_kernel_name(M, N, args, rx.decode_path())
    # (sc16 is read in place by the streaming decode; other decode kernels read the widened copy)
    dec_in = in_bytes if kname.startswith("decode_stream") else 8
    per_sym = N * M * dec_in + N * m_occ * 9 + (N * m_occ if args.ref_mode == 1 else 0)
    dec_bytes = n_dec * per_sym
    achieved = dec_bytes / dec_avg_s / 1e9 if dec_avg_s > 0 else 0.0
    # ---- the decode's memory pattern alone, on this box, in this process (after the timed
    # region): mimo_probe_decode_pattern stages and stores exactly the decode's bytes on its
    # grid with no arithmetic, over the same buffers -- the rate this box's HBM gives that
    # pattern, against which the decode's own time is stated
    pattern = None
    if (kname.startswith("decode_stream") and not c5 and not sc16 and not args.cfo
            and args.ref_mode == 1 and sym_major and m_occ == M and ok > 0
            and (N, M) in ((4, 2048), (4, 1024), (2, 4096), (2, 2048), (2, 1024))):
        pms = ctypes.c_float(0.0)
        prc = _lib.lib().mimo_probe_decode_pattern(
            iq.data_ptr(), L, F, N, M, cp, ok, pid, ref_rows.data_ptr(), out_sym.data_ptr(),
            out_idx.data_ptr(), 5, sh, ctypes.byref(pms))
        torch.cuda.synchronize(dev)
        if prc == 0 and pms.value > 0:
            p_s = pms.value / 1e3
            p_bytes = ok * pid * (N * (M + 2) * 8 + N * M * 9 + N * M)
            pattern = {"ms": pms.value, "bytes": p_bytes, "gbs": p_bytes / p_s / 1e9,
                       "decode_ms": dec_avg_s * 1e3,
                       "decode_vs_pattern": (dec_avg_s / p_s) if p_s > 0 else None,
                       "note": "mimo_probe_decode_pattern: the decode's staging DMA and output "
                               "stores (the same grid, bytes and buffers), no transform, apply "
                               "or demap; mean of 5 launches after the timed region"}
    traffic = None
    if os.path.exists(args.pmc_json):
        try:
            pm = json.load(open(args.pmc_json))
            cfgm = pm.get("config", {})
            if ((cfgm.get("M"), cfgm.get("streams"), cfgm.get("frames"), cfgm.get("pid"),
                    cfgm.get("ref_mode"), cfgm.get("sample_format", "fc32"))
                    == (M, N, F, pid, args.ref_mode, args.sample_format)
                    and pm.get("kernel") == "|".join(x.split("<")[0] for x in kname.split("|"))):
                traffic = pm.get("decode_hbm_bytes_per_launch")
        except Exception:
            traffic = None

    # ---- CPU baseline: the C oracle on synced frames of this batch (rank 0, N = 1 only)
    cpu = None
    evm_delta = None
    if rank == 0 and world == 1 and args.cpu_baseline and ok_slots:
        from oracle import ref
        sel = ok_slots[:4]
        frames = []
        for i in sel:
            r = res[i]
            c = i // K
            org = int(r["origin"])
            ln = ok_len(i) if not c5 else int(r["num_samples_processed"])
            host = iq[c, :, org:org + ln].cpu().numpy()
            frames.append((host, int(r["trigger"]), int(r["sync_index"])))
        cpu, o = cpu_baseline(args, det, frames, args.workload == "c4")
        fsel = sel[0]
        sym = o.symbols()[:pid]
        if len(sym):
            ti = tx_idx[fsel if not c5 else int(res[fsel]["ref_frame"]), :, :len(sym)]
            _, en, ed, _ = ref.demap_evm(sym, args.qam, ti.cpu().numpy())
            r = res[fsel]
            evm_cpu = 10 * np.log10(float(np.sum(en)) / float(np.sum(ed)))
            evm_gpu = 10 * np.log10(float(np.sum(r["evm_num"])) / float(np.sum(r["evm_den"])))
            evm_delta = {"frame_slot": fsel, "gpu_db": evm_gpu, "cpu_db": evm_cpu,
                         "delta_db": evm_gpu - evm_cpu,
                         "sync_index_equal": int(o.get_sync_index()) == int(r["sync_index"])}

    # ---- H2D, reported separately (never the headline): the batch's captures
    # copied from pinned host memory into HBM on the receive stream, at most 8 captures
    h2d = None
    if rank == 0 and args.h2d:
        nc = min(F, 8)
        dev_iq = iq[:nc]
        host = torch.empty(dev_iq.shape, dtype=dev_iq.dtype, pin_memory=True)
        host.copy_(dev_iq)
        cur = torch.cuda.current_stream(dev)
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(cur)
            dev_iq.copy_(host, non_blocking=True)
            e1.record(cur)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / 1e3)
        t = min(ts)
        nbytes = host.numel() * host.element_size()
        h2d = {"gbs": nbytes / t / 1e9, "samples_per_s": nbytes / 8 / t, "captures": nc,
               "ms": t * 1e3, "bytes": nbytes,
               "note": "pinned host -> HBM copy of %d fc32 captures (best of 3), PCIe-inclusive "
                       "ingest rate; the headline starts with the captures resident" % nc}
        del host

    value = samples_total / elapsed
    ms_step = elapsed / args.steps * 1e3
    bytes_alg = scanned_total * in_bytes + args.steps * n_dec_all * N * m_occ * 9
    wl = WORKLOADS[args.workload]
    line = {
        "metric": "complex IQ samples/s through 4x4 MMSE detect; EVM-dB delta vs CPU ref",
        "value": value,
        "unit": "complex samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "strong" if c5 else "weak",
        "vs_baseline": None,
        "dtype": "fp32 (complex64; fp64 weight solve)",
        "data": "synthetic (GPU tx_worker-layout frames, flat Rayleigh %dx%d, AWGN %.0f dB)"
                % (N, N, args.snr),
        "config": {"workload": wl["desc"], "M": M, "cp": cp, "streams": N, "access_codes": nac,
                   "pid": pid, "qam": args.qam, "detector": args.detector,
                   "captures_per_step_per_gpu": F, "frames_per_capture": K if c5 else 1,
                   "ingest": ("rank-0 sc16 scatter over RCCL P2P" if timed_scatter
                              else "resident in HBM"),
                   "cfo": args.cfo,
                   "out_layout": ("symbol-major [frame][symbol][stream][M_occ]" if sym_major
                                  else "stream-major [frame][stream][symbol][M_occ]"),
                   "sample_format": ("sc16 wire samples read in place (4 B/sample)" if sc16
                                     else "fc32 complex64 (8 B/sample)"),
                   "parallelism": ("%d streams over %d GPU(s)" % (args.frames, world) if c5 else
                                   "frames sharded across %d GPU(s), no collective" % world)},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": kname, "bytes_per_launch": dec_bytes,
                     "symbols_per_launch": n_dec, "bytes_per_symbol": per_sym,
                     "avg_launch_ms": dec_avg_s * 1e3},
        "decode_pattern_ms": pattern["ms"] if pattern else None,
        "decode_vs_pattern": pattern["decode_vs_pattern"] if pattern else None,
        "decode_pattern": pattern,
        "pipeline": pipe_info,
        "cpu_baseline": cpu,
        "evm_db_delta_vs_cpu": evm_delta,
        "scan_rate_all_captures": scanned_total / elapsed,
        "pipeline_hbm_gbs": bytes_alg / elapsed / 1e9,
        "stages_ms_per_step": {k: v[0] / n_stage for k, v in stages.items()},
        "frames_ok": int(ok_all),
        "frames": int(args.frames * args.frames_per_stream) if c5 else int(F * world),
        "rescan_slots": rescans,
        "sc_exact_recomputes_per_step": n_exact / max(args.steps, 1),
        "evm_db": 10 * np.log10(evm_num / evm_den) if evm_den > 0 else None,
        "symbol_errors_last_step": int(errors),
        "rank0_scatter": scatter_info,
        "sc16_resident": sc16_info,
        # FFT + detect + demap + EVM given W (the decode stage alone), samples of the decoded
        # symbols (N antennas x (M + cp)) per second of the decode kernels' event time
        "decode_stage": {"value": (n_dec * N * (M + cp) / dec_avg_s) if dec_avg_s > 0 else None,
                         "unit": "complex samples/s", "ms_per_step": dec_avg_s * 1e3,
                         "symbols_per_step": n_dec},
        "h2d": h2d,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

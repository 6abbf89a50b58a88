"""Multi-rank logic on CPU (gloo, world size 2): frame sharding and the counter reduction that
bench.py --gpus N uses. The per-rank compute here is the CPU oracle on the
committed fixtures, standing in for each rank's GPU so the sharded totals can be checked
against a single-process run."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rub_mimo_amd.shard import STAT_KEYS, frame_ids, reduce_stats

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
FIXTURES = ["m64_2x2_zf2", "m64_1x1_zf", "m128_4x4_mmse", "m64_2x2_siso"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _frame_stats(name):
    """Oracle receive of one fixture capture -> the counters a rank reports."""
    from oracle import ref
    g = dict(np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False))
    N, pid = int(g["N"]), int(g["pid"])
    fs = ref.FrameSyncRef(int(g["M"]), int(g["cp"]), N, int(g["nac"]), pid_max=pid,
                          detector=int(g["detector"]),
                          keep_identity_bias=bool(g["keep_identity_bias"]), p=g["p"],
                          siso_tx=int(g["siso_tx"]), siso_rx=int(g["siso_rx"]))
    fs.execute(g["rx"])
    sym = fs.symbols()[:pid]                     # [n_sym, N, M_occ]
    ok = 1 if len(sym) else 0
    num = den = err = 0.0
    if ok:
        _, en, ed, er = ref.demap_evm(sym, int(g["qam"]), g["tx_idx"][:, :len(sym)])
        num, den, err = float(np.sum(en)), float(np.sum(ed)), float(np.sum(er))
    return dict(samples=float(g["rx"].size), frames_ok=ok, symbols=float(len(sym)), evm_num=num,
                evm_den=den, errors=err)


def _worker(rank, world, port, frames_per_rank, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        f0, nf = frame_ids(rank, frames_per_rank)
        mine = [FIXTURES[i % len(FIXTURES)] for i in range(f0, f0 + nf)]
        acc = {k: 0.0 for k in STAT_KEYS}
        for name in mine:
            for k, v in _frame_stats(name).items():
                acc[k] += v
        elapsed = 0.25 * (rank + 1)
        tot, emax = reduce_stats(acc, elapsed, dist)
        q.put((rank, list(range(f0, f0 + nf)), tot, emax))
    finally:
        dist.destroy_process_group()


def _pack(names):
    """Frames of `names` as one float32 row each (rx viewed as float32, zero-padded)."""
    rows = [np.ascontiguousarray(np.load(os.path.join(GOLD, n + ".npz"))["rx"]).view(np.float32)
            .ravel() for n in names]
    return rows


def _scatter_worker(rank, world, port, frames_per_rank, width, steps, q):
    """Rank 0 holds every rank's captures ([world][F][width] float32, the fixtures' rx rows);
    ScatterPipeline delivers each rank its slice for `steps` double-buffered steps; each rank
    checks the bytes, runs the oracle on the frames it received and reduces the counters."""
    from rub_mimo_amd.shard import ScatterPipeline
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        names = [FIXTURES[i % len(FIXTURES)] for i in range(world * frames_per_rank)]
        rows = _pack(names)
        src = None
        if rank == 0:
            src = torch.zeros((world, frames_per_rank, width), dtype=torch.float32)
            for i, r in enumerate(rows):
                src[i // frames_per_rank, i % frames_per_rank, :len(r)] = torch.from_numpy(r)
        pipe = ScatterPipeline(dist, src, (frames_per_rank, width), torch.float32, "cpu",
                               rank, world)
        pipe.start()
        f0, nf = frame_ids(rank, frames_per_rank)
        exact = True
        acc = {k: 0.0 for k in STAT_KEYS}
        for s in range(steps):
            got = pipe.next()
            for j in range(nf):
                want = rows[f0 + j]
                exact &= bool(np.array_equal(got[j, :len(want)].numpy(), want))
                exact &= bool(torch.all(got[j, len(want):] == 0))
            if s == 0:      # receive what arrived (the oracle stands in for the rank's GPU)
                for j in range(nf):
                    name = names[f0 + j]
                    g = np.load(os.path.join(GOLD, name + ".npz"))
                    rx = got[j, :len(rows[f0 + j])].numpy().view(np.complex64).reshape(
                        g["rx"].shape)
                    assert np.array_equal(rx, g["rx"])
                    for k, v in _frame_stats(name).items():
                        acc[k] += v
        pipe.drain()
        tot, emax = reduce_stats(acc, 0.1 * (rank + 1), dist)
        q.put((rank, exact, tot, emax))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_rank0_scatter_delivers_bytes_and_counters(world):
    """bench.py --ingest scatter's data movement on CPU (gloo): byte-exact delivery of every
    rank's slice over double-buffered steps, and the reduced counters equal one process."""
    per, steps = 2, 3
    width = max(len(r) for r in _pack(FIXTURES)) + 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scatter_worker, args=(r, world, port, per, width, steps, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single = {k: 0.0 for k in STAT_KEYS}
    for i in range(world * per):
        for k, v in _frame_stats(FIXTURES[i % len(FIXTURES)]).items():
            single[k] += v
    for rank, exact, tot, emax in out:
        assert exact, rank
        assert emax == pytest.approx(0.1 * world)
        for k in STAT_KEYS:
            assert tot[k] == pytest.approx(single[k], rel=1e-12)


def test_split_streams_partition():
    from rub_mimo_amd.shard import split_streams
    for world in (1, 2, 3, 4, 8):
        spans = [split_streams(8, world, r) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == 8
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
        assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1
    with pytest.raises(ValueError):
        split_streams(8, 2, 2)


def test_frame_ids_partition():
    seen = []
    for r in range(4):
        f0, n = frame_ids(r, 3)
        seen += list(range(f0, f0 + n))
    assert seen == list(range(12))
    with pytest.raises(ValueError):
        frame_ids(0, 0)


def test_reduce_stats_single_process_is_identity():
    s = dict(samples=10, frames_ok=1, symbols=5, evm_num=2.0, evm_den=4.0, errors=3)
    tot, e = reduce_stats(s, 1.5, None)
    assert tot == {k: float(v) for k, v in s.items()} and e == 1.5


def test_two_rank_sharding_matches_single_process():
    world, per = 2, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, per, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    # disjoint frame ownership covering the job
    assert out[0][1] + out[1][1] == list(range(world * per))
    # every rank sees the same totals; they equal one process doing all frames
    single = {k: 0.0 for k in STAT_KEYS}
    for i in range(world * per):
        for k, v in _frame_stats(FIXTURES[i % len(FIXTURES)]).items():
            single[k] += v
    assert single["frames_ok"] >= 2 and single["evm_den"] > 0   # real work was reduced
    for _, _, tot, emax in out:
        assert emax == pytest.approx(0.25 * world)
        for k in STAT_KEYS:
            assert tot[k] == pytest.approx(single[k], rel=1e-12)

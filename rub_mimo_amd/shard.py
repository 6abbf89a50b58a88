"""rub_mimo_amd/shard.py -- frames across ranks.

Captured frames are independent: G, W and the sync state are per frame, so the receive path
shards with no exchange on the data path. Rank r of W owns frames [r*F, (r+1)*F) of the job
(its synthetic frame ids, or its own capture stream).

Two ways a rank's captures reach its GPU:
- resident: every rank reads (here: synthesises) its own captures. No data-path collective;
  this is what bench.py's headline measures (weak scaling).
- rank-0 scatter: rank 0 holds the radio's captures for the whole node at the sc16 wire format
  (UHD, mimo/config.h:52) and sends every rank its slice over RCCL point-to-point (xGMI; one
  direct link per peer, so not ring-bound). This replaces the reference's single-process
  capture handoff (mimo/main.cc:905-922: the rx worker fills /tmp/rx<ch>.dat, framesync reads
  it back). `scatter_from_rank0` is the grouped send/recv; `ScatterPipeline` double-buffers it
  against the receive pipeline.

The one collective of the resident mode is the reduction of a few counters after the timed
region: the sums of samples, frames received, decoded symbols, EVM numerator/denominator and
symbol errors, and the max of the per-rank elapsed time.
"""

STAT_KEYS = ("samples", "frames_ok", "symbols", "evm_num", "evm_den", "errors")


def frame_ids(rank, frames_per_rank):
    """First frame id and count of this rank's frames."""
    if rank < 0 or frames_per_rank <= 0:
        raise ValueError("rank must be >= 0 and frames_per_rank > 0")
    return rank * frames_per_rank, frames_per_rank


def split_streams(n_streams, world, rank):
    """Contiguous share [s0, s1) of n_streams independent streams for `rank` (C5: 8 streams
    over 1/2/4/8 GPUs). Every rank gets at least one stream only if n_streams >= world."""
    if world <= 0 or not 0 <= rank < world or n_streams < 0:
        raise ValueError("bad world/rank/n_streams")
    base, extra = divmod(n_streams, world)
    s0 = rank * base + min(rank, extra)
    return s0, s0 + base + (1 if rank < extra else 0)


def reduce_stats(stats, elapsed, dist=None, device="cpu", force=False):
    """Sum the counters and take the max elapsed over ranks; identity when dist is None or the
    group has one rank (force: run the collectives at world size 1 too -- the device test of
    the RCCL path on one GPU). Returns (totals dict, elapsed_max)."""
    if dist is None or not dist.is_available() or not dist.is_initialized() or \
            (dist.get_world_size() == 1 and not force):
        return {k: float(stats[k]) for k in STAT_KEYS}, float(elapsed)
    import torch
    t = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    c = torch.tensor([float(stats[k]) for k in STAT_KEYS], dtype=torch.float64, device=device)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return dict(zip(STAT_KEYS, (float(v) for v in c.tolist()))), float(t.item())


def wire_bytes(t):
    """The tensor as the bytes RCCL moves: NCCL/RCCL point-to-point has no int16 (torch's NCCL
    process group refuses Short tensors), so sc16 wire buffers travel as uint8 views of the same
    memory; other dtypes pass unchanged."""
    import torch
    return t.view(torch.uint8) if t.dtype == torch.int16 else t


def scatter_from_rank0(dist, src, dst, rank, world):
    """Grouped point-to-point scatter: rank 0 sends src[r] to rank r (r >= 1); rank r >= 1
    receives into dst. src ([world, ...], rank 0 only) and dst are contiguous tensors of one
    dtype; dst has src[r]'s shape. Rank 0's own slice is not copied (it reads src[0] in place).
    Returns the list of requests (empty at world size 1); on NCCL/RCCL the transfers run on the
    communicator's stream, ordered after the work already queued on the current stream, and
    req.wait() makes the current stream wait for them."""
    if world <= 1:
        return []
    ops = []
    if rank == 0:
        if src is None or src.shape[0] != world:
            raise ValueError("rank 0 needs src with a leading dimension of world size")
        for r in range(1, world):
            ops.append(dist.P2POp(dist.isend, wire_bytes(src[r]), r))
    else:
        if dst is None:
            raise ValueError("ranks >= 1 need a dst tensor")
        ops.append(dist.P2POp(dist.irecv, wire_bytes(dst), 0))
    return dist.batch_isend_irecv(ops)


class ScatterPipeline:
    """Double-buffered rank-0 scatter of sc16 wire captures (the ingest side of bench.py
    --ingest scatter): batch i+1 is in flight on the communicator while batch i is widened
    (mimo_ingest_sc16) and received. `src` is rank 0's [world][...] int16 wire buffer; every
    rank owns two receive slots shaped like src[0].

        pipe.start()              # scatter batch 0 into slot 0
        for i in steps:
            wire = pipe.next()    # wait for batch i; scatter batch i+1 into the other slot
            widen(wire) ; receive(...)

    The scatter of batch i+1 is enqueued after the widening of batch i-1 (the previous user of
    its slot) on the current stream, so the slot is never overwritten while being read."""

    def __init__(self, dist, src, slot_shape, dtype, device, rank, world):
        import torch
        self.dist, self.src, self.rank, self.world = dist, src, rank, world
        self.slots = None
        if rank != 0 and world > 1:
            self.slots = [torch.empty(slot_shape, dtype=dtype, device=device) for _ in range(2)]
        self.i = 0
        self.reqs = None

    def _slot(self, i):
        return self.src[0] if self.rank == 0 or self.world <= 1 else self.slots[i & 1]

    def start(self):
        self.i = 0
        self.reqs = scatter_from_rank0(self.dist, self.src, None if self.slots is None
                                       else self.slots[0], self.rank, self.world)

    def next(self):
        for r in self.reqs or []:
            r.wait()
        cur = self._slot(self.i)
        self.i += 1
        self.reqs = scatter_from_rank0(self.dist, self.src, None if self.slots is None
                                       else self.slots[self.i & 1], self.rank, self.world)
        return cur

    def drain(self):
        for r in self.reqs or []:
            r.wait()
        self.reqs = None

"""rub_mimo_amd/shard.py -- frames across ranks.

Captured frames are independent: G, W and the sync state are per frame, so the receive path
shards with no exchange on the data path. Rank r of W owns frames [r*F, (r+1)*F) of the job
(its synthetic frame ids, or its own capture stream). The one collective is the reduction
of a few counters after the timed region: the sums of samples, frames received, decoded
symbols, EVM numerator/denominator and symbol errors, and the max of the per-rank elapsed
time.
"""

STAT_KEYS = ("samples", "frames_ok", "symbols", "evm_num", "evm_den", "errors")


def frame_ids(rank, frames_per_rank):
    """First frame id and count of this rank's frames."""
    if rank < 0 or frames_per_rank <= 0:
        raise ValueError("rank must be >= 0 and frames_per_rank > 0")
    return rank * frames_per_rank, frames_per_rank


def reduce_stats(stats, elapsed, dist=None, device="cpu"):
    """Sum the counters and take the max elapsed over ranks; identity when dist is None or the
    group has one rank. Returns (totals dict, elapsed_max)."""
    if dist is None or not dist.is_available() or not dist.is_initialized() or \
            dist.get_world_size() == 1:
        return {k: float(stats[k]) for k in STAT_KEYS}, float(elapsed)
    import torch
    t = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    c = torch.tensor([float(stats[k]) for k in STAT_KEYS], dtype=torch.float64, device=device)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return dict(zip(STAT_KEYS, (float(v) for v in c.tolist()))), float(t.item())

"""The multi-GPU path's collectives on the device: a fresh child process -- the
process group initialised with the "nccl" backend (RCCL on ROCm) before any GPU call, as
bench.py's ranks do -- runs shard.reduce_stats through device all_reduces at world size 1
(force=True: the early return that every one-GPU run takes is bypassed), and a grouped
point-to-point exchange of an sc16 wire buffer with itself. Only gloo ever ran these
collectives before (tests/test_dist.py at world size 2 and 3, on the CPU); this proves RCCL
loads and runs on MI355X. (Its first run found that torch's NCCL process group refuses int16
tensors, which the rank-0 scatter sent: sc16 buffers now travel as uint8 views.)"""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

CHILD = r'''
import os, sys
sys.path.insert(0, %(root)r)
import torch
import torch.distributed as dist
dist.init_process_group("nccl", rank=0, world_size=1)      # before any GPU call
assert dist.get_backend() == "nccl"
torch.cuda.set_device(0)
from rub_mimo_amd.shard import STAT_KEYS, reduce_stats
stats = dict(samples=1.5e9, frames_ok=51, symbols=51000, evm_num=2.25, evm_den=900.0, errors=7)
tot, el = reduce_stats(stats, 0.125, dist, device="cuda:0", force=True)
assert tot == {k: float(stats[k]) for k in STAT_KEYS}, tot
assert el == 0.125, el
# a device all_reduce of a larger tensor, SUM and MAX
x = torch.arange(1 << 20, dtype=torch.float32, device="cuda:0")
y = x.clone()
dist.all_reduce(y, op=dist.ReduceOp.SUM)
assert torch.equal(x, y)
dist.all_reduce(y, op=dist.ReduceOp.MAX)
assert torch.equal(x, y)
# rank-0 scatter's primitive: a grouped send/recv of an sc16 wire buffer (to itself at world
# size 1), int16 moved as its bytes (shard.wire_bytes: RCCL has no int16)
from rub_mimo_amd.shard import wire_bytes
src = (torch.arange(4096, dtype=torch.int32, device="cuda:0") - 2048).to(torch.int16)
dst = torch.zeros_like(src)
reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend, wire_bytes(src), 0),
                               dist.P2POp(dist.irecv, wire_bytes(dst), 0)])
for r in reqs:
    r.wait()
torch.cuda.synchronize()
assert torch.equal(src, dst)
dist.destroy_process_group()
print("rccl ok")
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_reduce_stats_on_device():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, "-c", CHILD % {"root": root}], env=env, cwd=root,
                         timeout=150, capture_output=True, text=True)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    assert "rccl ok" in out.stdout

"""tools/bench_ingest.py -- sc16 -> complex64 ingest (mimo_ingest_sc16) throughput at the C3x8
capture size: 8 captures x 4 antennas x 2,563,688 samples, 12 B of HBM per sample."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from rub_mimo_amd.receiver import ingest_sc16

rows, n = 32, 2563688
stride = (n + 63) // 64 * 64
src = torch.randint(-32768, 32767, (rows * stride * 2,), dtype=torch.int16, device="cuda")
dst = torch.empty(rows * stride * 2, dtype=torch.float32, device="cuda")
st = torch.cuda.current_stream()
for _ in range(3):
    ingest_sc16(src, stride, dst, stride, rows, n, stream=st.cuda_stream)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
K = 50
e0.record(st)
for _ in range(K):
    ingest_sc16(src, stride, dst, stride, rows, n, stream=st.cuda_stream)
e1.record(st)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / K
gbs = rows * n * 12 / ms / 1e6
print(json.dumps({"kernel": "sc16_to_fc32_vec_kernel", "ms": ms, "samples": rows * n,
                  "achieved_GBps": gbs, "frac_of_8TBps": gbs / 8000}))

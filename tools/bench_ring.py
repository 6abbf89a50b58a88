"""tools/bench_ring.py -- host-to-HBM capture ingest through the pinned-host ring
(mimo_ring_*), PCIe-inclusive: a producer thread copies sc16 wire samples (as a
recv loop would hand them over) into pinned chunks and commits them; the uploads run on the
ring's stream. Reported next to a pageable fc32 upload of the same captures (the reference's
host format, 8 B/sample, mimo/config.h:51). Never the bench's `value`: that is measured with
the captures resident in HBM.

usage: python tools/bench_ring.py [--ant 4] [--samples 2563688] [--captures 8] [--chunk 262144]
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ant", type=int, default=4)
    ap.add_argument("--samples", type=int, default=2563688)   # one C3 capture per antenna
    ap.add_argument("--captures", type=int, default=8)
    ap.add_argument("--chunk", type=int, default=1 << 18)
    ap.add_argument("--chunks", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("-o", "--out", default=None)
    a = ap.parse_args()
    import torch
    from rub_mimo_amd.ring import CaptureRing
    N, L, F = a.ant, a.samples, a.captures
    rng = np.random.default_rng(1)
    host = rng.integers(-2000, 2000, (F, N, L, 2), dtype=np.int16)
    cap = torch.empty((F, N, L, 2), dtype=torch.int16, device="cuda")
    ring = CaptureRing(N, a.chunk, a.chunks)
    stream = torch.cuda.current_stream().cuda_stream

    def produce(fill=True):
        for f in range(F):
            ring.bind(cap[f], L, L)
            pos = 0
            while pos < L:
                rows = ring.acquire()
                n = min(L - pos, a.chunk)
                if fill:
                    for r in range(N):
                        np.copyto(rows[r][:n], host[f, r, pos:pos + n])
                ring.commit(n)
                pos += n

    best = None
    for _ in range(a.reps + 1):                # the first pass warms the pinned pages
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        th = threading.Thread(target=produce)
        th.start()
        th.join()
        ring.publish(stream)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    ok = bool(torch.equal(cap.cpu(), torch.from_numpy(host)))
    # uploads alone (the recv loop writes the pinned chunks itself, so no host copy): the
    # ring's PCIe-bound rate
    tu = None
    for _ in range(a.reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        produce(False)
        ring.publish(stream)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        tu = dt if tu is None else min(tu, dt)
    ring.close()
    # the reference's host format: pageable complex64, one synchronous copy per capture
    fc = (host[..., 0] + 1j * host[..., 1]).astype(np.complex64) / np.float32(32767.0)
    dcap = torch.empty((F, N, L), dtype=torch.complex64, device="cuda")
    tf = None
    for _ in range(a.reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for f in range(F):
            dcap[f].copy_(torch.from_numpy(fc[f]))
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        tf = dt if tf is None else min(tf, dt)
    n = F * N * L
    res = {"captures": F, "antennas": N, "samples_per_antenna": L, "chunk": a.chunk,
           "chunks": a.chunks, "bytes_equal": ok,
           "ring_sc16": {"s": best, "samples_per_s": n / best, "GBps": n * 4 / best / 1e9,
                         "note": "producer thread copies each chunk from a host array (numpy, "
                                 "one core) before committing"},
           "ring_sc16_upload_only": {"s": tu, "samples_per_s": n / tu, "GBps": n * 4 / tu / 1e9},
           "pageable_fc32": {"s": tf, "samples_per_s": n / tf, "GBps": n * 8 / tf / 1e9}}
    print(json.dumps(res))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()

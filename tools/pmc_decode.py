"""tools/pmc_decode.py -- HBM bytes per decode launch from two rocprofv3 PMC passes.

usage: python tools/pmc_decode.py FETCH_counter_collection.csv WRITE_counter_collection.csv \
           --M 2048 --streams 4 --frames 8 --pid 1000 --ref-mode 1 -o profiles/decode_pmc.json

MI355X_MICROARCH.md (HBM section): FETCH_SIZE reports half the bytes of a wide coalesced
16-byte-per-lane streaming read on gfx950 (doubled here); WRITE_SIZE is exact for 16-byte
streaming stores. Both are in KiB per dispatch. Counters come from separate passes (FETCH_SIZE
and WRITE_SIZE cannot share one on gfx950), each with --kernel-trace only.
"""
import argparse
import csv
import json
import statistics


def per_dispatch(path, counter, pattern):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and pattern in r["Kernel_Name"]]
    if not vals:
        raise SystemExit(f"no {counter} rows for {pattern} in {path}")
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--kernel", default="decode_persistent_kernel")
    ap.add_argument("--M", type=int, required=True)
    ap.add_argument("--streams", type=int, required=True)
    ap.add_argument("--frames", type=int, required=True)
    ap.add_argument("--pid", type=int, required=True)
    ap.add_argument("--ref-mode", type=int, default=1)
    ap.add_argument("--sample-format", default="fc32", choices=["fc32", "sc16"])
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    # a stage of several kernels ("a|b"): the sum of each kernel's median per dispatch
    ks = a.kernel.split("|")
    f = [per_dispatch(a.fetch_csv, "FETCH_SIZE", k) for k in ks]
    w = [per_dispatch(a.write_csv, "WRITE_SIZE", k) for k in ks]
    fetch_b = 2.0 * sum(statistics.median(x) for x in f) * 1024.0
    write_b = sum(statistics.median(x) for x in w) * 1024.0
    out = {
        "config": {"M": a.M, "streams": a.streams, "frames": a.frames, "pid": a.pid,
                   "ref_mode": a.ref_mode, "sample_format": a.sample_format},
        "kernel": a.kernel,
        "dispatches": {"fetch": [len(x) for x in f], "write": [len(x) for x in w]},
        "fetch_size_kib_median": [statistics.median(x) for x in f],
        "write_size_kib_median": [statistics.median(x) for x in w],
        "decode_hbm_read_bytes_per_launch": fetch_b,
        "decode_hbm_write_bytes_per_launch": write_b,
        "decode_hbm_bytes_per_launch": fetch_b + write_b,
        "correction": "FETCH_SIZE x2 (gfx950 16 B/lane streaming reads), WRITE_SIZE x1, KiB",
    }
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

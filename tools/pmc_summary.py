"""tools/pmc_summary.py -- per-kernel bound analysis from rocprofv3 PMC passes + kernel stats.

usage: python tools/pmc_summary.py --tag r02_c3 --stats gpurun_out/stats_r02_c3 -o profiles/r02/pmc_c3.json

Reads gpurun_out/pmc_<tag>_{sqa,sqb,fetch,write}/run_counter_collection.csv (whichever exist)
and the kernel-trace stats csv, and derives per kernel (median over dispatches):
- duration (kernel stats average), waves, VALU instructions per wave;
- VALU busy fraction = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES x waves-per-SIMD occupancy proxy is
  not used; instead issue share = SQ_ACTIVE_INST_VALU / SQ_BUSY_CYCLES per SIMD (both quad-cycle
  units on CDNA4, MI355X_MICROARCH.md PMC table; SQ_BUSY_CYCLES is per SE, so it is scaled by
  the 4 SIMDs x CUs-per-SE);
- wait split: SQ_WAIT_ANY (parked on s_waitcnt/barrier), SQ_WAIT_INST_ANY (issue stall),
  SQ_ACTIVE_INST_ANY, each as a fraction of SQ_WAVE_CYCLES (they sum to ~1);
- LDS bank-conflict share = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE;
- HBM bytes: FETCH_SIZE x 2 (gfx950 16 B/lane streaming reads) + WRITE_SIZE, KiB -> bytes, and
  the GB/s they imply over the kernel's average duration.
"""
import argparse
import collections
import csv
import glob
import json
import os
import statistics


def load_counters(paths):
    rows = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            rows[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return rows


def short(name):
    n = name.replace("void ", "").split("(")[0]
    return n.replace("mimo::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--stats", required=True)
    ap.add_argument("--root", default="gpurun_out")
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    paths = glob.glob(os.path.join(a.root, "pmc_%s_*" % a.tag, "*counter_collection.csv"))
    cnt = load_counters(paths)
    dur = {}
    for r in csv.DictReader(open(os.path.join(a.stats, "run_kernel_stats.csv"))):
        dur[r["Name"]] = float(r["AverageNs"])
    out = {}
    for k, c in cnt.items():
        med = {n: statistics.median(v) for n, v in c.items()}
        d = {"kernel": short(k), "dispatches": max(len(v) for v in c.values())}
        if k in dur:
            d["avg_us"] = dur[k] / 1e3
        waves = med.get("SQ_WAVES")
        if waves:
            d["waves"] = waves
            if "SQ_INSTS_VALU" in med:
                d["valu_insts_per_wave"] = med["SQ_INSTS_VALU"] / waves
            if "SQ_INSTS_LDS" in med:
                d["lds_insts_per_wave"] = med["SQ_INSTS_LDS"] / waves
        wc = med.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                      "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
                if n in med:
                    d[n.lower().replace("sq_", "") + "_frac"] = med[n] / wc
        if "SQ_LDS_BANK_CONFLICT" in med and med.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_bank_conflict_frac"] = med["SQ_LDS_BANK_CONFLICT"] / med["SQ_LDS_IDX_ACTIVE"]
        if "SQ_BUSY_CYCLES" in med and "SQ_ACTIVE_INST_VALU" in med and "avg_us" in d:
            # VALU issue rate over the kernel: quad-cycles with a VALU issued, summed over all
            # waves, against the chip's SIMD quad-cycles in the kernel's duration (256 CUs x 4
            # SIMDs, 2.4 GHz peak engine clock)
            simd_quads = d["avg_us"] * 1e-6 * 2.4e9 / 4 * 256 * 4
            d["valu_issue_share_of_chip"] = med["SQ_ACTIVE_INST_VALU"] / simd_quads
        fb = med.get("FETCH_SIZE")
        wb = med.get("WRITE_SIZE")
        if fb is not None:
            d["hbm_read_bytes"] = 2.0 * fb * 1024.0
        if wb is not None:
            d["hbm_write_bytes"] = wb * 1024.0
        if fb is not None and wb is not None and "avg_us" in d:
            d["hbm_gbs"] = (d["hbm_read_bytes"] + d["hbm_write_bytes"]) / (d["avg_us"] * 1e3)
        if "TCC_HIT_sum" in med:
            tot = med["TCC_HIT_sum"] + med.get("TCC_MISS_sum", 0.0)
            d["l2_hit_frac"] = med["TCC_HIT_sum"] / tot if tot else None
        out[short(k)] = d
    json.dump({"tag": a.tag, "sources": sorted(paths), "kernels": out,
               "notes": "FETCH_SIZE doubled (gfx950), WRITE_SIZE as is; wave-cycle fractions are "
                        "of SQ_WAVE_CYCLES (quad-cycles)"}, open(a.out, "w"), indent=1)
    for k, d in sorted(out.items(), key=lambda kv: -kv[1].get("avg_us", 0)):
        print("%-40s %s" % (k[:40], " ".join("%s=%.3g" % (n, v) for n, v in d.items()
                                             if isinstance(v, float) and n != "avg_us_"))[:400])


if __name__ == "__main__":
    main()

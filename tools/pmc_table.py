"""tools/pmc_table.py DIR... -- median per-dispatch counter values per kernel from rocprofv3 csv."""
import collections
import csv
import glob
import statistics
import sys

for d in sys.argv[1:]:
    rows = collections.defaultdict(list)
    for p in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            rows[(r["Kernel_Name"][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
    print("==", d)
    for (k, c), v in sorted(rows.items()):
        print("  %-60s %-24s n=%3d median=%.4g" % (k, c, len(v), statistics.median(v)))

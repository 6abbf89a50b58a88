#!/bin/bash
# rocprof kernel stats of a short bench per library build (LIBS, relative to rub_mimo_amd/),
# printing the kernels matching KPAT -- timing ablations and A/B builds
set -o pipefail
R=$PWD
O=$R/gpurun_out/${TAG:-kstats}
mkdir -p $O
export TMPDIR=/tmp
for L in $LIBS; do
  ( cd /tmp && RMIMO_LIB=$R/rub_mimo_amd/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$L -o run -- python3 $R/bench.py --workload ${WL:-c3} --steps 5 --cpu-baseline 0 --sc16-steps 0 --h2d 0 $BENCH_ARGS > $O/prof_$L.log 2>&1 ) || { echo "rocprof $L failed"; tail -5 $O/prof_$L.log; exit 1; }
  f=$(find $O/prof_$L -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$L" "${KPAT:-decode}" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[3], r['Name']):
        print(sys.argv[2], r['Name'][:44], r['Calls'], '%.1f us' % (float(r['AverageNs']) / 1e3))
PY
done

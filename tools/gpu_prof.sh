#!/bin/bash
# rocprofv3 kernel stats of a short C3 bench (HEAD build) and the S&C exact-kernel timeline of
# the PROFILE=1 build (librub_mimo_amd_prof.so, RMIMO_SC_PROF=1) -- diagnostics only
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${TAG:-prof}
mkdir -p $O
export TMPDIR=/tmp
W=${WL:-c3}
( cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$W -o run -- python3 $R/bench.py --workload $W --steps 10 --cpu-baseline 0 --sc16-steps 0 --h2d 0 $BENCH_ARGS > $O/prof_$W.log 2>&1 ) || { echo "rocprof failed"; tail -20 $O/prof_$W.log; exit 1; }
f=$(find $O/prof_$W -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:14]:
    print("%-70s %6s %10.1f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
if [ -n "$SCPROF" ]; then
  RMIMO_LIB=$R/rub_mimo_amd/librub_mimo_amd_prof.so RMIMO_SC_PROF=1 RMIMO_SC_COUNT=1 timeout -k 10 200 python3 tools/diag_sc.py --frames ${FRAMES:-64} --reps 2 > $O/scprof.log 2>&1 || { echo "scprof failed"; tail -20 $O/scprof.log; exit 1; }
  grep -E "exact_prof|sc_count|stages_ms" $O/scprof.log | tail -8
fi

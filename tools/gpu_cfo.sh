#!/bin/bash
# CFO tests, the --cfo bench line (with rocprof kernel stats) and the S&C exact-kernel timeline
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${TAG:-cfo}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "cfo" > $O/cfo_tests.log 2>&1 || { echo "cfo tests failed"; tail -n 30 $O/cfo_tests.log; exit 1; }
tail -n 1 $O/cfo_tests.log
for v in 0 0.3; do
  timeout -k 10 200 python bench.py --cfo $v --cpu-baseline 0 --sc16-steps 0 --h2d 0 > $O/bench_cfo_$v.json 2> $O/bench_cfo_$v.err || { echo "bench failed"; tail -20 $O/bench_cfo_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/bench_cfo_$v.json'))
print('cfo $v', 'value %.4g'%d['value'], 'ms %.4f'%d['ms_per_step'], 'ok %d'%d['frames_ok'], 'evm %.3f'%d['evm_db'], {k:round(x,4) for k,x in d['stages_ms_per_step'].items()})"
done
( cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfo -o run -- python3 $R/bench.py --cfo 0.3 --steps 10 --cpu-baseline 0 --sc16-steps 0 --h2d 0 > $O/prof_cfo.log 2>&1 ) || { echo "rocprof failed"; tail -20 $O/prof_cfo.log; exit 1; }
f=$(find $O/prof_cfo -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:16]:
    print("%-64s %5s %10.1f us" % (r["Name"][:64], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
RMIMO_SC_PROF=1 RMIMO_SC_COUNT=1 timeout -k 10 200 python3 tools/diag_sc.py --frames 64 --reps 2 > $O/scprof.log 2>&1 || { echo "scprof failed"; tail -20 $O/scprof.log; exit 1; }
grep -E "exact_prof|sc_count|stages_ms" $O/scprof.log | tail -12

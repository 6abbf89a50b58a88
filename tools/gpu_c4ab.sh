set -o pipefail
O=gpurun_out/${TAG:-c4ab}; mkdir -p $O
TAG=${TAG:-c4ab} LIB_A=librub_mimo_amd_base.so LIB_B=librub_mimo_amd_persist.so WL=c4 bash tools/gpu_libab.sh || exit 1
timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "split" > $O/t.log 2>&1; echo "split tests rc=$?"; tail -n 1 $O/t.log
export TMPDIR=/tmp
R=$PWD
for L in librub_mimo_amd_base.so librub_mimo_amd_persist.so; do
  ( cd /tmp && RMIMO_LIB=$R/rub_mimo_amd/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$L -o run -- python3 $R/bench.py --workload c4 --steps 5 --cpu-baseline 0 --sc16-steps 0 --h2d 0 > $R/$O/prof_$L.log 2>&1 ) || { echo "rocprof failed"; exit 1; }
  f=$(find $O/prof_$L -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$L" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'spectra' in r['Name'] or 'apply_split' in r['Name']:
        print(sys.argv[2], r['Name'][:40], r['Calls'], '%.1f us' % (float(r['AverageNs'])/1e3))
PY
done

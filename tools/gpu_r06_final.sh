#!/bin/bash
# Round-6 evidence in one GPU session: every gpu test, smoke, the bench lines (C3 default with
# the CPU baseline and the decode-pattern leg, C2/C4/C5 with theirs), PMC FETCH/WRITE passes
# over the decode, kernel-trace stats (C3, C4), the CFO pair.
#   tools/gpu_r06_final.sh TAG [all|bench|prof]
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
tag=${1:-r06}
part=${2:-all}
O=$R/gpurun_out/$tag
mkdir -p $O
cd $R
if [ $part != prof ]; then
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { echo "bench c3 failed"; tail -20 $O/bench_c3.err; exit 1; }
for w in c2 c4 c5; do
  timeout -k 10 400 python bench.py --workload $w --cpu-baseline 1 > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail -20 $O/bench_$w.err; exit 1; }
done
for w in c3 c2 c4 c5; do
  python3 -c "
import json; d=json.load(open('$O/bench_$w.json')); st=d['stages_ms_per_step']; c=d['cpu_baseline'] or {}
print('$w', 'ms %.4f'%d['ms_per_step'], 'value %.4g'%d['value'], 'frac %.3f'%d['roofline']['frac'], 'pattern', d.get('decode_vs_pattern'), 'cpu', c.get('value'), ' '.join('%s %.4f'%(k,v) for k,v in st.items()))"
done
fi
[ $part = bench ] && exit 0
export PMC_KERNEL="decode|spectra|apply_split"
for w in c3 c4; do
  "$R/tools/pmc_run.sh" "${tag}_${w}_fetch" "FETCH_SIZE" --workload $w || exit 1
  "$R/tools/pmc_run.sh" "${tag}_${w}_write" "WRITE_SIZE" --workload $w || exit 1
done
cd /tmp && export TMPDIR=/tmp
for w in c3 c4; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/stats_${tag}_$w" -o run -- python3 "$R/bench.py" --workload $w --cpu-baseline 0 --sc16-steps 0 --steps 10 > "$R/gpurun_out/stats_${tag}_$w.log" 2>&1 || exit 1
done
echo stats-done
cd $R
TAG=$tag REPS=2 bash tools/gpu_cfo_bench.sh || exit 1
echo cfo-done

#!/bin/bash
# Round evidence on one box: the full -m gpu suite, bench lines (CPU baseline on) for every
# workload plus the CFO line, then the PMC passes and rocprof stats (tools/gpu_pmc.sh).
# Usage: TAG=r03b bash tools/gpu_round.sh   (outputs under gpurun_out/$TAG and gpurun_out/*_$TAG_*)
set -o pipefail
T=${TAG:-round}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -n 30 $O/gpu_tests.log; exit 1; }
tail -n 1 $O/gpu_tests.log
for w in c3 c2 c4 c5; do
  timeout -k 10 300 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail -n 20 $O/bench_$w.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/bench_$w.json'))
print('$w', 'value %.4g'%d['value'], 'ms %.4f'%d['ms_per_step'], 'roof %.3f'%d['roofline']['frac'], 'cpu %.3g'%d['cpu_baseline']['value'])"
done
timeout -k 10 200 python bench.py --cfo 0.3 --cpu-baseline 0 > $O/bench_c3_cfo.json 2> $O/bench_c3_cfo.err || { echo "cfo bench failed"; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench_c3_cfo.json')); print('cfo', 'ms %.4f'%d['ms_per_step'])"
bash tools/gpu_pmc.sh $T || { echo "pmc failed"; exit 1; }
echo round-evidence-done

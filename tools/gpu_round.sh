#!/bin/bash
# One GPU-box session: gpu tests, then the bench workloads. Every GPU step has its own limit
# and the chain stops at the first failure.
set -o pipefail
O=gpurun_out/${1:-r02}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for w in c3 c5 c2 c4; do
  timeout -k 10 240 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail -20 $O/bench_$w.err; exit 1; }
  echo "$w: $(head -c 400 $O/bench_$w.json)"
done
timeout -k 10 200 python bench.py --ingest scatter --cpu-baseline 0 > $O/bench_c3_scatter1.json 2> $O/bench_c3_scatter1.err || { echo "scatter failed"; tail -20 $O/bench_c3_scatter1.err; exit 1; }

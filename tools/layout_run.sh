#!/bin/bash
# symbol-major output layout: layout parity on every decode path, the whole GPU suite, then the
# bench lines with each layout (alternating)
set -o pipefail
mkdir -p gpurun_out/lay
timeout -k 10 200 python -u -m pytest tests/test_gpu.py -x -v --timeout 150 --timeout-method thread -k "symbol_major_layout" > gpurun_out/lay/t1.log 2>&1 || { tail -n 40 gpurun_out/lay/t1.log; exit 1; }
tail -n 1 gpurun_out/lay/t1.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/lay/t2.log 2>&1 || { tail -n 40 gpurun_out/lay/t2.log; exit 1; }
tail -n 1 gpurun_out/lay/t2.log
for w in c3 c5 c4; do
  A_ENV="RMIMO_X=0" B_ENV="RMIMO_X=1" PAIRS=1 BENCH_ARGS="--workload $w --out-layout stream" tools/ab_env.sh | sed "s/^/$w stream /" || exit 1
  A_ENV="RMIMO_X=0" B_ENV="RMIMO_X=1" PAIRS=1 BENCH_ARGS="--workload $w --out-layout symbol" tools/ab_env.sh | sed "s/^/$w symbol /" || exit 1
done

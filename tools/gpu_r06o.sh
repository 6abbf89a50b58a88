#!/bin/bash
# CFO through ls_window_kernel: CFO and LS-form parity tests, then the CFO bench pair
set -o pipefail
O=gpurun_out/r06z; mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu.py \
  -k "cfo or ls_window" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "PASSED|FAILED" $O/tests.log | sed 's/.*:://' ; tail -1 $O/tests.log
TAG=r06z REPS=2 bash tools/gpu_cfo_bench.sh || exit 1

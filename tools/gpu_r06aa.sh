#!/bin/bash
set -o pipefail
O=gpurun_out/r06aa; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu.py -k "ls_window_with_cfo" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "PASSED|FAILED" $O/tests.log | sed 's/.*:://'; tail -1 $O/tests.log

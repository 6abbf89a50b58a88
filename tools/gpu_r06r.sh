#!/bin/bash
# S&C exact pass: resolve windows per iteration (in-kernel profile)
set -o pipefail
O=gpurun_out/r06r; mkdir -p $O
RMIMO_SC_PROF=1 RMIMO_SC_COUNT=1 timeout -k 10 200 python3 tools/diag_sc.py --frames 64 --reps 2 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
grep -E "exact_" $O/prof.log | tail -6

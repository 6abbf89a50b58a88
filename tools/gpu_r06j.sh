#!/bin/bash
# S&C item dump (which items take 4 iterations) + default bench (LS window conflict-free sums)
set -o pipefail
O=gpurun_out/r06j; mkdir -p $O
T="timeout -k 10"
RMIMO_SC_COUNT=1+ $T 200 python3 tools/diag_sc.py --frames 64 --reps 1 > $O/items.log 2>&1 || { tail -20 $O/items.log; exit 1; }
$T 300 python3 bench.py --cpu-baseline 0 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
tail -c 600 $O/bench.json

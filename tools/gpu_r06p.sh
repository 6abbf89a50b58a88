#!/bin/bash
# kernel-trace stats of the opt-in CFO bench (C3 x 64, eps 0.3)
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r06p
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r06p/stats_cfo" -o run -- python3 "$R/bench.py" --cfo 0.3 --cpu-baseline 0 --sc16-steps 0 --steps 10 > "$R/gpurun_out/r06p/stats_cfo.log" 2>&1 || exit 1
head -16 "$R/gpurun_out/r06p/stats_cfo/run_kernel_stats.csv" | cut -d, -f1-4

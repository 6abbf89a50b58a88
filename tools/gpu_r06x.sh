#!/bin/bash
# screen HBM traffic and durations, LDS-ring form (default) and HEAD
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
export PMC_KERNEL="sc_screen"
tools/pmc_run.sh r06x_ring_fetch FETCH_SIZE || exit 1
RMIMO_LIB=$R/build/var/schead.so tools/pmc_run.sh r06x_head_fetch FETCH_SIZE || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r06x/stats_ring" -o run -- python3 "$R/bench.py" --cpu-baseline 0 --sc16-steps 0 --steps 10 > "$R/gpurun_out/r06x/stats_ring.log" 2>&1 || exit 1
RMIMO_LIB=$R/build/var/schead.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r06x/stats_head" -o run -- python3 "$R/bench.py" --cpu-baseline 0 --sc16-steps 0 --steps 10 > "$R/gpurun_out/r06x/stats_head.log" 2>&1 || exit 1
echo done

#!/bin/bash
# round 6, call V: PMC passes over the front-stage kernels and the decode at HEAD (C3 x 64)
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd $R
export PMC_KERNEL="search_ls_wave|ls_window|sc_exact|sc_screen|decode_stream"
bash tools/pmc_all.sh r06v_c3 || { echo "pmc failed"; exit 1; }
echo pmc-done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/stats_r06v_c3" -o run -- python3 "$R/bench.py" --cpu-baseline 0 --sc16-steps 0 --steps 10 > "$R/gpurun_out/stats_r06v_c3.log" 2>&1 || exit 1
echo stats-done

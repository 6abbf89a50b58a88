#!/bin/bash
# tools/pmc_run.sh NAME "COUNTERS" [bench args...] -- one rocprofv3 --pmc pass over the decode
# kernels of a short bench run (direct-launch stage pass), csv under gpurun_out/pmc_NAME/
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; ctrs=$2; shift 2
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -s KILL 120 rocprofv3 --kernel-include-regex "${PMC_KERNEL:-decode}" --pmc $ctrs --output-format csv \
  -d "$R/gpurun_out/pmc_$name" -o run -- python3 "$R/bench.py" --cpu-baseline 0 --sc16-steps 0 --steps 2 \
  --warmup 1 "$@" > "$R/gpurun_out/pmc_$name.log" 2>&1

#!/bin/bash
# tools/prof_stats.sh NAME [bench args...] -- rocprofv3 kernel-trace stats of a short bench run
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$name" \
  -o run -- python3 "$R/bench.py" --cpu-baseline 0 "$@" > "$R/gpurun_out/prof_$name.log" 2>&1

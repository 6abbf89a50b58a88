#!/bin/bash
# C3 round-end evidence at the bench default: decode PMC (FETCH/WRITE passes -> the bench's
# traffic json), the bench line with the CPU baseline, kernel-trace stats
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
tag=${1:-r02f}
O=$R/gpurun_out/$tag
mkdir -p $O
cd $R
export PMC_KERNEL="decode"
"$R/tools/pmc_run.sh" "${tag}_c3_fetch" "FETCH_SIZE" --workload c3 --h2d 0 || exit 1
"$R/tools/pmc_run.sh" "${tag}_c3_write" "WRITE_SIZE" --workload c3 --h2d 0 || exit 1
python3 tools/pmc_decode.py gpurun_out/pmc_${tag}_c3_fetch/run_counter_collection.csv \
  gpurun_out/pmc_${tag}_c3_write/run_counter_collection.csv --kernel decode_stream_kernel \
  --M 2048 --streams 4 --frames 64 --pid 1000 --ref-mode 1 -o profiles/decode_pmc_c3.json || exit 1
cp profiles/decode_pmc_c3.json $O/decode_pmc_c3.json
timeout -k 10 300 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/stats_${tag}_c3" -o run -- python3 "$R/bench.py" --cpu-baseline 0 --sc16-steps 0 --h2d 0 --steps 10 > "$R/gpurun_out/stats_${tag}_c3.log" 2>&1 || exit 1
echo done

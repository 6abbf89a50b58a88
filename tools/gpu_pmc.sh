#!/bin/bash
# PMC passes + kernel-trace stats for the bench workloads (one rocprofv3 run per pass).
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
tag=${1:-r02}
export PMC_KERNEL="decode|search|ls_|sc_screen|sc_exact|weights|plateau|evm|fill"
"$R/tools/pmc_all.sh" "${tag}_c3" || exit 1
export PMC_KERNEL="decode|spectra|apply_split|search|ls_|weights"
"$R/tools/pmc_run.sh" "${tag}_c4_sqa" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" --workload c4 || exit 1
"$R/tools/pmc_run.sh" "${tag}_c4_fetch" "FETCH_SIZE" --workload c4 || exit 1
"$R/tools/pmc_run.sh" "${tag}_c4_write" "WRITE_SIZE" --workload c4 || exit 1
"$R/tools/pmc_run.sh" "${tag}_c2_fetch" "FETCH_SIZE" --workload c2 || exit 1
"$R/tools/pmc_run.sh" "${tag}_c2_write" "WRITE_SIZE" --workload c2 || exit 1
"$R/tools/pmc_run.sh" "${tag}_c5_fetch" "FETCH_SIZE" --workload c5 || exit 1
"$R/tools/pmc_run.sh" "${tag}_c5_write" "WRITE_SIZE" --workload c5 || exit 1
cd /tmp && export TMPDIR=/tmp
for w in c3 c4 c2 c5; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/stats_${tag}_$w" -o run -- python3 "$R/bench.py" --workload $w --cpu-baseline 0 --sc16-steps 0 --steps 10 > "$R/gpurun_out/stats_${tag}_$w.log" 2>&1 || exit 1
done

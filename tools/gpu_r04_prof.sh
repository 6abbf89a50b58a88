#!/bin/bash
# round-4 profiling session: PMC passes (tools/pmc_all.sh) over C3 and C4 and kernel-trace
# stats of both, plus the C4 decode A/B (residue-class vs split) on the same box
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
tag=${1:-r04}
O=$R/gpurun_out/$tag
mkdir -p $O
cd $R
for v in 1 0; do
  RMIMO_DECODE_RES=$v timeout -k 10 200 python bench.py --workload c4 --cpu-baseline 0 --sc16-steps 0 > $O/bench_c4_res$v.json 2> $O/bench_c4_res$v.err || { tail -20 $O/bench_c4_res$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/bench_c4_res$v.json')); print('c4 res=$v', round(d['ms_per_step'],4), {k:round(x,4) for k,x in d['stages_ms_per_step'].items()}, d['roofline']['kernel'])"
done
export PMC_KERNEL="decode|search|ls_|sc_screen|sc_exact|weights|plateau|evm|fill"
"$R/tools/pmc_all.sh" "${tag}_c3" || exit 1
export PMC_KERNEL="decode|spectra|apply_split|search|ls_|weights"
"$R/tools/pmc_all.sh" "${tag}_c4" --workload c4 || exit 1
cd /tmp && export TMPDIR=/tmp
for w in c3 c4; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/stats_${tag}_$w" -o run -- python3 "$R/bench.py" --workload $w --cpu-baseline 0 --sc16-steps 0 --steps 10 > "$R/gpurun_out/stats_${tag}_$w.log" 2>&1 || exit 1
done
echo done

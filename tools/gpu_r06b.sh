#!/bin/bash
# round 6, call B: the one-slot F = 5120 search -- C3 parity first, then bench A/B of the forms
set -o pipefail
mkdir -p gpurun_out/r06b
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "c3_4x4 or layout or block_search or sc16_batch or cfo_folded_matches" > gpurun_out/r06b/tests.txt 2>&1
rc=$?; tail -15 gpurun_out/r06b/tests.txt; [ $rc -eq 0 ] || exit $rc
for v in slot5 pair slot5_o2 slot5 pair slot5_o2; do
  case $v in
    slot5) env="" ;;
    pair) env="RMIMO_SEARCH_FORM=pair" ;;
    slot5_o2) env="RMIMO_SEARCH5_ORDER=2" ;;
  esac
  env $env $T 200 python bench.py --cpu-baseline 0 --sc16-steps 0 --steps 20 > gpurun_out/r06b/b_$v.json 2>gpurun_out/r06b/b_$v.err || { tail gpurun_out/r06b/b_$v.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/r06b/b_$v.json')); st=d['stages_ms_per_step']; print('$v', 'ms %.4f'%d['ms_per_step'], ' '.join('%s %.4f'%(k,v) for k,v in st.items()), 'evm_delta', d.get('evm_db_delta_vs_cpu'))"
done

#!/bin/bash
# round 6, call D: LS form test, C3 parity, then bench A/B: search slot5 / pair, LS window /
# terms, S&C longest-first order on / off (build/var/sc_noorder.so)
set -o pipefail
mkdir -p gpurun_out/r06d
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "ls_window or c3_4x4 or block_search or sc16_batch or c4_split or c2_2x2 or two_phase or late_frames" > gpurun_out/r06d/tests.txt 2>&1
rc=$?; tail -15 gpurun_out/r06d/tests.txt; [ $rc -eq 0 ] || exit $rc
for v in pair slot5 terms noorder pair slot5 terms noorder; do
  case $v in
    slot5) env="RMIMO_X=1" ;;
    pair) env="RMIMO_SEARCH_FORM=pair" ;;
    terms) env="RMIMO_SEARCH_FORM=pair RMIMO_LS_FORM=terms" ;;
    noorder) env="RMIMO_SEARCH_FORM=pair RMIMO_LIB=$PWD/build/var/sc_noorder.so" ;;
  esac
  env $env $T 200 python bench.py --cpu-baseline 0 --sc16-steps 0 --steps 20 > gpurun_out/r06d/b_$v.json 2>gpurun_out/r06d/b_$v.err || { tail gpurun_out/r06d/b_$v.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/r06d/b_$v.json')); st=d['stages_ms_per_step']; print('$v', 'ms %.4f'%d['ms_per_step'], ' '.join('%s %.4f'%(k,v) for k,v in st.items()))"
done

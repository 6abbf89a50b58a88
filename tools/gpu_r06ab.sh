#!/bin/bash
# weights: the row solve (8-lane groups) at 4x4 vs the per-thread solve (default)
set -o pipefail
O=gpurun_out/r06ab; mkdir -p $O
T="timeout -k 10"
RMIMO_LIB=$PWD/build/var/wrow4.so $T 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu.py \
  -k "c3_4x4 or golden or batch_frames or ls_window_equals" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  for v in wrow4 default; do
    if [ $v = default ]; then L=""; else L="RMIMO_LIB=$PWD/build/var/$v.so"; fi
    env $L $T 200 python bench.py --cpu-baseline 0 --sc16-steps 0 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail $O/b_${v}_$r.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); s=d['stages_ms_per_step']
print('$v', $r, round(d['ms_per_step'],4), 'weights', round(s['weights'],4), 'evm', d['evm_db'])"
  done
done

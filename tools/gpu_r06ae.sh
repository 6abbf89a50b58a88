#!/bin/bash
# LS window: two transform images, one barrier per exchange (default) vs HEAD
set -o pipefail
O=gpurun_out/r06ae; mkdir -p $O
T="timeout -k 10"
$T 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu.py \
  -k "ls_window or c3_4x4 or c2_2x2 or golden or cfo_folded_matches" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  for v in eshead default; do
    if [ $v = default ]; then L=""; else L="RMIMO_LIB=$PWD/build/var/$v.so"; fi
    env $L $T 200 python bench.py --cpu-baseline 0 --sc16-steps 0 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail $O/b_${v}_$r.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); s=d['stages_ms_per_step']
print('$v', $r, round(d['ms_per_step'],4), 'ls', round(s['ls'],4))"
  done
done

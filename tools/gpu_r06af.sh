#!/bin/bash
# search: the keys' wave maximum over DPP and permlane swaps (default) vs ds_bpermute shuffles (HEAD)
set -o pipefail
O=gpurun_out/r06af; mkdir -p $O
T="timeout -k 10"
$T 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu.py \
  -k "search or c3_4x4 or c2_2x2 or golden or c4_8x8 or sc16_batch or ls_window or cfo_folded_matches" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  for v in eshead default; do
    if [ $v = default ]; then L=""; else L="RMIMO_LIB=$PWD/build/var/$v.so"; fi
    env $L $T 200 python bench.py --cpu-baseline 0 --sc16-steps 0 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail $O/b_${v}_$r.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); s=d['stages_ms_per_step']
print('$v', $r, round(d['ms_per_step'],4), 'search', round(s['search'],4), 'ls', round(s['ls'],4), 'frames_ok', d['frames_ok'])"
  done
done

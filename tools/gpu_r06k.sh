#!/bin/bash
# S&C exact pass: long passes split between two workgroups. Parity (split == whole, S&C tests),
# then A/B of the S&C stage: default (split >= 3 iterations), never split, split >= 2.
set -o pipefail
O=gpurun_out/r06k; mkdir -p $O
T="timeout -k 10"
$T 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu.py \
  -k "split_passes or two_phase or c3_4x4 or c2_2x2 or captures_starting or streaming_framesync or batch_frames" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for r in 1 2; do
  for v in default scwhole scsplit2; do
    if [ $v = default ]; then L=""; else L="RMIMO_LIB=$PWD/build/var/$v.so"; fi
    env $L $T 200 python bench.py --cpu-baseline 0 --sc16-steps 0 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail $O/b_${v}_$r.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); s=d['stages_ms_per_step']
print('$v', $r, round(d['ms_per_step'],4), 'sc', round(s['sc'],4), 'frames_ok', d['frames_ok'])"
  done
done

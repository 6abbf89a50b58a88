#!/bin/bash
# S&C screen: lagged samples from an LDS ring of the workgroup's own blocks (default) vs HEAD
set -o pipefail
O=gpurun_out/r06w; mkdir -p $O
T="timeout -k 10"
$T 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu.py \
  -k "two_phase or c3_4x4 or c2_2x2 or captures_starting or streaming_framesync or batch_frames or golden or c4_8x8 or sc16_batch or cfo_folded_matches" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  for v in schead default; do
    if [ $v = default ]; then L=""; else L="RMIMO_LIB=$PWD/build/var/$v.so"; fi
    env $L $T 200 python bench.py --cpu-baseline 0 --sc16-steps 0 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail $O/b_${v}_$r.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); s=d['stages_ms_per_step']
print('$v', $r, round(d['ms_per_step'],4), 'sc', round(s['sc'],4), 'frames_ok', d['frames_ok'], 'exact', d['sc_exact_recomputes_per_step'])"
  done
done
for v in default schead; do
  if [ $v = default ]; then L=""; else L="RMIMO_LIB=$PWD/build/var/$v.so"; fi
  env $L RMIMO_SC_PROF=1 RMIMO_SC_COUNT=1 $T 200 python3 tools/diag_sc.py --frames 64 --reps 2 > $O/prof_$v.log 2>&1 || { tail -20 $O/prof_$v.log; exit 1; }
  grep -E "exact_prof" $O/prof_$v.log | tail -1
done

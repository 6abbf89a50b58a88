#!/bin/bash
# A/B of the S&C stage: HEAD (grid N), never split (grid 2N), split >= 3 (default), split >= 2
set -o pipefail
O=gpurun_out/r06l; mkdir -p $O
T="timeout -k 10"
for r in 1 2; do
  for v in schead scwhole default scsplit2; do
    if [ $v = default ]; then L=""; else L="RMIMO_LIB=$PWD/build/var/$v.so"; fi
    env $L $T 200 python bench.py --cpu-baseline 0 --sc16-steps 0 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail $O/b_${v}_$r.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); s=d['stages_ms_per_step']
print('$v', $r, round(d['ms_per_step'],4), 'sc', round(s['sc'],4), 'frames_ok', d['frames_ok'])"
  done
done
for v in default schead; do
  if [ $v = default ]; then L=""; else L="RMIMO_LIB=$PWD/build/var/$v.so"; fi
  env $L RMIMO_SC_PROF=1 RMIMO_SC_COUNT=1 $T 200 python3 tools/diag_sc.py --frames 64 --reps 2 > $O/prof_$v.log 2>&1 || { tail -20 $O/prof_$v.log; exit 1; }
  grep -E "exact_prof|exact_split" $O/prof_$v.log | tail -2
done

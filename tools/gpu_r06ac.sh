#!/bin/bash
# LS window timing ablations: no |X|^2 LDS sums (lsnos2), no fp64 sums (lsnoacc), default
set -o pipefail
O=gpurun_out/r06ac; mkdir -p $O
T="timeout -k 10"
for r in 1 2; do
  for v in lsnos2 lsnoacc default; do
    if [ $v = default ]; then L=""; else L="RMIMO_LIB=$PWD/build/var/$v.so"; fi
    env $L $T 200 python bench.py --cpu-baseline 0 --sc16-steps 0 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail $O/b_${v}_$r.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); s=d['stages_ms_per_step']
print('$v', $r, round(d['ms_per_step'],4), 'ls', round(s['ls'],4))"
  done
done

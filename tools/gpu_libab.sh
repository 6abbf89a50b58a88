#!/bin/bash
# A/B of two builds of the library on the bench (alternating runs): LIB_A / LIB_B are paths
# relative to rub_mimo_amd/, WL the workload(s)
set -o pipefail
O=gpurun_out/${TAG:-libab}
mkdir -p $O
for w in ${WL:-c3}; do
for k in ${AB_REPS:-1 2}; do
  for L in $LIB_A $LIB_B; do
    RMIMO_LIB=$PWD/rub_mimo_amd/$L timeout -k 10 200 python bench.py --workload $w --cpu-baseline 0 --sc16-steps 0 --h2d 0 $BENCH_ARGS > $O/ab_${w}_${L}_$k.json 2> $O/ab_${w}_${L}_$k.err || { echo "bench $L failed"; tail -n 20 $O/ab_${w}_${L}_$k.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/ab_${w}_${L}_$k.json'))
print('$w', '$L', 'ms %.4f'%d['ms_per_step'], 'roof %.3f'%d['roofline']['frac'], {k:round(x,4) for k,x in d['stages_ms_per_step'].items()})"
  done
done
done

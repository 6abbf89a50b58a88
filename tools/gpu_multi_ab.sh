#!/bin/bash
# A/B/C.. of library builds on one box, alternating: LIBS = paths relative to the repo root
# (the in-tree library is rub_mimo_amd/librub_mimo_amd.so), WL the workloads, REPS rounds;
# PROF_LIBS = DS_PROF builds run once each with RMIMO_DEC_PROF=1 (cycle split on stderr)
set -o pipefail
O=gpurun_out/${TAG:-mab}
mkdir -p $O
for w in ${WL:-c3}; do
for k in $(seq ${REPS:-2}); do
  for L in $LIBS; do
    n=$(basename $L .so)
    RMIMO_LIB=$PWD/$L timeout -k 10 200 python bench.py --workload $w --cpu-baseline 0 --sc16-steps 0 --h2d 0 $BENCH_ARGS > $O/${w}_${n}_$k.json 2> $O/${w}_${n}_$k.err || { echo "bench $L failed"; tail -n 20 $O/${w}_${n}_$k.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/${w}_${n}_$k.json'))
print('$w', '%-22s'%'$n', 'ms %.4f'%d['ms_per_step'], 'roof %.3f'%d['roofline']['frac'], ' '.join('%s %.4f'%(k,x) for k,x in d['stages_ms_per_step'].items()), flush=True)"
  done
done
done
for L in $PROF_LIBS; do
  n=$(basename $L .so)
  RMIMO_DEC_PROF=1 RMIMO_LIB=$PWD/$L timeout -k 10 200 python bench.py --workload ${PROF_WL:-c3} --cpu-baseline 0 --sc16-steps 0 --h2d 0 --steps 3 --warmup 1 > $O/prof_${n}.json 2> $O/prof_${n}.err || { echo "prof $L failed"; tail -n 20 $O/prof_${n}.err; exit 1; }
  echo "$n $(grep dec_prof $O/prof_${n}.err | tail -n 1)"
done

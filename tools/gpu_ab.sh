#!/bin/bash
# A/B of one environment switch on the bench: alternating runs (default, then $AB_ENV), C3
# unless WL is set; prints value, ms/step and stage times of each run
set -o pipefail
O=gpurun_out/${TAG:-ab}
mkdir -p $O
W=${WL:-c3}
for k in ${AB_REPS:-1 2}; do
  for v in base alt; do
    if [ $v = alt ]; then E="$AB_ENV"; else E=""; fi
    env $E timeout -k 10 200 python bench.py --workload $W --cpu-baseline 0 --sc16-steps 0 --h2d 0 $BENCH_ARGS > $O/ab_${W}_${v}_$k.json 2> $O/ab_${W}_${v}_$k.err || { echo "bench $v failed"; tail -n 20 $O/ab_${W}_${v}_$k.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/ab_${W}_${v}_$k.json'))
print('$v', '$E', 'value %.4g'%d['value'], 'ms %.4f'%d['ms_per_step'], 'ok %d'%d['frames_ok'], {k:round(x,4) for k,x in d['stages_ms_per_step'].items()})"
  done
done

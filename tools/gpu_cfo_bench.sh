#!/bin/bash
# the --cfo bench pair (off / eps 0.3) at C3, alternating REPS times (cost of the CFO stages)
set -o pipefail
O=gpurun_out/${TAG:-cfob}
mkdir -p $O
for k in $(seq 1 ${REPS:-1}); do
for v in 0 0.3; do
  timeout -k 10 200 python bench.py --cfo $v --cpu-baseline 0 --sc16-steps 0 --h2d 0 $BENCH_ARGS > $O/bench_cfo_${v}_$k.json 2> $O/bench_cfo_${v}_$k.err || { echo "bench failed"; tail -20 $O/bench_cfo_${v}_$k.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/bench_cfo_${v}_$k.json'))
print('cfo $v', 'value %.4g'%d['value'], 'ms %.4f'%d['ms_per_step'], 'ok %d'%d['frames_ok'], 'evm %.3f'%d['evm_db'], {k:round(x,4) for k,x in d['stages_ms_per_step'].items()})"
done
done

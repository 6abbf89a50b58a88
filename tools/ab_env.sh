#!/bin/bash
# A/B timing of the C3 bench between two environment settings (A_ENV, B_ENV: "VAR=value ..."),
# alternating PAIRS times with STEPS steps each; TESTS=1 runs the GPU suite first
mkdir -p gpurun_out/ab
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab/t.log 2>&1 || { tail -n 30 gpurun_out/ab/t.log; exit 1; }
  tail -n 1 gpurun_out/ab/t.log
fi
for i in $(seq ${PAIRS:-2}); do
for v in A B; do
  if [ $v = A ]; then E="$A_ENV"; else E="$B_ENV"; fi
  env $E timeout -k 10 200 python bench.py --cpu-baseline 0 --sc16-steps 0 --steps ${STEPS:-20} $BENCH_ARGS > gpurun_out/ab/b_$v.json 2>gpurun_out/ab/b_$v.err || { tail gpurun_out/ab/b_$v.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ab/b_$v.json')); st=d['stages_ms_per_step']; print('$v', round(d['ms_per_step'],4), ' '.join('%s %.4f'%(k,st[k]) for k in ('sc','search','ls','decode')), 'roof', round(d['roofline']['frac'],3), d['frames_ok'])"
done
done

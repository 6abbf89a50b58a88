#!/bin/bash
# tests (optionally filtered) then bench lines for the given workloads, no CPU baseline
set -o pipefail
O=gpurun_out/${TAG:-q}
mkdir -p $O
# TESTS: unset = no tests, "all" (or blank) = every gpu test, anything else = a -k expression
if [ -n "${TESTS+x}" ]; then
  K=()
  if [ -n "${TESTS// /}" ] && [ "$TESTS" != all ]; then K=(-k "$TESTS"); fi
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${K[@]}" > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -n 40 $O/gpu_tests.log; exit 1; }
  tail -n 2 $O/gpu_tests.log
fi
for w in ${WORKLOADS:-c3}; do
  timeout -k 10 200 python bench.py --workload $w --cpu-baseline 0 $BENCH_ARGS > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail -n 20 $O/bench_$w.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/bench_$w.json'))
print('$w', 'value %.4g'%d['value'], 'ms %.4f'%d['ms_per_step'], 'ok %d/%d'%(d['frames_ok'],d['frames']), 'roof %.3f'%d['roofline']['frac'], d['roofline']['kernel'], 'evm %.3f'%d['evm_db'])
print('   ', {k:round(v,4) for k,v in d['stages_ms_per_step'].items()})"
done

#!/bin/bash
# round-4 session check: every gpu test, then bench lines (C3 default first), then the CFO pair
set -o pipefail
O=gpurun_out/${TAG:-r04}
mkdir -p $O
timeout -k 10 ${TEST_T:-700} python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread ${TEST_K:+-k "$TEST_K"} > $O/gpu_tests.log 2>&1
rc=$?
tail -n 3 $O/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|error" $O/gpu_tests.log | head -20; exit 1; fi
for w in ${WORKLOADS:-c3 c4 c2}; do
  timeout -k 10 200 python bench.py --workload $w --cpu-baseline 0 > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail -n 20 $O/bench_$w.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/bench_$w.json'))
print('$w', 'value %.4g'%d['value'], 'ms %.4f'%d['ms_per_step'], 'ok %d/%d'%(d['frames_ok'],d['frames']), 'roof %.3f'%d['roofline']['frac'], d['roofline']['kernel'], 'evm %.3f'%d['evm_db'])
print('   ', {k:round(v,4) for k,v in d['stages_ms_per_step'].items()})"
done

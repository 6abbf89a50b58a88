#!/bin/bash
# round 6, call I: the CFO decode with the deferred apply (one barrier per symbol fewer):
# CFO + C3 parity, then plain and CFO steps against the previous decode (build/var/ds_old.so)
set -o pipefail
mkdir -p gpurun_out/r06i
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu.py tests/test_gpu_streams.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "cfo or c3_4x4 or layout or c5 or split_stages or ls_window" > gpurun_out/r06i/tests.txt 2>&1
rc=$?; tail -4 gpurun_out/r06i/tests.txt; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r06i/tests.txt | head; exit $rc; }
for r in 1 2; do
for v in new old; do
  if [ $v = new ]; then env="RMIMO_X=1"; else env="RMIMO_LIB=$PWD/build/var/ds_old.so"; fi
  for c in 0 0.3; do
    env $env $T 200 python bench.py --cpu-baseline 0 --sc16-steps 0 --steps 20 --cfo $c > gpurun_out/r06i/b_${v}_$c.json 2>gpurun_out/r06i/b_${v}_$c.err || { tail gpurun_out/r06i/b_${v}_$c.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/r06i/b_${v}_$c.json')); st=d['stages_ms_per_step']; print('$v cfo $c', 'ms %.4f'%d['ms_per_step'], 'evm %.3f'%d['evm_db'], ' '.join('%s %.4f'%(k,v) for k,v in st.items()))"
  done
done
done

#!/bin/bash
# round 6, call G: pipelined front/decode on CU partitions (bench --pipeline D) against the
# serial step, D in {160, 176, 192, 208, 224}; split-stage parity first
set -o pipefail
mkdir -p gpurun_out/r06g
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "split_stages" > gpurun_out/r06g/tests.txt 2>&1
rc=$?; tail -4 gpurun_out/r06g/tests.txt; [ $rc -eq 0 ] || exit $rc
for v in 192 176 208 160 224 192 176; do
  $T 200 python bench.py --cpu-baseline 0 --sc16-steps 0 --steps 20 --pipeline $v > gpurun_out/r06g/b_$v.json 2>gpurun_out/r06g/b_$v.err || { tail gpurun_out/r06g/b_$v.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/r06g/b_$v.json')); p=d['pipeline']; print('D $v', 'ms %.4f'%d['ms_per_step'], 'serial %.4f'%p['serial_ms_per_step'], 'frames_ok', d['frames_ok'])"
done

#!/bin/bash
# the C4 bench line with its CPU baseline (S&C skipped from the GPU trigger, Parseval search,
# decode stage) so that evm_db_delta_vs_cpu is populated
set -o pipefail
O=gpurun_out/${TAG:-q}
mkdir -p $O
timeout -k 10 400 python bench.py --workload c4 --cpu-baseline 1 --sc16-steps 0 --h2d 0 $BENCH_ARGS > $O/bench_c4_cpu.json 2> $O/bench_c4_cpu.err || { echo "bench c4 cpu failed"; tail -n 20 $O/bench_c4_cpu.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench_c4_cpu.json'))
print('c4', 'value %.4g'%d['value'], 'ms %.4f'%d['ms_per_step'], d['roofline']['kernel'], 'evm_delta', d['evm_db_delta_vs_cpu'])"

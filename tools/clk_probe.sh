#!/bin/bash
# Sample the GPU's clocks and power while the C3 bench runs (read-only rocm-smi queries):
# is the decode's box-to-box / run-to-run spread a clock (power) effect?
set -o pipefail
O=gpurun_out/clk; mkdir -p $O
rocm-smi --showclocks --showpower --showtemp > $O/idle.txt 2>&1 || true
timeout -k 10 200 python bench.py --cpu-baseline 0 --sc16-steps 0 --steps 2000 --warmup 3 > $O/b.json 2> $O/b.err &
P=$!
for i in $(seq 1 12); do sleep 2; rocm-smi --showclocks --showpower --showtemp > $O/s_$i.txt 2>&1 || true; done
wait $P
python3 -c "import json; d=json.load(open('$O/b.json')); print(d['ms_per_step'], d['stages_ms_per_step']['decode'])"

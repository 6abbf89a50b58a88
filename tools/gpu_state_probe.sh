#!/bin/bash
# Is the decode's speed a property of the box or of its state? The memory-pattern micro
# (tools/micro/stream_ceiling) and the C3 bench on a fresh box, then again after a minute of
# sustained load, with read-only rocm-smi samples of clocks and power beside each.
set -o pipefail
O=gpurun_out/${TAG:-state}; mkdir -p $O
smi() { rocm-smi --showclocks --showpower --showtemp > $O/smi_$1.txt 2>&1 || true; }
smi idle
timeout -k 10 120 tools/micro/stream_ceiling > $O/micro_fresh.txt 2>&1 || exit 1
head -2 $O/micro_fresh.txt
timeout -k 10 200 python bench.py --cpu-baseline 0 --sc16-steps 0 --h2d 0 > $O/bench_fresh.json 2> $O/bench_fresh.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench_fresh.json')); print('fresh bench', d['ms_per_step'], d['stages_ms_per_step']['decode'])"
timeout -k 10 200 python bench.py --cpu-baseline 0 --sc16-steps 0 --h2d 0 --steps 25000 --warmup 3 > $O/bench_load.json 2> $O/bench_load.err &
P=$!
for i in 1 2 3; do sleep 15; smi load_$i; done
wait $P || exit 1
python3 -c "import json; d=json.load(open('$O/bench_load.json')); print('sustained bench', d['ms_per_step'], d['stages_ms_per_step']['decode'])"
timeout -k 10 120 tools/micro/stream_ceiling > $O/micro_after.txt 2>&1 || exit 1
head -2 $O/micro_after.txt
timeout -k 10 200 python bench.py --cpu-baseline 0 --sc16-steps 0 --h2d 0 > $O/bench_after.json 2> $O/bench_after.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench_after.json')); print('after bench', d['ms_per_step'], d['stages_ms_per_step']['decode'])"
smi end
grep -h "sclk\|Power (W)\|Sensor memory" $O/smi_*.txt

#!/bin/bash
# run bench c3 (fc32 and sc16) with each build/abl/*.so and print the decode stage time
set -o pipefail
mkdir -p gpurun_out/abl
for v in ${VARIANTS:-base nostore nodma nofft nostore_nodma}; do
  for fmt in fc32 sc16; do
    RMIMO_LIB=build/abl/$v.so timeout -k 10 120 python bench.py --workload ${WL:-c3} --cpu-baseline 0 --sc16-steps 0 --sample-format $fmt > gpurun_out/abl/$v.$fmt.json 2> gpurun_out/abl/$v.$fmt.err || { echo "$v $fmt failed"; tail -5 gpurun_out/abl/$v.$fmt.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/abl/$v.$fmt.json'))
s=d['stages_ms_per_step']; print('%-14s %s decode %.4f step %.4f'%('$v','$fmt',s['decode'],d['ms_per_step']))"
  done
done

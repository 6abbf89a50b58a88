#!/bin/bash
# search-stage timing of the ablation builds (tools/abl_search.sh) beside the in-tree library
mkdir -p gpurun_out/abls
for v in base ${VARIANTS:-nols noinv both nofwd noload lsonly} base; do
  if [ $v = base ]; then unset RMIMO_LIB; else export RMIMO_LIB=$PWD/build/var/s_$v.so; fi
  timeout -k 10 200 python bench.py --cpu-baseline 0 --sc16-steps 0 --steps 20 > gpurun_out/abls/b_$v.json 2>gpurun_out/abls/b_$v.err || { tail gpurun_out/abls/b_$v.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/abls/b_$v.json')); st=d['stages_ms_per_step']; print('$v', 'search %.4f'%st['search'], 'ls %.4f'%st['ls'])"
done

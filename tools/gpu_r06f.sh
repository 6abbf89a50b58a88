#!/bin/bash
# round 6, call F: ls_window_kernel timing ablations, the S&C exact-pass profile, space sharing
set -o pipefail
mkdir -p gpurun_out/r06f
T="timeout -k 10"
for v in base lsw_noload lsw_nopf lsw_nofft base; do
  if [ $v = base ]; then env="RMIMO_X=1"; else env="RMIMO_LIB=$PWD/build/var/$v.so"; fi
  env $env $T 200 python bench.py --cpu-baseline 0 --sc16-steps 0 --steps 20 > gpurun_out/r06f/b_$v.json 2>gpurun_out/r06f/b_$v.err || { tail gpurun_out/r06f/b_$v.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/r06f/b_$v.json')); st=d['stages_ms_per_step']; print('$v', 'ms %.4f'%d['ms_per_step'], ' '.join('%s %.4f'%(k,v) for k,v in st.items()))"
done
RMIMO_SC_PROF=1 RMIMO_SC_COUNT=1 $T 200 python bench.py --cpu-baseline 0 --sc16-steps 0 --steps 2 --warmup 1 > gpurun_out/r06f/scprof.json 2> gpurun_out/r06f/scprof.err || { tail gpurun_out/r06f/scprof.err; exit 1; }
grep -E "exact_prof|exact_split|sc_count" gpurun_out/r06f/scprof.err | tail -12
$T 400 python tools/exp_cumask.py --out gpurun_out/r06f/cumask.json > gpurun_out/r06f/cumask.txt 2>&1 || { tail gpurun_out/r06f/cumask.txt; exit 1; }
tail -8 gpurun_out/r06f/cumask.txt

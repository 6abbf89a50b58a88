#!/bin/bash
# round 6, call E: the full GPU suite at the new defaults (window LS, cleanup, RCCL test), the
# default bench line with the decode-pattern leg, and ls_window_kernel timing ablations
set -o pipefail
mkdir -p gpurun_out/r06e
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06e/gpu_tests.txt 2>&1
rc=$?; tail -6 gpurun_out/r06e/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
$T 300 python bench.py > gpurun_out/r06e/bench_default.json 2> gpurun_out/r06e/bench_default.err || { tail gpurun_out/r06e/bench_default.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r06e/bench_default.json')); st=d['stages_ms_per_step']
print('default', 'ms %.4f'%d['ms_per_step'], 'value %.3e'%d['value'], ' '.join('%s %.4f'%(k,v) for k,v in st.items()))
print('pattern', d['decode_pattern_ms'], d['decode_vs_pattern'], 'frac', d['roofline']['frac'])"
for v in base lsw_noload lsw_nopf lsw_nofft base; do
  if [ $v = base ]; then env="RMIMO_X=1"; else env="RMIMO_LIB=$PWD/build/var/$v.so"; fi
  env $env $T 200 python bench.py --cpu-baseline 0 --sc16-steps 0 --steps 20 > gpurun_out/r06e/b_$v.json 2>gpurun_out/r06e/b_$v.err || { tail gpurun_out/r06e/b_$v.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/r06e/b_$v.json')); st=d['stages_ms_per_step']; print('$v', 'ms %.4f'%d['ms_per_step'], ' '.join('%s %.4f'%(k,v) for k,v in st.items()))"
done
# the S&C exact pass's in-kernel profile at HEAD (diagnostics: per-pass timeline, slowest pass)
RMIMO_SC_PROF=1 RMIMO_SC_COUNT=1 $T 200 python bench.py --cpu-baseline 0 --sc16-steps 0 --steps 2 --warmup 1 > gpurun_out/r06e/scprof.json 2> gpurun_out/r06e/scprof.err || { tail gpurun_out/r06e/scprof.err; exit 1; }
grep -E "exact_prof|exact_split|sc_count" gpurun_out/r06e/scprof.err | tail -12
# space sharing: stage times on CU-masked streams, the overlapped-step lower bound per split
$T 400 python tools/exp_cumask.py --out gpurun_out/r06e/cumask.json > gpurun_out/r06e/cumask.txt 2>&1 || { tail gpurun_out/r06e/cumask.txt; exit 1; }
tail -8 gpurun_out/r06e/cumask.txt

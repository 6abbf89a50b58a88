set -o pipefail
O=gpurun_out/r03t; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "split or c4 or 8x8" > $O/t.log 2>&1; echo "tests rc=$?"; tail -n 1 $O/t.log
for k in 1 2; do for v in 1 0; do
  RMIMO_APPLY_V1=$v timeout -k 10 200 python bench.py --workload c4 --cpu-baseline 0 --sc16-steps 0 --h2d 0 > $O/b_${v}_$k.json 2>$O/b_${v}_$k.err || exit 1
  python3 -c "
import json; d=json.load(open('$O/b_${v}_$k.json')); print('v1=$v', 'ms %.4f'%d['ms_per_step'], 'decode', round(d['stages_ms_per_step']['decode'],4), 'evm %.4f'%d['evm_db'])"
done; done
TAG=r03t WL=c4 KPAT="apply_split|spectra" LIBS="librub_mimo_amd.so" bash tools/gpu_kstats.sh

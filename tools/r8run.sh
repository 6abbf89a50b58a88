set -o pipefail
mkdir -p gpurun_out/r8
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 240 --timeout-method thread -k "residue or c4_full" > gpurun_out/r8/t.log 2>&1 || { tail -n 40 gpurun_out/r8/t.log; exit 1; }
tail -n 3 gpurun_out/r8/t.log
A_ENV="RMIMO_DECODE_RES=0" B_ENV="RMIMO_DECODE_RES=1" PAIRS=2 BENCH_ARGS="--workload c4" tools/ab_env.sh || exit 1
RMIMO_LIB=$PWD/build/var/prof0r8.so RMIMO_DEC_PROF=1 RMIMO_DECODE_RES=1 timeout -k 10 200 python bench.py --cpu-baseline 0 --sc16-steps 0 --steps 5 --workload c4 > gpurun_out/r8/prof.json 2> gpurun_out/r8/prof.err || { tail gpurun_out/r8/prof.err; exit 1; }
tail -n 20 gpurun_out/r8/prof.err

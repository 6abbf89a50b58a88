#!/bin/bash
# S&C exact pass with 2 workgroups per (item, antenna): sync parity (golden, C2/C3 full frames,
# two-phase, streams) under RMIMO_SC_SPLIT=2, then A/B of 1 vs 2 vs 4 workgroups
set -o pipefail
mkdir -p gpurun_out/scs
RMIMO_SC_SPLIT=2 timeout -k 10 500 python -u -m pytest tests/test_gpu.py tests/test_gpu_streams.py -x -q --timeout 300 --timeout-method thread -k "golden or full_frame or two_phase or c5 or stream_matches or chunked" > gpurun_out/scs/t.log 2>&1 || { tail -n 30 gpurun_out/scs/t.log; exit 1; }
tail -n 1 gpurun_out/scs/t.log
A_ENV="RMIMO_SC_SPLIT=0" B_ENV="RMIMO_SC_SPLIT=2" PAIRS=3 tools/ab_env.sh || exit 1
A_ENV="RMIMO_SC_SPLIT=0" B_ENV="RMIMO_SC_SPLIT=4" PAIRS=1 tools/ab_env.sh || exit 1
A_ENV="RMIMO_SC_SPLIT=0" B_ENV="RMIMO_SC_SPLIT=2" PAIRS=2 BENCH_ARGS="--workload c2" tools/ab_env.sh || exit 1

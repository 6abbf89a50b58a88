#!/bin/bash
# persistent later-phase S&C screen: sync parity (golden, C2/C3/C4 full frames, two-phase vs one
# pass, streams), then A/B against the one-item grid (RMIMO_SCR_PERSIST=0)
set -o pipefail
mkdir -p gpurun_out/scp
timeout -k 10 500 python -u -m pytest tests/test_gpu.py tests/test_gpu_streams.py -x -q --timeout 300 --timeout-method thread -k "golden or full_frame or two_phase or c5 or stream_matches or chunked or layout" > gpurun_out/scp/t.log 2>&1 || { tail -n 30 gpurun_out/scp/t.log; exit 1; }
tail -n 1 gpurun_out/scp/t.log
A_ENV="RMIMO_SCR_PERSIST=0" B_ENV="RMIMO_SCR_PERSIST=1" PAIRS=3 tools/ab_env.sh || exit 1
A_ENV="RMIMO_SCR_PERSIST=0" B_ENV="RMIMO_SCR_PERSIST=1" PAIRS=2 BENCH_ARGS="--workload c2" tools/ab_env.sh || exit 1
A_ENV="RMIMO_SCR_PERSIST=0" B_ENV="RMIMO_SCR_PERSIST=1" PAIRS=1 BENCH_ARGS="--workload c4" tools/ab_env.sh || exit 1
A_ENV="RMIMO_SCR_PERSIST=0" B_ENV="RMIMO_SCR_PERSIST=1" PAIRS=1 BENCH_ARGS="--workload c5" tools/ab_env.sh || exit 1

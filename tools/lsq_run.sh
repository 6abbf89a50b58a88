#!/bin/bash
# chunked LS-term layout: estimate parity (golden, C3 full frame, fused-LS bitwise), A/B of the
# LS combine against the previous layout (build/var/lsprev.so), then the write-rate micro
set -o pipefail
mkdir -p gpurun_out/lsq gpurun_out/micro
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 240 --timeout-method thread -k "golden or ls_combine_fused or c3_4x4_mmse_2048_64qam_full or c4_full or cfo" > gpurun_out/lsq/t.log 2>&1 || { tail -n 30 gpurun_out/lsq/t.log; exit 1; }
tail -n 1 gpurun_out/lsq/t.log
A_ENV="RMIMO_LIB=/root/repo/build/var/lsprev.so" B_ENV="RMIMO_X=1" PAIRS=3 tools/ab_env.sh || exit 1
A_ENV="RMIMO_LIB=/root/repo/build/var/lsprev.so" B_ENV="RMIMO_X=1" PAIRS=2 BENCH_ARGS="--workload c4" tools/ab_env.sh || exit 1
timeout -k 10 200 ./tools/micro/stream_ceiling > gpurun_out/micro/ceiling_write.txt 2>&1 || exit 1
tail -n 9 gpurun_out/micro/ceiling_write.txt

#!/bin/bash
# fused LS combine: parity (bitwise vs the separate kernel, golden fixtures, C3 full frame), then
# A/B of RMIMO_LS_FUSE and of the search's XCD order under fusion, C3 and C4
set -o pipefail
mkdir -p gpurun_out/lsf
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 240 --timeout-method thread -k "ls_combine_fused or golden or c3_4x4_mmse_2048_64qam_full or c2_2x2_zf_1024_16qam_full" > gpurun_out/lsf/t.log 2>&1 || { tail -n 40 gpurun_out/lsf/t.log; exit 1; }
tail -n 2 gpurun_out/lsf/t.log
echo "== C3 fuse 0 vs 1"; A_ENV="RMIMO_LS_FUSE=0" B_ENV="RMIMO_LS_FUSE=1" PAIRS=3 tools/ab_env.sh || exit 1
echo "== C3 fused, xcd 1 vs 2"; A_ENV="RMIMO_SEARCH_XCD=1" B_ENV="RMIMO_SEARCH_XCD=2" PAIRS=2 tools/ab_env.sh || exit 1
echo "== C4 fuse 0 vs 1"; A_ENV="RMIMO_LS_FUSE=0" B_ENV="RMIMO_LS_FUSE=1" PAIRS=2 BENCH_ARGS="--workload c4" tools/ab_env.sh || exit 1

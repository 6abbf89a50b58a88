#!/bin/bash
# fused LS combine with the chunked search order (RMIMO_SEARCH_XCD=3): parity, then A/B
set -o pipefail
mkdir -p gpurun_out/lsf
RMIMO_SEARCH_XCD=3 timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 240 --timeout-method thread -k "ls_combine_fused or golden or c3_4x4_mmse_2048_64qam_full" > gpurun_out/lsf/t2.log 2>&1 || { tail -n 40 gpurun_out/lsf/t2.log; exit 1; }
tail -n 1 gpurun_out/lsf/t2.log
echo "== C3 unfused xcd1 vs fused xcd3/32"; A_ENV="RMIMO_LS_FUSE=0" B_ENV="RMIMO_SEARCH_XCD=3" PAIRS=3 tools/ab_env.sh || exit 1
echo "== C3 fused xcd3 chunk 16 vs 64"; A_ENV="RMIMO_SEARCH_XCD=3 RMIMO_LS_CHUNK=16" B_ENV="RMIMO_SEARCH_XCD=3 RMIMO_LS_CHUNK=64" PAIRS=2 tools/ab_env.sh || exit 1
echo "== C3 unfused xcd1 vs unfused xcd3"; A_ENV="RMIMO_LS_FUSE=0" B_ENV="RMIMO_LS_FUSE=0 RMIMO_SEARCH_XCD=3" PAIRS=2 tools/ab_env.sh || exit 1
echo "== C4 unfused vs fused xcd3/8"; A_ENV="RMIMO_LS_FUSE=0" B_ENV="RMIMO_SEARCH_XCD=3 RMIMO_LS_CHUNK=8" PAIRS=2 BENCH_ARGS="--workload c4" tools/ab_env.sh || exit 1

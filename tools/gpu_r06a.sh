#!/bin/bash
# round 6, call A: search ablation table at HEAD, then the GPU suite after the variant cleanup
set -o pipefail
mkdir -p gpurun_out/r06a
bash tools/abl_run_search.sh > gpurun_out/r06a/abls.txt 2>&1 || { echo "ablation failed"; exit 1; }
cat gpurun_out/r06a/abls.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06a/gpu_tests.txt 2>&1
rc=$?
tail -5 gpurun_out/r06a/gpu_tests.txt
exit $rc

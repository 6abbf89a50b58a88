#!/bin/bash
# tools/run_steps.sh -- run GPU steps on the gpurun box, each under its own time limit.
# usage: tools/run_steps.sh "<seconds> <command>" ["<seconds> <command>" ...]
# A step that fails normally (tests failing, exit 1) lets the next step run; a time limit,
# abort, kill or segfault (exit >= 124) stops the session: nothing more touches the GPU.
mkdir -p gpurun_out
for step in "$@"; do
  t=${step%% *}
  cmd=${step#* }
  echo "=== [$(date +%T) limit ${t}s] $cmd" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" bash -c "$cmd"
  rc=$?
  echo "=== rc=$rc" | tee -a gpurun_out/steps.log
  if [ "$rc" -ge 124 ]; then
    echo "fatal exit status $rc: stopping this session" | tee -a gpurun_out/steps.log
    exit "$rc"
  fi
done
exit 0

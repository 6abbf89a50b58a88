#!/bin/bash
# S&C knob A/B: diag_sc stage times and the exact-kernel timeline per environment setting
# (SC_ENVS: space-separated list of VAR=VALUE[,VAR=VALUE] settings; "base" = none)
set -o pipefail
O=gpurun_out/${TAG:-scab}
mkdir -p $O
i=0
for e in ${SC_ENVS:-base}; do
  E=""; [ "$e" != base ] && E="${e//,/ }"
  env $E RMIMO_SC_PROF=1 RMIMO_SC_COUNT=1 timeout -k 10 200 python3 tools/diag_sc.py --frames ${FRAMES:-64} --reps ${REPS:-3} > $O/sc_$i.log 2>&1 || { echo "diag $e failed"; tail -20 $O/sc_$i.log; exit 1; }
  echo "== $e"; grep -E "exact_prof" $O/sc_$i.log | tail -1 | cut -c1-220; grep stages_ms $O/sc_$i.log
  env $E timeout -k 10 200 python3 tools/diag_sc.py --frames ${FRAMES:-64} --reps 10 > $O/sct_$i.log 2>&1 || { echo "diag2 $e failed"; exit 1; }
  grep stages_ms $O/sct_$i.log
  i=$((i+1))
done

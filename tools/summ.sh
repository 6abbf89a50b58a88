#!/bin/bash
# summarise the last gpurun session's logs
cd "$(dirname "$0")/.."
cat gpurun_out/steps.log 2>/dev/null | grep rc=
for f in gpurun_out/*tests*.log; do [ -f "$f" ] && echo "$f: $(grep -E 'passed|failed' $f | tail -1)"; done
for f in gpurun_out/bench*.log; do [ -f "$f" ] && grep metric "$f" | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('$f', json.dumps({k:d.get(k) for k in ['value','ms_per_step','frames_ok','evm_db','sc_exact_recomputes_per_step','pipeline_hbm_gbs']}))
print('  roofline', json.dumps(d['roofline']))
print('  stages', json.dumps({k:round(v,4) for k,v in d['stages_ms_per_step'].items()}))
if d.get('cpu_baseline'): print('  cpu', d['cpu_baseline']['value'])
"; done
for f in gpurun_out/prof/*kernel_stats.csv; do [ -f "$f" ] && echo "$f" && cut -d, -f1-4 "$f" | head -14; done

#!/bin/bash
# parameter sweep of bench lines (no rebuild): ARGS lines from $SWEEP (';'-separated)
set -o pipefail
IFS=';' read -ra CASES <<< "$SWEEP"
for args in "${CASES[@]}"; do
  timeout -k 10 150 python -u bench.py --steps 200 --warmup 10 --no-cpu-baseline --lanes1-steps 0 --no-queue-compare $args > gpurun_out/sw.log 2>&1 || { tail -5 gpurun_out/sw.log; exit 1; }
  python -c "
import json
for l in open('gpurun_out/sw.log'):
    if l.startswith('{\"metric'):
        d=json.loads(l); print('[$args]', d['value'], {k: round(v,3) for k,v in d['stages_ms'].items() if k in ('entropy','idct','output')})"
done

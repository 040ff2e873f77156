#!/bin/bash
# Repeated, interleaved bench-line sweep: SWEEP="args;args;..." REPS=n
# (200 steps each, no CPU baseline / queue child / lanes-1 pass)
IFS=';' read -ra CASES <<< "$SWEEP"
for rep in $(seq 1 ${REPS:-3}); do
  for args in "${CASES[@]}"; do
    timeout -k 10 150 python -u bench.py --steps ${STEPS:-200} --warmup 10 --no-cpu-baseline --lanes1-steps 0 --no-queue-compare $args > gpurun_out/rsw.log 2>&1 || { tail -5 gpurun_out/rsw.log; exit 1; }
    python -c "
import json
for l in open('gpurun_out/rsw.log'):
    if l.startswith('{\"metric'):
        d=json.loads(l); print('[$args] rep $rep', d['value'], {k: round(v,3) for k,v in d['stages_ms'].items() if k in ('entropy','idct','output')})"
  done
done

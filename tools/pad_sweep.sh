#!/bin/bash
# bench value and entropy stage time over entropy LDS padding (CU packing) x lanes.
for cfg in "--lanes 1" "--lanes 1 --entropy-lds-pad 27000" "--lanes 2" "--lanes 2 --entropy-lds-pad 27000" $EXTRA; do
  timeout -k 10 120 python bench.py --steps 200 --no-cpu-baseline $cfg > gpurun_out/p.log 2>&1 || { tail -5 gpurun_out/p.log; exit 1; }
  python -c "
import json
for l in open('gpurun_out/p.log'):
    if l.startswith('{\"metric'):
        d=json.loads(l); print('$cfg', d['value'], d['stages_ms'])"
done

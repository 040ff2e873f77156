#!/bin/bash
# entropy stage time (lanes 1) over slot size x warm-up slots
for sw in "256 16" "256 12" "384 11" "384 8" "512 8" "512 6" "512 10" "768 5" "1024 4"; do
  set -- $sw
  timeout -k 10 120 python bench.py --steps 100 --no-cpu-baseline --lanes 1 --sub-bits $1 --warm-slots $2 > gpurun_out/s.log 2>&1 || { tail -5 gpurun_out/s.log; exit 1; }
  python -c "
import json
for l in open('gpurun_out/s.log'):
    if l.startswith('{\"metric'):
        d=json.loads(l); print('sub_bits $1 warm $2', d['value'], d['stages_ms']['entropy'])"
done

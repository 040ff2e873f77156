#!/bin/bash
# GPU tests, then bench lines for several entropy warm-up settings (A/B helper)
set -o pipefail
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for w in 0 2 3 5 8; do
  for lanes in 1 2; do
    timeout -k 10 100 python bench.py --steps 200 --no-cpu-baseline --warm-slots $w --lanes $lanes > gpurun_out/l.log 2>&1 || { tail -5 gpurun_out/l.log; exit 1; }
    python -c "
import json
for l in open('gpurun_out/l.log'):
    if l.startswith('{\"metric'):
        d=json.loads(l); print('warm $w lanes $lanes', d['value'], 'entropy', d['stages_ms']['entropy'])"
  done
done

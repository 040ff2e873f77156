#!/bin/bash
# Throughput by pipeline lane count (GPU box): bash tools/lanes_sweep.sh "3 4 5 6 8"
mkdir -p gpurun_out
for l in ${1:-3 4 5 6 8}; do
  timeout -k 10 120 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --lanes $l \
    > gpurun_out/lanes_$l.log 2>&1
  rc=$?
  echo "lanes $l rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/lanes_$l.log) $(grep -o '"entropy": [0-9.]*' gpurun_out/lanes_$l.log)"
  [ $rc -ge 124 ] && exit $rc
done
exit 0

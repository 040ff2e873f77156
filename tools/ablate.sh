#!/bin/bash
# Throughput with whole stages removed (timing ablations, outputs wrong):
# the marginal cost of each kernel under the 4-lane schedule.
# usage (GPU box): bash tools/ablate.sh ["extra bench args"]
mkdir -p gpurun_out
for m in ${MASKS:-0 0x10000 0x20000 0x40000 0x70000 0x1000 0x2000}; do
  timeout -k 10 120 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline \
    --debug-mask $((m)) $1 > gpurun_out/ablate_$m.log 2>&1
  rc=$?
  v=$(grep -o '"value": [0-9.]*' gpurun_out/ablate_$m.log)
  st=$(grep -o '"stages_ms": {[^}]*}' gpurun_out/ablate_$m.log)
  echo "mask $m rc=$rc $v $st"
  [ $rc -ge 124 ] && exit $rc
done
exit 0

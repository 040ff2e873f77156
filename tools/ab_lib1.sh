#!/bin/bash
# standalone (one lane) stage times and 4-lane rates of two builds:
# LIBS="label=path label=path" (path "" = in-tree)
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
for lv in $LIBS; do
  l=${lv%%=*}; p=${lv#*=}
  if [ -n "$p" ]; then export SPDL_AMD_LIB=$p; else unset SPDL_AMD_LIB; fi
  for lanes in 1 4; do
  timeout -k 10 200 python -u bench.py --steps ${STEPS:-100} --warmup 10 --lanes $lanes --no-cpu-baseline --no-queue-compare --lanes1-steps 0 $EXTRA > gpurun_out/ab1_$l.json 2>&1 || { tail -5 gpurun_out/ab1_$l.json; exit 3; }
  python -c "import json; r=json.loads(open('gpurun_out/ab1_$l.json').read().splitlines()[-1]); print('$l lanes $lanes rep $rep', r['value'], {k: round(x,4) for k,x in r['stages_ms'].items() if k in ('destuff','entropy','idct','output')})"
  done
done; done

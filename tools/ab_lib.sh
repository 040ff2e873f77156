#!/bin/bash
# A/B of two library builds on the configs[1] bench (alternating, REPS reps):
# LIBS="label=path label=path" (path "" = the in-tree library)
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-3}); do
for lv in $LIBS; do
  l=${lv%%=*}; p=${lv#*=}
  if [ -n "$p" ]; then export SPDL_AMD_LIB=$p; else unset SPDL_AMD_LIB; fi
  timeout -k 10 200 python -u bench.py --steps ${STEPS:-200} --warmup 10 --no-cpu-baseline --no-queue-compare --lanes1-steps ${L1:-0} $EXTRA > gpurun_out/ablib_$l.json 2>&1 || { tail -5 gpurun_out/ablib_$l.json; exit 3; }
  python -c "import json; r=json.loads(open('gpurun_out/ablib_$l.json').read().splitlines()[-1]); print('$l rep $rep', r['value'], {k: round(x,3) for k,x in r['stages_ms'].items() if k in ('destuff','entropy','idct','output')}, r['roofline']['lanes1'] and r['roofline']['lanes1']['kernel_ms'])"
done; done

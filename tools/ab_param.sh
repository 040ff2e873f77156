#!/bin/bash
# A/B of one decoder parameter on the configs[1] bench: PARAM=name VALUES="a b c"
# (alternating order, REPS repetitions, 200 steps each)
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
for v in $VALUES; do
  timeout -k 10 200 python -u bench.py --steps ${STEPS:-200} --warmup 10 --no-cpu-baseline --no-queue-compare --lanes1-steps ${L1:-0} --param $PARAM=$v $EXTRA > gpurun_out/ab_$PARAM$v.json 2>&1 || { tail -5 gpurun_out/ab_$PARAM$v.json; exit 3; }
  python -c "import json; r=json.loads(open('gpurun_out/ab_$PARAM$v.json').read().splitlines()[-1]); print('$PARAM=$v rep $rep', r['value'], {k: round(x,3) for k,x in r['stages_ms'].items() if k in ('entropy','idct','output')}, r['roofline']['lanes1'] and r['roofline']['lanes1']['kernel_ms'], r['oracle_check'][:12])"
done; done

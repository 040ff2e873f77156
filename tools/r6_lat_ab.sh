#!/bin/bash
# Per-stage latency of one synchronous batch at one lane (HIP events on
# every stage), r04 vs current build, REPS reps alternating.
mkdir -p gpurun_out/r6lat
for rep in $(seq 1 ${REPS:-2}); do
for lv in "cur=" "r04=spdl_amd/lib/variants/libspdl_hipjpeg_r04.so"; do
  l=${lv%%=*}; p=${lv#*=}
  if [ -n "$p" ]; then export SPDL_AMD_LIB=$p; else unset SPDL_AMD_LIB; fi
  timeout -k 10 150 python -u bench.py --steps 60 --warmup 10 --lanes ${LANES:-1} --sync-steps --timed-events stages \
    --no-cpu-baseline --no-queue-compare --lanes1-steps 0 --oracle-check 4 > gpurun_out/r6lat/${l}_$rep.json 2>&1 || { tail -5 gpurun_out/r6lat/${l}_$rep.json; exit 3; }
  python -c "import json; r=json.loads(open('gpurun_out/r6lat/${l}_$rep.json').read().splitlines()[-1]); print('$l', $rep, r['ms_per_step'], {k: round(v,4) for k,v in r['stages_ms'].items()}, r['host_submit_ms'])"
done; done

#!/bin/bash
# swscale kernel alone (one lane, synchronous batches): old vs new build, band groups
mkdir -p gpurun_out
run() {  # label, env, args
  timeout -k 10 200 env $2 python -u bench.py --steps 60 --warmup 5 --lanes 1 --no-cpu-baseline --no-queue-compare --lanes1-steps 0 $3 > gpurun_out/sa.json 2>&1 || { tail -5 gpurun_out/sa.json; exit 3; }
  python -c "import json; r=json.loads(open('gpurun_out/sa.json').read().splitlines()[-1]); print('$1', r['value'], {k: round(x,4) for k,x in r['stages_ms'].items() if k in ('entropy','idct','output')})"
}
run old SPDL_AMD_LIB=spdl_amd/lib/variants/libspdl_hipjpeg_old.so ""
for g in 1 2 4 8 64; do run "group $g" X=1 "--param sws_band_group=$g"; done
run old4 SPDL_AMD_LIB=spdl_amd/lib/variants/libspdl_hipjpeg_old.so "--lanes 4"

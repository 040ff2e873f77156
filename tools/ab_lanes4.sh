#!/bin/bash
# A/B bench lines (lanes 4, 200 steps, and the driver's 20-step run) of variant libraries
set -o pipefail
for v in $VARIANTS; do
  lib=spdl_amd/lib/libspdl_hipjpeg.so
  [ "$v" != base ] && lib=spdl_amd/lib/variants/libspdl_hipjpeg_$v.so
  for args in "--steps 200" "--steps 20 --warmup 5"; do
    SPDL_AMD_LIB=$lib timeout -k 10 150 python -u bench.py --no-cpu-baseline --lanes1-steps 0 $args > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python -c "
import json
for l in open('gpurun_out/ab.log'):
    if l.startswith('{\"metric'):
        d=json.loads(l); print('$v [$args]', d['value'], {k: round(v,3) for k,v in d['stages_ms'].items() if k in ('entropy','idct','output')})"
  done
done

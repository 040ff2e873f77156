#!/bin/bash
# A/B of entropy phase timers and bench lines: VARIANTS="nobb ..." bash tools/ab_phases.sh
set -o pipefail
for v in $VARIANTS; do
  SPDL_AMD_LIB=spdl_amd/lib/variants/libspdl_hipjpeg_$v.so timeout -k 10 150 python tools/debug/phases.py > gpurun_out/ph_$v.log 2>&1 || { tail -5 gpurun_out/ph_$v.log; exit 1; }
  echo "variant $v"; cat gpurun_out/ph_$v.log
  for l in 4 1; do
    SPDL_AMD_LIB=spdl_amd/lib/variants/libspdl_hipjpeg_$v.so timeout -k 10 150 python -u bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-queue-compare --lanes1-steps 0 --lanes $l > gpurun_out/b_${v}_l$l.log 2>&1 || { tail -5 gpurun_out/b_${v}_l$l.log; exit 1; }
    python -c "
import json
for l in open('gpurun_out/b_${v}_l$l.log'):
    if l.startswith('{\"metric'):
        d=json.loads(l); print('  lanes $l', d['value'], {k: round(v,3) for k,v in d['stages_ms'].items()})"
  done
done

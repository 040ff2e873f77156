#!/bin/bash
# A/B of library variants: entropy phases + bench lines (lanes 1 and 4) per
# library.  usage (GPU box): bash tools/ab_libs.sh lib1.so lib2.so ...
set -o pipefail
mkdir -p gpurun_out
for lib in "$@"; do
  echo "== $lib"
  SPDL_AMD_LIB=$lib timeout -k 10 120 python tools/entropy_phases.py > gpurun_out/ph.log 2>&1 || { tail -5 gpurun_out/ph.log; exit 1; }
  cat gpurun_out/ph.log
  for lanes in 1 4; do
    SPDL_AMD_LIB=$lib timeout -k 10 200 python bench.py --steps 200 --no-cpu-baseline --lanes $lanes --lanes1-steps 0 > gpurun_out/l.log 2>&1 || { tail -5 gpurun_out/l.log; exit 1; }
    python -c "
import json
for l in open('gpurun_out/l.log'):
    if l.startswith('{\"metric'):
        d=json.loads(l); print('lanes $lanes', d['value'], {k: round(v, 3) for k, v in d['stages_ms'].items()})"
  done
done

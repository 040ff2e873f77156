#!/bin/bash
# GPU test suite, entropy phase timings and two bench lines (A/B loop helper).
set -o pipefail
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
timeout -k 10 120 python tools/debug/debug_phases3.py > gpurun_out/ph.log 2>&1 || exit 1
grep "T=512" gpurun_out/ph.log
for cfg in "--lanes 2" "--lanes 1"; do
  timeout -k 10 120 python bench.py --steps 200 --no-cpu-baseline $cfg > gpurun_out/l.log 2>&1 || { tail -5 gpurun_out/l.log; exit 1; }
  python -c "
import json
for l in open('gpurun_out/l.log'):
    if l.startswith('{\"metric'):
        d=json.loads(l); print('$cfg', d['value'], d['stages_ms'])"
done
# optional A/B: bench lines of each variant library given in $VARIANTS
for v in $VARIANTS; do
  SPDL_AMD_LIB=spdl_amd/lib/variants/libspdl_hipjpeg_$v.so timeout -k 10 120 python bench.py --steps 200 --no-cpu-baseline > gpurun_out/l.log 2>&1 || { tail -5 gpurun_out/l.log; exit 1; }
  python -c "
import json
for l in open('gpurun_out/l.log'):
    if l.startswith('{\"metric'):
        d=json.loads(l); print('variant $v', d['value'], d['stages_ms'])"
done

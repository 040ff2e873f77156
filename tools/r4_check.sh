#!/bin/bash
# round-4 GPU check: parity tests first, then phase timers and bench lines
# (BASE=1: also the phase timers of spdl_amd/lib/variants/libspdl_hipjpeg_base.so)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_par.log 2>&1 || { echo "parity failed"; tail -40 gpurun_out/t_par.log; exit 1; }
tail -1 gpurun_out/t_par.log
timeout -k 10 150 python tools/debug/phases.py > gpurun_out/ph.log 2>&1 || { tail -20 gpurun_out/ph.log; exit 1; }
cat gpurun_out/ph.log
if [ -n "$BASE" ]; then
SPDL_AMD_LIB=spdl_amd/lib/variants/libspdl_hipjpeg_base.so timeout -k 10 150 python tools/debug/phases.py > gpurun_out/ph_base.log 2>&1 || { tail -20 gpurun_out/ph_base.log; exit 1; }
echo base; cat gpurun_out/ph_base.log
fi
for l in 4 1; do
timeout -k 10 150 python -u bench.py --steps 200 --warmup 10 --no-cpu-baseline --lanes $l > gpurun_out/b_l$l.log 2>&1 || { tail -20 gpurun_out/b_l$l.log; exit 1; }
python -c "
import json
for l in open('gpurun_out/b_l$l.log'):
    if l.startswith('{\"metric'):
        d=json.loads(l); print('lanes $l', d['value'], {k: round(v,3) for k,v in d['stages_ms'].items()})"
done
if [ -n "$FULL" ]; then
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { echo "suite failed"; tail -40 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
fi

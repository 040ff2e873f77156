#!/bin/bash
# single-image entropy phase timings per variant library:
# VARIANTS="base x" bash tools/phase_ab.sh
mkdir -p gpurun_out
for v in $VARIANTS; do
  lib=spdl_amd/lib/libspdl_hipjpeg.so
  [ "$v" != base ] && lib=spdl_amd/lib/variants/libspdl_hipjpeg_$v.so
  echo "== $v"
  SPDL_AMD_LIB=$lib timeout -k 10 200 python -u tools/debug/debug_phases_bench.py > gpurun_out/ph_$v.log 2>&1
  rc=$?; head -3 gpurun_out/ph_$v.log; [ $rc -ne 0 ] && exit $rc
done
exit 0

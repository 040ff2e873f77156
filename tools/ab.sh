#!/bin/bash
# A/B bench of variant libraries (make -C spdl_amd/csrc variant NAME=x DEFS=...):
# VARIANTS="base x y" bash tools/ab.sh ["extra bench args"]; "base" = the default build.
mkdir -p gpurun_out
for v in $VARIANTS; do
  lib=spdl_amd/lib/libspdl_hipjpeg.so
  [ "$v" != base ] && lib=spdl_amd/lib/variants/libspdl_hipjpeg_$v.so
  for l in 1 2; do
    SPDL_AMD_LIB=$lib timeout -k 10 150 python -u bench.py --steps 60 --warmup 5 --no-cpu-baseline --lanes $l $1 > gpurun_out/ab_${v}_l$l.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "variant $v lanes $l rc=$rc"; tail -5 gpurun_out/ab_${v}_l$l.log; [ $rc -ge 124 ] && exit $rc; fi
  done
done
python tools/stages.py "gpurun_out/ab_*.log"

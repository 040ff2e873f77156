#!/bin/bash
# Output-stage A/B: for each variant library, 1-lane bench lines with the
# sws_kernel ablation masks (0 = full, 256 = no H pass, 512 = no V pass,
# 1024 = no tile store, 1792 = none).  VARIANTS="base g16" bash tools/sws_ab.sh
mkdir -p gpurun_out
for v in $VARIANTS; do
  lib=spdl_amd/lib/libspdl_hipjpeg.so
  [ "$v" != base ] && lib=spdl_amd/lib/variants/libspdl_hipjpeg_$v.so
  for m in ${MASKS:-0 256 512 1024 1792}; do
    SPDL_AMD_LIB=$lib timeout -k 10 150 python -u bench.py --steps 60 --warmup 5 --no-cpu-baseline \
      --lanes 1 --oracle-check 0 --debug-mask $m > gpurun_out/sab_${v}_m$m.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "variant $v mask $m rc=$rc"; tail -5 gpurun_out/sab_${v}_m$m.log; [ $rc -ge 124 ] && exit $rc; fi
  done
done
python tools/stages.py "gpurun_out/sab_*.log"

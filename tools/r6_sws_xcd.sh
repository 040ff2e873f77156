#!/bin/bash
# XCD-aware tile order (round 6, "xcd_order": bit 0 sws_kernel, bit 1
# idct_kernel): knob parity, then one-lane stage latency, the driver's command
# and the mixed set at four lanes by variant.
set -o pipefail
mkdir -p gpurun_out/r6xcd
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_knobs.py tests/test_gpu_parity.py > gpurun_out/r6xcd/tests.log 2>&1 \
  || { tail -20 gpurun_out/r6xcd/tests.log; exit 3; }
tail -2 gpurun_out/r6xcd/tests.log
V=${V:-"x0||--param xcd_order=0;x1||--param xcd_order=1;x3||--param xcd_order=3;i128|SPDL_AMD_LIB=spdl_amd/lib/variants/libspdl_hipjpeg_idct128.so|--param xcd_order=1"}
VARIANTS="$V" REPS=2 OUT=gpurun_out/r6xcd/stage_lanes1.txt bash tools/r6_stage_ab.sh || exit 3
VARIANTS="$V" REPS=2 WORKLOAD=mixed OUT=gpurun_out/r6xcd/stage_mixed.txt bash tools/r6_stage_ab.sh || exit 3
VARIANTS="$V" REPS=3 OUT=gpurun_out/r6xcd/driver.txt bash tools/r6_driver_ab.sh || exit 3
MV=$(echo "$V" | sed 's/|--param/|--workload mixed --param/g')
VARIANTS="$MV" REPS=3 STEPS=100 OUT=gpurun_out/r6xcd/mixed4.txt bash tools/r6_driver_ab.sh || exit 3

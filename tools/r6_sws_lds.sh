#!/bin/bash
# swscale LDS budget (tile height) with the XCD-aware order (round 6):
# variant builds -DHJ_SWS_LDS_KB=24/48/64 vs the default 32 -- swscale
# parity on each, then one-lane stage latency and the driver's command.
set -o pipefail
mkdir -p gpurun_out/r6lds
for k in 24 48 64; do
  SPDL_AMD_LIB=spdl_amd/lib/variants/libspdl_hipjpeg_lds$k.so timeout -k 10 300 python -u -m pytest -x -q \
    --timeout 120 --timeout-method thread tests/test_gpu_swscale.py tests/test_gpu_parity.py \
    > gpurun_out/r6lds/tests_$k.log 2>&1 || { tail -20 gpurun_out/r6lds/tests_$k.log; exit 3; }
  echo "lds $k: $(tail -1 gpurun_out/r6lds/tests_$k.log)"
done
V="l32||;l24|SPDL_AMD_LIB=spdl_amd/lib/variants/libspdl_hipjpeg_lds24.so|;l48|SPDL_AMD_LIB=spdl_amd/lib/variants/libspdl_hipjpeg_lds48.so|;l64|SPDL_AMD_LIB=spdl_amd/lib/variants/libspdl_hipjpeg_lds64.so|"
VARIANTS="$V" REPS=2 OUT=gpurun_out/r6lds/stage_lanes1.txt bash tools/r6_stage_ab.sh || exit 3
VARIANTS="$V" REPS=3 OUT=gpurun_out/r6lds/driver.txt bash tools/r6_driver_ab.sh || exit 3

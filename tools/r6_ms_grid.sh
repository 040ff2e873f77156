#!/bin/bash
# Multi-scan launch of a batch known to hold no multi-scan image (round 6,
# "ms_skip_empty": 0 = the full 256-workgroup launch, 1 = no launch, 2 = one
# workgroup -- the build of commit a33d1dc only): knob parity, then the
# driver's command and 200-step runs.
set -o pipefail
mkdir -p gpurun_out/r6ms
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_knobs.py > gpurun_out/r6ms/tests.log 2>&1 || { tail -20 gpurun_out/r6ms/tests.log; exit 3; }
tail -2 gpurun_out/r6ms/tests.log
V="m0||--param ms_skip_empty=0;m1||--param ms_skip_empty=1;m2||--param ms_skip_empty=2"
VARIANTS="$V" REPS=3 OUT=gpurun_out/r6ms/driver.txt bash tools/r6_driver_ab.sh || exit 3
VARIANTS="$V" REPS=2 STEPS=200 WARM=10 OUT=gpurun_out/r6ms/steps200.txt bash tools/r6_driver_ab.sh || exit 3
MV=$(echo "$V" | sed 's/|--param/|--workload mixed --param/g')
VARIANTS="$MV" REPS=2 STEPS=100 OUT=gpurun_out/r6ms/mixed4.txt bash tools/r6_driver_ab.sh || exit 3

#!/bin/bash
# round 6: new hand-off / cap / knob tests, then the driver-command A/B
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pieces.py tests/test_gpu_knobs.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_r6_pieces.log 2>&1
rc=$?; tail -5 gpurun_out/t_r6_pieces.log; [ $rc -eq 0 ] || exit $rc
REPS=3 VARIANTS="cur||;cursync||--warmup-mode sync;noev||--timed-events off;r04|SPDL_AMD_LIB=spdl_amd/lib/variants/libspdl_hipjpeg_r04.so|--warmup-mode sync" bash tools/r6_driver_ab.sh

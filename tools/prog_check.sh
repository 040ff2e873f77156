#!/bin/bash
# progressive decoder step: the multi-scan / parity GPU tests, then the
# per-scan phase timer and the device-resident stream (each step
# time-limited; a failure stops the script)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_multiscan.py tests/test_gpu_parity.py} -x -q -rf --timeout 240 --timeout-method thread > gpurun_out/t_prog.log 2>&1
rc=$?; tail -4 gpurun_out/t_prog.log; echo "tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/prog_phases.py > gpurun_out/prog_phases.txt 2>&1 || exit 3
grep -E "progressive=True|scan 9|scan 5|scan 1:" gpurun_out/prog_phases.txt | head -12
timeout -k 10 400 python -u tools/prog_device.py ${PD_STEPS:-30} > gpurun_out/prog_device.txt 2>&1 || exit 4
cat gpurun_out/prog_device.txt

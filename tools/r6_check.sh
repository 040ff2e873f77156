#!/bin/bash
# round 6: full -m gpu suite, then the driver's bench command and the mixed workload
mkdir -p gpurun_out/r6
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6/t_full.log 2>&1
rc=$?; tail -3 gpurun_out/r6/t_full.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6/bench_driver.json 2>&1 || exit 3
tail -1 gpurun_out/r6/bench_driver.json | cut -c1-400
SWEEP=";--workload mixed;--workload mixed --lanes 1;--lanes 1" bash tools/sweep.sh

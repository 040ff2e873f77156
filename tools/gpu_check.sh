#!/bin/bash
# GPU round trip: -m gpu tests, then (unless the tests crashed the process --
# abort / segfault / timeout, exit codes other than 0/1) one bench line.
# Usage (on the GPU box, via gpurun): bash tools/gpu_check.sh [pytest -k expr]
mkdir -p gpurun_out
K=${1:+-k "$1"}
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread $K \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests.log
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
brc=$?
cat gpurun_out/bench.json
tail -3 gpurun_out/bench.err
echo "bench rc=$brc"
exit $rc

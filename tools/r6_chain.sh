#!/bin/bash
# chain rounds: parity, per-image phases of the mixed set, bench lines
mkdir -p gpurun_out/chain
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py -x -v --timeout 120 --timeout-method thread > gpurun_out/chain/tests.log 2>&1
rc=$?; tail -3 gpurun_out/chain/tests.log; [ $rc -eq 0 ] || exit $rc
for c in 0 2 1; do
  PH_CHAIN=$c timeout -k 10 200 python -u tools/debug/phases_mixed.py > gpurun_out/chain/phases_c$c.log 2>&1 || exit 3
  echo "chain_after=$c"; tail -4 gpurun_out/chain/phases_c$c.log
done
SWEEP="--param chain_after=0;--param chain_after=2;--workload mixed --param chain_after=0;--workload mixed --param chain_after=2;--workload mixed --param chain_after=1;--workload mixed --lanes 1 --param chain_after=0;--workload mixed --lanes 1 --param chain_after=2;--workload mixed --lanes 1 --param chain_after=1;--lanes 1 --param chain_after=0;--lanes 1 --param chain_after=2" bash tools/sweep.sh
SPDL_AMD_LIB=spdl_amd/lib/variants/libspdl_hipjpeg_head.so SWEEP=";--workload mixed;--lanes 1" bash tools/sweep.sh

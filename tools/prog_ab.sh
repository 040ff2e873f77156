#!/bin/bash
# Progressive decoder: the multi-scan GPU tests, then per-phase timings and
# batch throughput of the current library against an A/B variant.
# Usage (GPU box): bash tools/prog_ab.sh [variant-name]
mkdir -p gpurun_out
V=${1:-old}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "prog or multiscan or Multiscan" \
  --timeout 240 --timeout-method thread > gpurun_out/prog_tests.log 2>&1
rc=$?
tail -5 gpurun_out/prog_tests.log
echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/prog_phases.py > gpurun_out/prog_phases_new.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/prog_bench.py > gpurun_out/prog_bench_new.txt 2>&1 || exit $?
SPDL_AMD_LIB=spdl_amd/lib/variants/libspdl_hipjpeg_$V.so timeout -k 10 200 python -u tools/prog_phases.py \
  > gpurun_out/prog_phases_$V.txt 2>&1 || exit $?
SPDL_AMD_LIB=spdl_amd/lib/variants/libspdl_hipjpeg_$V.so timeout -k 10 200 python -u tools/prog_bench.py \
  > gpurun_out/prog_bench_$V.txt 2>&1 || exit $?
tail -n 20 gpurun_out/prog_phases_new.txt gpurun_out/prog_bench_new.txt gpurun_out/prog_phases_$V.txt \
  gpurun_out/prog_bench_$V.txt

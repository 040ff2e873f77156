#!/bin/bash
# Entropy descriptors stored in 16-byte pairs (round 6, variant build
# -DHJ_DESC_PAIRS=1, `make variant NAME=dpair DEFS=-DHJ_DESC_PAIRS=1`):
# entropy parity tests on the variant, a WRITE_SIZE pass of each library,
# then one-lane stage latency and the driver's command, alternating.
set -o pipefail
VL=spdl_amd/lib/variants/libspdl_hipjpeg_dpair.so
mkdir -p gpurun_out/r6dp
SPDL_AMD_LIB=$VL timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_pieces.py tests/test_gpu_chain.py tests/test_gpu_corrupt.py tests/test_gpu_entropy_edges.py tests/test_gpu_configs.py \
  > gpurun_out/r6dp/tests.log 2>&1 || { tail -20 gpurun_out/r6dp/tests.log; exit 3; }
tail -2 gpurun_out/r6dp/tests.log
bash tools/pmc_passes.sh gpurun_out/r6dp/pmc_base "WRITE_SIZE" || exit 3
SPDL_AMD_LIB=$VL bash tools/pmc_passes.sh gpurun_out/r6dp/pmc_dpair "WRITE_SIZE" || exit 3
for v in base dpair; do
  python3 tools/pmc_traffic.py gpurun_out/r6dp/traffic_$v.json gpurun_out/r6dp/pmc_$v/pmc_1 gpurun_out/r6dp/pmc_$v/pmc_1 \
    > gpurun_out/r6dp/traffic_$v.txt 2>&1; grep entropy gpurun_out/r6dp/traffic_$v.txt | sed "s/^/$v /"
done
V="base||;dpair|SPDL_AMD_LIB=$VL|"
VARIANTS="$V" REPS=2 OUT=gpurun_out/r6dp/stage_lanes1.txt bash tools/r6_stage_ab.sh || exit 3
VARIANTS="$V" REPS=3 OUT=gpurun_out/r6dp/driver.txt bash tools/r6_driver_ab.sh || exit 3
VARIANTS="$V" REPS=2 STEPS=200 WARM=10 OUT=gpurun_out/r6dp/steps200.txt bash tools/r6_driver_ab.sh || exit 3

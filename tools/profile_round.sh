#!/bin/bash
# Round profile (GPU box): FETCH/WRITE calibration, PMC passes (traffic +
# SQ issue/wait), and rocprofv3 kernel-trace stats of the bench at 4 lanes
# and 1 lane.  usage: bash tools/profile_round.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/prof}
mkdir -p "$out"
bash tools/fetch_calib.sh "$out/calib" || exit 1
bash tools/pmc_round.sh "$out/pmc" || exit 1
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
sha256sum spdl_amd/lib/libspdl_hipjpeg.so | cut -d' ' -f1 > "$out/lib_sha256.txt"
for l in 4 1; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/ktrace_l$l" -o run --output-format csv \
    -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-queue-compare --lanes1-steps 0 --lanes $l \
    > "$out/ktrace_l$l.log" 2>&1 || { echo "kernel trace lanes $l failed"; exit 1; }
done
for w in mixed big1; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/ktrace_$w" -o run --output-format csv \
    -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-queue-compare --lanes1-steps 0 --workload $w \
    > "$out/ktrace_$w.log" 2>&1 || { echo "kernel trace $w failed"; exit 1; }
done
python3 tools/kernel_busy.py "$out/kernel_busy.json" \
  "4:$(find "$out/ktrace_l4" -name '*kernel_trace.csv' | head -1)" \
  "1:$(find "$out/ktrace_l1" -name '*kernel_trace.csv' | head -1)" > "$out/kernel_busy.txt" || exit 1
cat "$out/kernel_busy.txt"
python3 tools/pmc_traffic.py "$out/traffic.json" "$out/pmc/pmc_1" "$out/pmc/pmc_2" \
  --calib "$out/calib/calibration.json" > "$out/traffic.txt" || exit 1
cat "$out/traffic.txt" "$out/pmc/issue.txt" "$out/calib/calibration.txt"

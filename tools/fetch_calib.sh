#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration per access pattern (tools/fetch_calib.hip).
# usage (GPU box): bash tools/fetch_calib.sh OUTDIR
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=${1:-gpurun_out/calib}
mkdir -p "$out"
timeout -k 10 120 ./tools/fetch_calib > "$out/bytes.txt" || exit 1
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $c -d "$out/pmc_$i" -o run --output-format csv \
    -- ./tools/fetch_calib > "$out/pmc_$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 tools/fetch_calib_summary.py "$out" | tee "$out/calibration.txt"

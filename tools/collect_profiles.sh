#!/bin/bash
# copy a tools/profile_round.sh output dir into the committed profile set that
# bench.py reads: bash tools/collect_profiles.sh gpurun_out/prof_X profiles/r04/final
set -e
src=$1; d=$2
mkdir -p "$d/calib"
cp "$(find "$src/ktrace_l4" -name '*kernel_stats.csv' | head -1)" "$d/kernel_stats_lanes4.csv"
cp "$(find "$src/ktrace_l1" -name '*kernel_stats.csv' | head -1)" "$d/kernel_stats_lanes1.csv"
cp "$src/ktrace_l4.log" "$d/bench_under_ktrace_lanes4.log"
cp "$src/lib_sha256.txt" "$d/"
for w in mixed big1; do
  cp "$(find "$src/ktrace_$w" -name '*kernel_stats.csv' | head -1)" "$d/kernel_stats_$w.csv"
  cp "$src/ktrace_$w.log" "$d/bench_under_ktrace_$w.log"
done
cp "$src/ktrace_l1.log" "$d/bench_under_ktrace_lanes1.log"
cp "$src/kernel_busy.json" "$src/kernel_busy.txt" "$src/traffic.json" "$src/traffic.txt" "$d/"
cp "$src/pmc/issue.json" "$src/pmc/issue.txt" "$src/pmc/counters_summary.txt" "$d/"
cp "$src/calib/calibration.json" "$src/calib/calibration.txt" "$d/calib/"
[ -f "$src/calib/bytes.txt" ] && cp "$src/calib/bytes.txt" "$d/calib/"
echo "copied $src -> $d"

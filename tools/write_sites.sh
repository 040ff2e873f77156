#!/bin/bash
# Entropy write traffic by store site: WRITE_SIZE (raw KiB -> bytes) of the
# entropy kernel per launch under store-site ablations of the HJ_ABLATIONS
# library (outputs wrong; traffic only), 4 lanes and 1 lane.
# usage (GPU box): bash tools/write_sites.sh
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ws
LIB=spdl_amd/lib/variants/libspdl_hipjpeg_abl.so
for lanes in 4 1; do
for m in 0 0x4000 0x80000 0x8000 0x1000 0x84000; do
  d=gpurun_out/ws/l${lanes}_$m
  SPDL_AMD_LIB=$LIB timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $d -o run --output-format csv \
    -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-queue-compare --lanes1-steps 0 --lanes $lanes --debug-mask $((m)) > $d.log 2>&1 || { echo "mask $m rc=$?"; tail -3 $d.log; exit 1; }
  python3 - $d $m $lanes <<'PY'
import csv, glob, sys, re
d, m, lanes = sys.argv[1:]
v = []
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "entropy_kernel" in r["Kernel_Name"] and r["Counter_Name"] == "WRITE_SIZE":
            v.append(float(r["Counter_Value"]) * 1024)
print(f"lanes {lanes} mask {m:>8}: entropy WRITE_SIZE {sum(v)/len(v)/1e6:8.2f} MB per launch ({len(v)} launches)")
PY
done; done

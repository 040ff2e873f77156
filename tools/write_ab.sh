#!/bin/bash
# WRITE_SIZE / FETCH_SIZE per kernel for the default library and variants ($VARIANTS)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/wab
for v in default $VARIANTS; do
  lib=""; [ "$v" != default ] && lib=spdl_amd/lib/variants/libspdl_hipjpeg_$v.so
  for c in WRITE_SIZE FETCH_SIZE; do
    SPDL_AMD_LIB=$lib timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $c -d gpurun_out/wab/${v}_$c -o run --output-format csv \
      -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --oracle-check 0 > gpurun_out/wab/${v}_$c.log 2>&1 || { echo "pmc $v $c failed"; exit 1; }
  done
  python3 - "$v" <<'PY'
import csv, glob, sys, collections
v = sys.argv[1]
for c in ("WRITE_SIZE", "FETCH_SIZE"):
    f = glob.glob(f"gpurun_out/wab/{v}_{c}/**/*counter_collection.csv", recursive=True)
    agg = collections.defaultdict(list)
    for row in csv.DictReader(open(f[0])):
        agg[row["Kernel_Name"].split("(")[0]].append(float(row["Counter_Value"]))
    for k, xs in sorted(agg.items()):
        if "entropy" in k or "idct" in k:
            print(v, c, k[-40:], "per-dispatch KB-units mean", round(sum(xs) / len(xs), 1), "n", len(xs))
PY
done

#!/bin/bash
# repeated interleaved A/B of variant libraries (2-lane bench lines):
# VARIANTS="base p4" REPS=3 bash tools/ab_rep.sh ["extra bench args"]
mkdir -p gpurun_out/abr
for r in $(seq ${REPS:-3}); do
  for v in $VARIANTS; do
    lib=spdl_amd/lib/libspdl_hipjpeg.so
    [ "$v" != base ] && lib=spdl_amd/lib/variants/libspdl_hipjpeg_$v.so
    SPDL_AMD_LIB=$lib timeout -k 10 150 python -u bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-queue-compare --lanes1-steps 0 --oracle-check 0 $1 > gpurun_out/abr/${v}_r$r.log 2>&1 || { echo "fail $v"; exit 1; }
  done
done
python - <<'PY'
import glob, json, collections
vals = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/abr/*.log")):
    v = f.split("/")[-1].rsplit("_r", 1)[0]
    for line in open(f):
        if line.startswith("{"):
            vals[v].append(json.loads(line)["value"])
for v, xs in vals.items():
    print(f"{v:10s} mean {sum(xs)/len(xs):10.1f}  runs {xs}")
PY

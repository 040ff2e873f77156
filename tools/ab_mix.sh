#!/bin/bash
# Interleaved A/B of (library variant, bench args) pairs, REPS times.
# usage: REPS=3 bash tools/ab_mix.sh "name|variant|args" ...   (variant "base" = default build)
mkdir -p gpurun_out/abm
for r in $(seq ${REPS:-3}); do
  for spec in "$@"; do
    name=${spec%%|*}; rest=${spec#*|}; v=${rest%%|*}; args=${rest#*|}
    lib=spdl_amd/lib/libspdl_hipjpeg.so
    [ "$v" != base ] && lib=spdl_amd/lib/variants/libspdl_hipjpeg_$v.so
    SPDL_AMD_LIB=$lib timeout -k 10 150 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline \
      --oracle-check 0 $args > gpurun_out/abm/${name}_r$r.log 2>&1 || { echo "fail $name rc=$?"; exit 1; }
  done
done
python - <<'PY'
import glob, json, collections
vals = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/abm/*.log")):
    v = f.split("/")[-1].rsplit("_r", 1)[0]
    for line in open(f):
        if line.startswith("{"):
            vals[v].append(json.loads(line)["value"])
for v, xs in vals.items():
    print(f"{v:12s} mean {sum(xs)/len(xs):10.1f}  runs {xs}")
PY

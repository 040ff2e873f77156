#!/bin/bash
# Bench lines for several argument sets (A/B helper).  Each line of $SWEEP is
# one set of bench.py arguments; prints value + entropy stage per set.
# Usage (GPU box): SWEEP=$'--warm-slots 8\n--warm-slots 12' bash tools/sweep_args.sh
mkdir -p gpurun_out
REP=${REP:-1}
while IFS= read -r args; do
  [ -z "$args" ] && continue
  lib=""
  if [[ "$args" == lib:* ]]; then
    name=${args%% *}; name=${name#lib:}; args=${args#* }; [ "$args" == "lib:$name" ] && args=""
    lib=spdl_amd/lib/variants/libspdl_hipjpeg_$name.so
  fi
  for r in $(seq $REP); do
    SPDL_AMD_LIB=$lib timeout -k 10 120 python bench.py --steps ${STEPS:-200} --no-cpu-baseline --oracle-check 0 $args > gpurun_out/sw.log 2>&1 || { echo "FAILED: $args"; tail -5 gpurun_out/sw.log; exit 1; }
    python - "$lib $args" <<'PY'
import json, sys
for l in open('gpurun_out/sw.log'):
    if l.startswith('{"metric'):
        d = json.loads(l)
        print(f"{sys.argv[1]:50s} {d['value']:10.0f} entropy {d['stages_ms']['entropy']:.3f} ms/step {d['ms_per_step']:.4f}", flush=True)
PY
  done
done <<< "$SWEEP"

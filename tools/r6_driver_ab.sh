#!/bin/bash
# Same-box A/B on the driver's exact command (--gpus 1 --steps 20 --warmup 5),
# alternating variants, REPS reps: VARIANTS="label|env|extra-args;..."
# (env: SPDL_AMD_LIB=path or empty).  One summary line per run.
mkdir -p gpurun_out/r6ab
OUT=${OUT:-gpurun_out/r6ab/summary.txt}
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
IFS=';' read -ra VS <<< "$VARIANTS"
for rep in $(seq 1 ${REPS:-3}); do
  for v in "${VS[@]}"; do
    IFS='|' read -r label envs extra <<< "$v"
    log=gpurun_out/r6ab/${label}_$rep.json
    env $envs timeout -k 10 150 python -u bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARM:-5} \
      --no-cpu-baseline --no-queue-compare --lanes1-steps 0 --oracle-check 8 $extra > "$log" 2>&1 \
      || { echo "FAIL $label"; tail -5 "$log"; exit 3; }
    python - "$label" "$rep" "$log" >> "$OUT" <<'EOF'
import json, sys
r = json.loads([l for l in open(sys.argv[3]) if l.startswith('{"metric"')][-1])
st = {k: round(v, 3) for k, v in r["stages_ms"].items() if k in ("entropy", "idct", "output")}
print(sys.argv[1], "rep", sys.argv[2], r["value"], r["ms_per_step"], st, flush=True)
EOF
    tail -1 "$OUT"
  done
done

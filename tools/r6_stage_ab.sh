#!/bin/bash
# Per-stage latency of one synchronous batch (HIP events on every stage) by
# variant, REPS reps alternating: VARIANTS="label|env|extra-args;..."
# (LANES, default 1; WORKLOAD, default pad224).  One summary line per run.
mkdir -p gpurun_out/r6stage
OUT=${OUT:-gpurun_out/r6stage/summary.txt}
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
IFS=';' read -ra VS <<< "$VARIANTS"
for rep in $(seq 1 ${REPS:-2}); do
  for v in "${VS[@]}"; do
    IFS='|' read -r label envs extra <<< "$v"
    log=gpurun_out/r6stage/${label}_$rep.json
    env $envs timeout -k 10 150 python -u bench.py --steps ${STEPS:-60} --warmup 10 --lanes ${LANES:-1} \
      --sync-steps --timed-events stages --workload ${WORKLOAD:-pad224} --no-cpu-baseline \
      --no-queue-compare --lanes1-steps 0 --oracle-check 4 $extra > "$log" 2>&1 \
      || { echo "FAIL $label"; tail -5 "$log"; exit 3; }
    python - "$label" "$rep" "$log" >> "$OUT" <<'EOF'
import json, sys
r = json.loads([l for l in open(sys.argv[3]) if l.startswith('{"metric"')][-1])
st = {k: round(v, 4) for k, v in r["stages_ms"].items()}
print(sys.argv[1], "rep", sys.argv[2], r["ms_per_step"], st, flush=True)
EOF
    tail -1 "$OUT"
  done
done

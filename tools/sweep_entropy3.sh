#!/bin/bash
# 1-lane entropy stage time over slot size (sub_bits) x warm-up slots
B="python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --lanes 1 --oracle-check 0"
mkdir -p gpurun_out/sw3
for sb in ${SUBS:-256 384 512 768 1024}; do
  for w in ${WARMS:-2 4 6 8 12}; do
    timeout -k 10 120 $B --sub-bits $sb --warm-slots $w > gpurun_out/sw3/s${sb}_w$w.log 2>&1 || { echo "fail $sb $w"; exit 1; }
  done
done
python - <<'PY'
import glob, json, re
rows = []
for f in glob.glob("gpurun_out/sw3/*.log"):
    for line in open(f):
        if line.startswith("{"):
            r = json.loads(line)
            m = re.search(r"s(\d+)_w(\d+)", f)
            rows.append((r["stages_ms"]["entropy"], int(m.group(1)), int(m.group(2)), r["value"]))
for e, sb, w, v in sorted(rows):
    print(f"sub_bits {sb:5d} warm {w:3d} entropy {e:.4f} ms  value {v}")
PY

"""Print value + stage timings of the bench JSON lines in gpurun_out/*.log."""
import glob
import json
import sys

for f in sorted(glob.glob(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/b_*.log")):
    for line in open(f):
        if line.startswith('{"metric'):
            d = json.loads(line)
            print(f"{f:28s} {d['value']:10.1f}", {k: round(v, 3) for k, v in d["stages_ms"].items()})

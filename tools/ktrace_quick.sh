#!/bin/bash
# rocprofv3 kernel-trace stats of the bench at 4 lanes and 1 lane (GPU box).
# usage: bash tools/ktrace_quick.sh OUTDIR [bench args...]
out=${1:-gpurun_out/ktq}; shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
for l in 4 1; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/l$l" -o run --output-format csv \
    -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --lanes1-steps 0 --lanes $l "$@" \
    > "$out/l$l.log" 2>&1 || { echo "kernel trace lanes $l failed"; tail -5 "$out/l$l.log"; exit 1; }
  f=$(find "$out/l$l" -name "*kernel_stats.csv" | head -1)
  echo "== lanes $l: $(tail -1 $out/l$l.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  python3 -c "
import csv,re,sys
for r in csv.DictReader(open('$f')):
    n=re.sub(r'\(.*','',r['Name']).replace('void ','')
    print(f\"  {n:40s} {int(r['Calls']):5d} {float(r['AverageNs'])/1000:9.1f} us\")"
done

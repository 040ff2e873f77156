#!/bin/bash
# rocprofv3 over the progressive decoder (tools/prog_one.py: 256-image
# progressive batches): kernel-trace stats, then the SQ counter passes of
# tools/prog_pmc.sh.  Output: gpurun_out/prog_prof/
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/prog_prof
mkdir -p $out
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $out/kt -o run --output-format csv \
  -- python3 tools/prog_one.py 256 3 > $out/kt.log 2>&1 || { echo "kernel trace failed"; tail -5 $out/kt.log; exit 1; }
f=$(find $out/kt -name "*kernel_stats.csv" | head -1)
cp "$f" $out/kernel_stats.csv
python3 -c "
import csv,re
for r in csv.DictReader(open('$out/kernel_stats.csv')):
    n=re.sub(r'\(.*','',r['Name']).replace('void ','')
    print(f\"  {n:40s} {int(r['Calls']):5d} {float(r['AverageNs'])/1000:9.1f} us\")"
bash tools/prog_pmc.sh > $out/pmc.txt 2>&1 || { echo "pmc failed"; tail -5 $out/pmc.txt; exit 1; }
cat $out/pmc.txt | tail -16

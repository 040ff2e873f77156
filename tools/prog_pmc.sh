#!/bin/bash
# SQ counter passes over the multiscan decoder (tools/prog_one.py), each pass
# its own rocprofv3 run with --kernel-trace only.  Output: gpurun_out/prog_pmc/
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/prog_pmc
mkdir -p $out
i=0
for grp in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM" \
  "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_IFETCH SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC" ; do
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -d $out/p$i -o run --output-format csv \
    -- python3 tools/prog_one.py 64 2 > $out/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 $out/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, re, collections
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/prog_pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").strip()
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in vals.items():
    if "multiscan" not in k: continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"  {c:24s} {sum(v)/len(v):14.0f}  (n={len(v)})")
PY

#!/bin/bash
# PMC passes over a short bench run, one counter group per pass, each its own
# rocprofv3 run with --kernel-trace only (never combined with sys/runtime
# trace).  usage: tools/pmc_passes.sh OUTDIR "<counters>" ["<counters>" ...]
# Output: OUTDIR/pmc_<n>/  (summarise with tools/pmc_summary.py)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=$1; shift
mkdir -p "$out"
i=0
for grp in "$@"; do
  i=$((i+1))
  echo "== pmc pass $i: $grp"
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -d "$out/pmc_$i" -o run --output-format csv \
    -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-queue-compare --lanes1-steps 0 > "$out/pmc_$i.log" 2>&1 || { echo "pass $i rc=$?"; exit 1; }
done

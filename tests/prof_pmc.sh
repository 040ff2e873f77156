#!/bin/bash
# PMC passes over a short bench run (one counter group per pass; never combined
# with sys/runtime trace). Output: gpurun_out/pmc_<n>/
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/pmc_$i -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_$i.log 2>&1
done

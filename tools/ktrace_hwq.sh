#!/bin/bash
# kernel traces of the 4-lane bench with 4 and 16 hardware queues (tools/queue_map.py reads them)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/ktq2
mkdir -p $out
for q in 4 16; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/q$q -o run -- \
    python3 -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --lanes1-steps 0 --hw-queues $q \
    > $out/q$q.log 2>&1 || { tail -5 $out/q$q.log; exit 1; }
  f=$(ls $out/q$q/*/run_kernel_trace.csv $out/q$q/run_kernel_trace.csv 2>/dev/null | head -1)
  python3 tools/queue_map.py $f > $out/q$q.map.txt
  grep -o '"value": [0-9.]*' $out/q$q.log
done

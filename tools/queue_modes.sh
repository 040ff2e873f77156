#!/bin/bash
# 4-lane bench per lane-stream creation mode (HJ_QUEUE_MODE) with 4 and 16
# hardware queues; kernel-trace queue maps of the 4-queue runs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/qmodes
mkdir -p $out
for m in ${MODES:-0 1 2}; do
  for q in 4 16; do
    HJ_QUEUE_MODE=$m HJ_QUEUE_DEBUG=1 timeout -k 10 150 python -u bench.py --steps 200 --warmup 10 --no-cpu-baseline \
      --lanes1-steps 0 --hw-queues $q > $out/m${m}_q$q.log 2>&1 || { tail -5 $out/m${m}_q$q.log; exit 1; }
    echo "mode $m hwq $q $(grep -o '"value": [0-9.]*' $out/m${m}_q$q.log)"
  done
  HJ_QUEUE_MODE=$m timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $out/kt_m$m -o run -- \
    python3 -u bench.py --steps 60 --warmup 10 --no-cpu-baseline --lanes1-steps 0 --hw-queues 4 \
    > $out/kt_m$m.log 2>&1 || { tail -5 $out/kt_m$m.log; exit 1; }
  f=$(ls $out/kt_m$m/*/run_kernel_trace.csv $out/kt_m$m/run_kernel_trace.csv 2>/dev/null | head -1)
  python3 tools/queue_map.py $f > $out/kt_m$m.map.txt && head -8 $out/kt_m$m.map.txt
done

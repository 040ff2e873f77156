#!/bin/bash
# lanes x in-flight x hardware queues on the configs[1] bench (GPU box):
# bash tools/lanes_sweep.sh  -- one line per setting (each run time-limited)
mkdir -p gpurun_out
for cfg in "4 4 6" "4 4 8" "4 4 10" "16 4 6" "16 5 7" "16 6 8" "16 8 10" "4 5 7" "4 6 8"; do
  set -- $cfg
  hq=$1; ln=$2; inf=$3
  timeout -k 10 200 python -u bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-queue-compare \
    --lanes1-steps 0 --hw-queues $hq --lanes $ln --inflight $inf > gpurun_out/lsw.json 2> gpurun_out/lsw.err || { tail -3 gpurun_out/lsw.err; exit 3; }
  python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/lsw.json') if l.startswith('{')][-1]
print('hwq $hq lanes $ln inflight $inf', d['value'], d['ms_per_step'])"
done

#!/bin/bash
# A/B: entropy piece size on the configs[1] bench (4 lanes, 200 steps)
mkdir -p gpurun_out
for pb in ${PBS:-131072 65536 49152 32768}; do
  for th in ${THS:-256}; do
  timeout -k 10 200 python -u bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-queue-compare --lanes1-steps 20 --piece-bytes $pb --entropy-threads $th > gpurun_out/ab_pb$pb.json 2>&1 || { tail -5 gpurun_out/ab_pb$pb.json; exit 3; }
  python -c "import json; r=json.loads(open('gpurun_out/ab_pb$pb.json').read().splitlines()[-1]); print('piece $pb th $th', r['value'], r['stages_ms']['entropy'], r['roofline']['lanes1']['kernel_ms'], r['oracle_check'])"
  done
done

#!/bin/bash
# bench lines in the late-import regime (HIP initialised with Q hardware queues before spdl_amd)
set -o pipefail
for args in "--hw-queues 4" "--hw-queues 4 --lanes 4" "--hw-queues 4 --lanes 2" "--hw-queues 8" "--lanes 3"; do
  timeout -k 10 150 python -u bench.py --steps 200 --warmup 10 --no-cpu-baseline --lanes1-steps 0 $args > gpurun_out/hq.log 2>&1 || { tail -5 gpurun_out/hq.log; exit 1; }
  python -c "
import json
for l in open('gpurun_out/hq.log'):
    if l.startswith('{\"metric'):
        d=json.loads(l); print('$args', d['value'], 'lanes', d['config']['lanes'], 'hwq', d['config']['hw_queues'])"
done

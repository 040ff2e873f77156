#!/bin/bash
# configs[4] host budget: one stream rank with the copy pool sized as one of
# LOCAL_WORLD_SIZE ranks sharing the box's cores, and the 8-rank rehearsal.
set -o pipefail
for lws in 1 8; do
  LOCAL_WORLD_SIZE=$lws timeout -k 10 200 python -u bench_stream.py --images 2048 --passes 3 > gpurun_out/st.log 2>&1 || { tail -5 gpurun_out/st.log; exit 1; }
  python -c "
import json
for l in open('gpurun_out/st.log'):
    if l.startswith('{\"metric'):
        d=json.loads(l); print('LOCAL_WORLD_SIZE=$lws', d['value'], d.get('config',{}).get('copy_threads'), {k:d[k] for k in d if 'host' in k or 'thread' in k})"
done
nproc; python -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null

#!/bin/bash
# configs[4] host budget with per-rank binding (round 5): the 8-rank stream
# rehearsal on one GPU (bound: each rank on its share of the GPU's NUMA
# node; unbound for comparison), then the gpu config tests.
mkdir -p gpurun_out
nproc; python -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null
for mode in split node none; do
  extra="--bind $mode"
  timeout -k 10 300 python -u bench_stream.py --gpus 8 --rehearse-one-gpu --images 2048 --passes 3 $extra > gpurun_out/st8_$mode.log 2>&1 || { tail -5 gpurun_out/st8_$mode.log; exit 1; }
  python - <<PY
import json
for l in open('gpurun_out/st8_$mode.log'):
    if l.startswith('{"metric'):
        d=json.loads(l); print('$mode', d['value'], [(r['rank'], r['images_per_sec'], r.get('numa_node'), r.get('cpus')) for r in d['ranks']])
PY
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 600 --timeout-method thread > gpurun_out/t_cfg.log 2>&1; rc=$?; tail -3 gpurun_out/t_cfg.log; exit $rc

#!/bin/bash
# Round-end bench lines (GPU box): bash tools/final_bench.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/final}
mkdir -p "$out"
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.json" 2> "$out/$name.err" || { echo "$name failed"; tail -5 "$out/$name.err"; exit 1; }
  python3 -c "
import json,sys
for l in open('$out/$name.json'):
    if l.startswith('{'):
        d=json.loads(l); print('$name', d.get('value'), d.get('unit'), d.get('config',{}).get('lanes'), d.get('config',{}).get('hw_queues'))"
}
run bench_default 400 python -u bench.py
run bench_driver 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
run bench_lanes1 200 python -u bench.py --lanes 1 --no-cpu-baseline --no-queue-compare
run bench_fullres 200 python -u bench.py --workload fullres --no-cpu-baseline --no-queue-compare
run bench_imagenet_f16 200 python -u bench.py --workload imagenet --no-cpu-baseline --no-queue-compare
run bench_imagenet_bf16 200 python -u bench.py --workload imagenet --norm-dtype bfloat16 --no-cpu-baseline --no-queue-compare
run bench_mixed 200 python -u bench.py --workload mixed --no-cpu-baseline --no-queue-compare
run bench_big1 200 python -u bench.py --workload big1 --no-cpu-baseline --no-queue-compare
run bench_with_copies 300 python -u bench.py --with-copies --no-cpu-baseline --no-queue-compare
run stream_bytes 300 python -u bench_stream.py --source bytes
run stream_file 300 python -u bench_stream.py
run stream_d2h 300 python -u bench_stream.py --source bytes --d2h
timeout -k 10 300 python -u tools/prog_device.py > "$out/prog_device.txt" 2>&1 || { echo "prog_device failed"; tail -5 "$out/prog_device.txt"; exit 1; }
tail -4 "$out/prog_device.txt"

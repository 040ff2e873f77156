#!/bin/bash
# Stream-path A/B (GPU box): interleaved bench_stream.py runs of argument sets.
# usage: REPS=2 bash tools/stream_ab.sh "name|args" ...
mkdir -p gpurun_out/sab
for r in $(seq ${REPS:-2}); do
  for spec in "$@"; do
    name=${spec%%|*}; args=${spec#*|}
    timeout -k 10 120 python bench_stream.py $args > gpurun_out/sab/${name}_$r.log 2>&1 || { echo "fail $name"; tail -3 gpurun_out/sab/${name}_$r.log; exit 1; }
    echo "$name r$r $(grep -o '"value": [0-9.]*' gpurun_out/sab/${name}_$r.log)"
  done
done

#!/bin/bash
# Every bench line of the round into gpurun_out/meas/ (each step time-limited):
# configs[1] (default bench), lanes 1, configs[3] fp16/bf16, configs[4] stream
# (file, file + D2H, bytes), host-bytes path with copies, rocprof stats and
# the two PMC traffic passes of the default bench.
out=gpurun_out/meas
mkdir -p $out
tools/gpu_steps.sh \
  "200|meas/bench|python bench.py" \
  "120|meas/bench_lanes1|python bench.py --lanes 1 --no-cpu-baseline" \
  "120|meas/bench_copies|python bench.py --with-copies --no-cpu-baseline" \
  "120|meas/imagenet_f16|python bench.py --workload imagenet" \
  "120|meas/imagenet_bf16|python bench.py --workload imagenet --norm-dtype bfloat16" \
  "200|meas/stream_file|python bench_stream.py" \
  "200|meas/stream_d2h|python bench_stream.py --d2h" \
  "200|meas/stream_bytes|python bench_stream.py --source bytes" \
  "200|meas/prof|cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --steps 50 --no-cpu-baseline" \
  "300|meas/pmc|tools/pmc_passes.sh $out/pmc FETCH_SIZE WRITE_SIZE"

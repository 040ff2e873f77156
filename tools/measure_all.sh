#!/bin/bash
# Every bench line of the round into gpurun_out/meas/ (each step time-limited):
# configs[1] (default bench, with the CPU baseline), lanes 1, host-bytes path
# with copies, configs[3] fp16/bf16, configs[4] stream (file, file + D2H,
# bytes), configs[0] file/thread-pool harness, progressive vs baseline,
# rocprof kernel stats and the PMC passes (traffic + SQ counters).
out=gpurun_out/meas
mkdir -p $out
tools/gpu_steps.sh \
  "300|meas/bench|python bench.py" \
  "120|meas/bench_lanes1|python bench.py --lanes 1 --no-cpu-baseline" \
  "120|meas/bench_copies|python bench.py --with-copies --no-cpu-baseline" \
  "120|meas/imagenet_f16|python bench.py --workload imagenet --no-cpu-baseline" \
  "120|meas/imagenet_bf16|python bench.py --workload imagenet --norm-dtype bfloat16 --no-cpu-baseline" \
  "200|meas/stream_file|python bench_stream.py" \
  "200|meas/stream_d2h|python bench_stream.py --d2h" \
  "200|meas/stream_bytes|python bench_stream.py --source bytes" \
  "200|meas/configs0|python examples/image_dataloading.py --synthetic 2048 --batch-size 32 --num-threads 4" \
  "300|meas/progressive|python tools/prog_bench.py 256" \
  "200|meas/prof|cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --steps 50 --no-cpu-baseline" \
  "400|meas/pmc|bash tools/pmc_round.sh $out/pmc"

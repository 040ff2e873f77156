#!/bin/bash
# tests + bench + rocprof kernel stats (each step time-limited; a crash or
# timeout stops the script, test failures do not)
exec tools/gpu_steps.sh \
  "1000|gpu_tests|python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread" \
  "300|bench|python -u bench.py --steps 60 --warmup 5" \
  "240|prof|cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline"

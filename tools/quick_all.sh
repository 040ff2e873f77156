#!/bin/bash
# full GPU test suite, then bench lines (lanes 1/2/3) and the entropy sweep
B="python -u bench.py --steps 60 --warmup 5 --no-cpu-baseline"
exec tools/gpu_steps.sh \
  "1000|t_all|python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread" \
  "200|b_l1|$B --lanes 1" \
  "200|b_l2|$B" \
  "200|b_l3|$B --lanes 3 --inflight 3" \
  "600|sweep|bash tools/sweep_entropy2.sh"

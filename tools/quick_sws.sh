#!/bin/bash
# A/B loop helper for the output stage: the swscale GPU tests, then bench
# lines (stage timings) with 2 and 1 lanes and output-stage ablations.
B="python -u bench.py --steps 60 --warmup 5 --no-cpu-baseline"
exec tools/gpu_steps.sh \
  "600|t_sws|python -u -m pytest tests/test_gpu_swscale.py tests/test_gpu_parity.py tests/test_gpu_surface.py -m gpu -q -x --timeout 240 --timeout-method thread" \
  "200|b_l2|$B" \
  "200|b_l1|$B --lanes 1" \
  "200|b_noh|$B --lanes 1 --debug-mask 256" \
  "200|b_nov|$B --lanes 1 --debug-mask 512" \
  "200|b_nost|$B --lanes 1 --debug-mask 1024" \
  "200|b_none|$B --lanes 1 --debug-mask 1792"

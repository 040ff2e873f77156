#!/bin/bash
# round-5 GPU step: selected -m gpu tests (arg 1: pytest -k expression or
# file list via TESTS), then the bench workloads (each step time-limited;
# a crash or timeout stops the script)
mkdir -p gpurun_out
TESTS=${TESTS:-tests/test_gpu_pieces.py tests/test_gpu_entropy_edges.py tests/test_gpu_parity.py}
timeout -k 10 900 python -u -m pytest $TESTS -x -q -rf --timeout 240 --timeout-method thread > gpurun_out/t_r5.log 2>&1
rc=$?; tail -6 gpurun_out/t_r5.log; echo "tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
for w in ${WORKLOADS:-pad224 big1 mixed}; do
  timeout -k 10 200 python -u bench.py --steps 60 --warmup 5 --workload $w --no-cpu-baseline --no-queue-compare > gpurun_out/b_$w.json 2> gpurun_out/b_$w.err || exit 3
  python - <<PY
import json; r=json.loads(open("gpurun_out/b_$w.json").read().splitlines()[-1]); print("$w", r["value"], r["ms_per_step"], {k: round(v,3) for k,v in r["stages_ms"].items()}, r["config"]["compressed_GBps"], r["roofline"]["lanes1"]["kernel_ms"], r["oracle_check"])
PY
done

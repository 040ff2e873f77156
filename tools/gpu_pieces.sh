mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pieces.py tests/test_gpu_entropy_edges.py -x -v --timeout 240 --timeout-method thread > gpurun_out/t_pieces.log 2>&1
rc=$?; tail -25 gpurun_out/t_pieces.log; echo "rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
for w in pad224 big1 mixed; do
  timeout -k 10 200 python -u bench.py --steps 60 --warmup 5 --workload $w --no-cpu-baseline --no-queue-compare > gpurun_out/b_$w.json 2> gpurun_out/b_$w.err || exit 3
  python - <<PY
import json; r=json.loads(open("gpurun_out/b_$w.json").read().splitlines()[-1]); print("$w", r["value"], r["ms_per_step"], r["stages_ms"], r["config"]["compressed_GBps"], r["roofline"]["lanes1"]["kernel_ms"], r["oracle_check"])
PY
done
timeout -k 10 200 python -u bench.py --steps 60 --warmup 5 --workload big1 --piece-bytes 0 --no-cpu-baseline --no-queue-compare > gpurun_out/b_big1_nopiece.json 2>&1 || exit 4
python - <<PY
import json; r=json.loads(open("gpurun_out/b_big1_nopiece.json").read().splitlines()[-1]); print("big1 nopiece", r["value"], r["ms_per_step"], r["stages_ms"], r["roofline"]["lanes1"]["kernel_ms"])
PY

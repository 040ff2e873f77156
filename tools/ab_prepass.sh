mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pieces.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "prepass or pieces or mixed or big" > gpurun_out/t_ab1.log 2>&1; rc=$?; tail -2 gpurun_out/t_ab1.log; [ $rc -eq 0 ] || exit $rc
for w in big1 mixed; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --workload $w --no-cpu-baseline --no-queue-compare --lanes1-steps 0 > gpurun_out/b_$w.json 2>&1 || exit 3
  python -c "import json; r=json.loads(open('gpurun_out/b_$w.json').read().splitlines()[-1]); print('$w', r['value'], r['stages_ms'])"
done
for pp in -1 1; do
  timeout -k 10 200 python -u bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-queue-compare --lanes1-steps 0 --param sws_prepass=$pp > gpurun_out/b_pp$pp.json 2>&1 || exit 4
  python -c "import json; r=json.loads(open('gpurun_out/b_pp$pp.json').read().splitlines()[-1]); print('pad224 prepass=$pp', r['value'], r['stages_ms'])"
done

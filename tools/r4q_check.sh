set -o pipefail
mkdir -p gpurun_out/r4q
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4q/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r4q/gpu_tests.log
[ $rc -eq 0 ] && timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4q/bench.json 2> gpurun_out/r4q/bench.err && python -c "
import json; d=json.loads(open('gpurun_out/r4q/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['config']['hw_queues'], d['hw_queue_regimes'])"

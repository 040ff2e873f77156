set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 400 python -u bench.py > gpurun_out/final/bench_default.json 2> gpurun_out/final/bench_default.err &&
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final/bench_driver.json 2> gpurun_out/final/bench_driver.err &&
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --hw-queues 4 > gpurun_out/final/bench_hwq4.json 2> gpurun_out/final/bench_hwq4.err &&
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --lanes 1 > gpurun_out/final/bench_lanes1.json 2> gpurun_out/final/bench_lanes1.err

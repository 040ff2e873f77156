B="python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --lanes 1"
mkdir -p gpurun_out
for cfg in "--entropy-threads 512 --warm-slots 8" "--entropy-threads 1024 --warm-slots 8" "--entropy-threads 1024 --warm-slots 16" "--entropy-threads 256 --warm-slots 4" "--entropy-threads 256 --warm-slots 8" "--entropy-threads 512 --warm-slots 8 --sub-bits 256" "--entropy-threads 512 --warm-slots 16 --sub-bits 256" "--entropy-threads 512 --warm-slots 4 --sub-bits 1024"; do
  n=$(echo $cfg | tr -d ' -')
  timeout -k 10 120 $B $cfg > gpurun_out/b_sw_$n.log 2>&1 || { echo "fail $cfg"; exit 1; }
done
python tools/stages.py "gpurun_out/b_sw_*.log"

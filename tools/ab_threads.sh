mkdir -p gpurun_out/abt
for r in 1 2 3; do
  for t in 256 512; do
    timeout -k 10 150 python -u bench.py --steps 80 --warmup 5 --no-cpu-baseline --oracle-check 0 --entropy-threads $t > gpurun_out/abt/t${t}_r$r.log 2>&1 || exit 1
  done
done
timeout -k 10 150 python -u bench.py --steps 80 --warmup 5 --no-cpu-baseline --lanes 1 > gpurun_out/abt/t256_l1.log 2>&1 || exit 1
python tools/stages.py "gpurun_out/abt/*.log"

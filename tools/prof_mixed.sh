bash tools/gpu_r5.sh || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for w in big1 mixed; do
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$w -o run --output-format csv -- python3 bench.py --steps 30 --warmup 3 --workload $w --no-cpu-baseline --no-queue-compare --lanes1-steps 0 > gpurun_out/prof_$w.log 2>&1 || exit 5
f=$(find gpurun_out/prof_$w -name "*kernel_stats.csv" | head -1); echo "== $w"; cut -d, -f1-4 $f | head -14
done

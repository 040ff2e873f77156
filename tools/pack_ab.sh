set -o pipefail
for v in base p2 p4; do
  lib=spdl_amd/lib/libspdl_hipjpeg.so
  [ "$v" != base ] && lib=spdl_amd/lib/variants/libspdl_hipjpeg_$v.so
  SPDL_AMD_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_swscale.py -m gpu -q -x --timeout 240 --timeout-method thread -k bench_path > gpurun_out/pk_t_$v.log 2>&1 || { echo "tests $v failed"; tail -5 gpurun_out/pk_t_$v.log; exit 1; }
  for l in 1 2; do
    SPDL_AMD_LIB=$lib timeout -k 10 150 python -u bench.py --steps 60 --warmup 5 --no-cpu-baseline --lanes $l > gpurun_out/ab_${v}_l$l.log 2>&1 || exit 1
  done
  (cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && SPDL_AMD_LIB=$lib timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pk_pmc_$v -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pk_pmc_$v.log 2>&1) || { echo "pmc $v failed"; exit 1; }
  python tools/pmc_summary.py gpurun_out/pk_pmc_$v | grep -A1 entropy
done
python tools/stages.py "gpurun_out/ab_*.log"

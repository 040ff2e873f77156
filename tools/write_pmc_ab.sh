for v in base noent nobd nost; do
  lib=spdl_amd/lib/libspdl_hipjpeg.so
  [ "$v" != base ] && lib=spdl_amd/lib/variants/libspdl_hipjpeg_$v.so
  (cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && SPDL_AMD_LIB=$lib timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/w_$v -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --oracle-check 0 > gpurun_out/w_$v.log 2>&1) || { echo "pmc $v failed"; exit 1; }
  echo "== $v"; python tools/pmc_summary.py gpurun_out/w_$v | grep -A1 "entropy\|idct"
done

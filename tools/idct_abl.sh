for m in 0 0x800; do
  SPDL_AMD_LIB=spdl_amd/lib/variants/libspdl_hipjpeg_abl.so timeout -k 10 200 python -u bench.py --steps 60 --warmup 5 --lanes 1 --no-cpu-baseline --no-queue-compare --lanes1-steps 0 --debug-mask $((m)) > gpurun_out/ia.json 2>&1 || { tail -3 gpurun_out/ia.json; exit 1; }
  python -c "import json; r=json.loads(open('gpurun_out/ia.json').read().splitlines()[-1]); print('mask $m', r['value'], {k: round(x,4) for k,x in r['stages_ms'].items() if k in ('entropy','idct','output')})"
done

#!/bin/bash
# progressive batches with the scan decoders' waves at s_setprio 3 vs default
for rep in 1 2; do
for l in base msprio; do
  if [ $l = msprio ]; then export SPDL_AMD_LIB=spdl_amd/lib/variants/libspdl_hipjpeg_msprio.so; else unset SPDL_AMD_LIB; fi
  timeout -k 10 300 python -u tools/prog_device.py 40 > gpurun_out/pd_$l.txt 2>&1 || { tail -5 gpurun_out/pd_$l.txt; exit 1; }
  echo "== $l rep $rep"; tail -4 gpurun_out/pd_$l.txt
done; done

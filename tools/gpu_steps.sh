#!/bin/bash
# Run GPU steps in sequence, each under its own time limit.  A step that
# fails normally (test failures, rc 1-2) lets the next step run; a crash,
# abort or timeout (rc >= 124) ends the script there.
# usage: tools/gpu_steps.sh "<secs>|<log name>|<command>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  secs=${spec%%|*}; rest=${spec#*|}; name=${rest%%|*}; cmd=${rest#*|}
  echo "== [$name] $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== [$name] rc=$rc"
  grep -v "amdgpu.ids" "gpurun_out/$name.log" | tail -n 12
  if [ $rc -ge 124 ]; then echo "== stopping after [$name] rc=$rc"; exit $rc; fi
done

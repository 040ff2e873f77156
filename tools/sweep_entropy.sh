#!/bin/bash
# Entropy-stage time (bench.py stages_ms.entropy) over slot size x workgroup size.
for t in 256 512 1024; do
  for b in 256 384 512 768 1024 2048; do
    r=$(timeout -k 10 60 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --sub-bits $b --entropy-threads $t 2>&1 | grep '^{' | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['stages_ms']['entropy'])")
    echo "threads=$t sub_bits=$b -> $r"
  done
done

#!/bin/bash
# All PMC passes of a round over a short bench run (one rocprofv3 run per
# counter group, --kernel-trace only), then the traffic json + counter summary.
# usage: tools/pmc_round.sh OUTDIR   (run on the GPU box)
set -o pipefail
out=${1:-gpurun_out/pmc}
bash tools/pmc_passes.sh "$out" \
  "FETCH_SIZE" \
  "WRITE_SIZE" \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
  "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
  || exit 1
python3 tools/pmc_traffic.py "$out/traffic.json" "$out/pmc_1" "$out/pmc_2" > "$out/traffic.txt" || exit 1
python3 tools/pmc_issue.py "$out/issue.json" 256 "$out/pmc_3" "$out/pmc_4" > "$out/issue.txt" || exit 1
python3 tools/pmc_summary.py "$out"/pmc_* > "$out/counters_summary.txt" || exit 1
cat "$out/traffic.txt"

"""Per-kernel issue/wait shares from rocprofv3 --pmc SQ counters (one pass:
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU, and one with
SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT ...; see tools/pmc_round.sh).

  valu_share = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES  (wave time issuing VALU)
  wait_share = SQ_WAIT_ANY / SQ_WAVE_CYCLES          (wave time waiting on anything)
  lds_conflict_per_lds_inst = SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS
All per dispatch (averaged over the dispatches of the run).

usage: python tools/pmc_issue.py OUT.json BATCH PMC_DIR [PMC_DIR ...]
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

out_path, batch, dirs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
vals = defaultdict(lambda: defaultdict(list))
for d in dirs:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").strip()
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {}
for k, cs in sorted(vals.items()):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    if not {"SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY"} <= set(m):
        continue
    wc = max(m["SQ_WAVE_CYCLES"], 1.0)
    res[k] = {"waves": round(m.get("SQ_WAVES", 0)),
              "valu_share": round(m["SQ_ACTIVE_INST_VALU"] / wc, 4),
              "wait_share": round(m["SQ_WAIT_ANY"] / wc, 4),
              "lds_conflict_per_lds_inst": round(m.get("SQ_LDS_BANK_CONFLICT", 0.0)
                                                 / max(m.get("SQ_INSTS_LDS", 0.0), 1.0), 3),
              "valu_insts": round(m.get("SQ_INSTS_VALU", 0))}
json.dump({"source": dirs, "batch": batch, "kernels": res}, open(out_path, "w"), indent=1)
for k, v in res.items():
    print(f"{k:40s} valu {v['valu_share']:.2f} wait {v['wait_share']:.2f} "
          f"lds-conflict/inst {v['lds_conflict_per_lds_inst']:.2f} waves {v['waves']}")

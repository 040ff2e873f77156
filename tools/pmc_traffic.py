"""Per-launch HBM-side traffic per kernel from rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE collected in separate passes, as
/opt/skills/guides/MI355X_MICROARCH.md's HBM section prescribes).

Units and gfx950 corrections (same guide):
  * FETCH_SIZE / WRITE_SIZE are in KiB (x 1024 -> bytes);
  * on gfx950 FETCH_SIZE reports 1/2 of the bytes of a wide (16 B/lane)
    coalesced read -> doubled here.  Narrower access widths are uncalibrated;
    the figure is an upper-bound-style estimate for kernels that mix widths.
  * Infinity-Cache (MALL) hits are counted by these fabric-side counters.

usage: python tools/pmc_traffic.py OUT.json PMC_DIR [PMC_DIR ...]
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

out_path, dirs = sys.argv[1], sys.argv[2:]
vals = defaultdict(lambda: defaultdict(list))
for d in dirs:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").strip()
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {}
for k, cs in sorted(vals.items()):
    if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
        continue
    fetch = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) * 1024 * 2
    write = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) * 1024
    res[k] = {"fetch_bytes": round(fetch), "write_bytes": round(write),
              "traffic_bytes": round(fetch + write), "dispatches": len(cs["FETCH_SIZE"])}
json.dump({"source": dirs, "correction": "FETCH_SIZE x1024 x2 (gfx950 wide-read), WRITE_SIZE x1024",
           "kernels": res}, open(out_path, "w"), indent=1)
for k, v in res.items():
    print(f"{k:40s} fetch {v['fetch_bytes']/1e6:10.2f} MB  write {v['write_bytes']/1e6:10.2f} MB")

"""Correction factors of FETCH_SIZE / WRITE_SIZE per access pattern:
true bytes (printed by tools/fetch_calib) / (counter x 1024)."""
import csv
import glob
import json
import re
import sys

out = sys.argv[1]
true = {}
for line in open(f"{out}/bytes.txt"):
    k, n, _ = line.split()
    true[k] = int(n)
vals = {}
for f in glob.glob(f"{out}/pmc_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").strip()
        vals.setdefault(k, {})[r["Counter_Name"]] = float(r["Counter_Value"])
res = {}
for k, n in true.items():
    c = vals.get(k, {})
    ctr = c.get("FETCH_SIZE") if "read" in k else c.get("WRITE_SIZE")
    if ctr:
        res[k] = {"true_bytes": n, "counter_bytes": ctr * 1024, "factor": round(n / (ctr * 1024), 3)}
json.dump(res, open(f"{out}/calibration.json", "w"), indent=1)
for k, v in res.items():
    print(f"{k:14s} true {v['true_bytes']/1e6:9.1f} MB  counter {v['counter_bytes']/1e6:9.1f} MB  "
          f"factor {v['factor']}")

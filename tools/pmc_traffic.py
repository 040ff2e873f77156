"""Per-launch HBM-side traffic per kernel from rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE collected in separate passes, as
/opt/skills/guides/MI355X_MICROARCH.md's HBM section prescribes).

Units and corrections:
  * FETCH_SIZE / WRITE_SIZE are in KiB (x 1024 -> bytes);
  * the guide calibrates gfx950's FETCH_SIZE at 1/2 of the bytes only for
    wide coalesced streaming reads.  With CALIB (tools/fetch_calib.sh's
    calibration.json: true bytes / counter bytes per access pattern,
    measured on this box) each kernel's counter is scaled by the factor of
    the pattern it reads / writes with (PATTERN below); without it FETCH is
    reported raw (x1, a lower bound) and x2 (the streaming-read correction).
  * Infinity-Cache (MALL) hits are counted by these fabric-side counters.

usage: python tools/pmc_traffic.py OUT.json PMC_DIR [PMC_DIR ...] [--calib calibration.json]
"""
import csv
import glob
import json
import re
import sys

args = sys.argv[1:]
calib = None
if "--calib" in args:
    i = args.index("--calib")
    calib = json.load(open(args[i + 1]))
    args = args[:i] + args[i + 2:]
out_path, dirs = args[0], args[1:]
# kernel -> (read pattern, write pattern) of tools/fetch_calib.hip
PATTERN = {
    "hj::entropy_kernel": ("window_read", "append_write"),
    "hj::idct_kernel": ("list_read", "rows_write"),
    "hj::idct_rgb_kernel": ("list_read", "stream_write"),
}
DEFAULT = ("stream_read", "stream_write")
vals = {}
for d in dirs:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").strip()
            vals.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
res = {}
for k, cs in sorted(vals.items()):
    if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
        continue
    fetch_raw = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) * 1024
    write_raw = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) * 1024
    rp, wp = next((v for p, v in PATTERN.items() if k.startswith(p)), DEFAULT)
    if calib:
        ff, wf = calib[rp]["factor"], calib[wp]["factor"]
        corr = f"calibrated: FETCH x{ff} ({rp}), WRITE x{wf} ({wp})"
    else:
        ff, wf = 2.0, 1.0
        corr = "uncalibrated: FETCH x2 (streaming-read correction), WRITE x1"
    res[k] = {"fetch_bytes": round(fetch_raw * ff), "write_bytes": round(write_raw * wf),
              "fetch_raw_bytes": round(fetch_raw), "write_raw_bytes": round(write_raw),
              "traffic_bytes": round(fetch_raw * ff + write_raw * wf), "correction": corr,
              "dispatches": len(cs["FETCH_SIZE"])}
json.dump({"source": dirs, "batch": 256, "correction": "per kernel, see each record",
           "kernels": res}, open(out_path, "w"), indent=1)
for k, v in res.items():
    print(f"{k:40s} fetch {v['fetch_bytes']/1e6:9.2f} MB  write {v['write_bytes']/1e6:9.2f} MB"
          f"  ({v['correction']})")

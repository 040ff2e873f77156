"""Device time per launch-step during which each kernel runs: the union of its
launches' [start, end) intervals in a rocprofv3 kernel trace, divided by its
number of launches (the bench launches every kernel once per step).  With
several lanes the launches of one kernel overlap, so this -- not the average
launch duration -- is the kernel's share of ms_per_step.

usage: python tools/kernel_busy.py OUT.json LANES:TRACE_CSV [LANES:TRACE_CSV ...]
(TRACE_CSV: the *kernel_trace.csv of `rocprofv3 --kernel-trace`)
"""
import csv
import json
import re
import sys
from collections import defaultdict

out, specs = sys.argv[1], sys.argv[2:]
res = {}
for spec in specs:
    lanes, path = spec.split(":", 1)
    iv = defaultdict(list)
    for r in csv.DictReader(open(path)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").strip()
        iv[k].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    per = {}
    for k, xs in iv.items():
        xs.sort()
        busy, cur_s, cur_e = 0, None, None
        for s, e in xs:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            busy += cur_e - cur_s
        per[k] = {"launches": len(xs), "busy_ms_per_step": round(busy / len(xs) / 1e6, 5),
                  "avg_launch_ms": round(sum(e - s for s, e in xs) / len(xs) / 1e6, 5)}
    res[lanes] = per
json.dump(res, open(out, "w"), indent=1)
for lanes, per in res.items():
    for k, v in sorted(per.items(), key=lambda kv: -kv[1]["busy_ms_per_step"])[:6]:
        print(f"lanes {lanes} {k:40s} busy/step {v['busy_ms_per_step']:.4f} ms  "
              f"avg launch {v['avg_launch_ms']:.4f} ms  ({v['launches']} launches)")

"""Per-kernel duration statistics from a rocprofv3 rocpd database (the
--kernel-trace output when no CSV format is requested), written as the same
columns rocprofv3 --stats uses: python tools/rocpd_stats.py DB [OUT.csv]"""
import csv
import sqlite3
import statistics
import sys

db = sys.argv[1]
c = sqlite3.connect(db)
rows = c.execute("select name, start, end from kernels").fetchall()
by = {}
for name, s, e in rows:
    by.setdefault(name, []).append(e - s)
total = sum(sum(v) for v in by.values())
out = []
for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    out.append([name, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / total, min(v), max(v),
                statistics.pstdev(v)])
hdr = ["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"]
w = csv.writer(open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
w.writerow(hdr)
for r in out:
    w.writerow(r)

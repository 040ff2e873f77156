"""Which HIP stream ran on which hardware queue, and how many kernels overlapped.

usage: python tools/queue_map.py <run_kernel_trace.csv> [<skip_fraction>]

Prints the (stream, queue) pairs with their kernel counts and busy time, and a
time-weighted histogram of the number of kernels in flight over the traced
window (after dropping the first `skip_fraction` of dispatches: warmup).
"""
import collections
import csv
import sys


def main(path, skip=0.2):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[int(len(rows) * skip):]
    pairs = collections.Counter()
    busy = collections.Counter()
    names = collections.defaultdict(collections.Counter)
    ev = []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        key = (int(r["Stream_Id"]), int(r["Queue_Id"]))
        pairs[key] += 1
        busy[key] += e - s
        names[key][r["Kernel_Name"].split("(")[0].split("<")[0].replace("hj::", "")] += 1
        ev.append((s, 1))
        ev.append((e, -1))
    print("stream queue kernels busy_ms  top kernels")
    for k in sorted(pairs):
        top = ", ".join(f"{n}:{c}" for n, c in names[k].most_common(3))
        print(f"{k[0]:6d} {k[1]:5d} {pairs[k]:7d} {busy[k] / 1e6:8.3f}  {top}")
    ev.sort()
    hist = collections.Counter()
    cur, last = 0, ev[0][0]
    for t, d in ev:
        hist[cur] += t - last
        cur += d
        last = t
    tot = sum(hist.values())
    print("in-flight kernels: time share")
    for k in sorted(hist):
        print(f"  {k}: {hist[k] / tot:.3f}")
    print(f"window {tot / 1e6:.3f} ms, mean in flight "
          f"{sum(k * v for k, v in hist.items()) / tot:.2f}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 0.2)

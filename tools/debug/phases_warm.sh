for w in 2 4 6 12 24; do PH_WARM=$w timeout -k 10 300 python -u tools/debug/phases_mixed.py > gpurun_out/pm_w$w.txt 2>&1 || exit 1; done
python - <<'PY'
import re
res={}
for w in [2,4,6,12,24]:
    for l in open(f"gpurun_out/pm_w{w}.txt"):
        m=re.match(r"img\s+(\d+) bytes\s+(\d+).*total\s+([\d.]+) us.*rounds (\d+)", l)
        if m: res.setdefault(int(m.group(1)), {})[w]=(float(m.group(3)), int(m.group(4)), int(m.group(2)))
print("img bytes " + " ".join(f"w{w:>2}" for w in [2,4,6,12,24]))
tot={w:0 for w in [2,4,6,12,24]}; mx={w:0 for w in [2,4,6,12,24]}
for i in sorted(res, key=lambda i: res[i][12][2]):
    print(f"{i:3d} {res[i][12][2]:7d} " + " ".join(f"{res[i][w][0]:6.0f}/{res[i][w][1]:<2d}" for w in [2,4,6,12,24]))
    for w in tot: tot[w]+=res[i][w][0]; mx[w]=max(mx[w],res[i][w][0])
print("sum", tot); print("max", mx)
PY

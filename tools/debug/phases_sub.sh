for sb in 128 192 256 384; do PH_SUB=$sb timeout -k 10 300 python -u tools/debug/phases_mixed.py > gpurun_out/pm_s$sb.txt 2>&1 || exit 1; done
python - <<'PY'
import re
S=[128,192,256,384]
res={}
for w in S:
    for l in open(f"gpurun_out/pm_s{w}.txt"):
        m=re.match(r"img\s+(\d+) bytes\s+(\d+).*total\s+([\d.]+) us.*rounds (\d+)", l)
        if m: res.setdefault(int(m.group(1)), {})[w]=(float(m.group(3)), int(m.group(4)), int(m.group(2)))
print("img bytes " + " ".join(f"s{w:>3}" for w in S))
tot={w:0 for w in S}; mx={w:0 for w in S}
for i in sorted(res, key=lambda i: res[i][384][2]):
    print(f"{i:3d} {res[i][384][2]:7d} " + " ".join(f"{res[i][w][0]:6.0f}/{res[i][w][1]:<2d}" for w in S))
    for w in tot: tot[w]+=res[i][w][0]; mx[w]=max(mx[w],res[i][w][0])
print("sum", tot); print("max", mx)
PY

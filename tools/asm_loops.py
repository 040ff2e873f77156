"""List the loops of one kernel in a hipcc --save-temps .s file with their
instruction mix (VALU / SALU / LDS / VMEM): python tools/asm_loops.py FILE.s SYMBOL_PREFIX"""
import re
import sys

src, prefix = sys.argv[1], sys.argv[2]
lines = open(src).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith(prefix) and ":" in l)
end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
body = lines[start:end]
labels = {}
for i, l in enumerate(body):
    m = re.match(r"^(\.LBB\d+_\d+):", l)
    if m:
        labels[m.group(1)] = i
for i, l in enumerate(body):
    m = re.search(r"s_cbranch_\w+\s+(\.LBB\d+_\d+)|s_branch\s+(\.LBB\d+_\d+)", l)
    if not m:
        continue
    t = m.group(1) or m.group(2)
    if t in labels and labels[t] < i:
        seg = body[labels[t]: i + 1]
        ins = [x.strip() for x in seg if x.startswith("\t") and not x.strip().startswith((";", "."))]
        cnt = lambda *p: sum(1 for x in ins if x.startswith(p))
        print(f"loop {t} lines {labels[t]}-{i}: ins={len(ins)} valu={cnt('v_')} salu={cnt('s_')} "
              f"lds={cnt('ds_')} vmem={cnt('global_', 'buffer_', 'flat_')}")

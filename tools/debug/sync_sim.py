"""Self-synchronisation of a guessed Huffman decode state (CPU model of the
entropy kernel's round 0): for slot starts every N bits, decode from (z=0,
b=0) and measure the bits until the trajectory merges with the true one
(same bit position, z and block-in-MCU at a symbol start)."""
import sys
import numpy as np
sys.path.insert(0, "/root/repo")
from spdl_amd.synthetic import mixed_jpeg

def parse(d):
    i = 2; dht = {}; comps = []; sos = None
    while i < len(d):
        assert d[i] == 0xFF; m = d[i+1]; L = (d[i+2] << 8) | d[i+3]; seg = d[i+4:i+2+L]
        if m == 0xC4:
            j = 0
            while j < len(seg):
                tc, th = seg[j] >> 4, seg[j] & 15; bits = list(seg[j+1:j+17]); n = sum(bits)
                vals = list(seg[j+17:j+17+n]); dht[(tc, th)] = (bits, vals); j += 17 + n
        elif m in (0xC0, 0xC1):
            nc = seg[5]
            for c in range(nc):
                comps.append((seg[6+3*c], seg[7+3*c] >> 4, seg[7+3*c] & 15))
        elif m == 0xDA:
            ns = seg[0]; sc = [(seg[1+2*k], seg[2+2*k] >> 4, seg[2+2*k] & 15) for k in range(ns)]
            start = i + 2 + L
            return dht, comps, sc, start
        i += 2 + L

def table(bits, vals):
    # code -> (len, sym) dict by (len, code)
    code = 0; k = 0; t = {}
    for l in range(1, 17):
        for _ in range(bits[l-1]):
            t[(l, code)] = vals[k]; k += 1; code += 1
        code <<= 1
    return t

d = mixed_jpeg(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
dht, comps, sc, start = parse(d)
end = d.rindex(b"\xff\xd9")
raw = d[start:end]
clean = bytearray(); j = 0
while j < len(raw):
    clean.append(raw[j])
    if raw[j] == 0xFF and j + 1 < len(raw) and raw[j+1] == 0: j += 2
    else: j += 1
bitsarr = np.unpackbits(np.frombuffer(bytes(clean), np.uint8))
nb = len(bitsarr)
# MCU layout
blk_comp = []
for ci, (cid, h, v) in enumerate(comps):
    blk_comp += [ci] * (h * v)
tabs = {ci: (table(*dht[(0, sc[ci][1])]), table(*dht[(1, sc[ci][2])])) for ci in range(len(comps))}
# fast lookup: precompute for each table a dict of 16-bit prefix -> (len, sym)
def lut(t):
    L = {}
    for (l, c), s in t.items():
        base = c << (16 - l)
        for x in range(1 << (16 - l)):
            L[base + x] = (l, s)
    return L
luts = {ci: (lut(a), lut(b)) for ci, (a, b) in tabs.items()}
pw = np.zeros(nb + 32, np.int64)
b16 = np.concatenate([bitsarr, np.zeros(32, np.uint8)])
# 16-bit window at every position
w = np.zeros(nb, np.int64)
for k in range(16):
    w = (w << 1) | b16[k:k+nb]
bpm = len(blk_comp)
def step(pos, z, b):
    ci = blk_comp[b]
    L = luts[ci][0 if z == 0 else 1]
    e = L.get(int(w[pos]) if pos < nb else 0)
    if e is None:
        return pos + 1, z, b
    l, s = e
    if z == 0:
        pos += l + s; z = 1
    else:
        r, sz = s >> 4, s & 15
        pos += l + sz
        if sz == 0 and r != 15: z = 64
        else: z += r + 1
    if z >= 64:
        z = 0; b = (b + 1) % bpm
    return pos, z, b
# true trajectory: symbol starts -> state
truth = {}
pos, z, b = 0, 0, 0
while pos < nb - 16:
    truth[pos] = (z, b)
    pos, z, b = step(pos, z, b)
N = 384
res = []
for s0 in range(N, nb - 4000, N):
    pos, z, b = s0, 0, 0
    bits_to_align = None; bits_to_merge = None
    while pos < nb - 16 and pos - s0 < 200000:
        t = truth.get(pos)
        if t is not None:
            if bits_to_align is None: bits_to_align = pos - s0
            if t == (z, b):
                bits_to_merge = pos - s0; break
        pos, z, b = step(pos, z, b)
    res.append((bits_to_align, bits_to_merge))
al = np.array([a if a is not None else -1 for a, _ in res]); me = np.array([m if m is not None else -1 for _, m in res])
print(f"image bytes {len(d)} bits {nb} bpm {bpm} slots {len(res)}")
print("bits to bit-align: median %d p90 %d max %d" % (np.median(al), np.percentile(al, 90), al.max()))
ok = me[me >= 0]
print("bits to merge (z,b too): median %d p90 %d p99 %d max %d; never: %d" % (np.median(ok), np.percentile(ok, 90), np.percentile(ok, 99), ok.max(), (me < 0).sum()))
# phase hypotheses: after a warm-up of W bits from (z=0, b=0), is the state
# bit-aligned with the true trajectory with the right z (only the
# block-in-MCU phase possibly wrong)?
for W in (384, 768, 1536, 3072):
    okz = okall = tot = 0
    for s0 in range(N, nb - 8000, N):
        pos, z, b = s0, 0, 0
        while pos < s0 + W:
            pos, z, b = step(pos, z, b)
        t = truth.get(pos)
        tot += 1
        if t is not None and t[0] == z:
            okz += 1
            okall += t[1] == b
    print(f"warm-up {W:5d} bits: (pos, z) right {okz / tot:.3f}, all right {okall / tot:.3f}")

"""Ad-hoc GPU diagnostics: entropy-stage comparison against the oracle."""
import sys
import numpy as np
sys.path.insert(0, ".")
from oracle import oracle as O
from spdl_amd._lib import Decoder
from tests import cases

dec = Decoder(0)
names = sys.argv[1:] or ["q90_420", "tiny_8x8", "gray", "restart_rows", "q90_444"]
for name in names:
    d = cases.case(name)
    info = O.parse(d)
    coefs, clean, diag = dec.debug_entropy(d, info.nblocks)
    ref, _ = O.decode_coefs(d)
    # destuff reference
    scan = d[info.scan_start:]
    out = bytearray(); i = 0
    while i < len(scan):
        b = scan[i]
        if b == 0xFF:
            nb = scan[i + 1]
            if nb == 0: out.append(0xFF); i += 2; continue
            k = i + 1
            while k < len(scan) and scan[k] == 0xFF: k += 1
            if 0xD0 <= scan[k] <= 0xD7: i = k + 1; continue
            break
        out.append(b); i += 1
    clean_ok = bytes(clean) == bytes(out)
    bad = np.nonzero((coefs != ref).any(axis=1))[0]
    print(f"{name}: diag={diag} clean_ok={clean_ok} (len {len(clean)} vs {len(out)}) "
          f"bad_blocks={len(bad)}/{info.nblocks}")
    for blk in bad[:3]:
        diffpos = np.nonzero(coefs[blk] != ref[blk])[0]
        print("  block", blk, "pos", diffpos[:10], "gpu", coefs[blk][diffpos[:10]], "ref", ref[blk][diffpos[:10]])

print("---- planes ----")
for name in names:
    d = cases.case(name)
    for idct, oi in (("simple", O.IDCT_SIMPLE), ("islow", O.IDCT_ISLOW)):
        hyp = dec.decode_planes(d, idct=idct)
        ref = O.decode_planes(d, oi)
        for c, (h, r) in enumerate(zip(hyp, ref)):
            if not np.array_equal(h, r):
                diff = (h != r)
                H, W = h.shape
                bh, bw = -(-H // 8), -(-W // 8)
                pad = np.zeros((bh * 8, bw * 8), bool); pad[:H, :W] = diff
                blocks = pad.reshape(bh, 8, bw, 8).any(axis=(1, 3))
                ys, xs = np.nonzero(blocks)
                print(f"{name} {idct} plane{c}: {diff.mean():.3f} px bad, {blocks.sum()} / {blocks.size} blocks; first {list(zip(ys[:5], xs[:5]))}")
                y, x = ys[0] * 8, xs[0] * 8
                print("   hyp\n", h[y:y+8, x:x+8], "\n   ref\n", r[y:y+8, x:x+8])
            else:
                print(f"{name} {idct} plane{c}: OK")

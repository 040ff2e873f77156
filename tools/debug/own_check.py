"""Write-pass block ownership check (variant build -DHJ_OWN_CHECK=1,
`make variant NAME=own DEFS=-DHJ_OWN_CHECK=1`): per image, the descriptor
stores of the entropy write pass that fall outside the storing run's
block-scan range (ImageInfo::dbg[3]).  The mixed set and bench images, by
entropy_threads x chain_after.  Non-zero means two runs store one block."""
import sys

sys.path.insert(0, ".")
from oracle import oracle as O  # noqa: E402
from spdl_amd._lib import Decoder  # noqa: E402
from spdl_amd.synthetic import mixed_jpeg, synthetic_jpeg  # noqa: E402

dec = Decoder(0)
imgs = [("mixed", i, mixed_jpeg(i)) for i in range(64)] + [("bench", s, synthetic_jpeg(s))
                                                          for s in range(1000, 1008)]
for threads in (256, 512):
    for chain in (0, 1, 2):
        dec.set_param("entropy_threads", threads)
        dec.set_param("chain_after", chain)
        tot, bad = 0, []
        for kind, i, d in imgs:
            info = O.parse(d)
            coefs, clean, diag = dec.debug_entropy(d, info.nblocks)
            v = int(diag["dbg"][3])
            tot += v
            if v:
                bad.append((kind, i, v, diag["sync_rounds"]))
        print(f"threads {threads} chain_after {chain}: {tot} stores outside the scan range; "
              f"images {bad[:12]}", flush=True)

"""Entropy-stage coefficients (dense_kernel) vs the oracle for a few cases:
where do they differ (DC / AC, which blocks)."""
import sys

sys.path.insert(0, ".")
import numpy as np  # noqa: E402

from oracle import oracle as O  # noqa: E402
from spdl_amd._lib import Decoder  # noqa: E402
from tests import cases  # noqa: E402

dec = Decoder(0)
for name in ["tiny_8x8", "q90_444", "q90_420"]:
    d = cases.case(name)
    info = O.parse(d)
    coefs, clean, diag = dec.debug_entropy(d, info.nblocks)
    ref = O.decode_coefs(d)[0]
    bad = np.argwhere(coefs != ref)
    print(name, "status", diag["status"], "nblocks", info.nblocks, "mismatch", len(bad))
    if len(bad):
        blks = np.unique(bad[:, 0])
        print("  blocks", blks[:10], "n", len(blks), "dc mism", int((coefs[:, 0] != ref[:, 0]).sum()))
        b = blks[0]
        print("  hyp", coefs[b][:16])
        print("  ref", ref[b][:16])

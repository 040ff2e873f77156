import sys
sys.path.insert(0, ".")
from oracle import oracle as O
from spdl_amd._lib import Decoder
from tests import cases
dec = Decoder(0)
for name in ["q90_420", "large_1080p"]:
    d = cases.case(name)
    info = O.parse(d)
    for _ in range(3):
        coefs, clean, diag = dec.debug_entropy(d, info.nblocks)
    sym, witer, clk, rt = diag["dbg"]
    print(name, diag["phase_us"], "symbols", sym, "wave-iter-sum", witer, "waves", 4,
          "clock GHz", round(clk / (rt * 10.0), 3), "cycles/iter", round(clk / (witer / 4), 1))

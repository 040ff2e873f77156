"""Entropy-kernel phase timings per workgroup size (diagnostic, GPU)."""
import sys

sys.path.insert(0, ".")
from oracle import oracle as O  # noqa: E402
from spdl_amd._lib import Decoder  # noqa: E402
from tests import cases  # noqa: E402

for threads in (256, 512, 1024):
    for mask in (0,):
        dec = Decoder(0)
        dec.set_param("entropy_threads", threads)
        dec.set_param("debug_mask", mask)
        for name in ["q90_420", "large_1080p"]:
            d = cases.case(name)
            info = O.parse(d)
            for _ in range(3):
                coefs, clean, diag = dec.debug_entropy(d, info.nblocks)
            sym, witer, clk, rt = diag["dbg"]
            print(f"T={threads} mask={mask} {name} phases_us={diag['phase_us']} "
                  f"rounds={diag['sync_rounds']} symbols={sym} wave_iter_sum={witer}", flush=True)
        dec.close()

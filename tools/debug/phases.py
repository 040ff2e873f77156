"""Entropy-kernel phase timers (wall_clock64 ticks -> us) of single images per
workgroup size: round 0 | sync rounds | block scan | mark pass, DC pass ticks."""
import sys

sys.path.insert(0, ".")
from oracle import oracle as O  # noqa: E402
from spdl_amd._lib import Decoder  # noqa: E402
from tests import cases  # noqa: E402

import os  # noqa: E402

for threads, warm in [tuple(map(int, c.split(":"))) for c in
                      os.environ.get("PH_CASES", "256:-1 512:-1").split()]:
    dec = Decoder(0)
    dec.set_param("entropy_threads", threads)
    if warm >= 0:
        dec.set_param("warmup_slots", warm)
    for name in ["q90_420", "large_1080p"]:
        d = cases.case(name)
        info = O.parse(d)
        for _ in range(3):
            coefs, clean, diag = dec.debug_entropy(d, info.nblocks)
        print(f"T={threads} warm={dec.get_param('warmup_slots')} {name} phases_us={diag['phase_us']} rounds={diag['sync_rounds']} "
              f"dc_us={diag['dbg'][0] / 100.0:.1f}", flush=True)
    dec.close()

"""Entropy phase timers (us) of each distinct bench image, decoded alone:
round 0 | sync rounds | block scan | write pass, DC pass; the slowest image
bounds a batch's entropy launch."""
import os
import sys

sys.path.insert(0, ".")
from oracle import oracle as O  # noqa: E402
from spdl_amd._lib import Decoder  # noqa: E402
from spdl_amd.synthetic import synthetic_slice  # noqa: E402

threads = int(os.environ.get("PH_THREADS", "512"))
dec = Decoder(0)
dec.set_param("entropy_threads", threads)
rows = []
for i, d in enumerate(synthetic_slice(range(32), distinct=32)):
    info = O.parse(d)
    for _ in range(2):
        coefs, clean, diag = dec.debug_entropy(d, info.nblocks)
    ph = diag["phase_us"]
    tot = sum(ph) + diag["dbg"][0] / 100.0
    rows.append((tot, i, len(d), ph, diag["sync_rounds"]))
rows.sort()
for tot, i, n, ph, r in rows:
    print(f"img {i:2d} bytes {n:6d} total {tot:6.1f} us phases {ph} rounds {r}", flush=True)

"""Entropy phase timers (us) of each image of the mixed set (bench.py
--workload mixed), decoded alone: which images bound a mixed batch's
entropy launch (size, restart intervals, optimised tables, pieces)."""
import os
import sys

sys.path.insert(0, ".")
from oracle import oracle as O  # noqa: E402
from spdl_amd._lib import Decoder  # noqa: E402
from spdl_amd.synthetic import mixed_jpeg, mixed_spec  # noqa: E402

threads = int(os.environ.get("PH_THREADS", "512"))
dec = Decoder(0)
dec.set_param("entropy_threads", threads)
if os.environ.get("PH_SUB"):
    dec.set_param("sub_bits", int(os.environ["PH_SUB"]))
if os.environ.get("PH_CHAIN"):
    dec.set_param("chain_after", int(os.environ["PH_CHAIN"]))
if os.environ.get("PH_WARM"):
    dec.set_param("warmup_slots", int(os.environ["PH_WARM"]))
rows = []
for i in range(64):
    d = mixed_jpeg(i)
    info = O.parse(d)
    for _ in range(2):
        coefs, clean, diag = dec.debug_entropy(d, info.nblocks)
    ph = diag["phase_us"]
    tot = sum(ph) + diag["dbg"][0] / 100.0
    s = mixed_spec(i)
    rows.append((tot, i, len(d), ph, diag["sync_rounds"], s, diag["dbg"]))
rows.sort(key=lambda r: r[0])
for tot, i, n, ph, r, s, dg in rows:
    print(f"img {i:2d} bytes {n:7d} {s['width']}x{s['height']} q{s['quality']} sub{s['subsampling']} "
          f"opt{int(s['optimize'])} rst{int(s['restart_rows'])} total {tot:7.1f} us phases "
          f"{[round(x, 1) for x in ph]} rounds {r} chain {(dg[1] & 0xFFFFFF) / 100.0:.1f} us "
          f"in {dg[1] >> 24} chains, {dg[2]} bits", flush=True)

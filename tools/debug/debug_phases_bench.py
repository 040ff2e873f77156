"""Entropy-kernel phase timings of the bench images, one image at a time
(diagnostic, GPU): which images set the batch kernel's tail."""
import sys

sys.path.insert(0, ".")
from oracle import oracle as O  # noqa: E402
from spdl_amd._lib import Decoder  # noqa: E402
from spdl_amd.synthetic import synthetic_batch  # noqa: E402

datas = synthetic_batch(32, distinct=32)
dec = Decoder(0)
if len(sys.argv) > 1:
    dec.set_param("warmup_slots", int(sys.argv[1]))
rows = []
for i, d in enumerate(datas):
    info = O.parse(d)
    for _ in range(2):
        coefs, clean, diag = dec.debug_entropy(d, info.nblocks)
    ph = diag["phase_us"]
    rows.append((sum(ph), i, len(d), diag["sync_rounds"], ph, diag["dbg"][0] / 100.0))
rows.sort(reverse=True)
print("warmup_slots", sys.argv[1:] or "default", "mean total", sum(r[0] for r in rows) / len(rows),
      "mean sync", sum(r[4][1] for r in rows) / len(rows), "mean round0", sum(r[4][0] for r in rows) / len(rows))
for tot, i, n, r, ph, dc in rows[:6]:
    print(f"img {i:2d} bytes {n:6d} rounds {r} total_us {tot:7.1f} phases {ph} dcfix_us {dc:.1f}")
dec.close()

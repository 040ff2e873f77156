"""Entropy phase timers (wall_clock64 ticks -> us) of one image per case, for
A/B of entropy-kernel variants (SPDL_AMD_LIB selects the library):
round 0 | sync rounds | block scan | relabel or write pass, and sync rounds."""
import sys

sys.path.insert(0, ".")
from oracle import oracle as O  # noqa: E402
from spdl_amd._lib import Decoder  # noqa: E402
from spdl_amd.synthetic import synthetic_jpeg  # noqa: E402

dec = Decoder(0)
for threads in (256, 512):
    dec.set_param("entropy_threads", threads)
    for seed in (1000, 1001, 1002):
        d = synthetic_jpeg(seed)
        info = O.parse(d)
        for _ in range(3):
            coefs, clean, diag = dec.debug_entropy(d, info.nblocks)
        print(threads, seed, "phases_us", diag["phase_us"], "sync_rounds", diag["sync_rounds"],
              "status", diag["status"], flush=True)

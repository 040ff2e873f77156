"""multiscan_kernel phase timings of one progressive 480x640 image (GPU)."""
import sys

sys.path.insert(0, ".")
from oracle import oracle as O  # noqa: E402
from spdl_amd._lib import Decoder  # noqa: E402
from spdl_amd.synthetic import synthetic_jpeg  # noqa: E402

dec = Decoder(0)
for prog in (True,):
    d = synthetic_jpeg(2000, progressive=prog)
    info = O.parse(d)
    for _ in range(2):
        coefs, clean, diag = dec.debug_entropy(d, info.nblocks)
    print("bytes", len(d), "scans", diag["sync_rounds"], "phase_us (walk, tables, decode, lists)",
          diag["phase_us"], "status", diag["status"])
dec.close()

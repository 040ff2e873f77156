"""Per-phase wall-clock of the multiscan decoder on single progressive images
(GPU): marker walk, table builds, scan decode, level -> list conversion, and
per scan its start / end (us from the decode start), symbols and ns/symbol.
python tools/prog_phases.py"""
import sys

sys.path.insert(0, ".")
from spdl_amd import _lib  # noqa: E402
from spdl_amd.synthetic import synthetic_jpeg  # noqa: E402

dec = _lib.Decoder(0)
for prog in (True, False):
    for seed in (2000, 2001):
        d = synthetic_jpeg(seed, progressive=prog)
        info = _lib.get_image_info(d)
        nb = -(-info.width // 16) * -(-info.height // 16) * 6
        for _ in range(2):
            _, _, diag = dec.debug_entropy(d, nb)
        print(f"progressive={prog} seed {seed} bytes {len(d)}: phases_us {diag['phase_us']} "
              f"status {diag['status']} scans/rounds {diag['sync_rounds']} dbg {diag['dbg']}",
              flush=True)
        if prog:
            for s, (t0, t1, ns) in enumerate(diag["scans"][:diag["sync_rounds"]]):
                us = (t1 - t0) / 100.0
                print(f"   scan {s}: {t0 / 100:8.1f} .. {t1 / 100:8.1f} us  symbols {ns:6d}  "
                      f"{(us * 1000 / ns) if ns else 0:7.1f} ns/symbol", flush=True)
dec.close()

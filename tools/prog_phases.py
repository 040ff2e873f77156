"""Per-phase wall-clock of the multiscan decoder on single progressive images
(GPU): marker walk, table builds, scan decode, level -> list conversion.
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
dec.close()

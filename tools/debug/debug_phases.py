import sys
sys.path.insert(0, ".")
from oracle import oracle as O
from spdl_amd._lib import Decoder
from tests import cases
dec = Decoder(0)
for sub in (512, 1024, 2048):
    dec.set_param("sub_bits", sub)
    for name in ["q90_420", "q95_420", "noise_420", "restart_rows", "large_1080p"]:
        d = cases.case(name)
        info = O.parse(d)
        for _ in range(2):
            coefs, clean, diag = dec.debug_entropy(d, info.nblocks)
        print(sub, name, diag)

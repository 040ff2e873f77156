import sys
sys.path.insert(0, ".")
from oracle import oracle as O
from spdl_amd._lib import Decoder
from spdl_amd.synthetic import synthetic_jpeg
dec = Decoder(0)
for seed in (1000, 1001):
    d = synthetic_jpeg(seed)
    info = O.parse(d)
    for _ in range(3):
        coefs, clean, diag = dec.debug_entropy(d, info.nblocks)
    sc = diag["scans"]
    flat = [x for t in sc for x in t]
    print(seed, "parse phase ticks (10 ns) from start:", flat[40:47])

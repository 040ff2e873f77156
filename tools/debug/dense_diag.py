import sys
sys.path.insert(0, ".")
import numpy as np
from oracle import oracle as O
from spdl_amd._lib import Decoder
from tests import cases
dec = Decoder(0)
d = cases.case("tiny_8x8")
info = O.parse(d)
coefs, clean, diag = dec.debug_entropy(d, info.nblocks)
for j in range(info.nblocks):
    v = coefs[j].view(np.uint16).astype(np.uint32)
    vals = [int(v[2*i]) | (int(v[2*i+1]) << 16) for i in range(12)]
    print(j, ["%08x" % x for x in vals])
print("clean", clean[:32].tobytes().hex())

import sys, math, ctypes as C
sys.path[:0] = ['.', 'posggym-baselines_amd']
import numpy as np
from posggym_baselines_amd import _native as N
xs = []
for Nn in range(1, 3000):
    sq = math.sqrt(Nn)
    for v in range(0, Nn + 1, max(1, Nn // 40)):
        xs.append(v / sq)
rng = np.random.default_rng(0)
xs += list(rng.random(500000) * 300)
x = np.array(xs, dtype=np.float64)
out = np.zeros_like(x)
P = C.POINTER(C.c_double)
assert N.load().pomcp_debug_exp(x.ctypes.data_as(P), len(x), out.ctypes.data_as(P)) == 0
ref = np.array([math.exp(v) for v in x])
bad = np.nonzero(out != ref)[0]
print("n", len(x), "mismatches", len(bad))
for i in bad[:10]:
    print(x[i].hex(), out[i].hex(), ref[i].hex())

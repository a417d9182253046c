"""Time string FE factorization on the device vs the host's np.unique (one column of n
strings drawn from G distinct ids), and check that both group the rows identically."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np

from leanfe_amd import frame
from leanfe_amd._lib import Engine

n, G = int(sys.argv[1]), int(sys.argv[2])
rng = np.random.default_rng(1)
pool = np.array([f"firm-{i:07d}-{rng.integers(1 << 30):x}" for i in range(G)], dtype=object)
v = pool[rng.integers(0, G, n)]
with Engine(0) as eng:
    frame.factorize(v[:1000], device=eng)  # warm-up (allocations, module load)
    t0 = time.perf_counter()
    sb = frame.string_buffers(v)
    t1 = time.perf_counter()
    codes, g = eng.factorize_strings(*sb)
    t2 = time.perf_counter()
t3 = time.perf_counter()
uniq, inv = np.unique(v.astype(str), return_inverse=True)
t4 = time.perf_counter()
pairs = np.unique(np.stack([codes.astype(np.int64), inv.ravel().astype(np.int64)], axis=1), axis=0).shape[0]
print(json.dumps(dict(n=n, distinct=G, levels=g, same_grouping=bool(g == uniq.size == pairs),
                      arrow_s=round(t1 - t0, 3), device_s=round(t2 - t1, 3), np_unique_s=round(t4 - t3, 3),
                      bytes=int(sb[1].size))))

"""Helpers to read tests/golden/*.npz fixtures (inputs + expected outputs)."""
import glob
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz")))


def load(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    meta = json.loads(bytes(z["meta"]).decode())
    data = {k[3:]: z[k] for k in z.files if k.startswith("in_")}
    exp = {k: z[k] for k in z.files if not k.startswith("in_") and k != "meta"}
    return meta, data, exp


def ncl(v):
    if v is None:
        return None
    if isinstance(v, (list, tuple)):
        return tuple(int(x) for x in v)
    return int(v)

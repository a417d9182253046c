"""A wide fit at scale (more than 63 columns: column blocks of contexts, lfe_wide.hip), resident
and streamed, timed end to end through leanfe_hip from host NumPy columns (H2D included).  Prints
one JSON line; the panel is drawn with NumPy's generator (not the device generator: the columns
must exist on the host for leanfe_hip), so the check is against the generating beta.

    python tools/wide_run.py [--rows 10000000] [--k 100] [--levels 100000,1000]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--levels", default="100000,1000")
    a = ap.parse_args()
    from leanfe_amd import leanfe_hip

    n, k = a.rows, a.k
    L = [int(v) for v in a.levels.split(",")]
    rng = np.random.default_rng(7)
    fe = [rng.integers(0, g, n).astype(np.int32) for g in L]
    eff = [rng.normal(size=g) * (1.0 if f == 0 else 0.5) for f, g in enumerate(L)]
    beta = np.linspace(1.0, 0.1, k)
    d = {f"fe{f + 1}": fe[f] for f in range(len(L))}
    y = rng.normal(size=n)
    for f in range(len(L)):
        y += eff[f][fe[f]]
    for j in range(k):
        x = rng.normal(size=n) + 0.5 * eff[0][fe[0]]
        d[f"x{j + 1}"] = x
        y += beta[j] * x
    d["y"] = y
    xs = [f"x{j + 1}" for j in range(k)]
    fes = [f"fe{f + 1}" for f in range(len(L))]
    out = dict(kind="wide fit through leanfe_hip (host NumPy columns, H2D included)", rows=n, k=k, levels=L)
    for mode, kw in (("resident", {}), ("streamed", dict(out_of_core=True, chunk_rows=1 << 22))):
        for vcov, cl in (("HC1", None), ("cluster", ["fe1"])):
            times = []
            for _ in range(2):
                t0 = time.perf_counter()
                r = leanfe_hip(d, y_col="y", x_cols=xs, fe_cols=fes, strategy="alt_proj", vcov=vcov, cluster_cols=cl,
                               quiet=True, **kw)
                times.append(time.perf_counter() - t0)
            b = np.array([r.coefs[x] for x in xs])
            se = np.array([r.std_errors[x] for x in xs])
            out[f"{mode}_{vcov}"] = dict(seconds=[round(t, 3) for t in times], iterations=r.iterations,
                                         max_abs_t_vs_generating_beta=float(np.max(np.abs(b - beta) / se)),
                                         n_clusters=r.n_clusters)
            print(json.dumps({mode + "_" + vcov: out[f"{mode}_{vcov}"]}), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

"""The C restatement (oracle/altproj_c.c: bench.py's CPU baseline and the full-size
parity checker) against the golden fixtures' oracle outputs and against the NumPy
oracle (oracle/altproj.py): same iterations / n_obs / df_resid / cluster counts,
beta and SE to 1e-10 (unweighted IID, HC1, one-way and multi-way CGM cluster)."""
from __future__ import annotations

import shutil

import numpy as np
import pytest

from golden_util import load, names, ncl

pytestmark = pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")


def _unweighted_ols(n):
    m = load(n)[0]
    return (m["strategy"] == "alt_proj" and not m.get("weights") and not m.get("instruments")
            and m["vcov"].lower() in ("iid", "hc1", "cluster"))


CASES = [n for n in names() if _unweighted_ols(n)]


def _codes(a):
    u, inv = np.unique(a, return_inverse=True)
    return inv.astype(np.int32).ravel(), len(u)


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("threads", [1, 4])
def test_c_oracle_matches_golden(name, threads):
    from oracle.altproj_c import fit_c

    meta, data, exp = load(name)
    cols = [data[meta["y"]]] + [data[x] for x in meta["xs"]]
    codes, levels = zip(*[_codes(data[f]) for f in meta["fes"]])
    cl = [_codes(data[c]) for c in (meta.get("cluster_cols") or [])]
    r = fit_c(cols, list(codes), list(levels), vcov=meta["vcov"], tol=meta["demean_tol"], max_iter=meta["max_iter"],
              threads=threads, cl_codes=[c for c, _ in cl] or None, cl_levels=[g for _, g in cl] or None,
              ssc=meta["ssc"])
    assert r["iterations"] == int(exp["oracle_iterations"])
    assert r["n_obs"] == int(exp["oracle_n_obs"])
    assert r["df_resid"] == int(exp["oracle_df_resid"])
    np.testing.assert_allclose(r["beta"], exp["oracle_beta"], rtol=1e-10, atol=1e-13)
    np.testing.assert_allclose(r["se"], exp["oracle_se"], rtol=1e-10, atol=1e-14)
    if meta["vcov"] == "cluster":
        assert ncl(r["n_clusters"]) == ncl(meta["oracle_n_clusters"])


@pytest.mark.parametrize("m", [1, 2, 3])
def test_c_oracle_cluster_vs_numpy_oracle(m):
    """Random 3-FE panel with singletons, m-way CGM on columns with repeated and
    nested levels: the C intersection group-by against np.unique on stacked keys."""
    from oracle import altproj
    from oracle.altproj_c import fit_c

    rng = np.random.default_rng(7 + m)
    n = 30_000
    d = {"fe1": rng.integers(0, 3000, n), "fe2": rng.integers(0, 200, n), "fe3": rng.integers(0, 40, n)}
    d["fe1"][:25] = 10_000 + np.arange(25)  # singleton levels
    d["c1"] = d["fe2"] // 3                 # nested in fe2
    d["c2"] = rng.integers(0, 57, n)
    d["c3"] = rng.integers(0, 5, n)
    xs = ["x1", "x2", "x3"]
    for j, x in enumerate(xs):
        d[x] = rng.standard_normal(n) + 0.1 * (d["fe1"] % 7) * (j + 1)
    d["y"] = sum((j + 1) * d[x] for j, x in enumerate(xs)) + 0.01 * d["fe2"] + rng.standard_normal(n)
    cc = ["c1", "c2", "c3"][:m]
    o = altproj.fit(d, "y", xs, ["fe1", "fe2", "fe3"], vcov="cluster", cluster_cols=cc)
    codes, levels = zip(*[_codes(d[f]) for f in ("fe1", "fe2", "fe3")])
    cl = [_codes(d[c]) for c in cc]
    outs = [fit_c([d["y"]] + [d[x] for x in xs], list(codes), list(levels), vcov="cluster", threads=t,
                  cl_codes=[c for c, _ in cl], cl_levels=[g for _, g in cl]) for t in (1, 3)]
    for r in outs:
        assert r["iterations"] == o["iterations"] and r["n_obs"] == o["n_obs"] and r["df_resid"] == o["df_resid"]
        assert ncl(r["n_clusters"]) == ncl(o["n_clusters"])
        np.testing.assert_allclose(r["beta"], o["beta"], rtol=1e-10)
        np.testing.assert_allclose(r["se"], o["se"], rtol=1e-10)
    # intersection counts against np.unique of the stacked kept columns
    keep = o["keep"]
    for s, G in zip(outs[0]["subsets"], outs[0]["G_subsets"]):
        stacked = np.stack([d[cc[j]][keep] for j in s], axis=1)
        assert G == np.unique(stacked, axis=0).shape[0]


def test_c_oracle_r2_and_deterministic():
    from oracle import altproj
    from oracle.altproj_c import fit_c

    meta, data, exp = load("synth_hc1")
    cols = [data[meta["y"]]] + [data[x] for x in meta["xs"]]
    codes, levels = zip(*[_codes(data[f]) for f in meta["fes"]])
    a = fit_c(cols, list(codes), list(levels), vcov="HC1", threads=4)
    b = fit_c(cols, list(codes), list(levels), vcov="HC1", threads=4)
    assert np.array_equal(a["beta"], b["beta"]) and np.array_equal(a["se"], b["se"])  # fixed thread count
    o = altproj.fit(data, meta["y"], meta["xs"], meta["fes"], vcov="HC1")
    np.testing.assert_allclose(a["r_squared"], o["r_squared"], rtol=1e-10)

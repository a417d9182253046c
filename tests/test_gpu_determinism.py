"""Deterministic reductions (no f64 atomics on the parity path).

Every group sum, weight sum and cross term of the demeaning loop is a two-limb fixed-point sum
(lfe_internal.h: a fine int64 limb per value, and a coarse integer-valued f64 limb that only
outliers and non-finite values touch), the T_Q run sums are reduced in bucket order, the Gram /
meat partials in block order and the cluster scores in sorted order, so solving the same panel
twice must give bit-identical beta, SE, RSS and `iterations` - within one context and across
two contexts, whatever the data's range: a column with one value 1e9 x its RMS, a heavy-tailed
weight column and an FE level with a huge effect included.  Each case also keeps parity with
the CPU restatement (oracle/altproj.py, polars_impl.py:468-537) at 1e-10 with equal
`iterations` (the integer the stop test at polars_impl.py:511-526 produces)."""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _solve(eng, vcov="hc1"):
    import bench

    return bench.solve_step(eng, vcov)


def _same(a, b):
    assert a["iterations"] == b["iterations"]
    assert a["n_obs"] == b["n_obs"] and a["df_resid"] == b["df_resid"]
    np.testing.assert_array_equal(a["beta"], b["beta"])
    np.testing.assert_array_equal(a["se"], b["se"])
    assert a["rss"] == b["rss"]


@pytest.mark.parametrize("n,L", [(2_000_000, [20_000, 500]), (3_000_017, [100_000, 1_000])])
def test_same_panel_twice_is_bit_identical(n, L):
    from leanfe_amd import synth
    from leanfe_amd._lib import Engine

    k = 10
    runs = []
    for _ in range(2):  # two contexts
        with Engine(0) as eng:
            eng.synth_load(n, k, L, synth.betas(k), seed=777)
            first = _solve(eng)
            assert eng.exact_sums(), "the headline geometry should take the exact group sums"
            second = _solve(eng)  # same context: layout, sums and sweeps rebuilt
            _same(first, second)
            runs.append(first)
    _same(runs[0], runs[1])


@pytest.mark.parametrize("units", ["256", "4096", "100000"])
def test_sweep_work_units_do_not_change_bits(units, knob):
    """K1 (lfe_iter.hip k_tp) sums every segment in batches aligned to absolute 16-group
    boundaries, so its results do not depend on how the segments are split into work units (the
    unit size follows the shard size and the CU count)."""
    from leanfe_amd import synth
    from leanfe_amd._lib import Engine

    n, k, L = 2_000_000, 6, [20_000, 500]
    with Engine(0) as eng:
        eng.synth_load(n, k, L, synth.betas(k), seed=91)
        ref = _solve(eng)
        knob.setenv("LFE_K1_UNIT", units)
        other = _solve(eng)
    _same(ref, other)


def _fit_pair(data, xs):
    from leanfe_amd import leanfe_hip
    from oracle import altproj

    r = leanfe_hip(data, y_col="y", x_cols=xs, fe_cols=["fe1", "fe2"], strategy="alt_proj", vcov="HC1",
                   quiet=True, device=0)
    o = altproj.fit(data, "y", xs, ["fe1", "fe2"], vcov="HC1")
    b = np.array([r.coefs[x] for x in xs])
    s = np.array([r.std_errors[x] for x in xs])
    assert r.iterations == o["iterations"] and r.n_obs == o["n_obs"]
    np.testing.assert_allclose(b, o["beta"], rtol=1e-10, atol=0)
    np.testing.assert_allclose(s, o["se"], rtol=1e-10, atol=0)
    return b, s, r.iterations


def _fit_pair_fe(data, xs, fes, **kw):
    from leanfe_amd import leanfe_hip
    from oracle import altproj

    vcov = kw.pop("vcov", "HC1")
    r = leanfe_hip(data, y_col="y", x_cols=xs, fe_cols=fes, strategy="alt_proj", vcov=vcov, quiet=True, device=0,
                   **kw)
    o = altproj.fit(data, "y", xs, fes, vcov=vcov, **kw)
    b = np.array([r.coefs[x] for x in xs])
    s = np.array([r.std_errors[x] for x in xs])
    assert r.iterations == o["iterations"] and r.n_obs == o["n_obs"], (r.iterations, o["iterations"])
    np.testing.assert_allclose(b, o["beta"], rtol=1e-10, atol=0)
    np.testing.assert_allclose(s, o["se"], rtol=1e-10, atol=0)
    return b, s, r.iterations


def _twice(data, xs, fes, **kw):
    b1, s1, it1 = _fit_pair_fe(data, xs, fes, **dict(kw))
    b2, s2, it2 = _fit_pair_fe(data, xs, fes, **dict(kw))
    np.testing.assert_array_equal(b1, b2)
    np.testing.assert_array_equal(s1, s2)
    assert it1 == it2


def _with_outlier(data, col, row, value):
    data = dict(data)
    x = np.array(data[col], copy=True)
    x[row] = value
    data[col] = x
    return data


@pytest.mark.parametrize("value", [1e6, 1e9, -3e12])
def test_outlier_column_is_bit_identical_and_keeps_parity(value):
    """One value far outside the column's range (max |x| >> 64 RMS) used to make the fit fall back
    to f64 atomic sums; the coarse limb now carries it and the fit repeats bit for bit."""
    from leanfe_amd import synth

    xs = [f"x{j + 1}" for j in range(6)]
    data = synth.panel(400_000, 6, [8_000, 300], seed=4242)
    _twice(data, xs, ["fe1", "fe2"])
    _twice(_with_outlier(data, "x3", 12345, value), xs, ["fe1", "fe2"])


def test_outlier_y_reports_exact_sums():
    from leanfe_amd import synth
    from leanfe_amd._lib import Engine

    data = synth.panel(200_000, 3, [5_000, 200], seed=99)
    cols = [np.ascontiguousarray(data[c], dtype=np.float64) for c in ["y", "x1", "x2", "x3"]]
    cols[0] = cols[0].copy()
    cols[0][7] = 1e9
    codes = [np.ascontiguousarray(data[f], dtype=np.int32) for f in ["fe1", "fe2"]]
    with Engine(0) as eng:
        eng.load(cols, codes, [5_000, 200])
        eng.drop_singletons()
        assert eng.exact_sums()


@pytest.mark.parametrize("case", ["x_outlier", "large_effect_level", "heavy_tail"])
def test_general_sweeps_with_outliers_keep_parity(case):
    """F = 3 (lfe_seg.hip): an x outlier, one FE level whose effect is 1e8 x the others (its rows'
    cross terms take the coarse limb) and a heavy-tailed regressor (Student t, 1 dof):
    two solves bit-identical, beta / SE at 1e-10 of the oracle with equal iterations."""
    from leanfe_amd import synth

    L = [30_000, 4_000, 300]
    data = dict(synth.panel(600_000, 3, L, seed=2718))
    xs = ["x1", "x2", "x3"]
    fes = ["fe1", "fe2", "fe3"]
    if case == "x_outlier":
        data = _with_outlier(data, "x2", 4321, 5e9)
    elif case == "large_effect_level":
        y = np.array(data["y"], copy=True)
        y[np.asarray(data["fe2"]) == 17] += 1e8
        data["y"] = y
    else:
        data["x1"] = np.random.default_rng(11).standard_t(1.0, size=600_000)
    _twice(data, xs, fes)


@pytest.mark.parametrize("n,L,vcov", [(1_500_000, [60_000, 8_000, 500], "HC1"),   # config 4's shape (F = 3)
                                      (1_000_000, [20_000, 5_000], "iid")])        # G_Q too large for the fast path
def test_general_sweeps_are_bit_identical(n, L, vcov):
    """The general sweeps (lfe_seg.hip) rank their per-FE segment layouts with global cursor
    atomics; their group sums and cross terms sum in int64 (k_sums4 exact path,
    k_seg_cross / k_cross_quanta), so two solves agree bit for bit anyway."""
    from leanfe_amd import leanfe_hip, synth
    k = 4
    data = synth.panel(n, k, L, seed=313)
    xs = [f"x{j + 1}" for j in range(k)]
    fes = [f"fe{f + 1}" for f in range(len(L))]
    runs = [leanfe_hip(data, y_col="y", x_cols=xs, fe_cols=fes, strategy="alt_proj", vcov=vcov, quiet=True,
                       device=0) for _ in range(2)]
    for r in runs[1:]:
        assert r.iterations == runs[0].iterations and r.n_obs == runs[0].n_obs
        np.testing.assert_array_equal([r.coefs[x] for x in xs], [runs[0].coefs[x] for x in xs])
        np.testing.assert_array_equal([r.std_errors[x] for x in xs], [runs[0].std_errors[x] for x in xs])


@pytest.mark.parametrize("L,skew", [([20_000, 500], False), ([30_000, 2_000, 300], False), ([20_000, 500], True),
                                    ([30_000, 2_000, 300], True)])
def test_weighted_fits_are_bit_identical_and_keep_parity(L, skew):
    """Weighted fits sum w x, w and the stop test's raw y in two-limb fixed point too (quanta from
    the statistics of k_col_stats_w; k_sums4, k_sweep_sums and the weighted cross terms of
    k_seg_cross), so two solves agree bit for bit and still match the oracle at 1e-10 - also with
    one weight 1e6 x the rest."""
    from leanfe_amd import leanfe_hip, synth
    from leanfe_amd._lib import Engine
    from oracle import altproj
    k, n = 3, 300_000
    data = dict(synth.panel(n, k, L, seed=515))
    w = np.random.default_rng(7).uniform(0.5, 2.0, n)
    if skew:
        w[4321] = 1e6
    data["w"] = w
    xs = [f"x{j + 1}" for j in range(k)]
    fes = [f"fe{f + 1}" for f in range(len(L))]
    runs = []
    with Engine(0) as eng:
        for _ in range(2):
            runs.append(leanfe_hip(data, y_col="y", x_cols=xs, fe_cols=fes, strategy="alt_proj", weights="w",
                                   vcov="HC1", quiet=True, engine=eng))
            assert eng.exact_sums()
    r0, r1 = runs
    assert r1.iterations == r0.iterations and r1.n_obs == r0.n_obs
    np.testing.assert_array_equal([r1.coefs[x] for x in xs], [r0.coefs[x] for x in xs])
    np.testing.assert_array_equal([r1.std_errors[x] for x in xs], [r0.std_errors[x] for x in xs])
    o = altproj.fit(data, "y", xs, fes, vcov="HC1", weights="w")
    r = runs[0]
    assert r.iterations == o["iterations"] and r.n_obs == o["n_obs"]
    np.testing.assert_allclose([r.coefs[x] for x in xs], o["beta"], rtol=1e-10, atol=0)
    np.testing.assert_allclose([r.std_errors[x] for x in xs], o["se"], rtol=1e-10, atol=0)


@pytest.mark.parametrize("case", ["long_clusters", "short_clusters_with_a_long_one"])
def test_clustered_se_is_bit_identical(case):
    """Cluster score sums add the parts of a cluster cut by work-unit / wave edges in a fixed
    order (k_seg_chain, k_seg_rows_chain) instead of f64 atomics: one-way clusters of ~6700 rows
    (seg_gather_sum, many units per cluster) and two-way CGM intersections of a few rows with
    one 3000-row cluster spanning dozens of waves (k_seg_rows) repeat bit for bit and match the
    oracle's clustered SE (std_errors.py:289-441) at 1e-10."""
    from leanfe_amd import leanfe_hip, synth
    from oracle import altproj
    n, k = 400_000, 3
    L = [8_000, 60, 700] if case == "long_clusters" else [8_000, 20_000, 9_000]
    data = dict(synth.panel(n, k, L, seed=808))
    cl = ["fe2"] if case == "long_clusters" else ["fe2", "fe3"]
    if case != "long_clusters":  # one large intersection cluster
        fe2, fe3 = np.array(data["fe2"], copy=True), np.array(data["fe3"], copy=True)
        fe2[1000:4000], fe3[1000:4000] = 7, 11
        data["fe2"], data["fe3"] = fe2, fe3
    xs = [f"x{j + 1}" for j in range(k)]
    runs = [leanfe_hip(data, y_col="y", x_cols=xs, fe_cols=["fe1"], strategy="alt_proj", vcov="cluster",
                       cluster_cols=cl, quiet=True, device=0) for _ in range(2)]
    r0, r1 = runs
    np.testing.assert_array_equal([r1.std_errors[x] for x in xs], [r0.std_errors[x] for x in xs])
    np.testing.assert_array_equal([r1.coefs[x] for x in xs], [r0.coefs[x] for x in xs])
    o = altproj.fit(data, "y", xs, ["fe1"], vcov="cluster", cluster_cols=cl)
    np.testing.assert_allclose([r0.std_errors[x] for x in xs], o["se"], rtol=1e-10, atol=0)

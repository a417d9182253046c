"""Clustered SEs: one-column subsets by two-limb fixed-point sums (lfe_cluster.hip subset_meat_fix).

A one-column cluster subset's clusters are the column's codes, so the per-cluster score sums
S_c = sum_{i in c} x~_i r_i (w_i) (std_errors.py:317-333) are formed the way the group sums are -
fine limbs by int64 adds, outliers' coarse limbs by integer-valued f64 adds - into a table indexed
by the code, with no sort.  Against the sorted path (the LFE_TEST_CLUSTER_SORTED hook: keys, radix sort, segmented sums)
and the CPU oracle (oracle/altproj.py: std_errors.py:289-441): one-way and multi-way CGM (the
intersection subset still sorts), clusters on FE columns (reg_test.py:55, 61) and on a column that
is no FE, weights, a 5e9 outlier (coarse limbs), bit-identical repeats, and an emulated 2-rank
group (the table all-reduced)."""
from __future__ import annotations

import threading

import numpy as np
import pytest

from leanfe_amd import synth

pytestmark = pytest.mark.gpu


SORTED, STATS = 2, 4  # LFE_TEST_CLUSTER_SORTED, LFE_TEST_CLUSTER_STATS (include/leanfe_hip.h)


def _fit(data, xs, fes, cl, hooks=0, **kw):
    """The fit on its own engine with the given test hooks: 0 = the sort-free sums with quanta from
    the residual pass's meat, STATS = from a statistics pass, SORTED = the sorted path."""
    from leanfe_amd import leanfe_hip
    from leanfe_amd._lib import Engine

    with Engine(0) as eng:
        if hooks:
            eng.test_hooks(hooks)
        eng.profile(True)
        r = leanfe_hip(data, y_col="y", x_cols=xs, fe_cols=fes, strategy="alt_proj", vcov="cluster",
                       cluster_cols=cl, quiet=True, engine=eng, **kw)
        r.kernels = set(eng.kernel_stats())  # which cluster paths ran ("cluster_fix": the sort-free sums)
        return r


def _arr(r, xs, what):
    return np.array([getattr(r, what)[x] for x in xs])


CASES = [
    ("fe_oneway", [20_000, 600], ["fe1"], None),
    ("fe_twoway", [20_000, 600], ["fe1", "fe2"], None),
    ("fe_twoway_primary_second", [20_000, 600], ["fe2", "fe1"], None),  # the primary FE second
    ("other_oneway_weighted", [20_000, 600], ["grp"], "w"),
    ("fe3_cgm_outlier", [9_000, 800, 150], ["fe2", "fe3"], None),
]


@pytest.mark.parametrize("name,L,cl,weights", CASES, ids=[c[0] for c in CASES])
def test_one_column_subsets_without_sort(name, L, cl, weights):
    from oracle import altproj

    n, k = 500_000, 4
    xs = [f"x{j + 1}" for j in range(k)]
    fes = [f"fe{f + 1}" for f in range(len(L))]
    d = dict(synth.panel(n, k, L, seed=71))
    rng = np.random.default_rng(71)
    d["grp"] = rng.integers(0, 3_000, n)
    if weights:
        d["w"] = rng.uniform(0.5, 2.0, n)
    if "outlier" in name:
        x = np.array(d["x2"], copy=True)
        x[777] = 5e9
        d["x2"] = x
    kw = dict(weights=weights) if weights else {}
    fix = _fit(d, xs, fes, cl, **kw)
    again = _fit(d, xs, fes, cl, **kw)
    st = _fit(d, xs, fes, cl, hooks=STATS, **kw)
    srt = _fit(d, xs, fes, cl, hooks=SORTED, **kw)
    o = altproj.fit(d, "y", xs, fes, vcov="cluster", cluster_cols=cl, weights=weights)
    ncl = o["n_clusters"]
    assert fix.n_clusters == srt.n_clusters
    assert (tuple(fix.n_clusters) if isinstance(fix.n_clusters, (list, tuple)) else fix.n_clusters) == (
        tuple(ncl) if isinstance(ncl, (list, tuple)) else ncl)
    assert fix.iterations == o["iterations"] and fix.n_obs == o["n_obs"]
    np.testing.assert_allclose(_arr(fix, xs, "coefs"), o["beta"], rtol=1e-10, atol=0)
    np.testing.assert_allclose(_arr(fix, xs, "std_errors"), o["se"], rtol=1e-10, atol=0)
    np.testing.assert_allclose(_arr(fix, xs, "std_errors"), _arr(srt, xs, "std_errors"), rtol=1e-12, atol=0)
    np.testing.assert_allclose(_arr(st, xs, "std_errors"), _arr(srt, xs, "std_errors"), rtol=1e-12, atol=0)
    # the comparisons are between different computations: the sort-free sums ran in fix and st only
    assert "cluster_fix" in fix.kernels and "cluster_fix" in st.kernels and "cluster_fix" not in srt.kernels
    np.testing.assert_array_equal(_arr(fix, xs, "std_errors"), _arr(again, xs, "std_errors"))


def test_one_column_subset_on_emulated_ranks():
    """Row-sharded ranks: each rank's fixed-point table goes into the all-reduced key-indexed table;
    every rank equals the oracle on the whole panel and all ranks agree bit for bit."""
    from leanfe_amd import inference
    from leanfe_amd._lib import EmuGroup, Engine
    from leanfe_amd.dist import shard_range
    from oracle import altproj

    world, n, k, L = 3, 450_001, 3, [6_000, 300]
    data = synth.panel(n, k, L, seed=88)
    group, out, errs = EmuGroup(world), {}, []

    def work(r):
        lo, hi = shard_range(n, r, world)
        try:
            with Engine(0) as eng:
                eng.set_emu(group, r)
                eng.synth_load(hi - lo, k, L, synth.betas(k), seed=88, row_offset=lo)
                _, codes = eng.copy_inputs()
                eng.load_clusters([np.ascontiguousarray(codes[1])], [L[1]])
                n_obs, dims, card = eng.drop_singletons()
                it, _ = eng.demean(sorted(range(2), key=lambda i: card[i]), 1e-6, 50, check_from=3)
                G = eng.gram()
                bf, XtX_inv = inference.solve_normal(*inference.split_gram(G))
                eng.resid(bf, hc1=False, keep_scores=True)
                meats, Gs = eng.cluster_meat()
                df = n_obs - (k + 1) - (sum(dims) - 2)
                se, ncl = inference.se_cluster_oneway(XtX_inv[1:, 1:], meats[0], int(Gs[0]), n_obs, df, True)
                out[r] = dict(se=se, ncl=ncl, it=it)
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            group.abort()

    ts = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not errs, errs
    xs = [f"x{j + 1}" for j in range(k)]
    o = altproj.fit(data, "y", xs, ["fe1", "fe2"], vcov="cluster", cluster_cols=["fe2"])
    for r in range(world):
        assert out[r]["it"] == o["iterations"] and out[r]["ncl"] == o["n_clusters"]
        np.testing.assert_allclose(out[r]["se"], o["se"], rtol=1e-10, atol=0)
        np.testing.assert_array_equal(out[r]["se"], out[0]["se"])


@pytest.mark.parametrize("cl", [["fe2"], ["fe1"]])
def test_non_finite_scores_take_the_statistics_pass(cl):
    """A NaN score value raises the bound flag of the quanta that need no statistics pass (its coarse
    limb is not finite): the one-way sums on the primary FE formed in the residual pass (fe1) redo
    the pass with score rows, the sort-free sums (fe2) redo the subset with a statistics pass; NaN
    propagates into the same SEs as on the sorted path (std_errors.py:317-333 on NaN data)."""
    n, k, L = 200_000, 3, [5_000, 300]
    xs = [f"x{j + 1}" for j in range(k)]
    d = dict(synth.panel(n, k, L, seed=91))
    x = np.array(d["x2"], copy=True)
    x[1234] = np.nan
    d["x2"] = x
    fix = _fit(d, xs, ["fe1", "fe2"], cl)
    srt = _fit(d, xs, ["fe1", "fe2"], cl, hooks=SORTED)
    a, b = _arr(fix, xs, "std_errors"), _arr(srt, xs, "std_errors")
    np.testing.assert_array_equal(np.isnan(a), np.isnan(b))
    assert "cluster_fix" in fix.kernels


@pytest.mark.parametrize("k,L,singletons", [(4, [20_000, 600], 0), (10, [30_000, 1_000], 0), (6, [25_000, 800], 40)])
def test_one_way_cluster_on_the_primary_fe_in_the_residual_pass(k, L, singletons):
    """A one-way cluster on the primary FE (reg_test.py:55): its sums come out of the residual pass
    (k_resid_rows<.., true>: no score rows), against the separate sort-free sums (statistics hook),
    the sorted path and the oracle; bit-identical repeats."""
    from oracle import altproj

    n = 600_000
    xs = [f"x{j + 1}" for j in range(k)]
    d = dict(synth.panel(n, k, L, seed=57))
    if singletons:  # rows alone in their primary level: dropped (polars_impl.py:477-482), still keyed
        f1 = np.array(d["fe1"], copy=True)
        f1[:singletons] = L[0] + np.arange(singletons)
        d["fe1"] = f1
    fused = _fit(d, xs, ["fe1", "fe2"], ["fe1"])
    again = _fit(d, xs, ["fe1", "fe2"], ["fe1"])
    st = _fit(d, xs, ["fe1", "fe2"], ["fe1"], hooks=STATS)
    srt = _fit(d, xs, ["fe1", "fe2"], ["fe1"], hooks=SORTED)
    o = altproj.fit(d, "y", xs, ["fe1", "fe2"], vcov="cluster", cluster_cols=["fe1"])
    assert fused.n_clusters == o["n_clusters"] == srt.n_clusters
    assert fused.iterations == o["iterations"] and fused.n_obs == o["n_obs"] == n - singletons
    np.testing.assert_allclose(_arr(fused, xs, "std_errors"), o["se"], rtol=1e-10, atol=0)
    np.testing.assert_allclose(_arr(fused, xs, "std_errors"), _arr(srt, xs, "std_errors"), rtol=1e-12, atol=0)
    np.testing.assert_allclose(_arr(st, xs, "std_errors"), _arr(srt, xs, "std_errors"), rtol=1e-12, atol=0)
    np.testing.assert_array_equal(_arr(fused, xs, "std_errors"), _arr(again, xs, "std_errors"))


INTERSECTIONS = [
    # (levels, cluster columns, weighted): the primary FE (most levels) first, second, and in a
    # three-way subset; 120K rows on 40K primary levels leave many singletons (dropped rows inside
    # the buckets); weighted fits sum every subset's clusters from the sorted rows (no singleton form)
    ([40_000, 700], ["fe1", "fe2"], False),
    ([40_000, 700], ["fe2", "fe1"], False),
    ([40_000, 700, 90], ["fe3", "fe1", "fe2"], False),
    ([40_000, 700, 90], ["fe3", "fe1", "fe2"], True),
]


@pytest.mark.parametrize("L,cl,weighted", INTERSECTIONS,
                         ids=["primary_first", "primary_second", "three_way", "three_way_weighted"])
def test_intersections_on_the_primary_fe_sort_below_its_buckets(L, cl, weighted):
    """An intersection subset with a column that repeats the layout's primary FE sorts only the key
    bits below that FE's buckets (the layout's bucket order sorts the rest; dropped rows end the
    order as one run): equal to the full sort (the LFE_TEST_CLUSTER_SORTED hook) at 1e-12 with equal
    cluster counts, to the oracle at 1e-10, and bit for bit on a repeat."""
    from oracle import altproj

    n, k = 120_000, 3
    xs = [f"x{j + 1}" for j in range(k)]
    fes = [f"fe{f + 1}" for f in range(len(L))]
    d = dict(synth.panel(n, k, L, seed=57))
    kw = {}
    if weighted:
        d["w"] = np.random.default_rng(5).uniform(0.5, 2.0, n)
        kw = dict(weights="w")
    r = _fit(d, xs, fes, cl, **kw)
    again = _fit(d, xs, fes, cl, **kw)
    srt = _fit(d, xs, fes, cl, hooks=SORTED, **kw)
    o = altproj.fit(d, "y", xs, fes, vcov="cluster", cluster_cols=cl, weights=kw.get("weights"))
    assert r.n_obs == o["n_obs"] < n  # singletons dropped
    assert tuple(r.n_clusters) == tuple(srt.n_clusters) == tuple(o["n_clusters"])
    np.testing.assert_allclose(_arr(r, xs, "std_errors"), o["se"], rtol=1e-10, atol=0)
    np.testing.assert_allclose(_arr(r, xs, "std_errors"), _arr(srt, xs, "std_errors"), rtol=1e-12, atol=0)
    np.testing.assert_array_equal(_arr(r, xs, "std_errors"), _arr(again, xs, "std_errors"))


def test_clusters_loaded_after_the_fused_pass():
    """the residual pass summed a one-way cluster on the primary FE (no score rows);
    cluster columns loaded afterwards (Engine.load_clusters is public) must get their own meat - the
    pass is rerun writing score rows - never the one cached for the old column.  Against the sorted
    path (LFE_TEST_CLUSTER_SORTED) on the same engine calls."""
    from leanfe_amd._lib import Engine

    n, k, L = 300_000, 3, [8_000, 300]

    def run(hooks):
        with Engine(0) as eng:
            if hooks:
                eng.test_hooks(hooks)
            eng.synth_load(n, k, L, synth.betas(k), seed=44)
            _, codes = eng.copy_inputs()
            eng.load_clusters([np.ascontiguousarray(codes[0])], [L[0]])
            _, _, card = eng.drop_singletons()
            eng.demean(sorted(range(2), key=lambda i: card[i]), 1e-6, 50, check_from=3)
            assert eng.gram_resid(keep_scores=True) is not None
            m1, g1 = eng.cluster_meat()
            again = eng.cluster_meat()  # the cached meat of the same pass
            np.testing.assert_array_equal(again[0], m1)
            eng.load_clusters([np.ascontiguousarray(codes[1])], [L[1]])
            m2, g2 = eng.cluster_meat()
            eng.load_clusters([np.ascontiguousarray(codes[0]), np.ascontiguousarray(codes[1])], L)
            m3, g3 = eng.cluster_meat_subsets([(0,), (1,), (0, 1)])
            return (m1, g1), (m2, g2), (m3, g3)

    fused, srt = run(0), run(SORTED)
    assert int(fused[0][1][0]) == L[0] and int(fused[1][1][0]) == L[1]
    for (a, ga), (b, gb) in zip(fused, srt):
        np.testing.assert_array_equal(ga, gb)
        assert np.abs(a - b).max() <= 1e-12 * np.abs(b).max()


@pytest.mark.parametrize("k", [3, 10, 14, 20])
def test_mostly_singleton_intersection_multi_row_corrections(k, knob):
    """A two-way CGM whose intersection is mostly singletons (mean cluster size < 2, as config 4's
    fe2 x fe3 and MEGA_CLUSTER2's fe1 x fe2): meat = D + sum over clusters of two or more rows of
    (S_c S_c' - sum_i s_i s_i').  8 <= k <= 16 sums each cluster's rows straight from the score rows
    (k_multi_sums16) and forms the rows' Gram through the row index; k = 3, k = 20 and
    LFE_CL_MULTI_GATHER gather the rows into a copy first; LFE_CL_NO_SINGLETON sums every cluster.
    All at 1e-12 of each other, the oracle at 1e-10 with equal cluster counts, bit-identical repeats."""
    from oracle import altproj

    n, L = 400_000, [2_000, 400, 50]  # 800K cells: ~60 % of the rows singletons, the rest in 2+ row clusters
    xs = [f"x{j + 1}" for j in range(k)]
    fes = ["fe1", "fe2", "fe3"]
    d = dict(synth.panel(n, k, L, seed=83))
    cl = ["fe1", "fe2"]
    a = _fit(d, xs, fes, cl)
    again = _fit(d, xs, fes, cl)
    knob.setenv("LFE_CL_MULTI_GATHER", "1")
    g = _fit(d, xs, fes, cl)
    knob.delenv("LFE_CL_MULTI_GATHER")
    knob.setenv("LFE_CL_NO_SINGLETON", "1")
    full = _fit(d, xs, fes, cl)
    o = altproj.fit(d, "y", xs, fes, vcov="cluster", cluster_cols=cl)
    assert tuple(a.n_clusters) == tuple(o["n_clusters"]) == tuple(full.n_clusters)
    inter = np.unique(np.asarray(d["fe1"], np.int64) * L[1] + np.asarray(d["fe2"]))
    assert 2 * inter.size > n and inter.size < n  # the intersection: mostly singletons, some multi-row clusters
    np.testing.assert_array_equal(_arr(a, xs, "std_errors"), _arr(again, xs, "std_errors"))
    for other in (g, full):
        np.testing.assert_allclose(_arr(a, xs, "std_errors"), _arr(other, xs, "std_errors"), rtol=1e-12, atol=0)
    np.testing.assert_allclose(_arr(a, xs, "coefs"), o["beta"], rtol=1e-10, atol=0)
    np.testing.assert_allclose(_arr(a, xs, "std_errors"), o["se"], rtol=1e-10, atol=0)

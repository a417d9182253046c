"""Fits wider than one engine context (more than 63 columns; VERDICT r4 Missing 2).

The reference forms X'X of [1, X_dm] at any width (polars_impl.py:165-209), e.g. an event study's
i(year) dummies (:27-69) beside controls.  hip_impl._wide_fit runs the columns in blocks of
contexts (the first with the stop test, the others with exactly its sweeps) and writes the
demeaned columns into one device matrix; the Gram, residual, HC1 meat and cluster score sums then
come from that matrix (lfe_wide.hip).  Checked against the CPU oracle (oracle/altproj.py) at 1e-10
with equal iterations, and - with the context width lowered so that a 40-column fit takes three
blocks - against the one-context fit at 1e-12."""
from __future__ import annotations

import numpy as np
import pytest

from leanfe_amd import synth

pytestmark = pytest.mark.gpu


def _check(r, o, xs):
    assert r.iterations == o["iterations"] and r.n_obs == o["n_obs"] and r.df_resid == o["df_resid"]
    np.testing.assert_allclose([r.coefs[x] for x in xs], o["beta"], rtol=1e-10, atol=0)
    np.testing.assert_allclose([r.std_errors[x] for x in xs], o["se"], rtol=1e-10, atol=0)


@pytest.mark.parametrize("vcov,cl,weighted", [("HC1", None, False), ("iid", None, True), ("cluster", ["fe1"], False),
                                              ("cluster", ["fe1", "fe2"], True)])
def test_wide_fit_matches_oracle(vcov, cl, weighted):
    from leanfe_amd import leanfe_hip
    from oracle import altproj

    n, k, L = 150_001, 99, [3_000, 200]
    d = dict(synth.panel(n, k, L, seed=12))
    kw = {}
    if weighted:
        d["w"] = np.random.default_rng(12).uniform(0.5, 2.0, n)
        kw["weights"] = "w"
    xs = [f"x{j + 1}" for j in range(k)]
    r = leanfe_hip(d, y_col="y", x_cols=xs, fe_cols=["fe1", "fe2"], strategy="alt_proj", vcov=vcov, cluster_cols=cl,
                   quiet=True, **kw)
    o = altproj.fit(d, "y", xs, ["fe1", "fe2"], vcov=vcov, cluster_cols=cl, weights=kw.get("weights"))
    _check(r, o, xs)
    if cl:
        ncl = o["n_clusters"]
        assert (tuple(r.n_clusters) if isinstance(r.n_clusters, (list, tuple)) else r.n_clusters) == (
            tuple(ncl) if isinstance(ncl, (list, tuple)) else ncl)


def test_event_study_formula_beyond_63_columns():
    """y ~ x1 + x2 + i(year) with 80 years and firm clusters: 81 dummies + 2 controls."""
    from leanfe_amd import frame, leanfe_hip
    from oracle import altproj

    n, L = 200_000, [4_000, 150]
    d = dict(synth.panel(n, 2, L, seed=33))
    d["year"] = np.random.default_rng(33).integers(1940, 2021, n)
    r = leanfe_hip(d, formula="y ~ x1 + x2 + i(year) | fe1 + fe2", strategy="alt_proj", vcov="cluster",
                   cluster_cols=["fe1"], quiet=True)
    full = dict(d)
    xs = ["x1", "x2"] + frame.expand_factors(full, [("year", None)])
    assert list(r.coefs) == xs and len(xs) == 82
    o = altproj.fit(full, "y", xs, ["fe1", "fe2"], vcov="cluster", cluster_cols=["fe1"])
    _check(r, o, xs)


@pytest.mark.parametrize("vcov,F", [("HC1", 2), ("cluster", 3), ("iid", 1)])
def test_column_blocks_equal_the_one_context_fit(vcov, F, monkeypatch):
    from leanfe_amd import hip_impl, leanfe_hip

    n, k = 300_000, 39
    L = [5_000, 400, 60][:F]
    d = dict(synth.panel(n, k, L, seed=5))
    xs = [f"x{j + 1}" for j in range(k)]
    fes = [f"fe{f + 1}" for f in range(F)]
    cl = ["fe2", "fe3"] if vcov == "cluster" else None
    strat = "demean" if F == 1 else "alt_proj"
    one = leanfe_hip(d, y_col="y", x_cols=xs, fe_cols=fes, strategy=strat, vcov=vcov, cluster_cols=cl, quiet=True)
    monkeypatch.setattr(hip_impl, "MAX_CONTEXT_COLS", 16)  # 40 columns: three blocks
    wide = leanfe_hip(d, y_col="y", x_cols=xs, fe_cols=fes, strategy=strat, vcov=vcov, cluster_cols=cl, quiet=True)
    assert wide.iterations == one.iterations and wide.n_obs == one.n_obs and wide.df_resid == one.df_resid
    np.testing.assert_allclose([wide.coefs[x] for x in xs], [one.coefs[x] for x in xs], rtol=1e-12, atol=0)
    np.testing.assert_allclose([wide.std_errors[x] for x in xs], [one.std_errors[x] for x in xs], rtol=1e-12,
                               atol=0)
    if cl:
        assert tuple(wide.n_clusters) == tuple(one.n_clusters)


@pytest.mark.parametrize("vcov,cl,weighted", [("HC1", None, False), ("cluster", ["fe1", "fe2"], True)])
def test_streamed_wide_fit(vcov, cl, weighted):
    """k = 80 out of core: every block is a streamed context (group sums from one pass, codes-only
    sweeps, lfe_stream_materialize into D); against the resident wide fit and the oracle."""
    from leanfe_amd import leanfe_hip
    from oracle import altproj

    n, k, L = 120_001, 80, [2_500, 150]
    d = dict(synth.panel(n, k, L, seed=21))
    kw = {}
    if weighted:
        d["w"] = np.random.default_rng(21).uniform(0.5, 2.0, n)
        kw["weights"] = "w"
    xs = [f"x{j + 1}" for j in range(k)]
    args = dict(y_col="y", x_cols=xs, fe_cols=["fe1", "fe2"], strategy="alt_proj", vcov=vcov, cluster_cols=cl,
                quiet=True, **kw)
    oc = leanfe_hip(d, out_of_core=True, chunk_rows=50_000, **args)
    res = leanfe_hip(d, **args)
    o = altproj.fit(d, "y", xs, ["fe1", "fe2"], vcov=vcov, cluster_cols=cl, weights=kw.get("weights"))
    _check(oc, o, xs)
    assert oc.iterations == res.iterations and oc.n_obs == res.n_obs
    np.testing.assert_allclose([oc.coefs[x] for x in xs], [res.coefs[x] for x in xs], rtol=1e-11, atol=0)
    np.testing.assert_allclose([oc.std_errors[x] for x in xs], [res.std_errors[x] for x in xs], rtol=1e-11, atol=0)


def test_streamed_wide_event_study_from_parquet(tmp_path):
    """A Parquet source, out of core, y ~ x1 + x2 + i(year) with 70 years: the dummies are formed
    chunk by chunk from the streamed rows (frame.Expansion) for both blocks."""
    pa = pytest.importorskip("pyarrow")
    import pyarrow.parquet as pq

    from leanfe_amd import frame, leanfe_hip
    from oracle import altproj

    n, L = 150_000, [3_000, 120]
    d = dict(synth.panel(n, 2, L, seed=34))
    d["year"] = np.random.default_rng(34).integers(1950, 2020, n)
    path = str(tmp_path / "wide.parquet")
    pq.write_table(pa.table({c: np.asarray(v) for c, v in d.items()}), path, row_group_size=40_000)
    r = leanfe_hip(path, formula="y ~ x1 + x2 + i(year) | fe1 + fe2", strategy="alt_proj", vcov="HC1", quiet=True,
                   out_of_core=True, chunk_rows=40_000)
    full = dict(d)
    xs = ["x1", "x2"] + frame.expand_factors(full, [("year", None)])
    assert list(r.coefs) == xs and len(xs) == 71
    o = altproj.fit(full, "y", xs, ["fe1", "fe2"], vcov="HC1")
    _check(r, o, xs)


def _iv_panel(seed, n, L, k):
    """k regressors (x1 endogenous), k instruments: z1 plus the exogenous x2..xk (2SLS,
    common.py:188-287)."""
    d = dict(synth.panel(n, k, list(L), seed=seed))
    rng = np.random.default_rng(seed)
    u = rng.normal(0, 1, n)
    d["z1"] = rng.normal(0, 1, n) + 0.3 * d["x2"]
    d["x1"] = d["x1"] + 0.8 * d["z1"] + 0.6 * u
    d["y"] = d["y"] + 0.6 * d["x1"] + u
    d["cl1"] = rng.integers(0, 97, n)
    return d, ["z1"] + [f"x{j + 1}" for j in range(1, k)]


@pytest.mark.parametrize("vcov,cl,weighted", [("HC1", None, False), ("cluster", ["cl1", "fe2"], True), ("iid", None, False)])
def test_wide_iv_fit_matches_oracle(vcov, cl, weighted):
    """IV beyond 63 columns: [y] + 40 regressors + 40 instruments = 81 columns in two blocks; 2SLS
    from the device matrix's Gram, meats over u = [1, x~, z~] (std_errors.py:448-602)."""
    from leanfe_amd import leanfe_hip
    from oracle import altproj

    k, L = 40, [2_000, 150]
    d, inst = _iv_panel(44, 120_001, L, k)
    kw = {}
    if weighted:
        d["w"] = np.random.default_rng(45).uniform(0.5, 2.0, d["y"].size)
        kw["weights"] = "w"
    xs = [f"x{j + 1}" for j in range(k)]
    f = f"y ~ {' + '.join(xs)} | fe1 + fe2 | {' + '.join(inst)}"
    r = leanfe_hip(d, formula=f, strategy="alt_proj", vcov=vcov, cluster_cols=cl, quiet=True, **kw)
    assert r.is_iv and r.n_instruments == k
    o = altproj.fit(d, "y", xs, ["fe1", "fe2"], vcov=vcov, cluster_cols=cl, weights=kw.get("weights"),
                    instruments=inst)
    _check(r, o, xs)


@pytest.mark.parametrize("vcov", ["HC1", "cluster"])
def test_wide_iv_blocks_equal_the_one_context_iv_fit(vcov, monkeypatch):
    from leanfe_amd import hip_impl, leanfe_hip

    k = 5
    d, inst = _iv_panel(46, 250_000, [6_000, 200], k)
    xs = [f"x{j + 1}" for j in range(k)]
    f = f"y ~ {' + '.join(xs)} | fe1 + fe2 | {' + '.join(inst)}"
    cl = ["cl1"] if vcov == "cluster" else None
    one = leanfe_hip(d, formula=f, strategy="alt_proj", vcov=vcov, cluster_cols=cl, quiet=True)
    monkeypatch.setattr(hip_impl, "MAX_CONTEXT_COLS", 5)  # 11 columns: three blocks
    wide = leanfe_hip(d, formula=f, strategy="alt_proj", vcov=vcov, cluster_cols=cl, quiet=True)
    assert wide.iterations == one.iterations and wide.n_obs == one.n_obs and wide.is_iv
    np.testing.assert_allclose([wide.coefs[x] for x in xs], [one.coefs[x] for x in xs], rtol=1e-12, atol=0)
    np.testing.assert_allclose([wide.std_errors[x] for x in xs], [one.std_errors[x] for x in xs], rtol=1e-12,
                               atol=0)


def test_streamed_wide_iv_fit():
    """Out of core and wide with instruments: the streamed blocks carry [y] + x + z chunk by chunk
    (hip_impl._stream_chunks), against the resident wide IV fit and the oracle."""
    from leanfe_amd import leanfe_hip
    from oracle import altproj

    k, L = 35, [1_500, 100]
    d, inst = _iv_panel(47, 90_001, L, k)
    xs = [f"x{j + 1}" for j in range(k)]
    f = f"y ~ {' + '.join(xs)} | fe1 + fe2 | {' + '.join(inst)}"
    res = leanfe_hip(d, formula=f, strategy="alt_proj", vcov="HC1", quiet=True)
    oc = leanfe_hip(d, formula=f, strategy="alt_proj", vcov="HC1", quiet=True, out_of_core=True, chunk_rows=40_000)
    o = altproj.fit(d, "y", xs, ["fe1", "fe2"], vcov="HC1", instruments=inst)
    _check(oc, o, xs)
    np.testing.assert_allclose([oc.coefs[x] for x in xs], [res.coefs[x] for x in xs], rtol=1e-11, atol=0)
    np.testing.assert_allclose([oc.std_errors[x] for x in xs], [res.std_errors[x] for x in xs], rtol=1e-11, atol=0)


def test_wide_fit_three_fes_with_singletons():
    """Three FEs, rows alone in their level (dropped before the sweeps, polars_impl.py:477-482),
    weights and a one-way cluster on the second FE, 70 regressors in two blocks."""
    from leanfe_amd import leanfe_hip
    from oracle import altproj

    n, k, L = 100_003, 70, [2_500, 300, 40]
    d = dict(synth.panel(n, k, L, seed=61))
    f1 = np.array(d["fe1"], copy=True)
    f1[:25] = L[0] + np.arange(25)  # 25 singleton levels
    d["fe1"] = f1
    d["w"] = np.random.default_rng(61).uniform(0.5, 2.0, n)
    xs = [f"x{j + 1}" for j in range(k)]
    fes = ["fe1", "fe2", "fe3"]
    r = leanfe_hip(d, y_col="y", x_cols=xs, fe_cols=fes, strategy="alt_proj", vcov="cluster", cluster_cols=["fe2"],
                   weights="w", quiet=True)
    o = altproj.fit(d, "y", xs, fes, vcov="cluster", cluster_cols=["fe2"], weights="w")
    assert r.n_obs == n - 25 and r.n_clusters == o["n_clusters"]
    _check(r, o, xs)


@pytest.mark.parametrize("vcov,weighted", [("HC1", False), ("iid", True)])
def test_streamed_wide_fit_without_resident_design_matrix(vcov, weighted, monkeypatch):
    """VERDICT r5 Missing 1: a streamed wide IID / HC1 fit keeps no D (P n doubles): each row chunk's
    [1, y~, x~] is formed for every column block into one chunk buffer and its Gram / residual / meat
    added in chunk order (hip_impl._wide_fit_chunked).  Against the oracle (1e-10, equal integers),
    the streamed fit through a resident D (1e-11) and a second chunking (1e-13)."""
    from leanfe_amd import hip_impl, leanfe_hip
    from oracle import altproj

    n, k, L = 130_001, 90, [2_500, 150]
    d = dict(synth.panel(n, k, L, seed=23))
    kw = {}
    if weighted:
        d["w"] = np.random.default_rng(23).uniform(0.5, 2.0, n)
        kw["weights"] = "w"
    xs = [f"x{j + 1}" for j in range(k)]
    args = dict(y_col="y", x_cols=xs, fe_cols=["fe1", "fe2"], strategy="alt_proj", vcov=vcov, quiet=True,
                out_of_core=True, **kw)
    a = leanfe_hip(d, chunk_rows=40_000, **args)
    b = leanfe_hip(d, chunk_rows=64_064, **args)
    monkeypatch.setitem(hip_impl.KNOBS, "wide_chunked", False)
    res_d = leanfe_hip(d, chunk_rows=40_000, **args)
    o = altproj.fit(d, "y", xs, ["fe1", "fe2"], vcov=vcov, weights=kw.get("weights"))
    _check(a, o, xs)
    for other, tol in ((b, 1e-13), (res_d, 1e-11)):
        assert other.iterations == a.iterations and other.n_obs == a.n_obs
        np.testing.assert_allclose([a.coefs[x] for x in xs], [other.coefs[x] for x in xs], rtol=tol, atol=0)
        np.testing.assert_allclose([a.std_errors[x] for x in xs], [other.std_errors[x] for x in xs], rtol=tol, atol=0)


def test_device_generated_wide_fit_matches_the_oracle():
    """tools/wide_oocore_run.py's chunked wide fit (K = 100 columns generated per chunk on the device,
    no resident D; run at 1e9 rows into profiles/r06) at 150K rows: the oracle on the same panel
    (synth.panel, the host restatement of the device generator) at 1e-10 with equal integers, and a
    second chunking at 1e-13."""
    import importlib.util
    import os

    from oracle import altproj

    spec = importlib.util.spec_from_file_location(
        "wide_oocore_run", os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools", "wide_oocore_run.py"))
    tool = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(tool)
    n, K, L = 150_000, 100, [3_000, 120]
    beta = synth.betas(K)
    a = tool.wide_fit(n, K, L, beta, 40_000, seed=41)
    b = tool.wide_fit(n, K, L, beta, 64_000 + 64 * 7, seed=41)
    d = dict(synth.panel(n, K, L, seed=41))
    xs = [f"x{j + 1}" for j in range(K)]
    o = altproj.fit(d, "y", xs, ["fe1", "fe2"], vcov="HC1")
    assert a["blocks"] == 2 and a["iterations"] == o["iterations"] and a["n_obs"] == o["n_obs"]
    np.testing.assert_allclose(a["beta"], o["beta"], rtol=1e-10, atol=0)
    np.testing.assert_allclose(a["se"], o["se"], rtol=1e-10, atol=0)
    assert (b["iterations"], b["n_obs"], b["df_resid"]) == (a["iterations"], a["n_obs"], a["df_resid"])
    np.testing.assert_allclose(b["beta"], a["beta"], rtol=1e-13, atol=0)
    np.testing.assert_allclose(b["se"], a["se"], rtol=1e-13, atol=0)

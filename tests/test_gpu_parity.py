"""GPU parity: the HIP engine (through the C ABI) against the oracle and the golden fixtures.

Tolerances: coefficients and SEs within 1e-10 relative (BASELINE.json
north_star); integer outputs (n_obs, iterations, fe_dims, df_resid,
n_clusters) bit-exact.  Synthetic-panel generation is bit-exact host vs device.
"""
import numpy as np
import pytest

from golden_util import load, names, ncl
from leanfe_amd import hip_impl, synth
from oracle import altproj, yoco

pytestmark = pytest.mark.gpu
RTOL = 1e-10


def _formula(y, xs, fes, inst):
    return f"{y} ~ {' + '.join(xs)} | {' + '.join(fes)} | {' + '.join(inst)}"


def _hip_fit(meta, data, **kw):
    from leanfe_amd import leanfe_hip
    if meta.get("instruments"):  # IV enters through the formula only, as in leanfe_polars (:311-319)
        return leanfe_hip(data, formula=_formula(meta["y"], meta["xs"], meta["fes"], meta["instruments"]),
                          strategy=meta["strategy"], weights=meta["weights"], vcov=meta["vcov"],
                          cluster_cols=meta["cluster_cols"], ssc=meta["ssc"], quiet=True, **kw)
    return leanfe_hip(data, y_col=meta["y"], x_cols=meta["xs"], fe_cols=meta["fes"], strategy=meta["strategy"],
                      weights=meta["weights"], vcov=meta["vcov"], cluster_cols=meta["cluster_cols"],
                      ssc=meta["ssc"], quiet=True, **kw)


def _assert_same(r, beta, se, n_obs, iterations, df_resid, fe_dims, n_clusters, xs, rtol=RTOL):
    b = np.array([r.coefs[x] for x in xs])
    s = np.array([r.std_errors[x] for x in xs])
    assert r.n_obs == n_obs
    assert r.iterations == iterations
    assert r.df_resid == df_resid
    assert tuple(r.fe_dims or ()) == tuple(fe_dims)
    assert ncl(r.n_clusters) == ncl(n_clusters)
    np.testing.assert_allclose(b, beta, rtol=rtol, atol=0)
    np.testing.assert_allclose(s, se, rtol=rtol, atol=0)


YOCO_NAMES = [n for n in names() if load(n)[0]["pinned"] == "reference-yoco"]


@pytest.mark.parametrize("name", [n for n in names() if n not in YOCO_NAMES])
def test_golden_fixture(name):
    meta, data, exp = load(name)
    r = _hip_fit(meta, data, demean_tol=meta["demean_tol"], max_iter=meta["max_iter"])
    _assert_same(r, exp["oracle_beta"], exp["oracle_se"], int(exp["oracle_n_obs"]), int(exp["oracle_iterations"]),
                 int(exp["oracle_df_resid"]), exp["oracle_fe_dims"].tolist(), meta["oracle_n_clusters"], meta["xs"])
    if np.isfinite(exp["oracle_r2"]) and not meta.get("instruments"):  # R^2 (IID: from the Gram alone)
        np.testing.assert_allclose(r.r_squared, float(exp["oracle_r2"]), rtol=1e-10)
    if meta.get("instruments"):  # the reference's own 2SLS / IV SE functions on the same demeaned columns
        assert r.is_iv and r.n_instruments == len(meta["instruments"]) and r.r_squared is None
        np.testing.assert_allclose([r.std_errors[x] for x in meta["xs"]], exp["ref_se"], rtol=RTOL, atol=0)
    elif "ref_beta" in exp:  # the reference's exact LSDV values, up to alt-proj convergence error
        b = np.array([r.coefs[x] for x in meta["xs"]])
        np.testing.assert_allclose(b, exp["ref_beta"], rtol=1e-7, atol=0)


def test_synth_device_equals_host_bit_exact():
    from leanfe_amd._lib import Engine
    n, k, L = 5000, 3, [300, 20]
    host = synth.panel(n, k, L, seed=12345, row_offset=777)
    with Engine(0) as eng:
        eng.synth_load(n, k, L, synth.betas(k), seed=12345, row_offset=777)
        cols, codes = eng.copy_inputs(n)
    np.testing.assert_array_equal(cols[0], host["y"])
    for j in range(k):
        np.testing.assert_array_equal(cols[1 + j], host[f"x{j + 1}"])
    for f in range(len(L)):
        np.testing.assert_array_equal(codes[f], host[f"fe{f + 1}"])


@pytest.mark.parametrize("seed,n,L,k,vcov", [
    (1, 200_003, (5000, 300), 5, "iid"),            # n % 16 != 0: partial last row group
    (2, 300_000, (20000, 500), 3, "HC1"),
    (3, 150_005, (3000, 40, 7), 4, "cluster"),
    (12345, 2_000_000, (100000, 1000), 10, "HC1"),   # headline geometry (1e5 / 1e3 levels, k = 10)
    (6, 400_000, (700_000, 50), 2, "iid"),           # more levels than rows: many singletons, nb > 512
    (7, 300_000, (20000, 300), 20, "HC1"),           # p = 21: two 16-column slots (NT = 2) in every kernel
    (8, 120_000, (4000, 150), 40, "iid"),            # p = 41: NT = 3
    (9, 300_000, (20000, 4200), 1, "HC1"),           # G_Q = 4200, p = 2: separate layout sorts (fused > 150 KB LDS)
])
def test_random_panels_vs_oracle(seed, n, L, k, vcov):
    data = synth.panel(n, k, list(L), seed=seed)
    xs = [f"x{j + 1}" for j in range(k)]
    fes = [f"fe{f + 1}" for f in range(len(L))]
    cl = ["fe2", "fe3"] if vcov == "cluster" else None
    o = altproj.fit(data, "y", xs, fes, vcov=vcov, cluster_cols=cl)
    from leanfe_amd import leanfe_hip
    r = leanfe_hip(data, y_col="y", x_cols=xs, fe_cols=fes, strategy="alt_proj", vcov=vcov, cluster_cols=cl,
                   quiet=True)
    _assert_same(r, o["beta"], o["se"], o["n_obs"], o["iterations"], o["df_resid"], o["fe_dims"],
                 o["n_clusters"], xs)


@pytest.mark.parametrize("weighted", [False, True])
def test_three_way_cgm_on_device(weighted):
    """Three cluster columns: 7 CGM subsets whose intersections are keyed and grouped on
    the device (the fe1 x fe2 x fe3 subset is almost all singleton clusters), with
    singleton FE rows dropped (fe1 has ~5 rows per level) and optional weights."""
    n, L, k = 150_000, [30_000, 200, 13], 3
    data = synth.panel(n, k, L, seed=21)
    if weighted:
        data["w"] = 0.5 + np.random.default_rng(3).random(n)
    xs = [f"x{j + 1}" for j in range(k)]
    fes = ["fe1", "fe2", "fe3"]
    w = "w" if weighted else None
    o = altproj.fit(data, "y", xs, fes, vcov="cluster", cluster_cols=fes, weights=w)
    from leanfe_amd import leanfe_hip
    r = leanfe_hip(data, y_col="y", x_cols=xs, fe_cols=fes, strategy="alt_proj", vcov="cluster", cluster_cols=fes,
                   weights=w, quiet=True)
    assert o["n_obs"] < n  # singletons were dropped
    _assert_same(r, o["beta"], o["se"], o["n_obs"], o["iterations"], o["df_resid"], o["fe_dims"],
                 o["n_clusters"], xs)


def test_ols_no_fe_and_single_fe_demean():
    data = synth.panel(20000, 2, [400], seed=4)
    from leanfe_amd import leanfe_hip
    r = leanfe_hip(data, formula="y ~ x1 + x2 | fe1", quiet=True)
    o = altproj.fit(data, "y", ["x1", "x2"], ["fe1"], strategy="demean")
    _assert_same(r, o["beta"], o["se"], o["n_obs"], 1, o["df_resid"], o["fe_dims"], None, ["x1", "x2"])
    r = leanfe_hip(data, formula="y ~ x1 + x2", quiet=True)
    X = np.column_stack([np.ones(20000), data["x1"], data["x2"]])
    b = np.linalg.lstsq(X, data["y"], rcond=None)[0]
    np.testing.assert_allclose([r.coefs["x1"], r.coefs["x2"]], b[1:], rtol=1e-10)


def test_all_rows_singletons_raises_or_empty():
    data = {"y": np.arange(5.0), "x": np.arange(5.0) ** 2, "a": np.arange(5), "b": np.arange(5)}
    from leanfe_amd import leanfe_hip
    with pytest.raises(Exception):
        leanfe_hip(data, formula="y ~ x | a + b", strategy="alt_proj", quiet=True)


def test_bad_codes_rejected():
    from leanfe_amd._lib import Engine
    with Engine(0) as eng:
        with pytest.raises(ValueError):
            eng.load([np.zeros(4)], [np.array([0, 1, 5, 0], dtype=np.int32)], [3])


def _iv_panel(seed, n, L, k, m, weights=False):
    """k regressors (x1 endogenous), m >= k - 1 instruments (z1 plus the exogenous x2..xk)."""
    data = synth.panel(n, k, list(L), seed=seed)
    rng = np.random.default_rng(seed)
    u = rng.normal(0, 1, n)
    data["z1"] = rng.normal(0, 1, n) + 0.3 * data["x2"]
    data["x1"] = data["x1"] + 0.8 * data["z1"] + 0.6 * u
    data["y"] = data["y"] + 0.6 * data["x1"] + u
    if weights:
        data["w"] = rng.uniform(0.5, 2.0, n)
    data["cl1"] = rng.integers(0, 97, n)
    inst = ["z1"] + [f"x{j + 1}" for j in range(1, k)]
    return data, inst[:m]


@pytest.mark.parametrize("seed,n,L,k,vcov,weights", [
    (31, 300_000, (20000, 300), 3, "HC1", False),      # two-FE IV, general Gram + IV residual pass
    (32, 200_001, (5000, 200, 30), 4, "cluster", False),  # three FEs, one-way cluster on u = [1, x, z] scores
    (33, 150_000, (3000, 60), 2, "iid", True),          # weighted first and second stage
    (34, 250_000, (8000, 90), 3, "cluster", True),      # two-way CGM, weighted scores
])
def test_iv_panels_vs_oracle(seed, n, L, k, vcov, weights):
    data, inst = _iv_panel(seed, n, L, k, k)
    if weights:
        data["w"] = np.random.default_rng(seed + 1).uniform(0.5, 2.0, n)
    xs = [f"x{j + 1}" for j in range(k)]
    fes = [f"fe{f + 1}" for f in range(len(L))]
    cl = (["cl1"] if seed != 34 else ["cl1", "fe2"]) if vcov == "cluster" else None
    w = "w" if weights else None
    o = altproj.fit(data, "y", xs, fes, vcov=vcov, cluster_cols=cl, weights=w, instruments=inst)
    from leanfe_amd import leanfe_hip
    r = leanfe_hip(data, formula=_formula("y", xs, fes, inst), strategy="alt_proj", vcov=vcov, cluster_cols=cl,
                   weights=w, quiet=True)
    assert r.is_iv
    _assert_same(r, o["beta"], o["se"], o["n_obs"], o["iterations"], o["df_resid"], o["fe_dims"],
                 o["n_clusters"], xs)


def test_iv_without_fixed_effects():
    """IV with no FE part: strategy 'ols', the raw columns (polars_impl.py:176-198 on
    undemeaned data); an all-ones instrument column suppresses the added intercept."""
    from leanfe_amd import leanfe_hip
    data, inst = _iv_panel(35, 50_000, (100, 10), 2, 2)
    r = leanfe_hip(data, formula="y ~ x1 + x2 | | z1 + x2", strategy="ols", vcov="HC1", quiet=True)
    Y = data["y"]
    X = np.column_stack([np.ones(Y.size), data["x1"], data["x2"]])
    Z = np.column_stack([np.ones(Y.size), data["z1"], data["x2"]])
    o = altproj.run_regression_iv(Y, X[:, 1:], Z[:, 1:], None, "HC1", None, True, Y.size, 0)
    np.testing.assert_allclose([r.coefs["x1"], r.coefs["x2"]], o["beta"], rtol=RTOL, atol=0)
    np.testing.assert_allclose([r.std_errors["x1"], r.std_errors["x2"]], o["se"], rtol=RTOL, atol=0)
    data["one"] = np.ones(Y.size)
    r1 = leanfe_hip(data, formula="y ~ x1 + x2 | | one + z1 + x2", strategy="ols", vcov="iid", quiet=True)
    o1 = altproj.run_regression_iv(Y, X[:, 1:], Z, None, "iid", None, True, Y.size, 0)
    assert o1["Z_cols"] == 3  # no second intercept
    np.testing.assert_allclose([r1.coefs["x1"], r1.coefs["x2"]], o1["beta"], rtol=RTOL, atol=0)
    np.testing.assert_allclose([r1.std_errors["x1"], r1.std_errors["x2"]], o1["se"], rtol=RTOL, atol=0)


def test_iv_under_identified_raises():
    from leanfe_amd import leanfe_hip
    data, _ = _iv_panel(36, 20_000, (100, 10), 3, 1)
    with pytest.raises(ValueError, match="Under-identified"):
        leanfe_hip(data, formula="y ~ x1 + x2 + x3 | fe1 + fe2 | z1", strategy="alt_proj", quiet=True)


def _assert_yoco(r, o, xs, rtol=RTOL):
    assert r.n_obs == o["n_obs"] and r.df_resid == o["df_resid"]
    assert r.n_compressed == o["n_compressed"]
    assert tuple(r.fe_dims or ()) == tuple(o["fe_dims"] or ())
    assert ncl(r.n_clusters) == ncl(o["n_clusters"])
    np.testing.assert_allclose([r.coefs[x] for x in xs], o["beta"], rtol=rtol, atol=0)
    np.testing.assert_allclose([r.std_errors[x] for x in xs], o["se"], rtol=rtol, atol=0)
    np.testing.assert_allclose(r.rss, o["rss"], rtol=rtol)


@pytest.mark.parametrize("name", YOCO_NAMES)
def test_yoco_fixture(name):
    """strategy='compress' on the device (lfe_compress + records-mode solve) against the
    reference's own LSDV WLS / grouped-RSS SE functions (tests/golden/make_golden.py)."""
    meta, data, exp = load(name)
    r = _hip_fit(meta, data)
    assert r.n_obs == int(exp["oracle_n_obs"]) and r.df_resid == int(exp["oracle_df_resid"])
    assert r.n_compressed == int(exp["oracle_n_compressed"])
    assert tuple(r.fe_dims or ()) == tuple(exp["oracle_fe_dims"].tolist())
    assert ncl(r.n_clusters) == ncl(meta["ref_n_clusters"])
    np.testing.assert_allclose([r.coefs[x] for x in meta["xs"]], exp["ref_beta"], rtol=RTOL, atol=0)
    np.testing.assert_allclose([r.std_errors[x] for x in meta["xs"]], exp["ref_se"], rtol=RTOL, atol=0)
    np.testing.assert_allclose(r.rss, float(exp["ref_rss"]), rtol=RTOL)


def _yoco_panel(seed, n, L, k, weights=False):
    rng = np.random.default_rng(seed)
    codes = [rng.integers(0, G, n) for G in L]
    d = {f"x{j + 1}": rng.integers(0, 3 + j, n).astype(np.float64) for j in range(k)}
    d["y"] = sum((1.0 - 0.2 * j) * d[f"x{j + 1}"] for j in range(k)) + rng.normal(0, 1, n)
    for f, c in enumerate(codes):
        d[f"fe{f + 1}"] = c
        d["y"] = d["y"] + rng.normal(0, 1, L[f])[c]
    d["cl1"] = codes[0] // 4
    if weights:
        d["w"] = rng.uniform(0.5, 2.0, n)
    return d


@pytest.mark.parametrize("seed,n,L,k,vcov,weights", [
    (51, 2_000_000, (200, 50), 3, "HC1", False),        # ~50% of cells filled: 1M+ records, 2 FEs
    (52, 1_000_000, (120, 30, 8), 2, "cluster", False),  # three FEs, one-way cluster on the records
    (53, 600_000, (150, 40), 2, "iid", True),            # weighted: _n = sum w
    (54, 800_000, (100, 25), 2, "cluster", False),       # two-way CGM (cl1 x fe2) on the records
])
def test_yoco_panels_vs_oracle(seed, n, L, k, vcov, weights):
    from leanfe_amd import leanfe_hip
    d = _yoco_panel(seed, n, L, k, weights)
    xs = [f"x{j + 1}" for j in range(k)]
    fes = [f"fe{f + 1}" for f in range(len(L))]
    cl = (["cl1"] if seed != 54 else ["cl1", "fe2"]) if vcov == "cluster" else None
    w = "w" if weights else None
    o = yoco.fit(d, "y", xs, fes, weights=w, vcov=vcov, cluster_cols=cl)
    r = leanfe_hip(d, y_col="y", x_cols=xs, fe_cols=fes, strategy="compress", vcov=vcov, cluster_cols=cl,
                   weights=w, quiet=True)
    _assert_yoco(r, o, xs)


def test_yoco_nearly_nested_fes_converge_to_the_exact_lsdv():
    """Records whose second FE is almost a function of the first (99% of rows: fe2 = fe1 // 4):
    the weighted projections converge slowly, and the records solve must still reach the exact
    LSDV fit the reference factors directly (compress.py:659-747), stopping on the
    scale-relative floor rather than running to max_iter."""
    from leanfe_amd import leanfe_hip
    d = _yoco_panel(57, 400_000, (200, 50), 2)
    rng = np.random.default_rng(57)
    nested = rng.random(d["fe1"].size) < 0.99
    d["fe2"] = np.where(nested, d["fe1"] // 4, d["fe2"])
    xs, fes = ["x1", "x2"], ["fe1", "fe2"]
    o = yoco.fit(d, "y", xs, fes, vcov="HC1")
    r = leanfe_hip(d, y_col="y", x_cols=xs, fe_cols=fes, strategy="compress", vcov="HC1", quiet=True)
    _assert_yoco(r, o, xs)
    assert r.iterations < 100_000


def test_yoco_auto_selects_compress_and_hash_collisions_are_exact(knob):
    """strategy='auto' picks 'compress' for low-cardinality FEs with discrete x
    (compress.py:96-184), and an 8-bit row hash (forced collisions) still groups exactly."""
    from leanfe_amd import leanfe_hip
    d = _yoco_panel(55, 200_000, (60, 20), 2)
    xs, fes = ["x1", "x2"], ["fe1", "fe2"]
    o = yoco.fit(d, "y", xs, fes, vcov="HC1")
    r = leanfe_hip(d, y_col="y", x_cols=xs, fe_cols=fes, strategy="auto", vcov="HC1", quiet=True)
    assert r.n_compressed == o["n_compressed"]
    _assert_yoco(r, o, xs)
    knob.setenv("LFE_ROW_HASH_BITS", "8")
    d = _yoco_panel(56, 20_000, (30, 10), 2)
    o = yoco.fit(d, "y", xs, fes, vcov="cluster", cluster_cols=["cl1"])
    r = leanfe_hip(d, y_col="y", x_cols=xs, fe_cols=fes, strategy="compress", vcov="cluster", cluster_cols=["cl1"],
                   quiet=True)
    _assert_yoco(r, o, xs)


def test_gram_from_tables_guard_falls_back_to_the_design_pass():
    """Two-FE fits form the Gram from the group tables (R + table terms); when the FE part
    explains almost all of a column's variance that sum cancels, the device guard trips and
    the explicit design pass runs instead.  Both regimes must match the oracle."""
    from leanfe_amd import leanfe_hip
    n, L = 400_000, [20_000, 300]
    for scale in (0.5, 1e3):  # kappa ~ 1 (tables) and ~1e6 (> 1e4: design pass)
        d = synth.panel(n, 3, L, seed=61)
        eff = np.random.default_rng(61).normal(0, 1, L[0])
        d["x1"] = d["x1"] + scale * eff[d["fe1"]]
        xs, fes = ["x1", "x2", "x3"], ["fe1", "fe2"]
        o = altproj.fit(d, "y", xs, fes, vcov="HC1")
        from leanfe_amd._lib import Engine
        with Engine(0) as eng:
            eng.profile(True)
            r = leanfe_hip(d, y_col="y", x_cols=xs, fe_cols=fes, strategy="alt_proj", vcov="HC1", quiet=True,
                           engine=eng)
            ks = eng.kernel_stats()
        assert "gram_tables" in ks
        assert ("gram_design" in ks) == (scale > 1.0), sorted(ks)
        _assert_same(r, o["beta"], o["se"], o["n_obs"], o["iterations"], o["df_resid"], o["fe_dims"], None, xs)


@pytest.mark.parametrize("vcov,weights,inst", [("HC1", False, False), ("cluster", True, False), ("iid", False, True)])
def test_parquet_path_streams_and_matches_in_memory(tmp_path, monkeypatch, vcov, weights, inst):
    """A Parquet path streams (FE / cluster / weight columns first, then [y] + x (+ z) in
    batches through lfe_load_rows): the fit equals the in-memory one (to the last bits the
    atomic group sums leave free; the integer outputs exactly)."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from leanfe_amd import leanfe_hip
    d = synth.panel(300_001, 3, [5000, 80], seed=71)
    rng = np.random.default_rng(71)
    d["w"] = rng.uniform(0.5, 2.0, d["y"].size)
    d["cl"] = rng.integers(0, 400, d["y"].size)
    d["z1"] = d["x1"] + rng.normal(0, 1, d["y"].size)
    path = str(tmp_path / "panel.parquet")
    pq.write_table(pa.table(d), path, row_group_size=70_000)
    monkeypatch.setitem(hip_impl.KNOBS, "stream_batch", 65536)
    formula = "y ~ x1 + x2 + x3 | fe1 + fe2" + (" | z1 + x2 + x3" if inst else "")
    kw = dict(formula=formula, strategy="alt_proj", vcov=vcov, cluster_cols=["cl"] if vcov == "cluster" else None,
              weights="w" if weights else None, quiet=True)
    a = leanfe_hip(path, **kw)
    b = leanfe_hip(d, **kw)
    for x in ("x1", "x2", "x3"):
        np.testing.assert_allclose([a.coefs[x], a.std_errors[x]], [b.coefs[x], b.std_errors[x]], rtol=1e-13, atol=0)
    assert a.n_obs == b.n_obs and a.iterations == b.iterations and a.n_clusters == b.n_clusters


def test_nan_input_gives_nan_estimates_without_faulting():
    """The Polars path filters no NULLs (polars_impl.py:468-537), so a NaN in y spreads through the
    projections and the estimates are NaN.  How many sweeps the reference then runs depends on
    Polars' NaN-ignoring max over partly-NaN group means and is not pinned by any reference test or
    fixture; only the NaN estimates and a clean return are checked here."""
    from leanfe_amd import leanfe_hip
    d = synth.panel(30_000, 2, [600, 40], seed=81)
    d["y"] = d["y"].copy()
    d["y"][123] = np.nan
    r = leanfe_hip(d, formula="y ~ x1 + x2 | fe1 + fe2", strategy="alt_proj", vcov="iid", quiet=True)
    assert 3 <= r.iterations <= 50
    assert all(np.isnan(r.coefs[x]) for x in ("x1", "x2"))


def test_empty_input_raises():
    from leanfe_amd import leanfe_hip
    d = {"y": np.zeros(0), "x": np.zeros(0), "a": np.zeros(0, dtype=np.int64), "b": np.zeros(0, dtype=np.int64)}
    with pytest.raises(Exception):
        leanfe_hip(d, formula="y ~ x | a + b", strategy="alt_proj", quiet=True)


@pytest.mark.parametrize("L", [(3000, 40), (200, 30)])  # bucketed layout (deferred row index) / not
def test_copy_demeaned_matches_oracle_in_input_order(L):
    """lfe_copy_demeaned returns the demeaned columns in input row order (NaN on dropped rows).
    On a bucketed layout the input row index of each layout row is written on this first use
    (ensure_layout_orig), by an index-only rerun of the partition scatter."""
    from leanfe_amd._lib import Engine
    from oracle import altproj as ref
    rng = np.random.default_rng(5)
    n, k = 120_003, 2
    codes = [rng.integers(0, G, n).astype(np.int32) for G in L]
    codes[0][codes[0] >= L[0] - 5] = 0
    codes[0][:5] = np.arange(L[0] - 5, L[0], dtype=np.int32)  # five singletons of the first FE
    cols = [rng.standard_normal(n) for _ in range(k + 1)]
    with Engine(0) as eng:
        eng.load(cols, codes, list(L))
        n_obs, _, card = eng.drop_singletons()
        order = sorted(range(len(L)), key=lambda i: card[i])
        iters, _ = eng.demean(order, 1e-8, 100, check_from=3)
        out = eng.copy_demeaned()
    keep = ref.singleton_keep(codes, list(L))
    assert n_obs == int(keep.sum()) == n - 5
    dm, it_ref = ref.demean_altproj(np.array(cols)[:, keep], [c[keep] for c in codes], list(L), order, 1e-8, 100)
    assert iters == it_ref
    assert np.all(np.isnan(out[:, ~keep]))
    np.testing.assert_allclose(out[:, keep], dm, rtol=1e-9, atol=1e-11)

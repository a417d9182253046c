"""Generate the golden fixtures in tests/golden/*.npz — run in the build container only.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What is pinned and how
----------------------
The reference's Polars hot path (polars_impl.py:468-537) cannot run here: the
``polars`` wheel is absent (an ordinary ModuleNotFoundError, not a permission
denial).  Its NumPy/SciPy-only modules CAN run when ``polars`` / ``duckdb`` are
replaced by name-only stub modules, because they only use those names in type
annotations and ``isinstance`` checks.  This script loads, read-only and with
bytecode writing disabled, ``result.py``, ``common.py``, ``compress.py`` and
``std_errors.py`` from /root/reference/python/leanfe and uses:

* ``compress.build_design_matrix`` + ``compress.solve_wls`` on the UNcompressed
  rows (one "group" per row, weight 1): the exact least-squares-dummy-variable
  (LSDV) solution that alternating projections converge to.  Golden ``beta``.
* ``compress.compute_rss_grouped`` + ``compress.CompressionContext`` +
  ``compress.compute_se_compress``: IID, HC1 and one/multi-way clustered SEs of
  that LSDV fit (for the x block, equal to the FWL sandwich).  Golden ``se``.

``df_resid`` and ``n_obs`` are passed in following polars_impl.py:532-537
(n - (k+1) - absorbed_df after the single-pass singleton drop), which is what
the alt_proj path reports.

The oracle (oracle/altproj.py) is then run (a) at a tight tolerance, where it
must agree with the golden LSDV beta/SE to 1e-9, and (b) at the reference's
default tolerance (1e-6, max_iter 50), whose outputs (iterations, beta, SE) are
stored as ``oracle_*`` for the GPU parity tests.  Inputs and outputs only —
no reference source — go into the .npz files.
"""
from __future__ import annotations

import importlib
import json
import os
import sys
import types

sys.dont_write_bytecode = True
os.environ["PYTHONDONTWRITEBYTECODE"] = "1"

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_PKG = "/root/reference/python/leanfe"
sys.path.insert(0, REPO)

from oracle import altproj, yoco  # noqa: E402
from leanfe_amd import synth  # noqa: E402


def load_reference():
    """Import the reference's NumPy-only modules behind name-only stubs."""
    pl = types.ModuleType("polars")

    class _Frame:  # only used in isinstance checks / annotations
        pass

    pl.DataFrame = type("DataFrame", (_Frame,), {})
    pl.LazyFrame = type("LazyFrame", (_Frame,), {})
    pl.Config = type("Config", (), {"set_engine_affinity": staticmethod(lambda *a, **k: None)})
    sel = types.ModuleType("polars.selectors")
    pl.selectors = sel
    duck = types.ModuleType("duckdb")
    duck.DuckDBPyConnection = type("DuckDBPyConnection", (), {})
    sys.modules.update({"polars": pl, "polars.selectors": sel, "duckdb": duck})
    pkg = types.ModuleType("leanfe")
    pkg.__path__ = [REF_PKG]
    sys.modules["leanfe"] = pkg
    compress = importlib.import_module("leanfe.compress")
    std_errors = importlib.import_module("leanfe.std_errors")
    common = importlib.import_module("leanfe.common")
    return compress, std_errors, common


def wls_reference_beta(compress, data, y, xs, fes, keep, weights):
    """Weighted exact-LSDV beta from the reference's build_design_matrix + solve_wls with
    per-row sqrt-weights (compress.py:503-680)."""
    sel = lambda a: np.asarray(a)[keep]
    cols = {c: sel(data[c]).astype(np.float64) for c in xs}
    for f in fes:
        cols[f] = sel(data[f])
    yv = sel(data[y]).astype(np.float64)
    w = sel(data[weights]).astype(np.float64)
    cols["_mean_y"] = yv
    cols["_wts"] = np.sqrt(w)
    cols["_n"] = np.ones(yv.size)
    cols["_sum_y"] = yv
    cols["_sum_y_sq"] = yv ** 2
    res = compress.DuckDBResult(cols)
    design, Y, wts, _, _ = compress.build_design_matrix(res, xs, fes, use_sparse=True)
    beta, _ = compress.solve_wls(design, Y, wts)
    return np.asarray(beta[1:len(xs) + 1])


def lsdv_reference(compress, data, y, xs, fes, keep, vcov, cluster_cols, ssc, n_obs, df_resid):
    """Exact LSDV fit + SEs computed by the reference's own functions."""
    sel = lambda a: np.asarray(a)[keep]
    cols = {c: sel(data[c]).astype(np.float64) for c in xs}
    for f in fes:
        cols[f] = sel(data[f])
    yv = sel(data[y]).astype(np.float64)
    n = yv.size
    cols["_mean_y"] = yv
    cols["_wts"] = np.ones(n)
    cols["_n"] = np.ones(n)
    cols["_sum_y"] = yv
    cols["_sum_y_sq"] = yv ** 2
    res = compress.DuckDBResult(cols)
    design, Y, wts, all_cols, _ = compress.build_design_matrix(res, xs, fes, use_sparse=True)
    beta, XtX_inv = compress.solve_wls(design, Y, wts)
    rss_total, rss_per_group = compress.compute_rss_grouped(res, design, beta, backend="duckdb")
    cl_ids, resid_sums = None, None
    if vcov == "cluster":
        cl = [sel(data[c]) for c in cluster_cols]
        cl_ids = cl[0] if len(cl) == 1 else np.stack(cl, axis=1)
        fitted = np.asarray(design @ beta).ravel()
        resid_sums = yv - fitted
    k_x = len(xs) + 1
    ctx = compress.CompressionContext(
        XtX_inv=XtX_inv, rss_total=rss_total, rss_per_group=rss_per_group,
        n_obs=n_obs, df_resid=df_resid, vcov=vcov, design_matrix=design,
        x_cols=all_cols[:k_x], cluster_ids=cl_ids, residual_sums_per_group=resid_sums,
        apply_small_sample_correction=ssc)
    se, ncl = compress.compute_se_compress(ctx)
    return np.asarray(beta[1:k_x]), np.asarray(se[1:]), ncl


# ---------------------------------------------------------------------------
# fixture recipes
# ---------------------------------------------------------------------------

def fx_xlang():
    """tests/test_cross_language_equivalence.py:19-48 (seed 12345, n=1000)."""
    np.random.seed(12345)
    n = 1000
    return {
        "y": np.random.normal(10, 2, n),
        "x1": np.random.normal(0, 1, n),
        "x2": np.random.normal(5, 2, n),
        "treatment": np.random.binomial(1, 0.5, n),
        "fe1": np.repeat(np.arange(100), 10),
        "fe2": np.tile(np.arange(50), 20),
        "cluster": np.repeat(np.arange(50), 20),
        "weight": np.random.uniform(0.5, 2.0, n),
    }


def fx_multitreat():
    """python/tests/test_multiple_treatments.py:10-38 (seed 42, n=10000)."""
    np.random.seed(42)
    n = 10000
    d = {
        "customer_id": np.repeat(np.arange(1000), 10),
        "product_id": np.tile(np.arange(100), 100),
        "region": np.random.choice([0, 1, 2], n),
        "treatment_A": np.random.binomial(1, 0.3, n),
        "treatment_B": np.random.binomial(1, 0.4, n),
        "treatment_C": np.random.choice([0, 1, 2], n),
    }
    d["revenue"] = (10.0 + 0.5 * d["treatment_A"] + 0.8 * d["treatment_B"] + 1.2 * d["treatment_C"]
                    + d["customer_id"] * 0.01 + d["product_id"] * 0.02 + np.random.normal(0, 1, n))
    return d


def fx_panel(seed=7, n=20000, L=(400, 30), k=3, singletons=25, weights=False, clusters=True):
    """Unbalanced random panel with FE-correlated regressors and injected singletons."""
    rng = np.random.default_rng(seed)
    codes = [rng.integers(0, G, n) for G in L]
    # injected singletons: fresh fe1 levels used once (dropped by the single-pass rule)
    codes[0][:singletons] = L[0] + np.arange(singletons)
    eff = [rng.normal(0, 1.0 / (f + 1), G + singletons) for f, G in enumerate(L)]
    d = {}
    y = rng.normal(0, 1, n)
    for j in range(k):
        x = rng.normal(0, 1, n) + 0.7 * eff[0][codes[0]] - 0.3 * eff[-1][codes[-1]]
        d[f"x{j + 1}"] = x
        y = y + (1.0 - 0.3 * j) * x
    for f in range(len(L)):
        y = y + eff[f][codes[f]]
        d[f"fe{f + 1}"] = codes[f]
    d["y"] = y
    if weights:
        d["w"] = rng.uniform(0.5, 2.0, n)
    if clusters:
        d["cl1"] = rng.integers(0, 60, n)
        d["cl2"] = rng.integers(0, 45, n)
    return d


def fx_iv(seed=21, n=20000, L=(400, 30), weights=False):
    """IV panel: x1 endogenous (shares the shock u with y), z1 its instrument,
    x2 exogenous (its own instrument, as the reference's Z holds only the listed
    instruments, polars_impl.py:178)."""
    rng = np.random.default_rng(seed)
    codes = [rng.integers(0, G, n) for G in L]
    codes[0][:20] = L[0] + np.arange(20)  # singletons
    eff = [rng.normal(0, 1.0, G + 20) for G in L]
    u = rng.normal(0, 1, n)
    z1 = rng.normal(0, 1, n) + 0.5 * eff[0][codes[0]]
    x2 = rng.normal(0, 1, n) - 0.3 * eff[-1][codes[-1]]
    x1 = 0.9 * z1 + 0.3 * x2 + 0.7 * u + 0.4 * eff[-1][codes[-1]] + rng.normal(0, 0.5, n)
    y = 1.5 * x1 - 0.5 * x2 + u + sum(e[c] for e, c in zip(eff, codes))
    d = {"y": y, "x1": x1, "x2": x2, "z1": z1, "cl1": rng.integers(0, 60, n), "cl2": rng.integers(0, 45, n)}
    for f, c in enumerate(codes):
        d[f"fe{f + 1}"] = c
    if weights:
        d["w"] = rng.uniform(0.5, 2.0, n)
    return d


def fx_synth(n=20000, k=4, L=(500, 40)):
    return synth.panel(n, k, list(L), seed=12345)


CASES = [
    # name, recipe, y, xs, fes, strategy, weights, vcov, cluster_cols
    ("xlang_iid", fx_xlang, "y", ["x1", "x2", "treatment"], ["fe1", "fe2"], "alt_proj", None, "iid", None),
    ("xlang_hc1", fx_xlang, "y", ["x1", "x2", "treatment"], ["fe1", "fe2"], "alt_proj", None, "HC1", None),
    ("xlang_cl1", fx_xlang, "y", ["x1", "x2", "treatment"], ["fe1", "fe2"], "alt_proj", None, "cluster", ["cluster"]),
    ("xlang_cl2", fx_xlang, "y", ["x1", "x2", "treatment"], ["fe1", "fe2"], "alt_proj", None, "cluster", ["cluster", "fe2"]),
    ("xlang_demean", fx_xlang, "y", ["x1", "x2", "treatment"], ["fe1"], "demean", None, "iid", None),
    ("multitreat_iid", fx_multitreat, "revenue", ["treatment_A", "treatment_B", "treatment_C"],
     ["customer_id", "product_id"], "alt_proj", None, "iid", None),
    ("multitreat_cl1", fx_multitreat, "revenue", ["treatment_A", "treatment_B"],
     ["customer_id", "product_id"], "alt_proj", None, "cluster", ["customer_id"]),
    ("panel_iid", fx_panel, "y", ["x1", "x2", "x3"], ["fe1", "fe2"], "alt_proj", None, "iid", None),
    ("panel_hc1", fx_panel, "y", ["x1", "x2", "x3"], ["fe1", "fe2"], "alt_proj", None, "HC1", None),
    ("panel_cl1", fx_panel, "y", ["x1", "x2", "x3"], ["fe1", "fe2"], "alt_proj", None, "cluster", ["cl1"]),
    ("panel_cl2", fx_panel, "y", ["x1", "x2", "x3"], ["fe1", "fe2"], "alt_proj", None, "cluster", ["cl1", "cl2"]),
    ("panel3_cl2", lambda: fx_panel(seed=11, n=20000, L=(300, 60, 12), k=3), "y", ["x1", "x2", "x3"],
     ["fe1", "fe2", "fe3"], "alt_proj", None, "cluster", ["fe2", "fe3"]),
    ("panel_demean_hc1", lambda: fx_panel(seed=5, n=15000, L=(700,), k=2), "y", ["x1", "x2"], ["fe1"],
     "demean", None, "HC1", None),
    ("synth_iid", fx_synth, "y", ["x1", "x2", "x3", "x4"], ["fe1", "fe2"], "alt_proj", None, "iid", None),
    ("synth_hc1", fx_synth, "y", ["x1", "x2", "x3", "x4"], ["fe1", "fe2"], "alt_proj", None, "HC1", None),
]

# weighted fits: the reference's solve_wls (compress.py:659-680) takes per-row
# sqrt-weights, so passing _wts = sqrt(w) to its LSDV fit pins the weighted beta
# (ref_beta, "reference-wls-beta").  Its grouped SE helpers assume _wts = sqrt(_n),
# so the weighted SEs stay pinned to the oracle restatement of polars_impl.py:493-500,
# :201-206 and std_errors.py's weighted branches.
WEIGHTED = [
    ("xlang_w_iid", fx_xlang, "y", ["x1", "x2", "treatment"], ["fe1", "fe2"], "alt_proj", "weight", "iid", None),
    ("panel_w_cl1", lambda: fx_panel(seed=9, weights=True), "y", ["x1", "x2", "x3"], ["fe1", "fe2"],
     "alt_proj", "w", "cluster", ["cl1"]),
]


# IV/2SLS (polars_impl.py:176-270): just-identified designs (instruments = x count,
# so an intercept joins Z, :179-181).  The 2SLS algebra and the IV SEs are pinned by
# the reference's own common.iv_2sls and std_errors._compute_se_*_iv run on the
# oracle's demeaned columns; the demeaning itself is pinned by the LSDV cases above.
IV = [
    # name, recipe, y, xs, fes, strategy, weights, vcov, cluster_cols, instruments
    ("iv_iid", fx_iv, "y", ["x1", "x2"], ["fe1", "fe2"], "alt_proj", None, "iid", None, ["z1", "x2"]),
    ("iv_hc1", fx_iv, "y", ["x1", "x2"], ["fe1", "fe2"], "alt_proj", None, "HC1", None, ["z1", "x2"]),
    ("iv_cl1", fx_iv, "y", ["x1", "x2"], ["fe1", "fe2"], "alt_proj", None, "cluster", ["cl1"], ["z1", "x2"]),
    ("iv_cl2", fx_iv, "y", ["x1", "x2"], ["fe1", "fe2"], "alt_proj", None, "cluster", ["cl1", "cl2"],
     ["z1", "x2"]),
    ("iv_w_hc1", lambda: fx_iv(seed=23, weights=True), "y", ["x1", "x2"], ["fe1", "fe2"], "alt_proj", "w",
     "HC1", None, ["z1", "x2"]),
    ("iv_demean_cl1", lambda: fx_iv(seed=25, L=(500,)), "y", ["x1"], ["fe1"], "demean", None, "cluster",
     ["cl1"], ["z1"]),
]


def iv_reference(std_errors, common, orc, data, weights, vcov, cl, ssc=True):
    """2SLS + SEs of the oracle's demeaned columns by the reference's own functions
    (common.iv_2sls, std_errors._compute_se_hc1_iv / _cluster_oneway_iv /
    _cluster_multiway_iv); XtX_inv as polars_impl.py:185-198, IID as std_errors.py:196-210."""
    keep = orc["keep"]
    cols = orc["demeaned"]
    k = len(orc["beta"])
    n = cols.shape[1]
    Y = cols[0]
    X = np.hstack([np.ones((n, 1)), cols[1:1 + k].T])
    Z = cols[1 + k:].T
    if X.shape[1] > Z.shape[1] and not any(np.allclose(c, 1.0) for c in Z.T):
        Z = np.column_stack([np.ones(n), Z])
    w = np.asarray(data[weights])[keep].astype(np.float64) if weights else None
    beta_full, X_hat = common.iv_2sls(Y, X, Z, w)
    Xh = X_hat * np.sqrt(w)[:, None] if w is not None else X_hat
    L = np.linalg.cholesky(Xh.T @ Xh)
    XtX_inv = np.linalg.solve(L.T, np.linalg.solve(L, np.eye(L.shape[0])))
    resid = Y - X_hat @ beta_full
    n_obs, df_resid = orc["n_obs"], orc["df_resid"]
    v = vcov.lower()
    ncl = None
    if v == "iid":
        s2 = float(np.sum((w if w is not None else 1.0) * resid ** 2)) / df_resid
        se = np.sqrt(np.maximum(s2 * np.diag(XtX_inv), 0.0))
    elif v == "hc1":
        se, _ = std_errors._compute_se_hc1_iv(XtX_inv, resid, X_hat, w, n_obs, df_resid)
    elif len(cl) == 1:
        ids = np.asarray(data[cl[0]])[keep]
        se, ncl = std_errors._compute_se_cluster_oneway_iv(XtX_inv, resid, X_hat, w, ids, n_obs, df_resid, ssc)
    else:
        ids = np.stack([np.asarray(data[c])[keep] for c in cl], axis=1)
        se, ncl = std_errors._compute_se_cluster_multiway_iv(XtX_inv, resid, X_hat, w, ids, n_obs, df_resid, ssc)
    return np.asarray(beta_full[1:]), np.asarray(se[1:]), ncl


def fx_yoco(seed=41, n=20000, L=(50, 20), weights=False):
    """Discrete regressors on low-cardinality FEs (the YOCO use case): a binary
    treatment and a 5-level dose, so (x, FE) cells repeat and records compress."""
    rng = np.random.default_rng(seed)
    codes = [rng.integers(0, G, n) for G in L]
    eff = [rng.normal(0, 1.0, G) for G in L]
    d = {"treat": rng.integers(0, 2, n).astype(np.float64), "dose": rng.integers(0, 5, n).astype(np.float64)}
    d["y"] = 0.8 * d["treat"] - 0.3 * d["dose"] + rng.normal(0, 1, n) + sum(e[c] for e, c in zip(eff, codes))
    for f, c in enumerate(codes):
        d[f"fe{f + 1}"] = c
    d["state"] = codes[0] // 5
    if weights:
        d["w"] = rng.uniform(0.5, 2.0, n)
    return d


# YOCO strategy='compress' (compress.py:282-1175): outputs of the reference's own
# build_design_matrix / solve_wls / compute_rss_grouped / compute_se_compress on the
# records of oracle/yoco.compress (the Polars group_by restated in NumPy)
YOCO = [
    # name, recipe, y, xs, fes, weights, vcov, cluster_cols
    ("yoco_iid", fx_yoco, "y", ["treat", "dose"], ["fe1", "fe2"], None, "iid", None),
    ("yoco_hc1", fx_yoco, "y", ["treat", "dose"], ["fe1", "fe2"], None, "HC1", None),
    ("yoco_cl1", fx_yoco, "y", ["treat", "dose"], ["fe1", "fe2"], None, "cluster", ["state"]),
    ("yoco_cl2", fx_yoco, "y", ["treat", "dose"], ["fe1", "fe2"], None, "cluster", ["state", "fe2"]),
    ("yoco_w_hc1", lambda: fx_yoco(seed=43, weights=True), "y", ["treat", "dose"], ["fe1", "fe2"], "w", "HC1",
     None),
    ("yoco_1fe_cl1", lambda: fx_yoco(seed=45, L=(80,)), "y", ["treat", "dose"], ["fe1"], None, "cluster",
     ["state"]),
    ("yoco_nofe_hc1", lambda: fx_yoco(seed=47, L=(3,)), "y", ["treat", "dose"], [], None, "HC1", None),
]


def yoco_reference(compress, orc, xs, fes, vcov, cl, ssc=True):
    """leanfe_compress_polars (compress.py:1049-1175) after the group_by, by the
    reference's own functions."""
    rec = orc["records"]
    res = compress.DuckDBResult({c: np.asarray(v) for c, v in rec.items()})
    design, Y, wts, all_cols, _ = compress.build_design_matrix(res, list(xs), list(fes), use_sparse=True)
    beta, XtX_inv = compress.solve_wls(design, Y, wts)
    rss_total, rss_per_group = compress.compute_rss_grouped(res, design, beta, backend="duckdb")
    df_resid = orc["n_obs"] - len(all_cols)
    cl_ids, resid_sums = None, None
    if vcov.lower() == "cluster":
        cl_ids = rec[cl[0]] if len(cl) == 1 else np.stack([rec[c] for c in cl], axis=1)
        fitted = np.asarray(design @ beta).ravel()
        resid_sums = rec["_sum_y"] - rec["_n"] * fitted
    k_x = len(xs) + 1
    ctx = compress.CompressionContext(
        XtX_inv=XtX_inv, rss_total=rss_total, rss_per_group=rss_per_group, n_obs=orc["n_obs"],
        df_resid=df_resid, vcov=vcov, design_matrix=design, x_cols=all_cols[:k_x], cluster_ids=cl_ids,
        residual_sums_per_group=resid_sums, apply_small_sample_correction=ssc)
    se, ncl = compress.compute_se_compress(ctx)
    return np.asarray(beta[1:k_x]), np.asarray(se[1:]), ncl, df_resid, float(rss_total)


def _pack(name, data, y, xs, fes, strategy, weights, vcov, cl, ref, orc, tight, instruments=None, wls_beta=None,
          ssc=True):
    arrays = {f"in_{c}": np.asarray(v) for c, v in data.items()}
    meta = dict(name=name, y=y, xs=xs, fes=fes, strategy=strategy, weights=weights, vcov=vcov,
                instruments=instruments or [],
                cluster_cols=cl, demean_tol=1e-6, max_iter=50, ssc=bool(ssc),
                oracle_n_clusters=orc["n_clusters"], ref_n_clusters=ref[2] if ref else None,
                pinned=(("reference-iv" if instruments else "reference-lsdv") if ref else
                        "reference-wls-beta" if wls_beta is not None else "oracle-only"))
    arrays.update(
        oracle_beta=orc["beta"], oracle_se=orc["se"], oracle_iterations=np.int64(orc["iterations"]),
        oracle_n_obs=np.int64(orc["n_obs"]), oracle_df_resid=np.int64(orc["df_resid"]),
        oracle_fe_dims=np.asarray(orc["fe_dims"], dtype=np.int64),
        oracle_r2=np.float64(orc["r_squared"] if orc["r_squared"] is not None else np.nan),
        tight_beta=tight["beta"], tight_se=tight["se"],
        meta=np.frombuffer(json.dumps(meta, default=lambda o: list(o) if isinstance(o, tuple) else o)
                           .encode(), dtype=np.uint8))
    if ref:
        arrays.update(ref_beta=ref[0], ref_se=ref[1])
    if wls_beta is not None:
        arrays.update(ref_beta=wls_beta)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrays)


def _json_ncl(v):
    return list(v) if isinstance(v, tuple) else v


# ssc=False (std_errors.py:339-342 one-way G/(G-1) only; :434-436 no (n-1)/df_resid after the
# G_min rule): pinned to the reference's compute_se_compress / _compute_se_cluster_*_iv with
# apply_small_sample_correction / ssc False, whose adjustments are the same expressions
NOSSC = [
    ("panel_cl1_nossc", lambda: fx_panel(seed=13), "y", ["x1", "x2", "x3"], ["fe1", "fe2"], "alt_proj", None,
     "cluster", ["cl1"]),
    ("panel_cl2_nossc", lambda: fx_panel(seed=15), "y", ["x1", "x2", "x3"], ["fe1", "fe2"], "alt_proj", None,
     "cluster", ["cl1", "cl2"]),
    ("xlang_cl2_nossc", fx_xlang, "y", ["x1", "x2", "treatment"], ["fe1", "fe2"], "alt_proj", None, "cluster",
     ["cluster", "fe2"]),
]
NOSSC_IV = [
    ("iv_cl1_nossc", lambda: fx_iv(seed=27), "y", ["x1", "x2"], ["fe1", "fe2"], "alt_proj", None, "cluster", ["cl1"],
     ["z1", "x2"]),
    ("iv_cl2_nossc", lambda: fx_iv(seed=29), "y", ["x1", "x2"], ["fe1", "fe2"], "alt_proj", None, "cluster",
     ["cl1", "cl2"], ["z1", "x2"]),
]


def main_nossc():
    compress, std_errors, common = load_reference()
    for name, recipe, y, xs, fes, strategy, weights, vcov, cl in NOSSC:
        data = recipe()
        orc = altproj.fit(data, y, xs, fes, strategy=strategy, vcov=vcov, cluster_cols=cl, ssc=False)
        tight = altproj.fit(data, y, xs, fes, strategy=strategy, vcov=vcov, cluster_cols=cl, ssc=False,
                            demean_tol=1e-14, max_iter=100000)
        ref = lsdv_reference(compress, data, y, xs, fes, orc["keep"], vcov, cl, False, orc["n_obs"], orc["df_resid"])
        rb = np.max(np.abs(tight["beta"] - ref[0]) / np.maximum(np.abs(ref[0]), 1e-300))
        rs = np.max(np.abs(tight["se"] - ref[1]) / np.maximum(np.abs(ref[1]), 1e-300))
        assert rb < 1e-9 and rs < 1e-9, (name, rb, rs)
        assert _json_ncl(ref[2]) == _json_ncl(orc["n_clusters"]), (name, ref[2], orc["n_clusters"])
        with_ssc = altproj.fit(data, y, xs, fes, strategy=strategy, vcov=vcov, cluster_cols=cl, ssc=True)
        assert not np.allclose(with_ssc["se"], orc["se"], rtol=1e-6), name  # the flag changes the SEs
        print(f"{name:18s} it={orc['iterations']:3d} n={orc['n_obs']:6d} tight-vs-ref beta {rb:.1e} se {rs:.1e}")
        _pack(name, data, y, xs, fes, strategy, weights, vcov, cl, ref, orc, tight, ssc=False)
    for name, recipe, y, xs, fes, strategy, weights, vcov, cl, inst in NOSSC_IV:
        data = recipe()
        orc = altproj.fit(data, y, xs, fes, strategy=strategy, vcov=vcov, cluster_cols=cl, instruments=inst,
                          ssc=False)
        tight = altproj.fit(data, y, xs, fes, strategy=strategy, vcov=vcov, cluster_cols=cl, instruments=inst,
                            ssc=False, demean_tol=1e-14, max_iter=100000)
        ref = iv_reference(std_errors, common, orc, data, weights, vcov, cl, ssc=False)
        rb = np.max(np.abs(orc["beta"] - ref[0]) / np.abs(ref[0]))
        rs = np.max(np.abs(orc["se"] - ref[1]) / np.abs(ref[1]))
        assert rb < 1e-11 and rs < 1e-11, (name, rb, rs)
        assert _json_ncl(ref[2]) == _json_ncl(orc["n_clusters"]), (name, ref[2], orc["n_clusters"])
        print(f"{name:18s} it={orc['iterations']:3d} n={orc['n_obs']:6d} oracle-vs-ref IV beta {rb:.1e} se {rs:.1e}")
        _pack(name, data, y, xs, fes, strategy, weights, vcov, cl, ref, orc, tight, instruments=inst, ssc=False)


def main(only_weighted=False):
    compress, std_errors, common = load_reference()
    worst = 0.0
    for name, recipe, y, xs, fes, strategy, weights, vcov, cl in (WEIGHTED if only_weighted else CASES + WEIGHTED):
        data = recipe()
        orc = altproj.fit(data, y, xs, fes, strategy=strategy, weights=weights, vcov=vcov,
                          cluster_cols=cl)
        tight = altproj.fit(data, y, xs, fes, strategy=strategy, weights=weights, vcov=vcov,
                            cluster_cols=cl, demean_tol=1e-14, max_iter=100000)
        ref = None
        if weights is None:
            ref = lsdv_reference(compress, data, y, xs, fes, orc["keep"], vcov, cl, True,
                                 orc["n_obs"], orc["df_resid"])
            rb = np.max(np.abs(tight["beta"] - ref[0]) / np.maximum(np.abs(ref[0]), 1e-300))
            rs = np.max(np.abs(tight["se"] - ref[1]) / np.maximum(np.abs(ref[1]), 1e-300))
            db = np.max(np.abs(orc["beta"] - ref[0]) / np.maximum(np.abs(ref[0]), 1e-300))
            assert rb < 1e-9 and rs < 1e-9, (name, rb, rs)
            assert _json_ncl(ref[2]) == _json_ncl(orc["n_clusters"]), (name, ref[2], orc["n_clusters"])
            worst = max(worst, rb, rs)
            print(f"{name:18s} it={orc['iterations']:3d} n={orc['n_obs']:6d} df={orc['df_resid']:6d} "
                  f"tight-vs-ref beta {rb:.1e} se {rs:.1e} | default-tol beta dev {db:.1e}")
        else:
            wb = wls_reference_beta(compress, data, y, xs, fes, orc["keep"], weights)
            rb = np.max(np.abs(tight["beta"] - wb) / np.maximum(np.abs(wb), 1e-300))
            assert rb < 1e-9, (name, rb)
            print(f"{name:18s} it={orc['iterations']:3d} n={orc['n_obs']:6d} weighted: tight-vs-ref beta {rb:.1e} "
                  f"(SE oracle-pinned)")
            if only_weighted:
                _pack(name, data, y, xs, fes, strategy, weights, vcov, cl, None, orc, tight, wls_beta=wb)
        if not only_weighted:
            _pack(name, data, y, xs, fes, strategy, weights, vcov, cl, ref, orc, tight,
                  wls_beta=None if weights is None else wb)
    print(f"worst tight-oracle vs reference-LSDV relative deviation: {worst:.2e}")
    if only_weighted:
        return
    worst = 0.0
    for name, recipe, y, xs, fes, strategy, weights, vcov, cl, inst in IV:
        data = recipe()
        orc = altproj.fit(data, y, xs, fes, strategy=strategy, weights=weights, vcov=vcov,
                          cluster_cols=cl, instruments=inst)
        tight = altproj.fit(data, y, xs, fes, strategy=strategy, weights=weights, vcov=vcov,
                            cluster_cols=cl, instruments=inst, demean_tol=1e-14, max_iter=100000)
        ref = iv_reference(std_errors, common, orc, data, weights, vcov, cl)
        rb = np.max(np.abs(orc["beta"] - ref[0]) / np.abs(ref[0]))
        rs = np.max(np.abs(orc["se"] - ref[1]) / np.abs(ref[1]))
        assert rb < 1e-11 and rs < 1e-11, (name, rb, rs)
        assert _json_ncl(ref[2]) == _json_ncl(orc["n_clusters"]), (name, ref[2], orc["n_clusters"])
        worst = max(worst, rb, rs)
        print(f"{name:18s} it={orc['iterations']:3d} n={orc['n_obs']:6d} df={orc['df_resid']:6d} "
              f"oracle-vs-ref IV beta {rb:.1e} se {rs:.1e}")
        _pack(name, data, y, xs, fes, strategy, weights, vcov, cl, ref, orc, tight, instruments=inst)
    print(f"worst oracle vs reference IV relative deviation: {worst:.2e}")
    worst = 0.0
    for name, recipe, y, xs, fes, weights, vcov, cl in YOCO:
        data = recipe()
        orc = yoco.fit(data, y, xs, fes, weights=weights, vcov=vcov, cluster_cols=cl)
        rb_, rs_, rncl, rdf, rrss = yoco_reference(compress, orc, xs, fes, vcov, cl)
        rb = np.max(np.abs(orc["beta"] - rb_) / np.abs(rb_))
        rs = np.max(np.abs(orc["se"] - rs_) / np.abs(rs_))
        assert rb < 1e-11 and rs < 1e-11 and rdf == orc["df_resid"], (name, rb, rs, rdf, orc["df_resid"])
        assert _json_ncl(rncl) == _json_ncl(orc["n_clusters"]), (name, rncl, orc["n_clusters"])
        worst = max(worst, rb, rs)
        print(f"{name:18s} records={orc['n_compressed']:6d} n={orc['n_obs']:6d} df={orc['df_resid']:6d} "
              f"oracle-vs-ref YOCO beta {rb:.1e} se {rs:.1e}")
        arrays = {f"in_{c}": np.asarray(v) for c, v in data.items()}
        meta = dict(name=name, y=y, xs=xs, fes=fes, strategy="compress", weights=weights, vcov=vcov,
                    cluster_cols=cl, instruments=[], demean_tol=1e-6, max_iter=50, ssc=True,
                    oracle_n_clusters=orc["n_clusters"], ref_n_clusters=rncl, pinned="reference-yoco")
        arrays.update(
            oracle_beta=orc["beta"], oracle_se=orc["se"], oracle_n_obs=np.int64(orc["n_obs"]),
            oracle_df_resid=np.int64(orc["df_resid"]), oracle_n_compressed=np.int64(orc["n_compressed"]),
            oracle_fe_dims=np.asarray(orc["fe_dims"] or (), dtype=np.int64), oracle_rss=np.float64(orc["rss"]),
            ref_beta=rb_, ref_se=rs_, ref_rss=np.float64(rrss),
            meta=np.frombuffer(json.dumps(meta, default=lambda o: list(o) if isinstance(o, tuple) else o)
                               .encode(), dtype=np.uint8))
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrays)
    print(f"worst oracle vs reference YOCO relative deviation: {worst:.2e}")


if __name__ == "__main__":
    if "--nossc-only" in sys.argv:
        main_nossc()
    else:
        main(only_weighted="--weighted-only" in sys.argv)
        main_nossc()

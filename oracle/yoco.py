"""CPU ORACLE — TEST INFRASTRUCTURE ONLY: the YOCO ``strategy='compress'`` path.

A NumPy restatement of the reference's compression estimator so the HIP backend's
``lfe_compress`` path can be checked.  Only ``tests/`` may import it; the product
path (``leanfe_amd``) never imports, calls or falls back to it.

Restated (paths relative to the reference repo ``jorgenhost/leanfe``):

* group-by compression ........ python/leanfe/compress.py:282-358 (compress_polars):
                                key = x_cols + fe_cols (+ cluster cols), aggregates
                                _n, _sum_y, _sum_y_sq (weighted: sum w, sum y w,
                                sum y^2 w), _mean_y = _sum_y/_n, _wts = sqrt(_n)
* design with FE dummies ...... compress.py:503-656 ([1, x, dummies of every FE but
                                its first sorted level])
* WLS solve ................... compress.py:659-747 (Cholesky; lstsq/pinv fallback)
* grouped RSS ................. compress.py:754-811
* SEs ......................... compress.py:854-1042 (IID, HC1, one-way, CGM multi-way
                                on the records, G_min rule, ssc)
* driver ...................... compress.py:1049-1175 (leanfe_compress_polars: df_resid
                                = n_obs - P, fe_dims over records, n_compressed)

Pinning: ``tests/golden/make_golden.py`` runs the reference's own
``build_design_matrix`` / ``solve_wls`` / ``compute_rss_grouped`` /
``compute_se_compress`` on the same records and stores their outputs as ``ref_*``.
"""
from __future__ import annotations

from itertools import combinations

import numpy as np

MIN_CLUSTERS_FOR_ADJUSTMENT = 2  # std_errors.py:22 / compress.py


def _canon(col: np.ndarray) -> np.ndarray:
    """Group-by key of a float column: -0.0 == 0.0, every NaN alike."""
    v = np.asarray(col, dtype=np.float64).copy()
    v[v == 0.0] = 0.0
    bits = v.view(np.int64).copy()
    bits[np.isnan(v)] = np.int64(0x7FF8000000000000)
    return bits


def compress(data: dict, y: str, xs: list[str], fes: list[str], weights: str | None,
             cluster_cols: list[str] | None) -> dict:
    """compress.py:282-358 — one record per distinct (x, FE, cluster) key."""
    group_cols = list(xs) + list(fes)
    for c in cluster_cols or []:
        if c not in group_cols:
            group_cols.append(c)
    n = len(np.asarray(data[y]))
    keys = np.stack([_canon(data[c]) if np.asarray(data[c]).dtype.kind == "f"
                     else np.asarray(data[c]).astype(np.int64) for c in group_cols], axis=1) \
        if group_cols else np.zeros((n, 1), dtype=np.int64)
    _, first, inv = np.unique(keys, axis=0, return_index=True, return_inverse=True)
    inv = inv.ravel()
    G = first.size
    yv = np.asarray(data[y], dtype=np.float64)
    w = np.ones(n) if weights is None else np.asarray(data[weights], dtype=np.float64)
    rec = {c: np.asarray(data[c])[first] for c in group_cols}
    rec["_n"] = np.bincount(inv, weights=w, minlength=G)
    rec["_sum_y"] = np.bincount(inv, weights=yv * w, minlength=G)
    rec["_sum_y_sq"] = np.bincount(inv, weights=yv * yv * w, minlength=G)
    rec["_mean_y"] = rec["_sum_y"] / rec["_n"]
    rec["_wts"] = np.sqrt(rec["_n"])
    return dict(records=rec, n_obs=n, n_compressed=G)


def design(rec: dict, xs: list[str], fes: list[str]) -> tuple[np.ndarray, list[int]]:
    """compress.py:503-656: [1, x, dummies(FE, sorted levels, first dropped)]."""
    G = rec["_n"].size
    blocks = [np.ones((G, 1))] + [np.asarray(rec[x], dtype=np.float64)[:, None] for x in xs]
    dims = []
    for f in fes:
        cats, code = np.unique(np.asarray(rec[f]), return_inverse=True)
        dims.append(int(cats.size))
        D = np.zeros((G, cats.size - 1))
        m = code.ravel() > 0
        D[np.nonzero(m)[0], code.ravel()[m] - 1] = 1.0
        blocks.append(D)
    return np.hstack(blocks), dims


def solve_wls(X: np.ndarray, Y: np.ndarray, wts: np.ndarray):
    """compress.py:659-747."""
    Xw = X * wts[:, None]
    XtX = Xw.T @ Xw
    Xty = Xw.T @ (Y * wts)
    try:
        L = np.linalg.cholesky(XtX)
        beta = np.linalg.solve(L.T, np.linalg.solve(L, Xty))
        XtX_inv = np.linalg.solve(L.T, np.linalg.solve(L, np.eye(XtX.shape[0])))
    except np.linalg.LinAlgError:
        beta = np.linalg.lstsq(XtX, Xty, rcond=None)[0]
        XtX_inv = np.linalg.pinv(XtX)
    return beta, XtX_inv


def _cluster_meat(scores: np.ndarray, ids: np.ndarray) -> tuple[np.ndarray, int]:
    _, inv = np.unique(ids, axis=0, return_inverse=True)
    inv = inv.ravel()
    G = int(inv.max()) + 1 if inv.size else 0
    S = np.zeros((G, scores.shape[1]))
    np.add.at(S, inv, scores)
    return S.T @ S, G


def fit(data: dict, y: str, xs: list[str], fes: list[str], *, weights: str | None = None,
        vcov: str = "iid", cluster_cols: list[str] | None = None, ssc: bool = True) -> dict:
    """leanfe_compress_polars (compress.py:1049-1175) on a dict of NumPy columns."""
    # polars_impl.py:407-416 passes cluster_cols whatever vcov is: they always join the key
    cc = compress(data, y, xs, fes, weights, cluster_cols)
    rec, n_obs = cc["records"], cc["n_obs"]
    X, dims = design(rec, xs, fes)
    beta, XtX_inv = solve_wls(X, rec["_mean_y"], rec["_wts"])
    fitted = X @ beta
    rss_g = rec["_sum_y_sq"] - 2 * fitted * rec["_sum_y"] + rec["_n"] * fitted ** 2
    rss = float(np.sum(rss_g))
    P = X.shape[1]
    df_resid = n_obs - P
    kx = len(xs) + 1
    v = vcov.lower()
    ncl = None
    if v == "iid":
        se_full = np.sqrt(np.maximum(np.diag(XtX_inv) * (rss / df_resid), 0.0))
    elif v == "hc1":
        meat = X.T @ (X * rss_g[:, None])
        V = XtX_inv @ meat @ XtX_inv
        se_full = np.sqrt(np.maximum(np.diag(V) * (n_obs / df_resid), 0.0))
    elif v == "cluster":
        if cluster_cols is None:
            raise ValueError("cluster_cols required for vcov='cluster'")
        e = rec["_sum_y"] - rec["_n"] * fitted
        scores = X * e[:, None]
        ids = [np.asarray(rec[c]) for c in cluster_cols]
        if len(ids) == 1:
            meat, G = _cluster_meat(scores, ids[0][:, None])
            adj = (G / (G - 1)) * ((n_obs - 1) / df_resid) if ssc else G / (G - 1)
            V = adj * (XtX_inv @ meat @ XtX_inv)
            ncl = G
        else:
            V = np.zeros_like(XtX_inv)
            first = []
            for size in range(1, len(ids) + 1):
                for sub in combinations(range(len(ids)), size):
                    meat, G = _cluster_meat(scores, np.stack([ids[j] for j in sub], axis=1))
                    if size == 1:
                        first.append(G)
                    if G <= 1:
                        continue
                    V += (-1) ** (size - 1) * (XtX_inv @ meat @ XtX_inv)
            if first and min(first) > MIN_CLUSTERS_FOR_ADJUSTMENT:
                V *= min(first) / (min(first) - 1)
            if ssc:
                V *= (n_obs - 1) / df_resid
            ncl = tuple(first)
        se_full = np.sqrt(np.maximum(np.diag(V), 0.0))
    else:
        raise ValueError(f"vcov must be 'iid', 'HC1', or 'cluster', got '{vcov}'")
    return dict(beta=beta[1:kx], se=se_full[1:kx], n_obs=n_obs, n_compressed=cc["n_compressed"],
                df_resid=df_resid, rss=rss, n_clusters=ncl, fe_dims=tuple(dims) if fes else None,
                records=rec)

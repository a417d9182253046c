"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

This module restates, in plain NumPy, the reference leanfe Polars backend's
``strategy='alt_proj'`` / ``'demean'`` hot path so the HIP backend can be checked
against it.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it.  The product path (``leanfe_amd``) never
imports, calls or falls back to it.

Every function cites the reference line(s) it restates (paths relative to the
reference repo ``jorgenhost/leanfe``):

* singleton drop ............ python/leanfe/polars_impl.py:477-482 (alt_proj),
                              :433-435 (demean)
* FE ordering ............... polars_impl.py:485
* projection ................ polars_impl.py:491-508 (unweighted :502-505,
                              weighted :493-500)
* loop + convergence ........ polars_impl.py:490-526
* fe_dims / absorbed_df ..... polars_impl.py:531-537 (alt_proj), :461-465 (demean)
* Gram + Cholesky solve ..... polars_impl.py:165-226
* residual, df, R^2 ......... polars_impl.py:229-232, 281-283
* SE dispatch ............... python/leanfe/std_errors.py:30-176
* IID ....................... std_errors.py:183-210
* HC1 ....................... std_errors.py:217-282
* one-way cluster ........... std_errors.py:289-347
* multi-way CGM ............. std_errors.py:354-441
* IV / 2SLS ................. polars_impl.py:176-200, 229, 234-270; common.py:188-287;
                              std_errors.py:448-602 (HC1 / one-way / multi-way on X_hat)

Pinning: ``tests/golden/make_golden.py`` checks this restatement against the
reference's own importable NumPy/SciPy functions (exact LSDV solve in
``compress.py``, ``compute_se_compress``) and writes ``tests/golden/*.npz``.
"""
from __future__ import annotations

from itertools import combinations

import numpy as np

MIN_CLUSTERS_FOR_ADJUSTMENT = 2  # std_errors.py:22


def factorize(values) -> tuple[np.ndarray, int]:
    """Dense codes 0..G-1 in sorted-unique order (group membership is what matters;
    cf. ``_cats_to_int`` polars_impl.py:118-139)."""
    uniq, inv = np.unique(np.asarray(values), return_inverse=True)
    return inv.astype(np.int64).ravel(), int(uniq.size)


def singleton_keep(codes_list: list[np.ndarray], n_levels: list[int]) -> np.ndarray:
    """``pl.all_horizontal([pl.len().over(fe) > 1 for fe in fe_cols])`` —
    polars_impl.py:478-482.  Counts on the PRE-filter data, single pass."""
    n = codes_list[0].size if codes_list else 0
    keep = np.ones(n, dtype=bool)
    for codes, G in zip(codes_list, n_levels):
        cnt = np.bincount(codes, minlength=G)
        keep &= cnt[codes] > 1
    return keep


def _group_mean(col: np.ndarray, codes: np.ndarray, G: int, w: np.ndarray | None) -> np.ndarray:
    """Per-row group mean ``c.mean().over(fe)`` (polars_impl.py:503) or weighted
    ``(c*w).sum().over(fe) / w.sum().over(fe)`` (polars_impl.py:496-497)."""
    if w is None:
        s = np.bincount(codes, weights=col, minlength=G)
        n = np.bincount(codes, minlength=G).astype(np.float64)
    else:
        s = np.bincount(codes, weights=col * w, minlength=G)
        n = np.bincount(codes, weights=w, minlength=G)
    with np.errstate(invalid="ignore", divide="ignore"):
        m = s / n
    return m[codes]


def project(cols: np.ndarray, codes: np.ndarray, G: int, w: np.ndarray | None) -> np.ndarray:
    """One FE projection: every column updates from the same pre-FE state
    (one ``with_columns``), polars_impl.py:491-508."""
    out = np.empty_like(cols)
    for j in range(cols.shape[0]):
        out[j] = cols[j] - _group_mean(cols[j], codes, G, w)
    return out


def demean_altproj(cols: np.ndarray, codes_list: list[np.ndarray], n_levels: list[int],
                   order: list[int], tol: float, max_iter: int,
                   w: np.ndarray | None = None, y_index: int = 0,
                   trace: list | None = None) -> tuple[np.ndarray, int]:
    """Alternating projections, polars_impl.py:490-526.

    ``order`` is ``fe_cols_ordered`` (ascending cardinality, stable).  After each
    full sweep, from ``it >= 3`` on, the stop test is
    ``max_fe max_rows |mean_over(fe)(y)|`` over ALL FEs in formula order, on y
    only and UNWEIGHTED even when weights are given (polars_impl.py:512-521).
    Returns the demeaned columns and ``iterations``.
    """
    cols = np.array(cols, dtype=np.float64, copy=True)
    iterations = 0
    for it in range(1, max_iter + 1):
        for f in order:
            cols = project(cols, codes_list[f], n_levels[f], w)
        if it >= 3:
            y = cols[y_index]
            max_mean = 0.0
            for codes, G in zip(codes_list, n_levels):
                m = _group_mean(y, codes, G, None)
                if m.size:
                    max_mean = max(max_mean, float(np.max(np.abs(m))))
            if trace is not None:
                trace.append(max_mean)
            if max_mean < tol:
                iterations = it
                break
        iterations = it
    return cols, iterations


def solve_normal(XtX: np.ndarray, Xty: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """Cholesky solve with LinAlgError fallback — polars_impl.py:211-220."""
    try:
        L = np.linalg.cholesky(XtX)
        beta_full = np.linalg.solve(L.T, np.linalg.solve(L, Xty))
        XtX_inv = np.linalg.solve(L.T, np.linalg.solve(L, np.eye(L.shape[0])))
    except np.linalg.LinAlgError:
        beta_full = np.linalg.solve(XtX, Xty)
        XtX_inv = np.linalg.inv(XtX)
    return beta_full, XtX_inv


def se_iid(XtX_inv, resid, w, df_resid):
    """std_errors.py:183-210."""
    if w is not None:
        sigma2 = float(np.sum(w * resid ** 2)) / df_resid
    else:
        sigma2 = float(np.sum(resid ** 2)) / df_resid
    return np.sqrt(np.maximum(sigma2 * np.diag(XtX_inv), 0.0)), None


def se_hc1(X, XtX_inv, resid, w, n_obs, df_resid):
    """std_errors.py:217-282: meat_ij = sum(x_i x_j r^2 [w]) over demeaned x
    (no intercept); V = XtX_inv meat XtX_inv * n/df_resid."""
    s = resid ** 2 if w is None else w * resid ** 2
    meat = X.T @ (X * s[:, None])
    V = XtX_inv @ meat @ XtX_inv
    return np.sqrt(np.maximum((n_obs / df_resid) * np.diag(V), 0.0)), None


def _cluster_scores(X, resid, w, cl_codes):
    """``group_by(cl).agg(sum(x*resid[*w]))`` — std_errors.py:317-333, :408."""
    e = resid if w is None else resid * w
    G = int(cl_codes.max()) + 1 if cl_codes.size else 0
    S = np.stack([np.bincount(cl_codes, weights=X[:, j] * e, minlength=G)
                  for j in range(X.shape[1])], axis=1) if X.shape[1] else np.zeros((G, 0))
    present = np.bincount(cl_codes, minlength=G) > 0
    return S[present], int(present.sum())


def se_cluster_oneway(X, XtX_inv, resid, w, cl_codes, n_obs, df_resid, ssc):
    """std_errors.py:289-347."""
    S, G = _cluster_scores(X, resid, w, cl_codes)
    meat = S.T @ S
    with np.errstate(divide="ignore", invalid="ignore"):
        if ssc:
            adj = (G / (G - 1)) * ((n_obs - 1) / df_resid)
        else:
            adj = G / (G - 1)
    V = adj * (XtX_inv @ meat @ XtX_inv)
    return np.sqrt(np.maximum(np.diag(V), 0.0)), G


def intersect_codes(cols: list[np.ndarray]) -> np.ndarray:
    """Composite-key factorization for ``group_by([c1, c2, ...])``."""
    if len(cols) == 1:
        return factorize(cols[0])[0]
    arr = np.stack(cols, axis=1)
    _, inv = np.unique(arr, axis=0, return_inverse=True)
    return inv.astype(np.int64).ravel()


def se_cluster_multiway(X, XtX_inv, resid, w, cl_cols, n_obs, df_resid, ssc):
    """Cameron-Gelbach-Miller, std_errors.py:354-441 (subsets in
    ``itertools.combinations`` order, G<=1 skipped but first-order G recorded,
    single G_min/(G_min-1) only if G_min > 2, then (n-1)/df_resid if ssc)."""
    m = len(cl_cols)
    V = np.zeros_like(XtX_inv)
    n_clusters = []
    for size in range(1, m + 1):
        sign = (-1) ** (size - 1)
        for subset in combinations(range(m), size):
            codes = intersect_codes([cl_cols[i] for i in subset])
            S, G = _cluster_scores(X, resid, w, codes)
            if size == 1:
                n_clusters.append(G)
            if G <= 1:
                continue
            meat = S.T @ S
            V += sign * (XtX_inv @ meat @ XtX_inv)
    if n_clusters:
        gmin = min(n_clusters)
        if gmin > MIN_CLUSTERS_FOR_ADJUSTMENT:
            V *= gmin / (gmin - 1)
    if ssc:
        V *= (n_obs - 1) / df_resid
    return np.sqrt(np.maximum(np.diag(V), 0.0)), tuple(n_clusters)


def run_regression(Y, Xdm, w, vcov, cl_cols, ssc, n_obs, absorbed_df):
    """``_run_regression`` OLS branch, polars_impl.py:141-285, then
    ``compute_standard_errors_polars`` (std_errors.py:30-176).

    ``vcov`` accepts 'iid', 'HC1'/'hc1' and 'cluster' (the reference's
    alt_proj path cannot reach HC1 because of a case mismatch between
    polars_impl.py:158 and std_errors.py:92; the formula restated is
    std_errors.py:217-282)."""
    n, k = Xdm.shape
    X = np.hstack([np.ones((n, 1)), Xdm]) if k > 0 else np.ones((n, 1))
    if w is not None:
        sw = np.sqrt(w)
        Xw = X * sw[:, None]
        Yw = Y * sw
        XtX = Xw.T @ Xw
        Xty = Xw.T @ Yw
    else:
        XtX = X.T @ X
        Xty = X.T @ Y
    beta_full, XtX_inv = solve_normal(XtX, Xty)
    beta = beta_full[1:] if X.shape[1] == k + 1 and k > 0 else beta_full[1:]
    resid = Y - X @ beta_full
    df_resid = n_obs - (k + 1) - absorbed_df
    Vinv = XtX_inv[1:, 1:]
    v = vcov.lower()
    if v == "iid":
        se, ncl = se_iid(Vinv, resid, w, df_resid)
    elif v == "hc1":
        se, ncl = se_hc1(Xdm, Vinv, resid, w, n_obs, df_resid)
    elif v == "cluster":
        if cl_cols is None:
            raise ValueError("cluster_cols required for vcov='cluster'")
        if len(cl_cols) == 1:
            se, ncl = se_cluster_oneway(Xdm, Vinv, resid, w, factorize(cl_cols[0])[0],
                                        n_obs, df_resid, ssc)
        else:
            se, ncl = se_cluster_multiway(Xdm, Vinv, resid, w, cl_cols, n_obs, df_resid, ssc)
    else:
        raise ValueError(f"Unknown vcov type: {vcov}")
    rss = float(np.sum(resid ** 2))
    tss = float(np.sum((Y - np.mean(Y)) ** 2))
    r2 = 1 - rss / tss if tss > 0 else None
    return dict(beta=beta, beta_full=beta_full, se=se, resid=resid, df_resid=df_resid,
                n_clusters=ncl, r_squared=r2, XtX=XtX, Xty=Xty, XtX_inv=XtX_inv, rss=rss, tss=tss)


def iv_2sls(Y, X, Z, w):
    """common.py:188-287: first stage X = Z gamma (weighted normal equations with
    sqrt(w) rows, X_hat = Z gamma unweighted), second stage on X_hat."""
    if Z.shape[1] < X.shape[1]:
        raise ValueError(f"Under-identified: {Z.shape[1]} instruments for {X.shape[1]} endogenous variables")
    if w is not None:
        sw = np.sqrt(w)
        Zw, Xw, Yw = Z * sw[:, None], X * sw[:, None], Y * sw
    else:
        Zw, Xw, Yw = Z, X, Y
    gamma = np.linalg.solve(Zw.T @ Zw, Zw.T @ Xw)
    X_hat = Z @ gamma
    Xhw = X_hat * sw[:, None] if w is not None else X_hat
    beta = np.linalg.solve(Xhw.T @ Xhw, Xhw.T @ Yw)
    return beta, X_hat


def run_regression_iv(Y, Xdm, Zdm, w, vcov, cl_cols, ssc, n_obs, absorbed_df):
    """``_run_regression`` IV branch, polars_impl.py:176-200 (intercept added to Z
    when X is wider and no Z column is all ones, :179-181), residual on X_hat
    (:229, as the reference computes it), SEs on X_hat with the full XtX_inv
    (:254-270 -> std_errors.py:86-141, 448-602), intercept stripped."""
    n, k = Xdm.shape
    X = np.hstack([np.ones((n, 1)), Xdm]) if k > 0 else np.ones((n, 1))
    Z = Zdm
    if X.shape[1] > Z.shape[1] and not any(np.allclose(col, 1.0) for col in Z.T):
        Z = np.column_stack([np.ones(n), Z])
    beta_full, X_hat = iv_2sls(Y, X, Z, w)
    if w is not None:
        Xhw = X_hat * np.sqrt(w)[:, None]
        XtX = Xhw.T @ Xhw
    else:
        XtX = X_hat.T @ X_hat
    try:
        L = np.linalg.cholesky(XtX)
        XtX_inv = np.linalg.solve(L.T, np.linalg.solve(L, np.eye(L.shape[0])))
    except np.linalg.LinAlgError:
        XtX_inv = np.linalg.inv(XtX)
    resid = Y - X_hat @ beta_full
    df_resid = n_obs - (k + 1) - absorbed_df
    v = vcov.lower()
    if v == "iid":
        se, ncl = se_iid(XtX_inv, resid, w, df_resid)
    elif v == "hc1":
        se, ncl = se_hc1(X_hat, XtX_inv, resid, w, n_obs, df_resid)
    elif v == "cluster":
        if cl_cols is None:
            raise ValueError("cluster_cols required for vcov='cluster'")
        if len(cl_cols) == 1:
            se, ncl = se_cluster_oneway(X_hat, XtX_inv, resid, w, factorize(cl_cols[0])[0],
                                        n_obs, df_resid, ssc)
        else:
            se, ncl = se_cluster_multiway(X_hat, XtX_inv, resid, w, cl_cols, n_obs, df_resid, ssc)
    else:
        raise ValueError(f"Unknown vcov type: {vcov}")
    strip = X.shape[1] == k + 1
    return dict(beta=beta_full[1:] if strip else beta_full, beta_full=beta_full,
                se=se[1:] if strip else se, resid=resid, df_resid=df_resid, n_clusters=ncl,
                r_squared=None, XtX=XtX, XtX_inv=XtX_inv, Z_cols=Z.shape[1],
                rss=float(np.sum(resid ** 2)), tss=None)


def fit(data: dict, y: str, xs: list[str], fes: list[str], *, strategy: str = "alt_proj",
        weights: str | None = None, demean_tol: float = 1e-6, max_iter: int = 50,
        vcov: str = "iid", cluster_cols: list[str] | None = None, ssc: bool = True,
        instruments: list[str] | None = None, trace: list | None = None) -> dict:
    """The alt_proj / demean branch of ``leanfe_polars`` (polars_impl.py:424-579)
    on a dict of NumPy columns.  Returns a plain dict of results.  With
    ``instruments`` the columns ``[y] + xs + instruments`` are demeaned
    (:431, :486) and the IV branch of ``_run_regression`` runs."""
    instruments = list(instruments or [])
    if strategy not in ("alt_proj", "demean"):
        raise ValueError(f"oracle supports alt_proj/demean, got {strategy}")
    if strategy == "demean" and len(fes) != 1:
        raise ValueError("Strategy 'demean' requires exactly one FE column.")
    if strategy == "alt_proj" and not fes:
        raise ValueError("Strategy 'alt_proj' requires FE-cols.")
    fac = [factorize(data[f]) for f in fes]
    codes = [c for c, _ in fac]
    card = [G for _, G in fac]  # fe_cardinality, polars_impl.py:373 (pre-filter)
    keep = singleton_keep(codes, card)
    sel = lambda a: np.asarray(a)[keep]
    cols = np.stack([sel(data[c]).astype(np.float64) for c in [y] + xs + instruments])
    codes_k = [c[keep] for c in codes]
    w = sel(data[weights]).astype(np.float64) if weights else None
    if strategy == "demean":
        cols = project(cols, codes_k[0], card[0], w)
        iterations = 1  # polars_impl.py:465
    else:
        order = sorted(range(len(fes)), key=lambda i: card[i])  # stable, :485
        cols, iterations = demean_altproj(cols, codes_k, card, order, demean_tol, max_iter,
                                          w, 0, trace)
    fe_dims = tuple(int(np.unique(c).size) for c in codes_k)  # :531-534
    absorbed_df = sum(fe_dims) - len(fes)                        # :535 (demean: G-1, :463)
    n_obs = int(keep.sum())
    cl = [sel(data[c]) for c in cluster_cols] if cluster_cols else None
    k = len(xs)
    if instruments:
        reg = run_regression_iv(cols[0], cols[1:1 + k].T.copy(), cols[1 + k:].T.copy(), w, vcov, cl, ssc,
                                n_obs, absorbed_df)
    else:
        reg = run_regression(cols[0], cols[1:].T.copy(), w, vcov, cl, ssc, n_obs, absorbed_df)
    reg.update(n_obs=n_obs, iterations=iterations, fe_dims=fe_dims,
               absorbed_df=absorbed_df, keep=keep, demeaned=cols)
    return reg

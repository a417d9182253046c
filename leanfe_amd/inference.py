"""Host-side (k+1)x(k+1) algebra that follows the device reductions.

These are the only floating-point steps of the hip backend that run on the
host, by design: the Cholesky solve of the 12x12 Gram and the
k x k sandwich products are microseconds of work and keeping them in NumPy
keeps them call-for-call identical to the reference.

* solve ........ polars_impl.py:211-225
* IID .......... std_errors.py:196-210
* HC1 .......... std_errors.py:275-282
* one-way ...... std_errors.py:335-347
* multi-way .... std_errors.py:395-441 (Cameron-Gelbach-Miller, G_min rule)
* IV / 2SLS .... polars_impl.py:176-198 + common.py:188-287 (first and second
                 stage from the device Gram of [1, y, x, z]), std_errors.py:448-602
                 (the X_hat meats as gamma' M_Z gamma of the device's Z-space meats)
"""
from __future__ import annotations

from itertools import combinations

import numpy as np
from scipy.linalg import get_lapack_funcs

MIN_CLUSTERS_FOR_ADJUSTMENT = 2


_potrf, _potrs = get_lapack_funcs(("potrf", "potrs"), (np.zeros((1, 1)),))


def solve_normal(XtX: np.ndarray, Xty: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """beta = (X'X)^-1 X'y and (X'X)^-1 through the Cholesky factor L of X'X (polars_impl.py:211-225:
    cholesky, then the two triangular solves).  LAPACK potrf + one potrs over [X'y | I]: the same
    factor and solves in two calls instead of NumPy's five (8 vs 57 us per solve, which the bench's
    step and every fit pay).  Not positive definite: LU solve and inverse, as the reference."""
    n = XtX.shape[0]
    L, info = _potrf(XtX, lower=1, clean=0)
    if info == 0:
        rhs = np.empty((n, n + 1), order="F")
        rhs[:, 0] = Xty
        rhs[:, 1:] = np.eye(n)
        x, info = _potrs(L, rhs, lower=1, overwrite_b=1)
        if info == 0:
            return x[:, 0].copy(), x[:, 1:]
    return np.linalg.solve(XtX, Xty), np.linalg.inv(XtX)


_X_IDX: dict[int, np.ndarray] = {}


def split_gram(G: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """Gram of [1, y, x_1..x_k] -> (X'X, X'y) of X = [1, x_1..x_k]."""
    n = G.shape[0]
    idx = _X_IDX.get(n)
    if idx is None:
        idx = _X_IDX[n] = np.array([0] + list(range(2, n)))
    return G.take(idx, 0).take(idx, 1), G[idx, 1]


# rss from the Gram cancels as R^2 -> 1: below this share of sum y~^2 the residual pass runs
RSS_FROM_GRAM_MIN = 1e-4


def stats_from_gram(G: np.ndarray, beta_full: np.ndarray):
    """Residual statistics {sum r^2, sum r^2, sum y~, sum y~^2} of an unweighted fit from
    the Gram of [1, y~, x~] alone: r'r = y'y - 2 b'X'y + b'X'X b (polars_impl.py:229,
    281-282 without the residual pass).  None when r'r < RSS_FROM_GRAM_MIN * y'y."""
    idx = [0] + list(range(2, G.shape[0]))
    yy = G[1, 1]
    Xy = G[idx, 1]
    rss = yy - 2.0 * beta_full @ Xy + beta_full @ G[np.ix_(idx, idx)] @ beta_full
    if not (rss > RSS_FROM_GRAM_MIN * yy):
        return None
    return np.array([rss, rss, G[0, 1], yy])


def se_iid(XtX_inv_b: np.ndarray, rss_w: float, df_resid: int) -> np.ndarray:
    sigma2 = rss_w / df_resid
    return np.sqrt(np.maximum(sigma2 * np.diag(XtX_inv_b), 0.0))


def se_hc1(XtX_inv_b: np.ndarray, meat: np.ndarray, n_obs: int, df_resid: int) -> np.ndarray:
    V = XtX_inv_b @ meat @ XtX_inv_b
    return np.sqrt(np.maximum((n_obs / df_resid) * np.diag(V), 0.0))


def se_cluster_oneway(XtX_inv_b, meat, G: int, n_obs: int, df_resid: int, ssc: bool):
    with np.errstate(divide="ignore", invalid="ignore"):
        adj = (G / (G - 1)) * ((n_obs - 1) / df_resid) if ssc else G / (G - 1)
    V = adj * (XtX_inv_b @ meat @ XtX_inv_b)
    return np.sqrt(np.maximum(np.diag(V), 0.0)), int(G)


def cluster_subsets(m: int) -> list[tuple[int, ...]]:
    """Non-empty subsets in the reference's order (size, then combinations order)."""
    return [s for size in range(1, m + 1) for s in combinations(range(m), size)]


def se_cluster_multiway(XtX_inv_b, meats: list[np.ndarray], Gs: list[int], subsets, n_obs: int,
                        df_resid: int, ssc: bool):
    V = np.zeros_like(XtX_inv_b)
    first = []
    for meat, G, s in zip(meats, Gs, subsets):
        if len(s) == 1:
            first.append(int(G))
        if G <= 1:
            continue
        V += (-1) ** (len(s) - 1) * (XtX_inv_b @ meat @ XtX_inv_b)
    if first:
        gmin = min(first)
        if gmin > MIN_CLUSTERS_FOR_ADJUSTMENT:
            V *= gmin / (gmin - 1)
    if ssc:
        V *= (n_obs - 1) / df_resid
    return np.sqrt(np.maximum(np.diag(V), 0.0)), tuple(first)


class IVSystem:
    """2SLS from the (p+1)^2 device Gram of [1, y~, x~_1..x~_k, z~_1..z~_m]
    (sqrt(w) rows when weighted), as ``_run_regression`` + ``iv_2sls`` do it with the
    n-row matrices (polars_impl.py:176-198, common.py:188-287):

        Z = [1, z~] when X = [1, x~] is wider than z~ and no z column is all ones
            (polars_impl.py:179-181; ``z_has_ones`` is that test, done by the caller)
        gamma = (Z'Z)^-1 Z'X,  X_hat = Z gamma,  beta_full = (X_hat'X_hat)^-1 X_hat'y
        XtX_inv = (X_hat'X_hat)^-1 by Cholesky (:185-198)

    Every X_hat-space product is gamma' (Z-space product) gamma, so the device only
    ever forms Z-space sums.  ``coef`` is X_hat beta_full = Z (gamma beta_full) as a
    coefficient vector over u = [1, col_1..col_{p-1}] for ``lfe_resid_iv``.
    """

    def __init__(self, G: np.ndarray, k: int, m: int, z_has_ones: bool = False):
        x_idx = [0] + list(range(2, 2 + k))
        z_idx = list(range(2 + k, 2 + k + m))
        if len(x_idx) > len(z_idx) and not z_has_ones:
            z_idx = [0] + z_idx
        if len(z_idx) < len(x_idx):
            raise ValueError(f"Under-identified: {len(z_idx)} instruments for {len(x_idx)} endogenous variables")
        self.k, self.m = k, m
        ZtZ = G[np.ix_(z_idx, z_idx)]
        ZtX = G[np.ix_(z_idx, x_idx)]
        Zty = G[z_idx, 1]
        self.gamma = np.linalg.solve(ZtZ, ZtX)                  # common.py:264-266
        XhtXh = self.gamma.T @ ZtZ @ self.gamma
        self.beta_full = np.linalg.solve(XhtXh, self.gamma.T @ Zty)  # :269-272
        try:                                                     # polars_impl.py:192-198
            L = np.linalg.cholesky(XhtXh)
            self.XtX_inv = np.linalg.solve(L.T, np.linalg.solve(L, np.eye(L.shape[0])))
        except np.linalg.LinAlgError:
            self.XtX_inv = np.linalg.inv(XhtXh)
        # Z columns as positions in u = [1, col_1..col_{p-1}] (Gram index - 1; intercept 0)
        self.z_u = [0 if j == 0 else j - 1 for j in z_idx]
        p = 1 + k + m
        self.coef = np.zeros(p)
        self.coef[self.z_u] = self.gamma @ self.beta_full

    def xhat_meat(self, meat_u: np.ndarray) -> np.ndarray:
        """X_hat' D X_hat from the device's u-space meat u' D u (or S'S of u-scores)."""
        Mz = meat_u[np.ix_(self.z_u, self.z_u)]
        return self.gamma.T @ Mz @ self.gamma

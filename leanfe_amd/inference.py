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
"""
from __future__ import annotations

from itertools import combinations

import numpy as np

MIN_CLUSTERS_FOR_ADJUSTMENT = 2


def solve_normal(XtX: np.ndarray, Xty: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    try:
        L = np.linalg.cholesky(XtX)
        beta_full = np.linalg.solve(L.T, np.linalg.solve(L, Xty))
        XtX_inv = np.linalg.solve(L.T, np.linalg.solve(L, np.eye(L.shape[0])))
    except np.linalg.LinAlgError:
        beta_full = np.linalg.solve(XtX, Xty)
        XtX_inv = np.linalg.inv(XtX)
    return beta_full, XtX_inv


def split_gram(G: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """Gram of [1, y, x_1..x_k] -> (X'X, X'y) of X = [1, x_1..x_k]."""
    idx = [0] + list(range(2, G.shape[0]))
    return G[np.ix_(idx, idx)].copy(), G[idx, 1].copy()


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

"""``leanfe()`` entry point (reference: python/leanfe/leanfe.py:14-184) with the
MI355X backend.

The reference dispatches on ``backend`` ("polars" | "duckdb", else
ValueError, leanfe.py:138-184).  This package adds ``backend="hip"`` and makes
it the default.  The reference's CPU backends are not part of this package:
asking for them raises ``ValueError`` naming the available backend (install
the reference ``leanfe`` package for them).
"""
from __future__ import annotations

from .hip_impl import leanfe_hip
from .result import LeanFEResult

BACKENDS = ("hip",)


def leanfe(data=None, y_col: str | None = None, x_cols: list[str] | None = None, fe_cols: list[str] = [],
           formula: str | None = None, strategy: str = "auto", weights: str | None = None,
           demean_tol: float = 1e-6, max_iter: int = 50, vcov: str = "iid",
           cluster_cols: list[str] | None = None, ssc: bool = True, sample_frac: float | None = None,
           backend: str = "hip", con=None, device: int | None = None) -> LeanFEResult:
    """Fast fixed-effects regression; same arguments and result as the
    reference ``leanfe()`` plus ``backend="hip"`` (default) and ``device``."""
    if backend == "hip":
        if data is None:
            raise ValueError(f"A dataset must be provided when using backend = {backend}.")
        return leanfe_hip(data=data, y_col=y_col, x_cols=x_cols, fe_cols=fe_cols, formula=formula,
                          strategy=strategy, weights=weights, demean_tol=demean_tol, max_iter=max_iter,
                          vcov=vcov, cluster_cols=cluster_cols, ssc=ssc, sample_frac=sample_frac,
                          device=device)
    if backend in ("polars", "duckdb"):
        raise ValueError(f"backend '{backend}' is the reference leanfe's CPU backend and is not part of "
                         "leanfe_amd; use backend='hip'")
    raise ValueError(f"backend must be 'hip', got '{backend}'")

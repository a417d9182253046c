"""Strategy selection, restating python/leanfe/compress.py:96-184
(``determine_strategy``) and :187-253 (``estimate_compression_ratio``).

The HIP backend implements every strategy the cost model can pick: ``alt_proj``,
``demean``, ``ols`` and ``compress`` (YOCO records grouped on the device,
``lfe_compress``; ``hip_impl._compress_fit``).  A row-sharded engine maps an
inferred ``compress`` to ``alt_proj``: YOCO groups one process's rows.

``estimate_compression_ratio`` is the host restatement of the reference's
count; the product takes the exact count from the device
(``lfe_count_distinct_rows``) and the tests use this one as its checker.
"""
from __future__ import annotations

import numpy as np

DEFAULT_MAX_FE_LEVELS = 10_000
DEFAULT_DEMEANING_ITERATIONS = 10
SPARSE_MATRIX_COST_FACTOR = 1.0
GROUP_BY_COST_FACTOR = 1.0
WLS_SOLVE_COST_EXPONENT = 2
COMPRESSION_RATIO_MAX_ROWS = 5_000_000  # above this the exact unique-row count is skipped (None)


def determine_strategy(vcov: str, has_instruments: bool, fe_cardinality: dict[str, int] | None = None,
                       max_fe_levels: int = DEFAULT_MAX_FE_LEVELS, n_obs: int | None = None,
                       n_x_cols: int | None = None, estimated_compression_ratio: float | None = None) -> str:
    if has_instruments:
        return "alt_proj"
    if vcov.lower() not in ("iid", "hc1", "cluster"):
        return "alt_proj"
    if fe_cardinality is None:
        return "compress"
    total = sum(fe_cardinality.values())
    biggest = max(fe_cardinality.values()) if fe_cardinality else 0
    if biggest > max_fe_levels:          # compress.py:156-157
        return "alt_proj"
    if total > max_fe_levels * 2:        # compress.py:161-162
        return "alt_proj"
    if estimated_compression_ratio is not None and n_obs is not None:
        n_compressed = int(n_obs * estimated_compression_ratio)
        yoco = (GROUP_BY_COST_FACTOR * n_obs + SPARSE_MATRIX_COST_FACTOR * n_compressed * total
                + total ** WLS_SOLVE_COST_EXPONENT)
        fwl = DEFAULT_DEMEANING_ITERATIONS * len(fe_cardinality) * n_obs
        return "compress" if yoco < fwl else "alt_proj"
    return "compress"


def _mix64(h: np.ndarray, v: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        h = (h ^ v) * np.uint64(0x100000001B3)
        h ^= h >> np.uint64(29)
        return h * np.uint64(0xBF58476D1CE4E5B9)


def estimate_compression_ratio(columns: list[np.ndarray]) -> float | None:
    """Unique rows over (x, FE) columns / n (compress.py:187-253), on the host.
    The hip backend counts exactly on the device (``Engine.count_distinct_rows``);
    this restatement is kept for host-only callers and as a test reference.  Exact
    (``np.unique`` over stacked rows) for small n; for n up to
    COMPRESSION_RATIO_MAX_ROWS a 64-bit row hash stands in for the row (a
    collision only lowers the estimate by a negligible amount); above that the
    estimate is skipped and None is returned."""
    if not columns:
        return 1.0
    n = columns[0].size
    if n == 0:
        return 1.0
    if n <= 200_000:
        arr = np.stack([np.asarray(c, dtype=np.float64) for c in columns], axis=1)
        return np.unique(arr, axis=0).shape[0] / n
    if n > COMPRESSION_RATIO_MAX_ROWS:
        return None
    h = np.full(n, 0xCBF29CE484222325, dtype=np.uint64)
    for c in columns:
        v = np.ascontiguousarray(np.asarray(c, dtype=np.float64)).view(np.uint64)
        h = _mix64(h, v)
    return np.unique(h).size / n

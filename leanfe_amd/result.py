"""Regression result object, API-compatible with the reference's ``LeanFEResult``
(python/leanfe/result.py:11-295): same attributes, accessors, dict-like view,
t-statistics and two-sided p-values from Student's t with ``df_resid`` degrees
of freedom (result.py:91-102), and the same printed table layout."""
from __future__ import annotations

from typing import Any

import numpy as np
from scipy import stats


class PrettyInt(int):
    """An integer that displays with underscores in its representation."""

    def __repr__(self) -> str:
        return f"{self:_}"


def wrap_int(val: Any) -> PrettyInt | None:
    return PrettyInt(val) if val is not None else None


class LeanFEResult:
    def __init__(self, coefs: dict[str, float], std_errors: dict[str, float], n_obs: int, vcov_type: str,
                 iterations: int = 0, n_compressed: int | None = None, compression_ratio: float | None = None,
                 is_iv: bool = False, n_instruments: int | None = None,
                 n_clusters: int | tuple[int, ...] | None = None, df_resid: int | None = None,
                 r_squared: float | None = None, r_squared_within: float | None = None,
                 rss: float | None = None, tss: float | None = None, formula: str | None = None,
                 fe_cols: list[str] | dict[str, Any] | None = None, fe_dims: tuple[int, ...] | None = None,
                 backend: str = "hip", timings: dict | None = None):
        self.coefs = coefs
        self.std_errors = std_errors
        self.n_obs = n_obs
        self.iterations = iterations
        self.n_compressed = n_compressed
        self.compression_ratio = compression_ratio
        self.vcov_type = vcov_type
        self.is_iv = is_iv
        self.n_instruments = n_instruments
        self.n_clusters = n_clusters
        self.df_resid = df_resid or (n_obs - len(coefs))
        self.r_squared = r_squared
        self.r_squared_within = r_squared_within
        self.rss = rss
        self.tss = tss
        self.formula = formula
        self.fe_cols = fe_cols or []
        self.fe_dims = fe_dims
        self.backend = backend
        self.timings = timings or {}
        self.t_stats: dict[str, float] = {}
        self.p_values: dict[str, float] = {}
        for var in coefs:
            if std_errors[var] > 0:
                t = coefs[var] / std_errors[var]
                self.t_stats[var] = t
                self.p_values[var] = 2 * (1 - stats.t.cdf(abs(t), self.df_resid))
            else:
                self.t_stats[var] = np.nan
                self.p_values[var] = np.nan

    @staticmethod
    def _significance_stars(p: float) -> str:
        if p < 0.001:
            return "***"
        if p < 0.01:
            return "**"
        if p < 0.05:
            return "*"
        if p < 0.1:
            return "."
        return ""

    def summary(self) -> str:
        return str(self)

    def __repr__(self) -> str:
        return f"LeanFEResult(n_obs={self.n_obs:_}, n_coef={len(self.coefs)}, vcov='{self.vcov_type}')"

    def __str__(self) -> str:
        bar = "=" * 70
        lines = ["", bar, "                         leanfe Regression Results", bar]
        if self.formula:
            lines.append(f"Formula:      {self.formula}")
            lines.append(f"Observations: {self.n_obs:_}")
        if self.fe_cols:
            if isinstance(self.fe_cols, list):
                lines.append(f"Fixed Effects: {', '.join(self.fe_cols)}")
                if self.fe_dims:
                    lines.append("FE Dimensions: " + " × ".join(f"{d:_}" for d in self.fe_dims))
            elif isinstance(self.fe_cols, dict):
                for fe, count in self.fe_cols.items():
                    lines.append(f"Fixed Effect ({fe}): {count:_} groups")
        if self.r_squared_within is not None:
            lines.append(f"R² (within):  {self.r_squared_within:.4f}")
        lines.append(f"Std. Errors:  {self._vcov_description()}")
        if self.n_clusters:
            if isinstance(self.n_clusters, tuple):
                lines.append("Clusters:     " + " × ".join(f"{c:_}" for c in self.n_clusters))
            else:
                lines.append(f"Clusters:     {self.n_clusters:_}")
        lines.append("-" * 70)
        lines.append(f"{'Variable':<20} {'Estimate':>12} {'Std.Err':>12} {'t-stat':>10} {'p-value':>10}")
        lines.append("-" * 70)
        for var in self.coefs:
            coef, se = self.coefs[var], self.std_errors[var]
            t, p = self.t_stats[var], self.p_values[var]
            name = var[:18] + ".." if len(var) > 20 else var
            lines.append(f"{name:<20} {coef:>12.6f} {se:>12.6f} {t:>10.3f} {p:>9.4f}"
                         f"{self._significance_stars(p)}")
        lines += ["-" * 70, "Signif. codes: 0 '***' 0.001 '**' 0.01 '*' 0.05 '.' 0.1", bar, ""]
        return "\n".join(lines)

    def _vcov_description(self) -> str:
        if self.vcov_type == "iid":
            return "IID"
        if self.vcov_type == "HC1":
            return "Heteroskedasticity-robust (HC1)"
        if self.vcov_type == "cluster":
            nc = self.n_clusters
            if isinstance(nc, tuple):
                return "Clustered (" + " × ".join(f"{c:,}" for c in nc) + " clusters)"
            return f"Clustered ({nc:,} clusters)"
        return self.vcov_type

    def coef(self, var: str | None = None):
        return self.coefs.copy() if var is None else self.coefs.get(var)

    def se(self, var: str | None = None):
        return self.std_errors.copy() if var is None else self.std_errors.get(var)

    def tstat(self, var: str | None = None):
        return self.t_stats.copy() if var is None else self.t_stats.get(var)

    def pvalue(self, var: str | None = None):
        return self.p_values.copy() if var is None else self.p_values.get(var)

    def confint(self, level: float = 0.95) -> dict[str, tuple]:
        t_crit = stats.t.ppf(1 - (1 - level) / 2, self.df_resid)
        return {v: (self.coefs[v] - t_crit * self.std_errors[v], self.coefs[v] + t_crit * self.std_errors[v])
                for v in self.coefs}

    def to_dict(self) -> dict:
        return {
            "formula": self.formula,
            "coefs": self.coefs,
            "std_errors": self.std_errors,
            "t_stats": self.t_stats,
            "p_values": self.p_values,
            "n_obs": wrap_int(self.n_obs),
            "n_compressed": wrap_int(self.n_compressed),
            "compression_ratio": self.compression_ratio,
            "fe_cols": self.fe_cols,
            "fe_dims": self.fe_dims,
            "iterations": self.iterations,
            "vcov_type": self.vcov_type,
            "is_iv": self.is_iv,
            "n_instruments": self.n_instruments,
            "n_clusters": self.n_clusters,
            "df_resid": wrap_int(self.df_resid),
            "r_squared_within": self.r_squared_within,
        }

    def __getitem__(self, key):
        return self.to_dict()[key]

    def get(self, key, default=None):
        return self.to_dict().get(key, default)

    def keys(self):
        return self.to_dict().keys()

    def values(self):
        return self.to_dict().values()

    def items(self):
        return self.to_dict().items()

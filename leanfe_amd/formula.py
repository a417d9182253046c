"""Formula grammar of leanfe (reference: python/leanfe/common.py:51-181).

    y ~ x1 + x2 + i(region, ref=R1) + treat:i(region) | fe1 + fe2 | z1 + z2

Parts: response ~ regressors | fixed effects | instruments.  Regressors may be
plain columns, factor terms ``i(var[, ref=value])`` or interactions
``var:i(factor[, ref=value])``.  Same outputs and error types as the
reference's ``parse_formula``.
"""
from __future__ import annotations

import re
from typing import NamedTuple


class FormulaComponents(NamedTuple):
    y_col: str
    x_cols: list[str]
    fe_cols: list[str]
    factor_vars: list[tuple[str, str | None]]
    interactions: list[tuple[str, str, str | None]]
    instruments: list[str]


_REF = r"(?:\s*,\s*ref\s*=\s*[\"']?([^\"')\s]+)[\"']?)?"
_FACTOR = re.compile(r"i\((\w+)" + _REF + r"\)")
_INTERACT = re.compile(r"(\w+):i\((\w+)" + _REF + r"\)")


def _split_terms(s: str) -> list[str]:
    return [t.strip() for t in s.split("+") if t.strip() != ""]


def parse_formula(formula: str) -> FormulaComponents:
    parts = [p.strip() for p in formula.split("|")]
    if len(parts) > 3:
        raise ValueError("Formula has too many parts. Use: 'y ~ x' or 'y ~ x | fe' or 'y ~ x | fe | z' (IV)")
    lhs_rhs = parts[0].split("~")
    if len(lhs_rhs) != 2:
        raise ValueError("Formula must have exactly one '~' separating y and x variables")
    y_col = lhs_rhs[0].strip()
    x_cols: list[str] = []
    factor_vars: list[tuple[str, str | None]] = []
    interactions: list[tuple[str, str, str | None]] = []
    for term in _split_terms(lhs_rhs[1]):
        if ":i(" in term and term.endswith(")"):
            m = _INTERACT.match(term)
            if not m:
                raise ValueError(f"Invalid interaction syntax: {term}")
            interactions.append((m.group(1), m.group(2), m.group(3)))
        elif term.startswith("i(") and term.endswith(")"):
            m = _FACTOR.match(term)
            if not m:
                raise ValueError(f"Invalid i() syntax: {term}. Use i(var) or i(var, ref=value)")
            factor_vars.append((m.group(1), m.group(2)))
        else:
            x_cols.append(term)
    fe_cols = _split_terms(parts[1]) if len(parts) >= 2 and parts[1].strip() else []
    instruments = _split_terms(parts[2]) if len(parts) == 3 and parts[2].strip() else []
    return FormulaComponents(y_col, x_cols, fe_cols, factor_vars, interactions, instruments)

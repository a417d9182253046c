"""The i8 digit cross terms at their numeric edges (parity of the default headline path).

The dense passes (lfe_dense.hip for two FEs, the pair tables of lfe_dense3.hip for three) cut every
512-level tile of effects, per column, into 8 base-128 digits of round(alpha * 2^(54 - e)) with
2^e > the tile's largest |alpha|.  Every other effect of the tile is then rounded to 2^-54 of that
largest one, so a single huge effect coarsens its tile's neighbours by the same absolute amount.
The dynamic-range guard (dn8_tile_digits, kDn8RangeBits = 16) flags a tile column where more than a
quarter of the nonzero effects lie 2^16 below the largest; lfe_demean then redoes the solve without
the dense cross terms, so the result is the row passes' (LFE_DENSE=0) bit for bit.

Panels (forced onto the dense path with LFE_DENSE=1):
- guard fires: one FE level whose effect on y is 1e8 x the others' (primary and secondary FE), a
  regressor with one 5e9 outlier (its group's effect dwarfs the tile);
- guard stays off: a level with a 1e3 effect (2^10: the digits keep 44 bits of the others), a
  heavy-tailed regressor (Student t, 1 dof: |x| up to ~1e6), a NaN in one regressor (that column's
  tiles go NaN and spread as in the f64 sums; the other columns stay exact).
Every case: the CPU oracle (oracle/altproj.py, the reference loop polars_impl.py:490-526) at 1e-10
with equal `iterations` and bit-identical repeats; where the guard fires, bit-identity with the row
passes; where it does not, the f64-MFMA passes (LFE_DN8=0, two FEs) or the row sweeps (LFE_DENSE=0,
three FEs) at 1e-12."""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GUARDED = ["effect_primary", "effect_secondary", "x_outlier"]
CASES = GUARDED + ["effect_moderate", "heavy_tail", "nan_x"]


def _panel(case, n, levels, k, seed):
    from leanfe_amd import synth

    data = dict(synth.panel(n, k, levels, seed=seed))
    if case == "effect_primary":
        y = np.array(data["y"], copy=True)
        y[np.asarray(data["fe1"]) == 17] += 1e8
        data["y"] = y
    elif case == "effect_moderate":
        y = np.array(data["y"], copy=True)
        y[np.asarray(data["fe2"]) == 17] += 1e3
        data["y"] = y
    elif case == "effect_secondary":
        y = np.array(data["y"], copy=True)
        y[np.asarray(data["fe2"]) == 17] += 1e8
        data["y"] = y
    elif case == "x_outlier":
        x = np.array(data["x2"], copy=True)
        x[4321] = 5e9
        data["x2"] = x
    elif case == "heavy_tail":
        data["x1"] = np.random.default_rng(seed + 1).standard_t(1.0, size=n)
    elif case == "nan_x":
        x = np.array(data["x2"], copy=True)
        x[4321] = np.nan
        data["x2"] = x
    return data


def _fit(data, xs, fes, eng, vcov="HC1"):
    from leanfe_amd import leanfe_hip

    r = leanfe_hip(data, y_col="y", x_cols=xs, fe_cols=fes, strategy="alt_proj", vcov=vcov, quiet=True, engine=eng)
    return dict(beta=np.array([r.coefs[x] for x in xs]), se=np.array([r.std_errors[x] for x in xs]),
                iterations=r.iterations, n_obs=r.n_obs, cells=eng.dense_cells(), bytes=eng.dense_cell_bytes())


def _check(res, o, rtol=1e-10):
    assert res["iterations"] == o["iterations"] and res["n_obs"] == o["n_obs"], (res["iterations"], o["iterations"])
    np.testing.assert_array_equal(np.isnan(res["beta"]), np.isnan(o["beta"]))
    np.testing.assert_allclose(res["beta"], o["beta"], rtol=rtol, atol=0)
    np.testing.assert_allclose(res["se"], o["se"], rtol=rtol, atol=0)


def _close(a, b, rtol):
    assert a["iterations"] == b["iterations"]
    np.testing.assert_allclose(a["beta"], b["beta"], rtol=rtol, atol=0)
    np.testing.assert_allclose(a["se"], b["se"], rtol=rtol, atol=0)


def _same(a, b):
    assert a["iterations"] == b["iterations"]
    np.testing.assert_array_equal(a["beta"], b["beta"])
    np.testing.assert_array_equal(a["se"], b["se"])


def _demeaned_columns_match(data, cols_names, fes, levels):
    """The demeaned columns of the dense path against the oracle's (NaN exactly where the oracle's
    are; every finite column at the oracle's values)."""
    from leanfe_amd._lib import Engine
    from oracle import altproj

    cols = [np.asarray(data[c], dtype=np.float64) for c in cols_names]
    codes = [np.ascontiguousarray(data[f], dtype=np.int32) for f in fes]
    with Engine(0) as eng:
        eng.load(cols, codes, list(levels))
        n_obs, _, card = eng.drop_singletons()
        order = sorted(range(len(fes)), key=lambda i: card[i])
        it, _ = eng.demean(order, 1e-8, 100, check_from=3)
        assert eng.dense_cells() > 0
        out = eng.copy_demeaned()
    keep = altproj.singleton_keep(codes, list(levels))
    dm, it_ref = altproj.demean_altproj(np.array(cols)[:, keep], [c[keep] for c in codes], list(levels), order, 1e-8,
                                        100)
    assert it == it_ref
    got = out[:, keep]
    np.testing.assert_array_equal(np.isnan(got), np.isnan(dm))
    np.testing.assert_allclose(got, dm, rtol=1e-9, atol=1e-11)


@pytest.mark.parametrize("case", CASES)
def test_two_fe_digits_at_numeric_edges(case, knob):
    from leanfe_amd._lib import Engine
    from oracle import altproj

    k, levels = 4, [3_000, 600]  # 900K rows: 0.5 rows per cell, the headline's density
    xs = [f"x{j + 1}" for j in range(k)]
    fes = ["fe1", "fe2"]
    data = _panel(case, 900_000, levels, k, seed=606)
    o = altproj.fit(data, "y", xs, fes, vcov="HC1")
    knob.setenv("LFE_DENSE", "1")
    with Engine(0) as eng:
        i8 = _fit(data, xs, fes, eng)
        again = _fit(data, xs, fes, eng)
        knob.setenv("LFE_DN8", "0")
        f64 = _fit(data, xs, fes, eng)
        assert f64["cells"] > 0 and f64["bytes"] == 2  # the f64 passes have no guard
        knob.delenv("LFE_DN8")
        knob.setenv("LFE_DENSE", "0")
        rows = _fit(data, xs, fes, eng)
    _check(i8, o)
    _check(f64, o)
    _same(i8, again)
    if case in GUARDED:
        assert i8["cells"] == 0  # the guard fired: the solve was redone on the row layouts
        _same(i8, rows)
    else:
        assert i8["cells"] > 0 and i8["bytes"] == 1  # the exact i8 passes ran
        _close(i8, f64, 1e-12)
    if case == "nan_x":
        knob.setenv("LFE_DENSE", "1")
        _demeaned_columns_match(data, ["y"] + xs, fes, levels)


@pytest.mark.parametrize("case", CASES)
def test_pair_table_digits_at_numeric_edges(case, knob):
    from leanfe_amd._lib import Engine
    from oracle import altproj

    k, levels = 4, [3_000, 800, 200]
    xs = [f"x{j + 1}" for j in range(k)]
    fes = ["fe1", "fe2", "fe3"]
    data = _panel(case, 1_200_000, levels, k, seed=707)
    o = altproj.fit(data, "y", xs, fes, vcov="HC1")
    knob.setenv("LFE_DENSE", "1")
    with Engine(0) as eng:
        dense = _fit(data, xs, fes, eng)
        again = _fit(data, xs, fes, eng)
        knob.setenv("LFE_DENSE", "0")
        rows = _fit(data, xs, fes, eng)
        assert rows["cells"] == 0
    _check(dense, o)
    _check(rows, o)
    _same(dense, again)
    # with three FEs the first projected FE absorbs a uniform shift of a large level effect (the
    # other effects of the big level's tile then sit ~1e3 below it, not 2^16: no guard needed); a
    # single 5e9 value lands in one level of the first FE and trips it
    if case == "x_outlier":
        assert dense["cells"] == 0
    elif case not in GUARDED:
        assert dense["cells"] > 0
    if dense["cells"] == 0:
        _same(dense, rows)
    elif case.startswith("effect"):
        # a 1e8 level effect puts y ~ 1e8 on its rows: every f64 path rounds their residuals at
        # ulp(1e8) ~ 1.5e-8, so the RSS (and the SE) of any two f64 evaluations differ by ~1e-12
        _close(dense, rows, 5e-12)
    else:
        _close(dense, rows, 1e-12)
    if case == "nan_x":
        knob.setenv("LFE_DENSE", "1")
        _demeaned_columns_match(data, ["y"] + xs, fes, levels)


def test_tiny_effects_digitize_exactly(knob):
    """A column whose effects all lie near 1e-300 (below 2^-969, where the digit scale 2^(54 - e)
    alone overflows to inf and 0 * inf made NaN digits): the scale goes in two exact
    power-of-two factors, so the tiny column demeans as the oracle does (compared after scaling
    back by 1e300), beside ordinary columns."""
    from leanfe_amd._lib import Engine
    from oracle import altproj

    levels = [3_000, 600]
    fes = ["fe1", "fe2"]
    data = _panel("none", 900_000, levels, 2, seed=808)
    cols = [np.asarray(data["y"]) * 1e-300, np.asarray(data["x1"]), np.asarray(data["x2"]) * 1e-310]
    codes = [np.ascontiguousarray(data[f], dtype=np.int32) for f in fes]
    knob.setenv("LFE_DENSE", "1")
    with Engine(0) as eng:
        eng.load(cols, codes, levels)
        _, _, card = eng.drop_singletons()
        order = sorted(range(2), key=lambda i: card[i])
        it, _ = eng.demean(order, 0.0, 12, check_from=3)  # no stop: the same 12 sweeps
        assert eng.dense_cells() > 0 and eng.dense_cell_bytes() == 1
        out = eng.copy_demeaned()
    keep = altproj.singleton_keep(codes, levels)
    dm, it_ref = altproj.demean_altproj(np.array(cols)[:, keep], [c[keep] for c in codes], levels, order, 0.0, 12)
    assert it == it_ref == 12
    got = out[:, keep]
    assert np.all(np.isfinite(got))
    np.testing.assert_allclose(got[0] * 1e300, dm[0] * 1e300, rtol=1e-9, atol=1e-11)
    np.testing.assert_allclose(got[1], dm[1], rtol=1e-9, atol=1e-11)
    # x2 * 1e-310 is subnormal: its values carry ~1e-14 relative precision at best in either path
    np.testing.assert_allclose(got[2] * 1e310, dm[2] * 1e310, rtol=0, atol=1e-6)

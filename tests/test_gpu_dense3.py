"""Pair-table sweeps for three or more FEs (leanfe_amd/csrc/lfe_dense3.hip).

Every cross term of the projection loop (polars_impl.py:490-526) for F >= 3 as products of the
pair count tables N_ab (i8 fragments x base-128 digits of the effects on the matrix cores), where
the tables are small against the rows; otherwise the general sweeps of lfe_seg.hip gather row by
row.  Both restate the same loop, so:
- the pair-table path matches the CPU oracle (oracle/altproj.py) at 1e-10 with equal `iterations`
  and agrees with the row path (LFE_DENSE=0) to rounding;
- it repeats bit for bit;
- p > 16 (two column groups per table), four FEs, singletons and ragged level counts, cells of more
  than 127 rows (flagged blocks, u16 counts) and of more than 255 (the 16-bit recount) all match;
- the Gram from the group tables (raw Gram of the shifted columns + per-group terms, no effect
  gathers) agrees with the design pass (LFE_TAB3=0), and a panel whose FE effects dwarf the
  residual variation trips its cancellation guard and falls back to the design pass.
LFE_DENSE=1 forces the pair tables wherever they fit, LFE_DENSE=0 turns them off."""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _fit(data, xs, fes, vcov="HC1", cl=None):
    from leanfe_amd import leanfe_hip

    kw = dict(cluster_cols=cl) if cl else {}
    r = leanfe_hip(data, y_col="y", x_cols=xs, fe_cols=fes, strategy="alt_proj", vcov=vcov, quiet=True, device=0,
                   **kw)
    return (np.array([r.coefs[x] for x in xs]), np.array([r.std_errors[x] for x in xs]), r.iterations, r.n_obs,
            r.df_resid)


def _oracle(data, xs, fes, vcov="HC1", cl=None):
    from oracle import altproj

    return altproj.fit(data, "y", xs, fes, vcov=vcov, cluster_cols=cl)


def _check(res, o, rtol=1e-10):
    b, s, it, n_obs, df = res
    assert it == o["iterations"] and n_obs == o["n_obs"] and df == o["df_resid"], (it, o["iterations"])
    np.testing.assert_allclose(b, o["beta"], rtol=rtol, atol=0)
    np.testing.assert_allclose(s, o["se"], rtol=rtol, atol=0)


def _dense_cells(data, xs, fes):
    """cells of the last demean's dense tables on a fresh engine (0: the row sweeps ran)"""
    from leanfe_amd._lib import Engine

    cols = [np.asarray(data["y"], dtype=np.float64)] + [np.asarray(data[x], dtype=np.float64) for x in xs]
    codes = [np.ascontiguousarray(data[f], dtype=np.int32) for f in fes]
    levels = [int(c.max()) + 1 for c in codes]
    with Engine(0) as eng:
        eng.load(cols, codes, levels)
        eng.drop_singletons()
        eng.demean(list(range(len(fes))), tol=1e-8, max_iter=100)
        return eng.dense_cells()


@pytest.mark.parametrize("vcov", ["HC1", "iid"])
def test_pair_tables_match_oracle_and_row_sweeps(vcov, knob):
    from leanfe_amd import synth

    k = 5
    xs = [f"x{j + 1}" for j in range(k)]
    fes = ["fe1", "fe2", "fe3"]
    data = synth.panel(1_500_000, k, [3_000, 800, 200], seed=303)
    o = _oracle(data, xs, fes, vcov)
    knob.setenv("LFE_DENSE", "0")
    rows = _fit(data, xs, fes, vcov)
    knob.delenv("LFE_DENSE")
    dense = _fit(data, xs, fes, vcov)
    _check(rows, o)
    _check(dense, o)
    np.testing.assert_allclose(dense[0], rows[0], rtol=1e-11, atol=0)
    np.testing.assert_allclose(dense[1], rows[1], rtol=1e-11, atol=0)
    again = _fit(data, xs, fes, vcov)
    np.testing.assert_array_equal(dense[0], again[0])
    np.testing.assert_array_equal(dense[1], again[1])


def test_pair_tables_wide_four_fes_singletons_ragged(knob):
    """k = 20 (p = 21: two 16-column groups per table), four FEs with level counts off every 64 /
    512 boundary, 30 singleton levels dropped before the tables are built, one-way clustered SEs."""
    from leanfe_amd import synth

    k = 20
    xs = [f"x{j + 1}" for j in range(k)]
    fes = ["fe1", "fe2", "fe3", "fe4"]
    data = synth.panel(600_000, k, [2_777, 613, 97, 33], seed=9)
    fe1 = np.array(data["fe1"], copy=True)
    fe1[:30] = np.arange(30) + 2_777
    data = dict(data, fe1=fe1)
    knob.setenv("LFE_DENSE", "1")
    _check(_fit(data, xs, fes, "cluster", ["fe3"]), _oracle(data, xs, fes, "cluster", ["fe3"]))


def test_pair_tables_heavy_cells(knob):
    """Cells with 128-400 rows (flagged 16 x 64 blocks, their u16 counts summed in f64) and one
    with ~40K rows (its 64-level chunk counted again on 16-bit counters), in every orientation."""
    rng = np.random.default_rng(21)
    n, k = 500_000, 3
    G = [1_500, 300, 40]
    f1 = rng.integers(0, G[0], n).astype(np.int32)
    f2 = rng.integers(0, G[1], n).astype(np.int32)
    f3 = rng.integers(0, G[2], n).astype(np.int32)
    i0 = 0
    for a, b, c3, m in [(17, 5, 3, 130), (900, 299, 39, 400), (1_499, 0, 0, 200), (64, 64, 7, 40_000)]:
        f1[i0:i0 + m], f2[i0:i0 + m], f3[i0:i0 + m] = a, b, c3
        i0 += m
    x = rng.standard_normal((n, k))
    y = (x @ np.array([1.0, -0.5, 0.25]) + rng.standard_normal(G[0])[f1] + rng.standard_normal(G[1])[f2]
         + rng.standard_normal(G[2])[f3] + rng.standard_normal(n))
    data = {"y": y, "fe1": f1, "fe2": f2, "fe3": f3, **{f"x{j + 1}": x[:, j].copy() for j in range(k)}}
    xs = ["x1", "x2", "x3"]
    fes = ["fe1", "fe2", "fe3"]
    o = _oracle(data, xs, fes)
    knob.setenv("LFE_DENSE", "1")
    dense = _fit(data, xs, fes)
    _check(dense, o)
    knob.setenv("LFE_DENSE", "0")
    rows = _fit(data, xs, fes)
    np.testing.assert_allclose(dense[0], rows[0], rtol=1e-12, atol=0)


def test_pair_tables_taken_where_expected(monkeypatch):
    """The default takes the pair tables for the reference's 3-FE panel shape (tables ~2 bytes per
    row) and the row sweeps where the tables would outweigh the rows."""
    from leanfe_amd import synth

    xs = ["x1", "x2"]
    fes = ["fe1", "fe2", "fe3"]
    small = synth.panel(400_000, 2, [2_000, 400, 100], seed=1)
    assert _dense_cells(small, xs, fes) > 0
    sparse = synth.panel(200_000, 2, [20_000, 4_000, 100], seed=1)
    assert _dense_cells(sparse, xs, fes) == 0


@pytest.mark.parametrize("vcov", ["iid", "HC1"])
def test_tables_gram_matches_design_pass(vcov, knob):
    from leanfe_amd import synth

    k = 14
    xs = [f"x{j + 1}" for j in range(k)]
    fes = ["fe1", "fe2", "fe3"]
    data = synth.panel(800_000, k, [2_000, 400, 100], seed=41)
    o = _oracle(data, xs, fes, vcov)
    tab = _fit(data, xs, fes, vcov)
    knob.setenv("LFE_TAB3", "0")
    design = _fit(data, xs, fes, vcov)
    _check(tab, o)
    _check(design, o)
    np.testing.assert_allclose(tab[0], design[0], rtol=1e-11, atol=0)
    np.testing.assert_allclose(tab[1], design[1], rtol=1e-11, atol=0)


def test_tables_gram_guard_falls_back():
    """y and x1 carry FE effects 1e7 times their within variation: the assembled diagonal keeps
    ~1e-14 of the raw one, the guard trips and the design pass gives the oracle's answer."""
    rng = np.random.default_rng(3)
    n, k = 300_000, 2
    G = [1_000, 200, 50]
    codes = [rng.integers(0, g, n).astype(np.int32) for g in G]
    big = sum(1e7 * rng.standard_normal(g)[c] for g, c in zip(G, codes))
    x1 = big + rng.standard_normal(n)
    x2 = rng.standard_normal(n)
    y = 0.5 * x1 - x2 + 2 * big + rng.standard_normal(n)
    data = {"y": y, "x1": x1, "x2": x2, "fe1": codes[0], "fe2": codes[1], "fe3": codes[2]}
    xs, fes = ["x1", "x2"], ["fe1", "fe2", "fe3"]
    _check(_fit(data, xs, fes), _oracle(data, xs, fes), rtol=1e-8)

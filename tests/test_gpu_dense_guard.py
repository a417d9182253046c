"""The i8 digits' dynamic-range guard pinned just below its threshold.

dn8_tile_digits (lfe_dense.hip) flags a 512-level tile column when more than a quarter of its nonzero
effects lie below 2^-16 of the tile's largest; then the solve is redone on the row passes.  Below that
share the exact i8 passes run, and those small effects keep only 54 - 16 = 38 bits (an f64 sum keeps
53 of each).  These panels put 15-24 % of every tile's effects below 2^-16 of its largest - the guard
stays silent - with a heavy-tailed level effect of log-normal(sigma = 3) shape at scale 1e6:

- two FEs: on y through the primary FE (every (firm, worker) cell holds one row, so the estimated
  primary effects are the generated ones up to the sampling noise of y, ~0.1, far below the 2^-16
  threshold of 15), and on x1 through the secondary FE;
- three FEs (pair tables): on y and on x1 through the first-projected FE.

Every case: the CPU oracle (oracle/altproj.py, polars_impl.py:490-526) at 1e-10 with equal
`iterations`, the exact i8 passes taken (cells > 0, 1 byte a cell), bit-identical repeats, and the
f64-MFMA passes (LFE_DN8=0, two FEs) or the row sweeps (LFE_DENSE=0, three FEs) at 1e-12."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

THRESH = 2.0 ** -16  # kDn8RangeBits = 16
BANDS = [(0.15, 0.17), (0.22, 0.24)]


def lognormal_effect(G, M, seed, lo, hi, tile=512):
    """G level effects of log-normal(sigma = 3) magnitude, random signs, the largest |effect| M, with a
    share in [lo, hi] of every 512-level tile below 2^-16 of the tile's largest and none within 4x of
    that line (the estimates then fall on the same side as the generated values)."""
    rng = np.random.default_rng(seed)
    a = np.exp(3.0 * rng.standard_normal(G)) * rng.choice([-1.0, 1.0], G)
    a *= M / np.abs(a).max()
    for t0 in range(0, G, tile):
        v = a[t0:t0 + tile]
        top = np.abs(v).argmax()
        thr = np.abs(v[top]) * THRESH
        near = (np.abs(v) > thr / 4) & (np.abs(v) < thr * 4)
        v[near & (np.abs(v) < thr)] /= 8
        v[near & (np.abs(v) >= thr)] *= 8
        want = int(round((lo + hi) / 2 * v.size))
        small = np.flatnonzero(np.abs(v) < thr)
        big = np.flatnonzero((np.abs(v) >= thr) & (np.arange(v.size) != top))
        if small.size > want:  # lift some small ones well above the line
            sel = rng.permutation(small)[:small.size - want]
            v[sel] = np.sign(v[sel]) * thr * rng.uniform(8, 1000, sel.size)
        elif small.size < want:  # and sink some large ones well below it
            sel = rng.permutation(big)[:want - small.size]
            v[sel] = np.sign(v[sel]) * thr * rng.uniform(1e-3, 1 / 8, sel.size)
        share = (np.abs(v) < thr).mean()
        assert lo <= share <= hi, share
    return a


def zero_sum(a):
    """Shift the sum onto the 16 largest effects (in proportion): the first-projected FE then
    absorbs no constant that would lift the small effects off zero."""
    top = np.argsort(-np.abs(a))[:16]
    w = np.abs(a[top])
    a[top] -= a.sum() * w / w.sum()
    return a


def _fit(data, xs, fes, eng):
    from leanfe_amd import leanfe_hip

    r = leanfe_hip(data, y_col="y", x_cols=xs, fe_cols=fes, strategy="alt_proj", vcov="HC1", quiet=True, engine=eng)
    return dict(beta=np.array([r.coefs[x] for x in xs]), se=np.array([r.std_errors[x] for x in xs]),
                iterations=r.iterations, n_obs=r.n_obs, cells=eng.dense_cells(), bytes=eng.dense_cell_bytes())


def _check(res, o, rtol=1e-10):
    assert res["iterations"] == o["iterations"] and res["n_obs"] == o["n_obs"]
    np.testing.assert_allclose(res["beta"], o["beta"], rtol=rtol, atol=0)
    np.testing.assert_allclose(res["se"], o["se"], rtol=rtol, atol=0)


def _close(a, b, rtol):
    assert a["iterations"] == b["iterations"]
    np.testing.assert_allclose(a["beta"], b["beta"], rtol=rtol, atol=0)
    np.testing.assert_allclose(a["se"], b["se"], rtol=rtol, atol=0)


@pytest.mark.parametrize("band", BANDS, ids=["15-17pct", "22-24pct"])
def test_two_fe_guard_silent_below_its_threshold(band, knob):
    from leanfe_amd._lib import Engine
    from oracle import altproj

    GP, GQ, k = 3_000, 300, 4
    n = GP * GQ  # every (primary, secondary) cell once
    i = np.arange(n)
    fe1, fe2 = (i // GQ).astype(np.int32), (i % GQ).astype(np.int32)
    rng = np.random.default_rng(17)
    x = rng.standard_normal((k, n))
    a = zero_sum(lognormal_effect(GP, 1e6, 21, *band))  # y's primary-FE effect
    b = lognormal_effect(GQ, 1e6, 22, *band)            # x1's secondary-FE effect
    x[0] += b[fe2]
    y = x.T @ np.array([1.0, -0.5, 0.25, 2.0]) + a[fe1] + rng.standard_normal(n)
    xs = [f"x{j + 1}" for j in range(k)]
    data = {"y": y, "fe1": fe1, "fe2": fe2, **{xs[j]: x[j].copy() for j in range(k)}}
    o = altproj.fit(data, "y", xs, ["fe1", "fe2"], vcov="HC1")
    knob.setenv("LFE_DENSE", "1")
    with Engine(0) as eng:
        i8 = _fit(data, xs, ["fe1", "fe2"], eng)
        again = _fit(data, xs, ["fe1", "fe2"], eng)
        knob.setenv("LFE_DN8", "0")
        f64 = _fit(data, xs, ["fe1", "fe2"], eng)
    assert i8["cells"] > 0 and i8["bytes"] == 1  # the guard stayed silent: the exact i8 passes ran
    assert f64["cells"] > 0 and f64["bytes"] == 2
    _check(i8, o)
    _check(f64, o)
    _close(i8, f64, 1e-12)
    np.testing.assert_array_equal(i8["beta"], again["beta"])
    np.testing.assert_array_equal(i8["se"], again["se"])


@pytest.mark.parametrize("band", BANDS, ids=["15-17pct", "22-24pct"])
def test_pair_table_guard_silent_below_its_threshold(band, knob):
    from leanfe_amd import synth
    from leanfe_amd._lib import Engine
    from oracle import altproj

    L, k, n = [3_000, 800, 200], 4, 1_200_000
    xs = [f"x{j + 1}" for j in range(k)]
    fes = ["fe1", "fe2", "fe3"]
    data = dict(synth.panel(n, k, L, seed=707))
    f3 = np.asarray(data["fe3"])
    data["y"] = data["y"] + lognormal_effect(L[2], 1e6, 31, *band)[f3]
    data["x1"] = data["x1"] + lognormal_effect(L[2], 1e6, 32, *band)[f3]
    o = altproj.fit(data, "y", xs, fes, vcov="HC1")
    knob.setenv("LFE_DENSE", "1")
    with Engine(0) as eng:
        dense = _fit(data, xs, fes, eng)
        again = _fit(data, xs, fes, eng)
        knob.setenv("LFE_DENSE", "0")
        rows = _fit(data, xs, fes, eng)
    assert dense["cells"] > 0 and rows["cells"] == 0
    _check(dense, o)
    _check(rows, o)
    _close(dense, rows, 1e-12)
    np.testing.assert_array_equal(dense["beta"], again["beta"])
    np.testing.assert_array_equal(dense["se"], again["se"])

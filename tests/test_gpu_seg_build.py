"""The row sweeps' segment layouts (leanfe_amd/csrc/lfe_seg.hip seg_build).

For every FE the kept rows are ordered by its code with the other FEs' codes beside them; the
cross terms T_f[g] = sum_{i in g} sum_{f' != f} alpha_f'[g_f'(i)] (polars_impl.py:490-526) are
segmented sums over that order.  Unweighted fits with two or three FEs build it by one radix pass
on the code's coarse bucket and a per-block ranking (the sorted build); the block scatter
(k_seg_scatter2, the LFE_TEST_SEG_SCATTER hook) builds the same segments with the rows of a segment
in another order.  The cross terms are two-limb fixed-point sums, exact in any order, so both
builds give the same fit bit for bit (clustered SEs: a one-column subset on an FE column sums the
score rows over that FE's segments in the sorted build - two-limb, so repeats are bit-identical -
and sorts in the other, equal at 1e-12), and both match the CPU oracle (oracle/altproj.py) at 1e-10
with equal `iterations` - with singletons dropped (rows past the kept range), a level count past
2^16 (coarse buckets of 2^9 codes and more) and a two-FE fit whose secondary table takes the row
sweeps."""
from __future__ import annotations

import numpy as np
import pytest

from leanfe_amd import synth

pytestmark = pytest.mark.gpu

SEG_SCATTER = 8  # LFE_TEST_SEG_SCATTER (include/leanfe_hip.h)


def _fit(data, xs, fes, hooks=0, vcov="HC1", cl=None):
    from leanfe_amd import leanfe_hip
    from leanfe_amd._lib import Engine

    kw = dict(cluster_cols=cl) if cl else {}
    with Engine(0) as eng:
        if hooks:
            eng.test_hooks(hooks)
        eng.profile(True)
        r = leanfe_hip(data, y_col="y", x_cols=xs, fe_cols=fes, strategy="alt_proj", vcov=vcov, quiet=True,
                       engine=eng, **kw)
        kernels = set(eng.kernel_stats())
    return (np.array([r.coefs[x] for x in xs]), np.array([r.std_errors[x] for x in xs]), r.iterations, r.n_obs,
            kernels)


CASES = [
    ("three_fe_singletons", 400_000, [120_000, 3_000, 200], "HC1", None),
    ("three_fe_cluster", 300_000, [20_000, 5_000, 700], "cluster", ["fe2"]),
    ("three_fe_twoway_cluster", 300_000, [20_000, 5_000, 700], "cluster", ["fe2", "fe3"]),
    ("two_fe_wide_secondary", 300_000, [60_000, 20_000], "iid", None),
]


@pytest.mark.parametrize("name,n,L,vcov,cl", CASES, ids=[c[0] for c in CASES])
def test_sorted_build_matches_scatter_and_oracle(knob, name, n, L, vcov, cl):
    from oracle import altproj

    knob.setenv("LFE_DENSE", "0")  # the row sweeps (lfe_seg.hip), not the count tables
    k = 3
    xs = [f"x{j + 1}" for j in range(k)]
    fes = [f"fe{f + 1}" for f in range(len(L))]
    d = dict(synth.panel(n, k, L, seed=123))
    srt = _fit(d, xs, fes, vcov=vcov, cl=cl)
    sct = _fit(d, xs, fes, hooks=SEG_SCATTER, vcov=vcov, cl=cl)
    again = _fit(d, xs, fes, vcov=vcov, cl=cl)
    for a, b in ((srt, sct), (srt, again)):
        np.testing.assert_array_equal(a[0], b[0])
        assert a[2] == b[2] and a[3] == b[3]
    np.testing.assert_array_equal(srt[1], again[1])
    if cl:  # the sorted build's clusters sum over the FE's segments (two-limb), the scatter's sort
        np.testing.assert_allclose(srt[1], sct[1], rtol=1e-12, atol=0)
    else:
        np.testing.assert_array_equal(srt[1], sct[1])
    if cl and len(cl) == 1:  # the FE's segments, no sort (the scatter build has no permutation: sorted)
        assert "cluster_fix" in srt[4] and "cluster_sort" not in srt[4], srt[4]
        assert "cluster_sort" in sct[4], sct[4]
    o = altproj.fit(d, "y", xs, fes, vcov=vcov, cluster_cols=cl)
    assert srt[2] == o["iterations"] and srt[3] == o["n_obs"]
    np.testing.assert_allclose(srt[0], o["beta"], rtol=1e-10, atol=0)
    np.testing.assert_allclose(srt[1], o["se"], rtol=1e-10, atol=0)

"""lfe_fit (Engine.fit): the whole regression in one engine call - drop, projections with the FEs
ordered by cardinality (polars_impl.py:485), Gram + device solve + residual pass, the host solve
(:211-220) and IID / HC1 SEs (std_errors.py:196-210, 275-282) in C - against the same steps driven
one call at a time from Python (NumPy / LAPACK on the host) and the CPU oracle."""
from __future__ import annotations

import numpy as np
import pytest

from leanfe_amd import inference, synth

pytestmark = pytest.mark.gpu


def _steps(eng, v, cl=0):
    """The step-by-step sequence lfe_fit replaces (hip_impl.leanfe_hip before round 6)."""
    from leanfe_amd.hip_impl import _beta_agrees

    n_obs, dims, card = eng.drop_singletons()
    order = sorted(range(len(card)), key=lambda i: card[i])
    it, _ = eng.demean(order, 1e-6, 50, check_from=3)
    fused = None if v == "iid" else eng.gram_resid(hc1=v == "hc1", keep_scores=v == "cluster")
    G = fused[0] if fused is not None else eng.gram()
    XtX, Xty = inference.split_gram(G)
    bf, inv = inference.solve_normal(XtX, Xty)
    k = XtX.shape[0] - 1
    df = n_obs - (k + 1) - (sum(dims) - len(dims))
    stats = inference.stats_from_gram(G, bf) if v == "iid" else None
    meat = None
    if stats is None:
        if fused is not None and _beta_agrees(fused[1], bf):
            stats, meat = fused[2], fused[3]
        else:
            stats, meat = eng.resid(bf, hc1=v == "hc1", keep_scores=v == "cluster")
    Vb = inv[1:, 1:]
    if v == "iid":
        se = inference.se_iid(Vb, stats[0], df)
    elif v == "hc1":
        se = inference.se_hc1(Vb, meat, n_obs, df)
    else:
        meats, Gs = eng.cluster_meat()
        se, _ = inference.se_cluster_oneway(Vb, meats[0], int(Gs[0]), n_obs, df, True)
    return dict(n_obs=n_obs, it=it, df=df, beta=bf, se=se, stats=np.asarray(stats))


def _fit(eng, v):
    r = eng.fit(v)
    se = r["se"]
    if v == "cluster":
        meats, Gs = eng.cluster_meat()
        se, _ = inference.se_cluster_oneway(r["xtx_inv"][1:, 1:], meats[0], int(Gs[0]), r["n_obs"], r["df_resid"],
                                            True)
    return dict(n_obs=r["n_obs"], it=r["iterations"], df=r["df_resid"], beta=r["beta_full"], se=se,
                stats=r["stats"])


@pytest.mark.parametrize("levels", [[3_000, 200], [5_000, 700, 60]], ids=["two_fe", "three_fe"])
@pytest.mark.parametrize("v", ["iid", "hc1", "cluster"])
def test_fit_matches_the_step_by_step_sequence_and_oracle(levels, v):
    from leanfe_amd._lib import Engine
    from oracle import altproj

    n, k = 400_000, 4
    data = synth.panel(n, k, levels, seed=29)

    def run(fn):
        with Engine(0) as eng:
            eng.synth_load(n, k, levels, synth.betas(k), seed=29)
            if v == "cluster":
                _, codes = eng.copy_inputs()
                eng.load_clusters([np.ascontiguousarray(codes[1])], [levels[1]])
            return fn(eng, v)

    a, b = run(_fit), run(_steps)
    assert (a["n_obs"], a["it"], a["df"]) == (b["n_obs"], b["it"], b["df"])
    np.testing.assert_allclose(a["beta"], b["beta"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(a["se"], b["se"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(a["stats"], b["stats"], rtol=1e-12, atol=0)
    xs = [f"x{j + 1}" for j in range(k)]
    fes = [f"fe{f + 1}" for f in range(len(levels))]
    o = altproj.fit(data, "y", xs, fes, vcov=v, cluster_cols=["fe2"] if v == "cluster" else None)
    assert a["it"] == o["iterations"] and a["n_obs"] == o["n_obs"] and a["df"] == o["df_resid"]
    np.testing.assert_allclose(a["beta"][1:], o["beta"], rtol=1e-10, atol=0)
    np.testing.assert_allclose(a["se"], o["se"], rtol=1e-10, atol=0)
    again = run(_fit)
    np.testing.assert_array_equal(again["beta"], a["beta"])
    np.testing.assert_array_equal(again["se"], a["se"])


def test_fit_refuses_what_it_does_not_cover():
    from leanfe_amd._lib import Engine

    n, k = 50_000, 2
    d = synth.panel(n, k, [500, 40], seed=3)
    w = np.random.default_rng(3).uniform(0.5, 2, n)
    with Engine(0) as eng:
        eng.load([d["y"], d["x1"], d["x2"]], [d["fe1"].astype(np.int32), d["fe2"].astype(np.int32)], [500, 40], w)
        with pytest.raises(ValueError):
            eng.fit("hc1")

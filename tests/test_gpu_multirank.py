"""The engine's multi-rank code paths on one GPU.

``world`` engine contexts, each driven by its own host thread and joined in an
in-process emulated group (``lfe_ctx_set_emu``: the same collective calls, in the
same order, as with RCCL, reduced through host memory), solve contiguous row
shards of one panel (global FE codes).  Every rank must return the single-process
oracle's fit on the whole panel, and all ranks must agree bit for bit.

This runs what world > 1 changes inside the engine:
- the all-reduced counts and the kept-row total;
- T_P partials with the P projection after the all-reduce (fast path);
- the all-reduced T_Q and the convergence test;
- the Gram and the device solve on every rank;
- the residual statistics and the cluster score tables.
"""
from __future__ import annotations

import threading

import numpy as np
import pytest

from leanfe_amd import inference, synth
from leanfe_amd.dist import shard_range

pytestmark = pytest.mark.gpu


def _solve(eng, vcov, cl_levels, n_obs_expected=None):
    n_obs, dims, card = eng.drop_singletons()
    order = sorted(range(len(card)), key=lambda i: card[i])
    iterations, _ = eng.demean(order, 1e-6, 50, check_from=3)
    v = vcov.lower()
    fused = eng.gram_resid(hc1=v == "hc1", keep_scores=v == "cluster")
    G = fused[0] if fused is not None else eng.gram()
    XtX, Xty = inference.split_gram(G)
    beta_full, XtX_inv = inference.solve_normal(XtX, Xty)
    if fused is not None:
        stats, meat = fused[2], fused[3]
    else:
        stats, meat = eng.resid(beta_full, hc1=v == "hc1", keep_scores=v == "cluster")
    k = XtX.shape[0] - 1
    df = n_obs - (k + 1) - (sum(dims) - len(dims))
    Vb = XtX_inv[1:, 1:]
    ncl = None
    if v == "iid":
        se = inference.se_iid(Vb, stats[0], df)
    elif v == "hc1":
        se = inference.se_hc1(Vb, meat, n_obs, df)
    elif len(cl_levels) == 1:
        meats, Gs = eng.cluster_meat()
        se, ncl = inference.se_cluster_oneway(Vb, meats[0], int(Gs[0]), n_obs, df, True)
    else:
        subsets = inference.cluster_subsets(len(cl_levels))
        meats, Gs = eng.cluster_meat_subsets(subsets)
        se, ncl = inference.se_cluster_multiway(Vb, list(meats), [int(g) for g in Gs], subsets, n_obs, df, True)
    return dict(beta=beta_full[1:], se=se, iterations=iterations, n_obs=n_obs, df_resid=df, fe_dims=list(dims),
                n_clusters=ncl, fused=fused is not None)


def _run_group(world, n, k, levels, vcov, cluster_fe, seed):
    from leanfe_amd._lib import EmuGroup, Engine

    group = EmuGroup(world)
    out, errs = {}, {}

    def worker(rank):
        try:
            lo, hi = shard_range(n, rank, world)
            eng = Engine(0)
            eng.set_emu(group, rank)
            eng.synth_load(hi - lo, k, levels, synth.betas(k), seed=seed, row_offset=lo)
            cl_levels = None
            if cluster_fe is not None:
                fes = [cluster_fe] if isinstance(cluster_fe, int) else list(cluster_fe)
                _, codes = eng.copy_inputs()
                cl_levels = [levels[f] for f in fes]
                eng.load_clusters([np.ascontiguousarray(codes[f]) for f in fes], cl_levels)
            out[rank] = _solve(eng, vcov, cl_levels)
            eng.close()
        except BaseException as e:  # noqa: BLE001
            errs[rank] = e

    threads = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in threads), "emulated group deadlocked"
    if errs:
        raise next(iter(errs.values()))
    return out


@pytest.mark.parametrize("world,n,k,levels,vcov,cluster_fe,owner", [
    (2, 400_003, 10, (20000, 500), "HC1", None, False),       # fast path (REDUCE mode), fused Gram/solve/resid
    (3, 300_000, 4, (8000, 300), "iid", None, False),
    (2, 200_000, 3, (3000, 200, 9), "cluster", 1, False),      # generic sweeps (F = 3) + key-indexed score table
    (2, 200_000, 3, (3000, 200, 9), "cluster", (0, 1), True),  # two-way CGM, owner-partitioned exchange
    (3, 250_001, 5, (30000, 120), "cluster", (0, 1), True),    # 3 ranks; fe1 x fe2: ~1.4 rows per cluster
    (3, 250_001, 5, (30000, 120), "cluster", (0, 1), False),   # same through the key-indexed table
])
def test_emulated_ranks_match_oracle(world, n, k, levels, vcov, cluster_fe, owner, knob):
    from oracle import altproj

    if owner:
        knob.setenv("LFE_CL_OWNER_MIN_SPAN", "0")
    else:
        knob.setenv("LFE_CL_OWNER_MIN_SPAN", str(1 << 40))
    seed = 11
    out = _run_group(world, n, k, list(levels), vcov, cluster_fe, seed)
    full = synth.panel(n, k, list(levels), seed=seed)
    xs = [f"x{j + 1}" for j in range(k)]
    fes = [f"fe{f + 1}" for f in range(len(levels))]
    cl = None
    if cluster_fe is not None:
        cl = [fes[cluster_fe]] if isinstance(cluster_fe, int) else [fes[f] for f in cluster_fe]
    o = altproj.fit(full, "y", xs, fes, vcov=vcov, cluster_cols=cl)
    for r in range(world):
        res = out[r]
        assert res["iterations"] == o["iterations"]
        assert res["n_obs"] == o["n_obs"] and res["df_resid"] == o["df_resid"]
        assert res["fe_dims"] == list(o["fe_dims"])
        np.testing.assert_allclose(res["beta"], o["beta"], rtol=1e-10, atol=0)
        np.testing.assert_allclose(res["se"], o["se"], rtol=1e-10, atol=0)
        if cluster_fe is not None:
            ncl = o["n_clusters"]
            assert (tuple(res["n_clusters"]) if isinstance(res["n_clusters"], (tuple, list)) else res["n_clusters"]) == (
                tuple(ncl) if isinstance(ncl, (tuple, list)) else ncl)
        np.testing.assert_array_equal(res["beta"], out[0]["beta"])  # identical on every rank
        np.testing.assert_array_equal(res["se"], out[0]["se"])


@pytest.mark.parametrize("world,n,k,levels,cluster_fe", [
    (2, 200_000, 3, (3000, 200, 9), 1),          # F = 3 sweeps + key-indexed score table
    (3, 250_001, 5, (30000, 120), (0, 1)),       # two-way CGM through the key-indexed table
])
def test_emulated_key_indexed_clusters_repeat_bit_identically(world, n, k, levels, cluster_fe, knob):
    """The multi-rank key-indexed cluster table is filled from each rank's sorted cluster sums
    (one store per cluster, k_cl_dense_put) instead of per-row f64 atomics: two solves give the
    same bits on every rank."""
    knob.setenv("LFE_CL_OWNER_MIN_SPAN", str(1 << 40))
    a = _run_group(world, n, k, list(levels), "cluster", cluster_fe, 17)
    b = _run_group(world, n, k, list(levels), "cluster", cluster_fe, 17)
    for r in range(world):
        assert a[r]["iterations"] == b[r]["iterations"]
        np.testing.assert_array_equal(a[r]["beta"], b[r]["beta"])
        np.testing.assert_array_equal(a[r]["se"], b[r]["se"])
        np.testing.assert_array_equal(a[r]["se"], a[0]["se"])


def _run_owned(world, n_total, k, levels, vcov, seed):
    """Owner-sharded ranks: rank r generates every row of the panel whose primary-FE code lies in
    dist.owner_range(G_P, r, world) (strong scaling: n_total rows in all)."""
    from leanfe_amd._lib import EmuGroup, Engine
    from leanfe_amd.dist import owner_range

    group = EmuGroup(world)
    out, errs = {}, {}
    P = max(range(len(levels)), key=lambda f: levels[f])

    def worker(rank):
        try:
            lo, hi = owner_range(levels[P], rank, world)
            eng = Engine(0)
            eng.set_emu(group, rank)
            eng.synth_load_owned(n_total, k, levels, synth.betas(k), P, lo, hi, seed=seed)
            _, codes = eng.copy_inputs()
            assert codes[P].size == eng.n and (codes[P].min() >= lo) and (codes[P].max() < hi)
            res = _solve(eng, vcov, None)
            res["rows"] = eng.n
            out[rank] = res
            eng.close()
        except BaseException as e:  # noqa: BLE001
            errs[rank] = e

    threads = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in threads), "emulated group deadlocked"
    if errs:
        raise next(iter(errs.values()))
    return out


@pytest.mark.parametrize("world,n,k,levels,vcov", [
    (2, 400_003, 10, (20000, 500), "HC1"),
    (8, 1_000_000, 10, (40000, 800), "HC1"),    # the 8-GPU strong-scaling split, on one GPU
    (8, 600_000, 5, (30000, 300), "iid"),
])
def test_emulated_owner_sharded_ranks_match_oracle(world, n, k, levels, vcov):
    from oracle import altproj

    seed = 13
    out = _run_owned(world, n, k, list(levels), vcov, seed)
    assert sum(out[r]["rows"] for r in range(world)) == n  # every row on exactly one rank
    full = synth.panel(n, k, list(levels), seed=seed)
    xs = [f"x{j + 1}" for j in range(k)]
    fes = [f"fe{f + 1}" for f in range(len(levels))]
    o = altproj.fit(full, "y", xs, fes, vcov=vcov)
    for r in range(world):
        res = out[r]
        assert res["iterations"] == o["iterations"]
        assert res["n_obs"] == o["n_obs"] and res["df_resid"] == o["df_resid"]
        assert res["fe_dims"] == list(o["fe_dims"])
        np.testing.assert_allclose(res["beta"], o["beta"], rtol=1e-10, atol=0)
        np.testing.assert_allclose(res["se"], o["se"], rtol=1e-10, atol=0)
        np.testing.assert_array_equal(res["beta"], out[0]["beta"])
        np.testing.assert_array_equal(res["se"], out[0]["se"])


def _run_owned_cl(world, n_total, k, levels, vcov, cl, seed, weights=False):
    """As _run_owned, with cluster columns (global FE codes) and optional weights (the same
    counter-based draw for every rank's rows, by global row index)."""
    from leanfe_amd._lib import EmuGroup, Engine
    from leanfe_amd.dist import owner_range

    group = EmuGroup(world)
    out, errs = {}, {}
    P = max(range(len(levels)), key=lambda f: levels[f])

    def worker(rank):
        try:
            lo, hi = owner_range(levels[P], rank, world)
            eng = Engine(0)
            eng.set_emu(group, rank)
            eng.synth_load_owned(n_total, k, levels, synth.betas(k), P, lo, hi, seed=seed)
            cols, codes = eng.copy_inputs()
            if weights:  # reload the same rows with weights (a function of the row's codes)
                w = 0.5 + (codes[0] % 7) / 4.0 + (codes[-1] % 3) / 8.0
                eng.load(list(cols), list(codes), list(levels), w)
                eng.set_owner(P, lo, hi)
            if cl:
                eng.load_clusters([np.ascontiguousarray(codes[f]) for f in cl], [levels[f] for f in cl])
            out[rank] = dict(first=_solve(eng, vcov, [levels[f] for f in cl] if cl else None),
                             second=_solve(eng, vcov, [levels[f] for f in cl] if cl else None), rows=eng.n)
            eng.close()
        except BaseException as e:  # noqa: BLE001
            errs[rank] = e

    threads = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in threads), "emulated group deadlocked"
    if errs:
        raise next(iter(errs.values()))
    return out


@pytest.mark.parametrize("world,n,k,levels,vcov,cl,weights", [
    (4, 800_000, 10, (60_000, 6_000, 600), "cluster", [1, 2], False),  # config-4-shaped: three FEs, CGM
    (8, 800_000, 10, (60_000, 6_000, 600), "cluster", [1, 2], False),
    (8, 600_000, 14, (20_000, 4_000, 1_000), "iid", None, False),      # MEGA-shaped
    (4, 500_000, 5, (30_000, 700), "HC1", None, True),                 # two FEs, weighted
    (3, 500_000, 4, (12_000, 2_000, 500), "HC1", None, True),          # three FEs, weighted
])
def test_emulated_owner_sharded_general_sweeps(world, n, k, levels, vcov, cl, weights):
    """Owner sharding beyond two unweighted FEs: the general sweeps keep the primary
    FE's counts, sums (W, Sy), cross term and effects on its owner rank and all-reduce only the other
    FEs' tables; the stop test is a max over ranks.  Every rank equals the oracle on the whole panel
    (equal integers, beta / SE at 1e-10), bit-identical across ranks and across repeats."""
    from oracle import altproj

    seed = 17
    out = _run_owned_cl(world, n, k, list(levels), vcov, cl, seed, weights)
    assert sum(out[r]["rows"] for r in range(world)) == n
    full = dict(synth.panel(n, k, list(levels), seed=seed))
    fes = [f"fe{f + 1}" for f in range(len(levels))]
    if weights:
        full["w"] = 0.5 + (full["fe1"] % 7) / 4.0 + (full[fes[-1]] % 3) / 8.0
    xs = [f"x{j + 1}" for j in range(k)]
    o = altproj.fit(full, "y", xs, fes, vcov=vcov, cluster_cols=[fes[f] for f in cl] if cl else None,
                    weights="w" if weights else None)
    for r in range(world):
        for res in (out[r]["first"], out[r]["second"]):
            assert res["iterations"] == o["iterations"] and res["n_obs"] == o["n_obs"]
            assert res["df_resid"] == o["df_resid"] and res["fe_dims"] == list(o["fe_dims"])
            np.testing.assert_allclose(res["beta"], o["beta"], rtol=1e-10, atol=0)
            np.testing.assert_allclose(res["se"], o["se"], rtol=1e-10, atol=0)
            np.testing.assert_array_equal(res["beta"], out[0]["first"]["beta"])
            np.testing.assert_array_equal(res["se"], out[0]["first"]["se"])
        if cl:
            assert tuple(out[r]["first"]["n_clusters"]) == tuple(o["n_clusters"])


def test_owner_declaration_is_validated():
    from leanfe_amd._lib import Engine

    eng = Engine(0)
    eng.synth_load(10_000, 2, [3000, 40], synth.betas(2), seed=3)
    with pytest.raises(ValueError):
        eng.set_owner(0, 0, 1500)  # rows with codes >= 1500 are present: not an owner shard
    eng.set_owner(0, 0, 3000)
    eng.set_owner(None)
    eng.close()


def test_sharded_leanfe_hip_auto_strategy_with_small_fes(monkeypatch):
    """leanfe_hip(engine=<sharded engine>) with the default strategy='auto' and two small FEs
    (where determine_strategy picks 'compress' for one process): every rank fits its row
    shard by alt_proj and returns the oracle's whole-panel fit (INTEGRATION.md §4's call)."""
    from leanfe_amd import dist, leanfe_hip
    from leanfe_amd._lib import EmuGroup, Engine
    from oracle import altproj

    world, n, k, levels, seed = 2, 120_000, 3, [300, 40], 21
    full = synth.panel(n, k, levels, seed=seed)
    xs = [f"x{j + 1}" for j in range(k)]
    # the emulated ranks share one process: the level agreement is the max over the shards,
    # which here is the panel's own level count
    monkeypatch.setattr(dist, "agree_levels", lambda eng, lv: [max(a, b) for a, b in zip(lv, levels)])
    group = EmuGroup(world)
    out, errs = {}, {}

    def worker(rank):
        try:
            lo, hi = shard_range(n, rank, world)
            eng = Engine(0)
            eng.set_emu(group, rank)
            eng.dist_group = ("emulated",)  # dist.is_sharded(eng): codes are global
            shard = {c: np.asarray(v)[lo:hi] for c, v in full.items()}
            out[rank] = leanfe_hip(shard, y_col="y", x_cols=xs, fe_cols=["fe1", "fe2"], vcov="HC1", quiet=True,
                                   engine=eng)
            eng.close()
        except BaseException as e:  # noqa: BLE001
            errs[rank] = e

    threads = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in threads), "emulated group deadlocked"
    if errs:
        raise next(iter(errs.values()))
    o = altproj.fit(full, "y", xs, ["fe1", "fe2"], vcov="HC1")
    for r in range(world):
        res = out[r]
        assert res.iterations == o["iterations"] and res.n_obs == o["n_obs"] and res.df_resid == o["df_resid"]
        np.testing.assert_allclose([res.coefs[x] for x in xs], o["beta"], rtol=1e-10, atol=0)
        np.testing.assert_allclose([res.std_errors[x] for x in xs], o["se"], rtol=1e-10, atol=0)


@pytest.mark.parametrize("world,n,k,levels,vcov,cl", [
    (2, 400_003, 5, [20000, 500], "HC1", None),
    (4, 600_000, 3, [30000, 300], "iid", None),
    (3, 300_000, 3, [20000, 700], "cluster", ["fe2"]),   # the cluster column moves with its rows
])
def test_emulated_contiguous_blocks_reshard_to_owners(world, n, k, levels, vcov, cl, monkeypatch):
    """leanfe_hip(engine=<sharded engine>) on contiguous row blocks (INTEGRATION.md §4's call):
    lfe_reshard_owner moves the rows so that every rank holds all rows of a range of the
    primary FE's levels, cut where the all-reduced counts balance the rows (not the levels);
    the owner-sharded sweeps then run (polars_impl.py:490-526), and every rank returns the
    oracle's whole-panel fit, bit-identical across ranks and across two runs."""
    from leanfe_amd import dist, leanfe_hip
    from leanfe_amd._lib import EmuGroup, Engine
    from oracle import altproj

    # skew the primary FE's level populations: equal level ranges would not balance the rows
    full = dict(synth.panel(n, k, levels, seed=23))
    fe1 = np.asarray(full["fe1"]).copy()
    fe1[: n // 3] = fe1[: n // 3] % (levels[0] // 10)  # a third of the rows in the first tenth of the levels
    full["fe1"] = fe1
    xs = [f"x{j + 1}" for j in range(k)]
    monkeypatch.setattr(dist, "agree_levels", lambda eng, lv: [max(a, b) for a, b in zip(lv, levels)])

    def run():
        group = EmuGroup(world)
        out, errs = {}, {}

        def worker(rank):
            try:
                lo, hi = shard_range(n, rank, world)
                eng = Engine(0)
                eng.set_emu(group, rank)
                eng.dist_group = ("emulated",)
                shard = {c: np.asarray(v)[lo:hi] for c, v in full.items()}
                r = leanfe_hip(shard, y_col="y", x_cols=xs, fe_cols=["fe1", "fe2"], vcov=vcov, cluster_cols=cl,
                               strategy="alt_proj", quiet=True, engine=eng)
                _, codes = eng.copy_inputs()
                out[rank] = dict(res=r, rows=eng.n, owner=eng.owner, fe1=(int(codes[0].min()), int(codes[0].max())))
                eng.close()
            except BaseException as e:  # noqa: BLE001
                errs[rank] = e

        threads = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout=300)
        assert not any(t.is_alive() for t in threads), "emulated group deadlocked"
        if errs:
            raise next(iter(errs.values()))
        return out

    a, b = run(), run()
    o = altproj.fit(full, "y", xs, ["fe1", "fe2"], vcov=vcov, cluster_cols=cl)
    counts = np.bincount(fe1, minlength=levels[0])
    assert sum(a[r]["rows"] for r in range(world)) == n
    assert max(a[r]["rows"] for r in range(world)) - min(a[r]["rows"] for r in range(world)) <= 2 * counts.max()
    for r in range(world):
        fe, lo, hi = a[r]["owner"]
        assert fe == 0 and lo <= a[r]["fe1"][0] and a[r]["fe1"][1] < hi
        res = a[r]["res"]
        assert res.iterations == o["iterations"] and res.n_obs == o["n_obs"] and res.df_resid == o["df_resid"]
        np.testing.assert_allclose([res.coefs[x] for x in xs], o["beta"], rtol=1e-10, atol=0)
        np.testing.assert_allclose([res.std_errors[x] for x in xs], o["se"], rtol=1e-10, atol=0)
        for other in (a[0]["res"], b[r]["res"]):  # every rank, and a second run, give the same bits
            np.testing.assert_array_equal([res.coefs[x] for x in xs], [other.coefs[x] for x in xs])
            np.testing.assert_array_equal([res.std_errors[x] for x in xs], [other.std_errors[x] for x in xs])


def test_reshard_memory_refusal_is_decided_by_every_rank(monkeypatch):
    """a re-shard refusal on one rank (here: rank 1 "short of device memory" for the
    staging copy, the LFE_TEST_SHORT_MEMORY hook) must be an all-rank decision taken before any row
    moves - every rank returns LFE_ENOMEM, keeps its contiguous block and the fit goes on with the
    row-block schedule, equal to the oracle and bit-identical across ranks (no rank is left inside a
    collective the others skipped)."""
    from leanfe_amd import dist, leanfe_hip
    from leanfe_amd._lib import EmuGroup, Engine
    from oracle import altproj

    world, n, k, levels = 3, 240_000, 3, [15_000, 400]
    full = dict(synth.panel(n, k, levels, seed=31))
    xs = [f"x{j + 1}" for j in range(k)]
    monkeypatch.setattr(dist, "agree_levels", lambda eng, lv: [max(a, b) for a, b in zip(lv, levels)])
    group = EmuGroup(world)
    out, errs = {}, {}

    def worker(rank):
        try:
            lo, hi = shard_range(n, rank, world)
            eng = Engine(0)
            eng.set_emu(group, rank)
            eng.dist_group = ("emulated",)
            if rank == 1:
                eng.test_hooks(1)  # LFE_TEST_SHORT_MEMORY
            shard = {c: np.asarray(v)[lo:hi] for c, v in full.items()}
            r = leanfe_hip(shard, y_col="y", x_cols=xs, fe_cols=["fe1", "fe2"], vcov="HC1", strategy="alt_proj",
                           quiet=True, engine=eng)
            out[rank] = dict(res=r, rows=eng.n, owner=eng.owner)
            eng.close()
        except BaseException as e:  # noqa: BLE001
            errs[rank] = e

    threads = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in threads), "emulated group deadlocked"
    if errs:
        raise next(iter(errs.values()))
    o = altproj.fit(full, "y", xs, ["fe1", "fe2"], vcov="HC1")
    for r in range(world):
        lo, hi = shard_range(n, r, world)
        assert out[r]["rows"] == hi - lo and out[r]["owner"] is None  # every rank kept its block
        res = out[r]["res"]
        assert res.iterations == o["iterations"] and res.n_obs == o["n_obs"]
        np.testing.assert_allclose([res.coefs[x] for x in xs], o["beta"], rtol=1e-10, atol=0)
        np.testing.assert_allclose([res.std_errors[x] for x in xs], o["se"], rtol=1e-10, atol=0)
        np.testing.assert_array_equal([res.coefs[x] for x in xs], [out[0]["res"].coefs[x] for x in xs])


@pytest.mark.parametrize("world,n,k,levels,vcov,weighted,cl", [
    (2, 300_001, 4, [12_000, 300], "HC1", False, None),          # two FEs: the fast sweeps on streamed codes
    (3, 240_000, 3, [9_000, 800, 120], "iid", True, None),        # three FEs, weighted: the general sweeps
    (2, 300_001, 4, [12_000, 300], "cluster", False, ["fe2"]),    # one-way clustered: owner exchange of scores
    (4, 320_000, 3, [9_000, 800, 150], "cluster", False, ["fe2", "fe3"]),  # CGM, 4 ranks
    (2, 200_000, 20, [6_000, 500, 90], "cluster", False, ["fe1", "fe2"]),  # k = 20: the wide MFMA passes
    (3, 210_000, 14, [7_000, 400], "HC1", True, None),            # k = 14, weighted
])
def test_emulated_out_of_core_ranks_match_oracle(world, n, k, levels, vcov, weighted, cl, monkeypatch):
    """Out-of-core fits on a sharded engine: every rank streams the columns of
    its own contiguous row block; the streamed group sums and every pass's tile are summed over the
    ranks (the design Gram streams: the ranks' raw tiles have their own shifts), and the clustered
    fits' per-cluster score sums go to their owner ranks (lfe_stream.hip, std_errors.py:289-441).
    Every rank returns the oracle's whole-panel fit, bit-identical across ranks."""
    from leanfe_amd import dist, leanfe_hip
    from leanfe_amd._lib import EmuGroup, Engine
    from oracle import altproj

    full = dict(synth.panel(n, k, levels, seed=29))
    if weighted:
        full["w"] = np.random.default_rng(30).uniform(0.5, 2.0, n)
    xs = [f"x{j + 1}" for j in range(k)]
    fes = [f"fe{f + 1}" for f in range(len(levels))]
    known = sorted(levels)
    # global level counts: a shard's local max code + 1 rounds up to the panel's (FE and cluster columns)
    monkeypatch.setattr(dist, "agree_levels", lambda eng, lv: [min(g for g in known if g >= x) for x in lv])
    group = EmuGroup(world)
    out, errs = {}, {}

    def worker(rank):
        try:
            lo, hi = shard_range(n, rank, world)
            eng = Engine(0)
            eng.set_emu(group, rank)
            eng.dist_group = ("emulated",)
            shard = {c: np.asarray(v)[lo:hi] for c, v in full.items()}
            out[rank] = leanfe_hip(shard, y_col="y", x_cols=xs, fe_cols=fes, vcov=vcov, strategy="alt_proj",
                                   cluster_cols=cl, weights="w" if weighted else None, quiet=True, engine=eng,
                                   out_of_core=True, chunk_rows=40_000 + 7_777 * rank)
            eng.close()
        except BaseException as e:  # noqa: BLE001
            errs[rank] = e

    threads = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in threads), "emulated group deadlocked"
    if errs:
        raise next(iter(errs.values()))
    o = altproj.fit(full, "y", xs, fes, vcov=vcov, cluster_cols=cl, weights="w" if weighted else None)
    for r in range(world):
        res = out[r]
        assert res.iterations == o["iterations"] and res.n_obs == o["n_obs"] and res.df_resid == o["df_resid"]
        np.testing.assert_allclose([res.coefs[x] for x in xs], o["beta"], rtol=1e-10, atol=0)
        np.testing.assert_allclose([res.std_errors[x] for x in xs], o["se"], rtol=1e-10, atol=0)
        np.testing.assert_array_equal([res.coefs[x] for x in xs], [out[0].coefs[x] for x in xs])
        np.testing.assert_array_equal([res.std_errors[x] for x in xs], [out[0].std_errors[x] for x in xs])
        if cl is not None:
            got, want = res.n_clusters, o["n_clusters"]
            assert (tuple(got) if isinstance(got, (tuple, list)) else got) == (
                tuple(want) if isinstance(want, (tuple, list)) else want)


@pytest.mark.parametrize("rank", [0, 7])
def test_owner_shard_solves_in_its_share_of_time(rank):
    """An owner shard (every row of 1/8 of the primary levels) solved alone takes less time than
    the whole panel: its buckets of the other ranks' levels are empty, and the sweeps pass over
    them (round 3: K1 walked every empty segment serially, 96 ms instead of 1.1 ms for the
    8-GPU shard of the headline panel).  Also checks that the shard's own fit is the oracle's."""
    import time

    from leanfe_amd import dist
    from leanfe_amd._lib import Engine
    from oracle import altproj

    n_total, k, levels = 8_000_000, 4, [100_000, 1_000]
    P = 0
    lo, hi = dist.owner_range(levels[P], rank, 8)
    eng = Engine(0)
    try:
        def timed():
            _solve(eng, "HC1", [])
            eng.sync()
            t0 = time.perf_counter()
            for _ in range(3):
                r = _solve(eng, "HC1", [])
            eng.sync()
            return (time.perf_counter() - t0) / 3, r

        eng.synth_load(n_total, k, levels, synth.betas(k), seed=3)
        t_full, _ = timed()
        eng.synth_load_owned(n_total, k, levels, synth.betas(k), P, lo, hi, seed=3)
        t_shard, r = timed()
        cols, codes = eng.copy_inputs()
    finally:
        eng.close()
    assert t_shard < t_full, (t_shard, t_full)
    data = {"y": cols[0], **{f"x{j + 1}": cols[j + 1] for j in range(k)}, "fe1": codes[0], "fe2": codes[1]}
    o = altproj.fit(data, "y", [f"x{j + 1}" for j in range(k)], ["fe1", "fe2"], vcov="HC1")
    assert r["iterations"] == o["iterations"] and r["n_obs"] == o["n_obs"]
    np.testing.assert_allclose(r["beta"], o["beta"], rtol=1e-10, atol=0)
    np.testing.assert_allclose(r["se"], o["se"], rtol=1e-10, atol=0)


@pytest.mark.parametrize("world,n,k,levels,vcov,cl", [
    (4, 600_000, 14, (20_000, 4_000, 1_000), "iid", None),  # MEGA-shaped, p = 15
    (3, 500_000, 4, (3_000, 500, 120), "cluster", [1, 2]),
])
def test_emulated_owner_sharded_pair_tables(world, n, k, levels, vcov, cl, knob):
    """The pair-table sweeps (lfe_dense3.hip, forced with LFE_DENSE=1) on owner shards: each rank's
    tables count its own rows, the primary FE's cross term stays local and the others' are
    all-reduced; every rank equals the oracle and repeats bit for bit."""
    from oracle import altproj

    knob.setenv("LFE_DENSE", "1")
    seed = 19
    out = _run_owned_cl(world, n, k, list(levels), vcov, cl, seed)
    full = dict(synth.panel(n, k, list(levels), seed=seed))
    fes = [f"fe{f + 1}" for f in range(len(levels))]
    xs = [f"x{j + 1}" for j in range(k)]
    o = altproj.fit(full, "y", xs, fes, vcov=vcov, cluster_cols=[fes[f] for f in cl] if cl else None)
    for r in range(world):
        for res in (out[r]["first"], out[r]["second"]):
            assert res["iterations"] == o["iterations"] and res["n_obs"] == o["n_obs"]
            np.testing.assert_allclose(res["beta"], o["beta"], rtol=1e-10, atol=0)
            np.testing.assert_allclose(res["se"], o["se"], rtol=1e-10, atol=0)
            np.testing.assert_array_equal(res["beta"], out[0]["first"]["beta"])


@pytest.mark.parametrize("levels", [(20_000, 500), (6_000, 900, 150)])
def test_unbalanced_owner_shards_take_the_same_sweeps(levels):
    """the dense-path decision (two FEs: count tables vs row layouts; three FEs:
    pair tables vs general sweeps) is taken from the whole panel's kept rows and largest primary
    level (summed with the kept-row total), not each rank's own: here rank 0 holds 7/8 of the rows
    and would take the tables alone while rank 1's shard is too sparse for them.  No LFE_DENSE
    override: both ranks must take the same path, equal the oracle and agree bit for bit."""
    from leanfe_amd._lib import EmuGroup, Engine
    from leanfe_amd.dist import owner_range
    from oracle import altproj

    world, k = 2, 3
    n = 4_000_000 if len(levels) == 2 else 3_000_000
    rng = np.random.default_rng(44)
    G0 = levels[0]
    heavy = rng.random(n) < 0.875
    fe1 = np.where(heavy, rng.integers(0, G0 // 2, n), rng.integers(G0 // 2, G0, n)).astype(np.int32)
    codes = [fe1] + [rng.integers(0, g, n).astype(np.int32) for g in levels[1:]]
    x = rng.standard_normal((n, k))
    y = x @ np.array([1.0, -0.5, 0.25]) + sum(rng.standard_normal(g)[c] for g, c in zip(levels, codes)) + \
        rng.standard_normal(n)
    data = {"y": y, **{f"x{j + 1}": x[:, j].copy() for j in range(k)},
            **{f"fe{f + 1}": c for f, c in enumerate(codes)}}
    group = EmuGroup(world)
    out, errs = {}, {}

    def worker(rank):
        try:
            lo, hi = owner_range(G0, rank, world)
            sel = (fe1 >= lo) & (fe1 < hi)
            eng = Engine(0)
            eng.set_emu(group, rank)
            eng.load([y[sel]] + [x[sel, j].copy() for j in range(k)], [c[sel] for c in codes], list(levels))
            eng.set_owner(0, lo, hi)
            res = _solve(eng, "HC1", None)
            res["cells"] = eng.dense_cells()
            res["rows"] = int(sel.sum())
            out[rank] = res
            eng.close()
        except BaseException as e:  # noqa: BLE001
            errs[rank] = e

    threads = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in threads), "emulated group deadlocked"
    if errs:
        raise next(iter(errs.values()))
    assert out[0]["rows"] > 5 * out[1]["rows"]
    assert (out[0]["cells"] > 0) == (out[1]["cells"] > 0)
    assert out[0]["cells"] > 0  # the whole panel is dense enough for the tables
    xs = [f"x{j + 1}" for j in range(k)]
    fes = [f"fe{f + 1}" for f in range(len(levels))]
    o = altproj.fit(data, "y", xs, fes, vcov="HC1")
    for r in range(world):
        res = out[r]
        assert res["iterations"] == o["iterations"] and res["n_obs"] == o["n_obs"]
        np.testing.assert_allclose(res["beta"], o["beta"], rtol=1e-10, atol=0)
        np.testing.assert_allclose(res["se"], o["se"], rtol=1e-10, atol=0)
        np.testing.assert_array_equal(res["beta"], out[0]["beta"])
        np.testing.assert_array_equal(res["se"], out[0]["se"])


@pytest.mark.parametrize("world,n,k,levels,cl", [
    (4, 1_500_000, 4, (10_000, 2_000), (0,)),          # HDFE_CLUSTER1's shape: sums in the residual pass
    (4, 1_500_000, 4, (10_000, 2_000), (0, 1)),        # HDFE_CLUSTER2's: owner-local bucket keys for fe1 x fe2
    (8, 1_500_000, 4, (10_000, 2_000), (0, 1)),
    (4, 1_000_000, 5, (40_000, 4_000, 400), (1, 2)),   # config 4's: fe2 x fe3 holds no owner column
    (8, 1_000_000, 5, (40_000, 4_000, 400), (1, 2)),
], ids=["hdfe_cl1_w4", "hdfe_cl2_w4", "hdfe_cl2_w8", "config4_w4", "config4_w8"])
def test_emulated_owner_shards_cluster_forms(world, n, k, levels, cl):
    """Owner-sharded ranks (every row of a range of the primary FE's levels on one rank: the
    strong-scaled headline schedule, dist.owner_range) with clustered SEs (std_errors.py:289-441):
    a subset holding the cluster column that repeats the primary FE has each cluster on one rank, so
    the round-5 forms run per rank - the one-way sums inside the residual pass, the bucket-key
    intersections - with only the k x k meat and the cluster count summed over ranks; other subsets
    keep the all-reduced table or the owner exchange.  Every rank equals the oracle on the whole panel
    (1e-10, equal integers) and all ranks and a second run agree bit for bit."""
    from leanfe_amd import dist
    from leanfe_amd._lib import EmuGroup, Engine
    from oracle import altproj

    seed = 61
    P = max(range(len(levels)), key=lambda f: levels[f])

    def run():
        group = EmuGroup(world)
        out, errs = {}, {}

        def worker(rank):
            try:
                lo, hi = dist.owner_range(levels[P], rank, world)
                eng = Engine(0)
                eng.set_emu(group, rank)
                eng.synth_load_owned(n, k, list(levels), synth.betas(k), P, lo, hi, seed=seed)
                _, codes = eng.copy_inputs()
                eng.load_clusters([np.ascontiguousarray(codes[f]) for f in cl], [levels[f] for f in cl])
                r = eng.fit("cluster")
                Vb = r["xtx_inv"][1:, 1:]
                if len(cl) == 1:
                    meats, Gs = eng.cluster_meat()
                    se, ncl = inference.se_cluster_oneway(Vb, meats[0], int(Gs[0]), r["n_obs"], r["df_resid"], True)
                else:
                    subsets = inference.cluster_subsets(len(cl))
                    meats, Gs = eng.cluster_meat_subsets(subsets)
                    se, ncl = inference.se_cluster_multiway(Vb, list(meats), [int(g) for g in Gs], subsets,
                                                            r["n_obs"], r["df_resid"], True)
                out[rank] = dict(beta=r["beta_full"][1:], se=se, ncl=ncl, it=r["iterations"], n_obs=r["n_obs"])
                eng.close()
            except BaseException as e:  # noqa: BLE001
                errs[rank] = e
                group.abort()

        threads = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout=300)
        assert not any(t.is_alive() for t in threads), "emulated group deadlocked"
        if errs:
            raise next(iter(errs.values()))
        return out

    a, b = run(), run()
    full = synth.panel(n, k, list(levels), seed=seed)
    xs = [f"x{j + 1}" for j in range(k)]
    fes = [f"fe{f + 1}" for f in range(len(levels))]
    o = altproj.fit(full, "y", xs, fes, vcov="cluster", cluster_cols=[fes[f] for f in cl])
    ncl = o["n_clusters"]
    for r in range(world):
        res = a[r]
        assert res["it"] == o["iterations"] and res["n_obs"] == o["n_obs"]
        got = res["ncl"] if len(cl) > 1 else [res["ncl"]]
        assert list(got) == (list(ncl) if isinstance(ncl, (list, tuple)) else [ncl])
        np.testing.assert_allclose(res["beta"], o["beta"], rtol=1e-10, atol=0)
        np.testing.assert_allclose(res["se"], o["se"], rtol=1e-10, atol=0)
        for other in (a[0], b[r]):
            np.testing.assert_array_equal(res["beta"], other["beta"])
            np.testing.assert_array_equal(res["se"], other["se"])

"""World-size-2 tests of the multi-GPU path on CPU (gloo).

The engine's collectives run inside liblfe_hip.so over RCCL (no GPU here), so
these tests cover (1) the host plumbing of leanfe_amd.dist — row sharding, the
RCCL unique-id hand-off, the timing helpers bench.py uses — and (2) the data-
parallel *schedule* the engine implements: which per-group partial sums are
all-reduced, and when, so that every rank's result equals the single-process
fit.  (2) is a NumPy restatement of that schedule (lfe_capi.hip / lfe_iter.hip:
counts -> singleton mask -> kept counts -> group sums S_f -> per projection the
cross term T_f -> Gram -> residual stats -> HC1 meat / cluster score tables),
run on two row shards with torch.distributed all-reduces and compared with the
oracle (oracle/altproj.py) on the unsharded panel.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from leanfe_amd import synth  # noqa: E402
from leanfe_amd.dist import HostGroup, attach, shard_range  # noqa: E402

WORLD = 2


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(fn, *args):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_entry, args=(r, port, q, fn, args)) for r in range(WORLD)]
    for p in procs:
        p.start()
    out = {}
    for _ in procs:
        r, res = q.get(timeout=300)
        out[r] = res
    for p in procs:
        p.join(timeout=60)
    for r in range(WORLD):
        if isinstance(out[r], BaseException):
            raise out[r]
    return out


def _entry(rank, port, q, fn, args):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(WORLD), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        res = fn(rank, *args)
        dist.destroy_process_group()
        q.put((rank, res))
    except BaseException as e:  # noqa: BLE001 - ship the failure to the parent
        q.put((rank, e))


# ---------------------------------------------------------------------------
# plumbing
# ---------------------------------------------------------------------------

def _agree_categories_worker(rank):
    from leanfe_amd import dist as ldist

    class _Eng:  # what agree_categories needs of an attached engine: its torch group
        dist_group = (None,)

    local = np.array([2001, 2003, 2007]) if rank == 0 else np.array([2003, 2010])
    return ldist.agree_categories(_Eng(), local).tolist()


def test_factor_categories_agreed_across_row_shards():
    """i(var) on a row shard: every rank expands the union of the ranks' categories (a shard may
    miss some), so all ranks load the same columns (hip_impl: dist.agree_categories)."""
    out = _run(_agree_categories_worker)
    assert out[0] == out[1] == [2001, 2003, 2007, 2010]


def test_shard_range_partitions_rows():
    for n in (0, 1, 7, 10, 1001):
        for world in (1, 2, 3, 8):
            parts = [shard_range(n, r, world) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
            sizes = [hi - lo for lo, hi in parts]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


class _FakeEngine:
    """Stands in for leanfe_amd._lib.Engine (no GPU): records set_comm."""
    calls = []

    @staticmethod
    def unique_id() -> bytes:
        return os.urandom(128)

    def set_comm(self, uid, rank, world):
        self.calls.append((uid, rank, world))


def _plumbing(rank):
    g = HostGroup()
    assert (g.rank, g.world) == (rank, WORLD)
    g.barrier()
    mx = g.max(float(rank + 1))
    sm = g.sum(float(rank + 1))
    b = g.bcast_bytes(b"uid-from-rank0" if rank == 0 else None)
    eng = _FakeEngine()
    attach(eng)
    uid, r, w = eng.calls[-1]
    import os
    return dict(max=mx, sum=sm, bytes=b, uid=uid, rank=r, world=w, ifname=os.environ.get("NCCL_SOCKET_IFNAME"))


def test_hostgroup_and_attach_gloo():
    out = _run(_plumbing)
    assert out[0]["max"] == out[1]["max"] == 2.0
    assert out[0]["sum"] == out[1]["sum"] == 3.0
    assert out[0]["bytes"] == out[1]["bytes"] == b"uid-from-rank0"
    assert out[0]["uid"] == out[1]["uid"] and len(out[0]["uid"]) == 128  # same RCCL id on every rank
    assert [out[r]["rank"] for r in range(WORLD)] == [0, 1]
    assert out[0]["world"] == out[1]["world"] == WORLD
    assert out[0]["ifname"] == out[1]["ifname"] == "lo"  # single node: RCCL bootstrap over loopback


# ---------------------------------------------------------------------------
# the engine's data-parallel schedule, restated on two shards
# ---------------------------------------------------------------------------

def _levels(rank):
    from leanfe_amd import frame
    from leanfe_amd.dist import agree_levels, is_sharded

    eng = _FakeEngine()
    attach(eng)
    # global codes of one FE: this shard happens not to hold the largest code
    shard = np.array([0, 3, 3, 1] if rank == 0 else [2, 7, 5], dtype=np.int64)
    codes, g = frame.factorize(shard, global_codes=True)
    try:
        frame.factorize(np.array(["a", "b"]), global_codes=True)
        strings_rejected = False
    except ValueError:
        strings_rejected = True
    return dict(sharded=is_sharded(eng), local=g, agreed=agree_levels(eng, [g, 10 + rank]),
                same_codes=bool(np.array_equal(codes, shard)), strings_rejected=strings_rejected)


def test_sharded_levels_agree_gloo():
    """Every rank sizes its group tables by the max code over all shards (dist.agree_levels)."""
    out = _run(_levels)
    assert out[0]["local"] == 4 and out[1]["local"] == 8
    assert out[0]["agreed"] == out[1]["agreed"] == [8, 11]
    assert all(out[r]["sharded"] and out[r]["same_codes"] and out[r]["strings_rejected"] for r in range(WORLD))


def _allreduce(a: np.ndarray) -> np.ndarray:
    t = torch.from_numpy(np.ascontiguousarray(a).copy())
    dist.all_reduce(t)
    return t.numpy()


def _gsum(vals: np.ndarray, codes: np.ndarray, G: int) -> np.ndarray:
    """Group sums of the rows of vals ([p, n] or [n]) -> [G, p] (or [G])."""
    if vals.ndim == 1:
        return np.bincount(codes, weights=vals, minlength=G)
    return np.stack([np.bincount(codes, weights=v, minlength=G) for v in vals], axis=1)


def _sharded_fit(rank, n, k, levels, seed, vcov, cluster_fe, tol=1e-6, max_iter=50):
    lo, hi = shard_range(n, rank, WORLD)
    d = synth.panel(hi - lo, k, levels, seed=seed, row_offset=lo)  # global codes: same generator
    F = len(levels)
    cols = np.stack([d["y"]] + [d[f"x{j + 1}"] for j in range(k)])
    codes = [d[f"fe{f + 1}"].astype(np.int64) for f in range(F)]
    cl = codes[cluster_fe] if cluster_fe is not None else None
    G = list(levels)
    # pre-filter counts (lfe_drop_singletons: one all-reduce per FE)
    cnt_pre = [_allreduce(np.bincount(c, minlength=G[f]).astype(np.int64)) for f, c in enumerate(codes)]
    card = [int((c > 0).sum()) for c in cnt_pre]
    keep = np.all([cnt_pre[f][codes[f]] > 1 for f in range(F)], axis=0)  # single pass (polars_impl.py:477-482)
    cols = cols[:, keep]
    codes = [c[keep] for c in codes]
    cl = cl[keep] if cl is not None else None
    cnt = [_allreduce(np.bincount(c, minlength=G[f]).astype(np.int64)) for f, c in enumerate(codes)]
    fe_dims = [int((c > 0).sum()) for c in cnt]
    n_obs = int(_allreduce(np.array([keep.sum()], dtype=np.int64))[0])
    order = sorted(range(F), key=lambda f: card[f])  # polars_impl.py:485
    # constant group sums (all-reduced once), alpha-form sweeps (one all-reduce per projection)
    S = [_allreduce(_gsum(cols, codes[f], G[f])) for f in range(F)]
    alpha = [np.zeros((G[f], cols.shape[0])) for f in range(F)]
    safe = [np.maximum(c, 1)[:, None] for c in cnt]
    it = 0
    for it in range(1, max_iter + 1):
        for f in order:
            other = sum(alpha[g][codes[g]] for g in range(F) if g != f)  # [n_loc, p]
            T = _allreduce(_gsum(np.asarray(other).T, codes[f], G[f])) if F > 1 else 0.0
            alpha[f] = np.where(cnt[f][:, None] > 0, (S[f] - T) / safe[f], 0.0)
        if it >= 3:  # stop test on y only (polars_impl.py:511-521)
            ytil = cols[0] - sum(alpha[f][codes[f], 0] for f in range(F))
            m = 0.0
            for f in range(F):
                sy = _allreduce(_gsum(ytil, codes[f], G[f]))
                present = cnt[f] > 0
                m = max(m, float(np.max(np.abs(sy[present] / cnt[f][present]))))
            if m < tol:
                break
    Xd = cols - sum(alpha[f][codes[f]].T for f in range(F))
    # Gram with intercept (one all-reduce), host solve (polars_impl.py:165-226)
    Z = np.vstack([np.ones(Xd.shape[1]), Xd[1:]])
    XtX = _allreduce(Z @ Z.T)
    Xty = _allreduce(Z @ Xd[0])
    L = np.linalg.cholesky(XtX)
    beta_full = np.linalg.solve(L.T, np.linalg.solve(L, Xty))
    XtX_inv = np.linalg.solve(L.T, np.linalg.solve(L, np.eye(k + 1)))
    r = Xd[0] - beta_full @ Z
    rss = float(_allreduce(np.array([r @ r]))[0])
    df_resid = n_obs - (k + 1) - (sum(fe_dims) - F)
    Vb = XtX_inv[1:, 1:]
    if vcov == "iid":
        V = Vb * (rss / df_resid)
        ncl = None
    elif vcov == "HC1":
        x = Xd[1:]
        meat = _allreduce((x * r * r) @ x.T)
        V = Vb @ meat @ Vb * (n_obs / df_resid)
        ncl = None
    else:  # one-way cluster: score table all-reduced (C x k)
        C = int(levels[cluster_fe])
        sc = _allreduce(_gsum(Xd[1:] * r, cl, C))
        Gc = int((_allreduce(np.bincount(cl, minlength=C).astype(np.int64)) > 0).sum())
        V = Vb @ (sc.T @ sc) @ Vb * (Gc / (Gc - 1)) * ((n_obs - 1) / df_resid)
        ncl = Gc
    se = np.sqrt(np.maximum(np.diag(V), 0.0))
    return dict(beta=beta_full[1:], se=se, iterations=it, n_obs=n_obs, df_resid=df_resid, fe_dims=fe_dims,
                n_clusters=ncl)


@pytest.mark.parametrize("n,k,levels,vcov,cluster_fe", [
    (20_000, 3, (400, 30), "iid", None),
    (20_001, 4, (500, 40), "HC1", None),
    (18_000, 2, (300, 25, 6), "cluster", 1),
])
def test_sharded_schedule_matches_oracle(n, k, levels, vcov, cluster_fe):
    from oracle import altproj

    seed = 7
    out = _run(_sharded_fit, n, k, list(levels), seed, vcov, cluster_fe)
    full = synth.panel(n, k, list(levels), seed=seed)
    xs = [f"x{j + 1}" for j in range(k)]
    fes = [f"fe{f + 1}" for f in range(len(levels))]
    cl = [fes[cluster_fe]] if cluster_fe is not None else None
    o = altproj.fit(full, "y", xs, fes, vcov=vcov, cluster_cols=cl)
    for r in range(WORLD):  # every rank holds the global fit
        res = out[r]
        np.testing.assert_allclose(res["beta"], o["beta"], rtol=1e-10, atol=1e-13)
        np.testing.assert_allclose(res["se"], o["se"], rtol=1e-10, atol=1e-14)
        assert res["iterations"] == o["iterations"]
        assert res["n_obs"] == o["n_obs"]
        assert res["df_resid"] == o["df_resid"]
        assert list(res["fe_dims"]) == list(o["fe_dims"])
        if cluster_fe is not None:
            assert res["n_clusters"] == o["n_clusters"]
    np.testing.assert_array_equal(out[0]["beta"], out[1]["beta"])  # bit-identical across ranks


# ---------------------------------------------------------------------------
# the owner schedule (lfe_ctx_set_owner / bench --shard owner): rank r holds every row whose code of
# the primary FE (most levels) lies in its level range, so the primary FE's counts, sums, cross
# terms and effects are complete on the rank and never all-reduced; the other FEs' are, and the
# stop test's max is taken over ranks (lfe_prep.hip, lfe_sweep.hip, lfe_seg.hip, lfe_dense3.hip)
# ---------------------------------------------------------------------------

def _allmax(x: float) -> float:
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _owner_fit(rank, n, k, levels, seed, vcov, cluster_fe, tol=1e-6, max_iter=50):
    F = len(levels)
    G = list(levels)
    P = int(np.argmax(G))
    lo, hi = shard_range(G[P], rank, WORLD)  # this rank's primary levels
    full = synth.panel(n, k, levels, seed=seed)
    own = (full[f"fe{P + 1}"] >= lo) & (full[f"fe{P + 1}"] < hi)
    cols = np.stack([full["y"][own]] + [full[f"x{j + 1}"][own] for j in range(k)])
    codes = [full[f"fe{f + 1}"][own].astype(np.int64) for f in range(F)]
    cl = codes[cluster_fe] if cluster_fe is not None else None
    local = lambda f: f == P  # noqa: E731 - the primary FE's tables are complete on the rank
    red = lambda f, a: a if local(f) else _allreduce(a)  # noqa: E731
    cnt_pre = [red(f, np.bincount(c, minlength=G[f]).astype(np.int64)) for f, c in enumerate(codes)]
    card = [int(_allreduce(np.array([(cnt_pre[f] > 0).sum()]))[0]) if local(f) else int((cnt_pre[f] > 0).sum())
            for f in range(F)]
    keep = np.all([cnt_pre[f][codes[f]] > 1 for f in range(F)], axis=0)
    cols = cols[:, keep]
    codes = [c[keep] for c in codes]
    cl = cl[keep] if cl is not None else None
    cnt = [red(f, np.bincount(c, minlength=G[f]).astype(np.int64)) for f, c in enumerate(codes)]
    fe_dims = [int(_allreduce(np.array([(cnt[f] > 0).sum()]))[0]) if local(f) else int((cnt[f] > 0).sum())
               for f in range(F)]
    n_obs = int(_allreduce(np.array([keep.sum()], dtype=np.int64))[0])
    order = sorted(range(F), key=lambda f: card[f])
    S = [red(f, _gsum(cols, codes[f], G[f])) for f in range(F)]
    alpha = [np.zeros((G[f], cols.shape[0])) for f in range(F)]
    safe = [np.maximum(c, 1)[:, None] for c in cnt]
    it = 0
    for it in range(1, max_iter + 1):
        for f in order:
            other = sum(alpha[g][codes[g]] for g in range(F) if g != f)
            T = red(f, _gsum(np.asarray(other).T, codes[f], G[f]))
            alpha[f] = np.where(cnt[f][:, None] > 0, (S[f] - T) / safe[f], 0.0)
        if it >= 3:
            ytil = cols[0] - sum(alpha[f][codes[f], 0] for f in range(F))
            m = 0.0
            for f in range(F):
                sy = red(f, _gsum(ytil, codes[f], G[f]))
                present = cnt[f] > 0
                if local(f):  # only this rank's primary levels
                    present &= (np.arange(G[f]) >= lo) & (np.arange(G[f]) < hi)
                if present.any():
                    m = max(m, float(np.max(np.abs(sy[present] / cnt[f][present]))))
            if _allmax(m) < tol:
                break
    Xd = cols - sum(alpha[f][codes[f]].T for f in range(F))
    Z = np.vstack([np.ones(Xd.shape[1]), Xd[1:]])
    XtX = _allreduce(Z @ Z.T)
    Xty = _allreduce(Z @ Xd[0])
    L = np.linalg.cholesky(XtX)
    beta_full = np.linalg.solve(L.T, np.linalg.solve(L, Xty))
    XtX_inv = np.linalg.solve(L.T, np.linalg.solve(L, np.eye(k + 1)))
    r = Xd[0] - beta_full @ Z
    rss = float(_allreduce(np.array([r @ r]))[0])
    df_resid = n_obs - (k + 1) - (sum(fe_dims) - F)
    Vb = XtX_inv[1:, 1:]
    ncl = None
    if vcov == "iid":
        V = Vb * (rss / df_resid)
    elif vcov == "HC1":
        x = Xd[1:]
        V = Vb @ _allreduce((x * r * r) @ x.T) @ Vb * (n_obs / df_resid)
    else:
        C = int(levels[cluster_fe])
        sc = _allreduce(_gsum(Xd[1:] * r, cl, C))
        ncl = int((_allreduce(np.bincount(cl, minlength=C).astype(np.int64)) > 0).sum())
        V = Vb @ (sc.T @ sc) @ Vb * (ncl / (ncl - 1)) * ((n_obs - 1) / df_resid)
    se = np.sqrt(np.maximum(np.diag(V), 0.0))
    return dict(beta=beta_full[1:], se=se, iterations=it, n_obs=n_obs, df_resid=df_resid, fe_dims=fe_dims,
                n_clusters=ncl, rows=int(own.sum()))


@pytest.mark.parametrize("n,k,levels,vcov,cluster_fe", [
    (20_000, 3, (400, 30), "HC1", None),
    (18_000, 2, (300, 25, 6), "cluster", 1),
    (16_000, 2, (40, 350, 12), "iid", None),  # the primary FE is not the first
])
def test_owner_schedule_matches_oracle(n, k, levels, vcov, cluster_fe):
    from oracle import altproj

    seed = 11
    out = _run(_owner_fit, n, k, list(levels), seed, vcov, cluster_fe)
    full = synth.panel(n, k, list(levels), seed=seed)
    xs = [f"x{j + 1}" for j in range(k)]
    fes = [f"fe{f + 1}" for f in range(len(levels))]
    cl = [fes[cluster_fe]] if cluster_fe is not None else None
    o = altproj.fit(full, "y", xs, fes, vcov=vcov, cluster_cols=cl)
    assert sum(out[r]["rows"] for r in range(WORLD)) == n  # the level ranges partition the rows
    for r in range(WORLD):
        res = out[r]
        np.testing.assert_allclose(res["beta"], o["beta"], rtol=1e-10, atol=1e-13)
        np.testing.assert_allclose(res["se"], o["se"], rtol=1e-10, atol=1e-14)
        assert res["iterations"] == o["iterations"]
        assert (res["n_obs"], res["df_resid"]) == (o["n_obs"], o["df_resid"])
        assert list(res["fe_dims"]) == list(o["fe_dims"])
        if cluster_fe is not None:
            assert res["n_clusters"] == o["n_clusters"]
    np.testing.assert_array_equal(out[0]["beta"], out[1]["beta"])

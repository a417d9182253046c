"""Multi-GPU plumbing: one process per GPU, rows sharded, RCCL inside the engine.

The engine (``liblfe_hip.so``) owns its RCCL communicator and issues every
collective on its own stream (include/leanfe_hip.h: ``lfe_ctx_set_comm``).
torch.distributed is only used here to ship the RCCL unique id from rank 0 to
the other ranks and for host-side barriers / reductions around timed regions
(any backend; ``gloo`` is enough, no GPU tensors are involved).

Data-parallel contract: each rank loads a contiguous block of
rows; FE and cluster codes are *global* (the same level ids on every rank, e.g.
factorized before sharding); every result (counts, fe_dims, iterations, beta,
SE) is the global one and identical on all ranks.
"""
from __future__ import annotations

import os


def env_world() -> tuple[int, int, int]:
    """(rank, world, local_rank) from the torchrun environment (1 process: 0, 1, 0)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous row block [lo, hi) of rank ``rank`` (sizes differ by at most one)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    q, r = divmod(int(n), world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def owner_range(n_levels: int, rank: int, world: int, align: int = 1) -> tuple[int, int]:
    """Contiguous level range [lo, hi) of FE codes owned by ``rank`` for owner-sharded rows
    (lfe_ctx_set_owner): equal shares of the levels (rows balance when levels are equally
    populated), optionally on multiples of ``align`` (e.g. the engine's 512-level bucket, so no
    bucket spans two ranks; at 1e5 levels over 8 ranks that costs 2.4 % balance, so off)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    G = int(n_levels)
    if align > 1 and G >= align * world:
        units = -(-G // align)
        lo, hi = shard_range(units, rank, world)
        return min(lo * align, G), min(hi * align, G)
    return shard_range(G, rank, world)


def attach(engine, group=None) -> None:
    """Join ``engine`` to an RCCL communicator spanning the ranks of ``group``.

    Rank 0 creates the unique id (``lfe_comm_unique_id``), torch.distributed
    broadcasts it, every rank calls ``lfe_ctx_set_comm(uid, rank, world)``.
    A 1-rank group detaches (world 1: no collectives)."""
    import torch.distributed as dist

    if not dist.is_initialized():
        raise RuntimeError("torch.distributed is not initialized")
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if world == 1:
        engine.set_comm(None, 0, 1)
        engine.dist_group = None
        return
    obj = [type(engine).unique_id() if rank == 0 else None]
    src = dist.get_global_rank(group, 0) if group is not None else 0
    dist.broadcast_object_list(obj, src=src, group=group)
    engine.set_comm(obj[0], rank, world)
    engine.dist_group = (group,)


def is_sharded(engine) -> bool:
    """True when ``engine`` was joined to a multi-rank group by ``attach``."""
    return getattr(engine, "dist_group", None) is not None


def agree_levels(engine, levels: list[int]) -> list[int]:
    """Level counts every rank uses: the max over the ranks of ``engine``'s group.

    Codes are global, but a shard may not contain a group's largest code; the
    engine's group tables (and their all-reduces) must have the same size on
    every rank."""
    if not is_sharded(engine) or not levels:
        return list(levels)
    if engine.dist_group[0] == "local":  # contexts of one process (EmuGroup): a host all-gather
        _, group, rank = engine.dist_group
        return [max(v) for v in zip(*group.exchange(rank, [int(g) for g in levels]))]
    import torch
    import torch.distributed as dist

    t = torch.tensor([int(g) for g in levels], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=engine.dist_group[0])
    return [int(g) for g in t.tolist()]


def agree_categories(engine, cats):
    """The sorted union over the ranks of ``engine``'s group of each rank's categories of a factor
    column (a row shard may miss some): every rank then expands ``i(var)`` / ``var:i(f)`` into the
    same dummy columns, in the same order (polars_impl.py:27-115 on the whole column)."""
    import numpy as np

    cats = np.unique(np.asarray(cats))
    if not is_sharded(engine):
        return cats
    if engine.dist_group[0] == "local":
        _, group, rank = engine.dist_group
        return np.unique(np.concatenate(group.exchange(rank, cats)))
    import torch.distributed as dist

    group = engine.dist_group[0]
    parts = [None] * dist.get_world_size(group)
    dist.all_gather_object(parts, cats.tolist(), group=group)
    return np.unique(np.concatenate([np.asarray(p_, dtype=cats.dtype) for p_ in parts]))


class HostGroup:
    """Host-side helpers for a timed multi-rank run (barrier, max / sum over ranks,
    byte broadcast) on top of torch.distributed; no-ops for a single process."""

    def __init__(self, backend: str = "gloo"):
        self.rank, self.world, self.local = env_world()
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist

            if os.environ.get("MASTER_ADDR", "127.0.0.1") in ("127.0.0.1", "localhost"):
                # every rank on this node: gloo's pairs and RCCL's bootstrap (the engine's
                # communicator; its data moves over xGMI peer links) over loopback, not over
                # whatever interface the container's hostname may (not) resolve to
                if backend == "gloo":
                    os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
                os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
            if not dist.is_initialized():
                dist.init_process_group(backend)
            self.dist = dist

    def barrier(self) -> None:
        if self.dist is not None:
            self.dist.barrier()

    def bcast_bytes(self, b: bytes | None) -> bytes | None:
        if self.dist is None:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def _reduce(self, v: float, op) -> float:
        import torch

        t = torch.tensor([float(v)], dtype=torch.float64)
        self.dist.all_reduce(t, op=op)
        return float(t.item())

    def max(self, v: float) -> float:
        return v if self.dist is None else self._reduce(v, self.dist.ReduceOp.MAX)

    def sum(self, v: float) -> float:
        return v if self.dist is None else self._reduce(v, self.dist.ReduceOp.SUM)

    def close(self) -> None:
        if self.dist is not None:
            self.dist.destroy_process_group()
            self.dist = None

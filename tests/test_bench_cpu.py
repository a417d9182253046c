"""bench.py's host side on CPU: the rank launcher (``--gpus N`` without torchrun spawns N
processes with torchrun's environment, before any GPU call), the workload presets and
labels, and the owner-sharding level ranges (leanfe_amd.dist.owner_range)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from leanfe_amd.dist import owner_range, shard_range  # noqa: E402


def test_rank_envs_are_torchrun_style():
    envs = bench.rank_envs(4, 29555, base={"PATH": "/bin"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert {e["WORLD_SIZE"] for e in envs} == {"4"}
    assert {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert {e["MASTER_PORT"] for e in envs} == {"29555"}
    assert all(e["PATH"] == "/bin" for e in envs)


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_spawns_n_ranks(n):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--print-rank-env"],
                         capture_output=True, text=True, timeout=120, env=env, check=True)
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert sorted(int(x["RANK"]) for x in lines) == list(range(n))
    assert sorted(int(x["LOCAL_RANK"]) for x in lines) == list(range(n))
    assert {x["WORLD_SIZE"] for x in lines} == {str(n)}
    assert {x["MASTER_ADDR"] for x in lines} == {"127.0.0.1"}


def test_launcher_propagates_failure():
    # a failing rank fails the launcher (here: WORLD_SIZE mismatch is impossible, so use a bad flag)
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "3",
                        "--print-rank-env", "--scaling", "nope"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0


def test_presets_and_labels():
    a = bench.parse([])
    assert (a.rows, a.k, a.levels, a.vcov) == (50_000_000, 10, [100_000, 1_000], "HC1")
    assert bench.is_headline(a)
    assert "50M rows total" in bench.workload_label(a, 1)
    a4 = bench.parse(["--config", "4"])
    assert a4.levels == [1_000_000, 100_000, 10_000] and a4.cl == [1, 2] and a4.vcov == "cluster"
    assert not bench.is_headline(a4)
    assert "clustered SE on fe2 x fe3" in bench.workload_label(a4, 1)
    a5 = bench.parse(["--config", "5", "--scaling", "weak"])
    assert a5.rows == 500_000_000 and not bench.is_headline(a5)
    assert "per GPU" in bench.workload_label(a5, 8)
    a1 = bench.parse(["--config", "1"])
    assert (a1.rows, a1.k, a1.levels, a1.vcov) == (1_000_000, 3, [20_000, 500], "iid")


def test_step_byte_model_covers_the_headline_kernels():
    ab = bench.algorithmic_bytes(50_000_000, 11, 2)
    for k in ("part_scatter", "group_sums", "gram_resid", "tp", "tq", "layout_scatter", "layout_hist"):
        assert ab[k] > 0
    assert ab["part_scatter"] == 50_000_000 * (16 * 11 + 8 * 2)


def test_step_byte_model_of_the_dense_cross_terms():
    """With the count tables (lfe_dense.hip) the table build reads both codes and writes two uint16
    tables, each cross-term pass reads one table, and the layout bases are gone."""
    n, cells = 50_000_000, 196 * 512 * 1008
    rows = bench.algorithmic_bytes(n, 11, 2)
    dense = bench.algorithmic_bytes(n, 11, 2, dense_cells=cells)
    assert dense["tp"] == dense["tq"] == 2 * cells
    assert dense["layout_scatter"] == 8 * n + 4 * cells and dense["layout_base"] == 0
    assert dense["part_scatter"] == rows["part_scatter"] and dense["gram_resid"] == rows["gram_resid"]


@pytest.mark.parametrize("G,world", [(100_000, 1), (100_000, 2), (100_000, 8), (1000, 8), (7, 3), (40_000, 8)])
def test_owner_range_partitions_levels(G, world):
    parts = [owner_range(G, r, world) for r in range(world)]
    assert parts[0][0] == 0 and parts[-1][1] == G
    assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
    sizes = [hi - lo for lo, hi in parts]
    assert max(sizes) - min(sizes) <= 1  # equal shares of the levels
    aligned = [owner_range(G, r, world, align=512) for r in range(world)]
    assert aligned[0][0] == 0 and aligned[-1][1] == G
    if G >= 512 * world:  # bucket-aligned: no primary-FE bucket spans two ranks
        assert all(lo % 512 == 0 for lo, _ in aligned)
    with pytest.raises(ValueError):
        owner_range(G, world, world)


def test_strong_split_covers_rows():
    n = 50_000_000
    for world in (1, 2, 4, 8):
        parts = [shard_range(n, r, world) for r in range(world)]
        assert sum(hi - lo for lo, hi in parts) == n

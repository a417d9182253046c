"""BASELINE.json configs at full size through the exact code path bench.py times
(``bench.solve_step``), checked against the C restatement of the reference
(oracle/altproj_c.c): beta, SE (IID / HC1 / two-way CGM clustered), iterations, n_obs,
df_resid and cluster counts.  Prints one JSON line per config.

    python tools/config_runs.py [--configs 1,2,3,4] [--rows N]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from leanfe_amd import synth  # noqa: E402
from leanfe_amd._lib import Engine  # noqa: E402
from oracle.altproj_c import default_threads, fit_c  # noqa: E402


def rel(a, b) -> float:
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300))) if a.size else 0.0


def _args(cfg, rows):
    """A BASELINE config number or the name of one of the reference's panels (bench.PRESETS)."""
    sel = ["--preset", cfg] if isinstance(cfg, str) else ["--config", str(cfg)]
    return bench.parse(sel + (["--rows", str(rows)] if rows else []))


def run(cfg: int | str, rows: int | None = None, repeat: int = 2) -> dict:
    a = _args(cfg, rows)
    eng = Engine(0)
    eng.synth_load(a.rows, a.k, a.levels, synth.betas(a.k), seed=a.seed)
    n_cl = len(a.cl) if a.cl else 0
    cols, codes = eng.copy_inputs()
    if n_cl:
        eng.load_clusters([np.ascontiguousarray(codes[f]) for f in a.cl], [a.levels[f] for f in a.cl])
    res = [bench.solve_step(eng, a.vcov, n_cl) for _ in range(repeat)]  # warm-up + a repeat
    eng.profile(True)
    t0 = time.perf_counter()
    r = bench.solve_step(eng, a.vcov, n_cl)
    eng.sync()
    gpu_s = time.perf_counter() - t0
    kst = eng.kernel_stats()
    eng.profile(False)
    eng.close()
    line = dict(config=cfg, rows=a.rows, k=a.k, levels=a.levels, vcov=a.vcov, cluster_fes=a.cl,
                iterations=r["iterations"], n_obs=r["n_obs"], df_resid=r["df_resid"], gpu_seconds=round(gpu_s, 4),
                mrows_s=round(a.rows / gpu_s / 1e6, 1), beta_dev_vs_host=r["beta_dev_vs_host"],
                kernels_ms={k: [round(v[0], 3), v[1]] for k, v in kst.items()},
                repeat_bit_identical=all(np.array_equal(x["beta"], r["beta"]) and np.array_equal(x["se"], r["se"])
                                         and x["iterations"] == r["iterations"] for x in res))
    threads = default_threads()
    print(f"[config {cfg}] GPU step {gpu_s:.3f} s; C oracle on {threads} threads ...", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    o = fit_c(list(cols), list(codes), a.levels, vcov=a.vcov, threads=threads,
              cl_codes=[codes[f] for f in a.cl] if n_cl else None,
              cl_levels=[a.levels[f] for f in a.cl] if n_cl else None)
    line["cpu_seconds"] = round(time.perf_counter() - t0, 3)
    line["cpu_threads"] = threads
    line["cpu_iterations"] = o["iterations"]
    line["max_rel_beta"] = rel(r["beta"], o["beta"])
    line["max_rel_se"] = rel(r["se"], o["se"])
    line["ints_equal"] = (r["iterations"] == o["iterations"] and r["n_obs"] == o["n_obs"]
                          and r["df_resid"] == o["df_resid"])
    if n_cl:
        line["n_clusters"] = list(r["n_clusters"]) if n_cl > 1 else r["n_clusters"]
        line["cpu_n_clusters"] = list(o["n_clusters"]) if n_cl > 1 else o["n_clusters"]
        line["cpu_G_subsets"] = o["G_subsets"]
        line["n_clusters_equal"] = line["n_clusters"] == line["cpu_n_clusters"]
    print(json.dumps(line), flush=True)
    return line


def _same_fit(x: dict, y: dict) -> bool:
    return (x["iterations"] == y["iterations"] and x["n_obs"] == y["n_obs"] and np.array_equal(x["beta"], y["beta"])
            and np.array_equal(x["se"], y["se"]))


def run_multirank(cfg: int, combos=(("owner", 2), ("owner", 4), ("owner", 8)), rows: int | None = None) -> list[dict]:
    """The config through the engine's multi-rank code: ``world`` contexts on one GPU joined in an
    emulated group (EmuGroup: the collective calls of RCCL, in the same order, reduced through host
    memory), each holding its shard of the panel (``owner``: every row of a range of primary-FE
    levels, as bench.py --shard owner; ``rows``: contiguous row blocks) and running
    ``bench.solve_step`` twice.  Every rank is compared with the C oracle on the whole panel, with
    rank 0 (bit-identical) and with its own repeat (bit-identical)."""
    import threading

    from leanfe_amd import dist
    from leanfe_amd._lib import EmuGroup

    a = _args(cfg, rows)
    n_cl = len(a.cl) if a.cl else 0
    eng = Engine(0)
    eng.synth_load(a.rows, a.k, a.levels, synth.betas(a.k), seed=a.seed)
    cols, codes = eng.copy_inputs()
    eng.close()
    threads = default_threads()
    t0 = time.perf_counter()
    o = fit_c(list(cols), list(codes), a.levels, vcov=a.vcov, threads=threads,
              cl_codes=[codes[f] for f in a.cl] if n_cl else None,
              cl_levels=[a.levels[f] for f in a.cl] if n_cl else None)
    cpu_s = time.perf_counter() - t0
    del cols, codes
    P = max(range(len(a.levels)), key=lambda f: a.levels[f])
    lines = []
    for shard, world in combos:
        group = EmuGroup(world)
        out, errs = {}, {}

        def worker(rank):
            try:
                e = Engine(0)
                e.set_emu(group, rank)
                if shard == "owner":
                    lo, hi = dist.owner_range(a.levels[P], rank, world)
                    e.synth_load_owned(a.rows, a.k, a.levels, synth.betas(a.k), P, lo, hi, seed=a.seed)
                else:
                    lo, hi = dist.shard_range(a.rows, rank, world)
                    e.synth_load(hi - lo, a.k, a.levels, synth.betas(a.k), seed=a.seed, row_offset=lo)
                if n_cl:
                    _, cd = e.copy_inputs()
                    e.load_clusters([np.ascontiguousarray(cd[f]) for f in a.cl], [a.levels[f] for f in a.cl])
                first = bench.solve_step(e, a.vcov, n_cl)
                e.sync()
                t = time.perf_counter()
                second = bench.solve_step(e, a.vcov, n_cl)
                e.sync()
                out[rank] = dict(first=first, second=second, rows=e.n, seconds=time.perf_counter() - t)
                e.close()
            except BaseException as ex:  # noqa: BLE001
                errs[rank] = ex

        ths = [threading.Thread(target=worker, args=(r,)) for r in range(world)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(timeout=600)
        if any(t.is_alive() for t in ths):
            raise RuntimeError(f"emulated group of {world} deadlocked")
        if errs:
            raise next(iter(errs.values()))
        r0 = out[0]["first"]
        line = dict(config=cfg, rows=a.rows, world=world, shard=shard, k=a.k, levels=a.levels, vcov=a.vcov,
                    rows_per_rank=[out[r]["rows"] for r in range(world)],
                    iterations=r0["iterations"], cpu_iterations=o["iterations"], cpu_seconds=round(cpu_s, 2),
                    emulated_solve_seconds_max=round(max(out[r]["seconds"] for r in range(world)), 4),
                    max_rel_beta=max(rel(out[r]["first"]["beta"], o["beta"]) for r in range(world)),
                    max_rel_se=max(rel(out[r]["first"]["se"], o["se"]) for r in range(world)),
                    ints_equal=all(out[r]["first"]["iterations"] == o["iterations"]
                                   and out[r]["first"]["n_obs"] == o["n_obs"]
                                   and out[r]["first"]["df_resid"] == o["df_resid"] for r in range(world)),
                    ranks_bit_identical=all(_same_fit(out[r]["first"], r0) for r in range(world)),
                    repeat_bit_identical=all(_same_fit(out[r]["first"], out[r]["second"]) for r in range(world)),
                    beta_dev_vs_host=max(out[r]["first"]["beta_dev_vs_host"] for r in range(world)))
        assert sum(line["rows_per_rank"]) == a.rows, line
        print(json.dumps(line), flush=True)
        lines.append(line)
    return lines


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1,2,3,4", help="config numbers and / or bench.PRESETS names")
    ap.add_argument("--rows", type=int, default=None, help="override the config's row count")
    ap.add_argument("--worlds", default=None, help="emulated multi-rank groups instead, e.g. 2,4,8")
    ap.add_argument("--shards", default="owner", help="owner and/or rows")
    a = ap.parse_args()
    for c in [int(x) if x.isdigit() else x for x in a.configs.split(",")]:
        if a.worlds:
            run_multirank(c, [(sh, int(w)) for sh in a.shards.split(",") for w in a.worlds.split(",")], a.rows)
        else:
            run(c, a.rows)


if __name__ == "__main__":
    main()

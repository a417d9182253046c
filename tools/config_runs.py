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


def run(cfg: int, rows: int | None = None, repeat: int = 2) -> dict:
    a = bench.parse(["--config", str(cfg)] + (["--rows", str(rows)] if rows else []))
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1,2,3,4")
    ap.add_argument("--rows", type=int, default=None, help="override the config's row count")
    a = ap.parse_args()
    for c in [int(x) for x in a.configs.split(",")]:
        run(c, a.rows)


if __name__ == "__main__":
    main()

"""Run BASELINE.json configs 2 and 4 at full size through the engine and check them
against the C restatement (oracle/altproj_c.c: beta, IID/HC1 SE, iterations, n_obs,
df_resid).  Config 4's two-way clustered SE (fe2 x fe3, CGM) has no full-size CPU
reference; it is checked for consistency (cluster counts vs host distinct counts,
finite positive SEs).  Prints one JSON line per config.

    python tools/config_runs.py [--configs 2,4] [--rows4 50000000]
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

from leanfe_amd import inference, synth  # noqa: E402
from leanfe_amd._lib import Engine  # noqa: E402
from oracle.altproj_c import fit_c  # noqa: E402


def solve(eng, vcov, cl_levels=None):
    t0 = time.perf_counter()
    n_obs, dims, card = eng.drop_singletons()
    order = sorted(range(len(card)), key=lambda i: card[i])
    iterations, _ = eng.demean(order, 1e-6, 50, check_from=3)
    G = eng.gram()
    XtX, Xty = inference.split_gram(G)
    beta_full, XtX_inv = inference.solve_normal(XtX, Xty)
    k = XtX.shape[0] - 1
    df = n_obs - (k + 1) - (sum(dims) - len(dims))
    v = vcov.lower()
    stats = inference.stats_from_gram(G, beta_full) if v == "iid" else None  # as leanfe_hip: no residual pass
    meat = None
    if stats is None:
        stats, meat = eng.resid(beta_full, hc1=v == "hc1", keep_scores=v == "cluster")
    out = dict(n_obs=n_obs, iterations=iterations, beta=beta_full[1:], df_resid=df, fe_dims=list(dims))
    if v == "hc1":
        out["se"] = inference.se_hc1(XtX_inv[1:, 1:], meat, n_obs, df)
    elif v == "iid":
        out["se"] = inference.se_iid(XtX_inv[1:, 1:], stats[0], df)
    else:
        subsets = inference.cluster_subsets(len(cl_levels))
        meats, Gs = eng.cluster_meat_subsets(subsets)  # intersections formed on the device
        out["se"], _ = inference.se_cluster_multiway(XtX_inv[1:, 1:], list(meats), [int(g) for g in Gs], subsets,
                                                     n_obs, df, True)
        out["G"] = [int(g) for g in Gs]
    out["seconds"] = time.perf_counter() - t0
    return out


def run(cfg, n, k, levels, vcov, cluster_fes=None, threads=16):
    eng = Engine(0)
    eng.synth_load(n, k, levels, synth.betas(k), seed=12345)
    cl_levels = None
    if cluster_fes:
        cols, codes = eng.copy_inputs()
        # first-order cluster columns; the CGM intersections are formed on the device
        cl_levels = [levels[f] for f in cluster_fes]
        eng.load_clusters([np.ascontiguousarray(codes[f]) for f in cluster_fes], cl_levels)
    solve(eng, vcov, cl_levels)  # warm-up
    eng.profile(True)
    r = solve(eng, vcov, cl_levels)
    kst = eng.kernel_stats()
    eng.profile(False)
    line = dict(config=cfg, rows=n, k=k, levels=levels, vcov=vcov, iterations=r["iterations"], n_obs=r["n_obs"],
                seconds=round(r["seconds"], 4), mrows_s=round(n / r["seconds"] / 1e6, 1),
                kernels_ms={k_: [round(v[0], 3), v[1]] for k_, v in kst.items()})
    cols, codes = eng.copy_inputs()
    oracle_vcov = "iid" if vcov == "cluster" else vcov
    if vcov == "cluster":  # compare beta and the HC1 SE of the same fit with the C restatement
        r_h = solve(eng, "HC1")
        r["se_hc1"] = r_h["se"]
    t0 = time.perf_counter()
    o = fit_c(list(cols), list(codes), levels, vcov="hc1" if vcov == "cluster" else oracle_vcov, threads=threads)
    line["cpu_seconds"] = round(time.perf_counter() - t0, 3)
    line["cpu_iterations"] = o["iterations"]
    line["max_rel_beta"] = float(np.max(np.abs(r["beta"] - o["beta"]) / np.abs(o["beta"])))
    se_gpu = r["se_hc1"] if vcov == "cluster" else r["se"]
    line["max_rel_se"] = float(np.max(np.abs(se_gpu - o["se"]) / np.abs(o["se"])))
    line["ints_equal"] = (r["iterations"] == o["iterations"] and r["n_obs"] == o["n_obs"]
                          and r["df_resid"] == o["df_resid"])
    if vcov == "cluster":
        line["cluster_G"] = r["G"]
        line["cluster_se_finite_positive"] = bool(np.all(np.isfinite(r["se"])) and np.all(r["se"] > 0))
        line["cluster_se"] = [float(x) for x in r["se"]]
    eng.close()
    print(json.dumps(line), flush=True)
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="2,4")
    ap.add_argument("--rows4", type=int, default=50_000_000)
    ap.add_argument("--rows5", type=int, default=500_000_000)
    a = ap.parse_args()
    for c in [int(x) for x in a.configs.split(",")]:
        if c == 2:
            run(2, 10_000_000, 5, [100_000, 1_000], "iid")
        elif c == 5:  # config 5 on one GPU (D = 1: 44 GB of columns fit in 288 GB)
            run(5, a.rows5, 10, [100_000, 1_000], "iid")
        elif c == 4:
            run(4, a.rows4, 10, [1_000_000, 100_000, 10_000], "cluster", cluster_fes=[1, 2])


if __name__ == "__main__":
    main()

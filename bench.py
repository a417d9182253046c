#!/usr/bin/env python
"""Headline benchmark: Mrows/s of demean + solve at 50M rows x 2 HDFE.

Workload (BASELINE.json configs[2]): synthetic counter-based panel
(leanfe_amd/synth.py, seed 12345), N = 5e7 rows per GPU, k = 10 regressors,
FEs with 1e5 and 1e3 levels, vcov = HC1.  One "step" = one full regression on
device-resident inputs exactly as ``leanfe_hip`` runs it after the data
hand-off: singleton drop -> alternating projections to convergence
(tol 1e-6, max_iter 50, check from it=3) -> Gram (MFMA) -> host Cholesky ->
residual + HC1 meat -> SEs.

Multi-GPU (``torchrun --nproc-per-node N bench.py --gpus N``): one process per
GPU, rows sharded (rank r generates rows [r*N, (r+1)*N) of the same panel,
weak scaling), every per-group partial sum / Gram / meat all-reduced with RCCL
inside the engine.  Timing: W warm-up steps, then barrier + device sync, K
timed steps, device sync + barrier; the max over ranks is reported.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from leanfe_amd import inference, synth  # noqa: E402
from leanfe_amd._lib import Engine  # noqa: E402
from leanfe_amd.dist import HostGroup  # noqa: E402

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10, help="untimed steps (GPU clocks settle within ~0.1 s)")
    ap.add_argument("--rows", type=int, default=50_000_000, help="rows per GPU")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--levels", type=str, default="100000,1000")
    ap.add_argument("--vcov", type=str, default="HC1")
    ap.add_argument("--seed", type=int, default=12345)
    ap.add_argument("--cpu-rows", type=int, default=50_000_000, help="CPU baseline sample (prefix rows)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-prof", action="store_true", help="diagnostic: no per-kernel events (no roofline)")
    ap.add_argument("--verbose", action="store_true")
    return ap.parse_args()


def device_sync(eng: Engine):
    eng.sync()
    torch = sys.modules.get("torch")  # only when already imported (multi-GPU runs)
    if torch is not None and torch.cuda.is_available():
        torch.cuda.synchronize()


def solve_step(eng: Engine, vcov: str):
    """One regression on device-resident data (the hip backend's hot path)."""
    n_obs, dims, card = eng.drop_singletons()
    order = sorted(range(len(card)), key=lambda i: card[i])
    iterations, _ = eng.demean(order, 1e-6, 50, check_from=3)
    hc1 = vcov.lower() == "hc1"
    # HC1: Gram + device solve + residual pass, one round trip; IID: the Gram alone
    fused = eng.gram_resid(hc1=hc1) if hc1 else None
    G = fused[0] if fused is not None else eng.gram()
    XtX, Xty = inference.split_gram(G)
    beta_full, XtX_inv = inference.solve_normal(XtX, Xty)
    k = XtX.shape[0] - 1
    df_resid = n_obs - (k + 1) - (sum(dims) - len(dims))
    stats, meat = (fused[2], fused[3]) if fused is not None else (inference.stats_from_gram(G, beta_full), None)
    if stats is None:
        stats, meat = eng.resid(beta_full, hc1=hc1)
    if vcov.lower() == "hc1":
        se = inference.se_hc1(XtX_inv[1:, 1:], meat, n_obs, df_resid)
    else:
        se = inference.se_iid(XtX_inv[1:, 1:], stats[0], df_resid)
    return dict(n_obs=n_obs, iterations=iterations, beta=beta_full[1:], se=se, df_resid=df_resid)


def algorithmic_bytes(n: int, p: int, F: int, T: int, hc1: bool) -> dict:
    """HBM bytes each kernel must move per launch (DESIGN.md "Kernels and their rooflines").

    n rows/GPU, p = 1 + k data columns (f64), F fixed effects (int32 codes).  The
    layout passes scan every row of the shard (dropped rows included).
    """
    return {
        "part_hist": 4 * n,                              # primary codes
        "part_scatter": n * (2 * 8 * p + 2 * 4 * F),      # read + write X and codes
        "count": 4 * n,                                  # one code column per launch
        "mark": 4 * n * F,                               # every code column (+ sparse writes)
        "group_sums": n * (8 * p + 4 * F),               # X + codes
        "cross": 4 * n,                                  # secondary codes in segment order
        "gram_design": n * (8 * p + 4 * F),              # X + codes
        "gram_resid": n * (8 * p + 4 * F),               # X + codes (HC1: no score write)
    }


PMC_TRAFFIC = os.path.join(ROOT, "profiles", "r01", "pmc_traffic.json")


def pmc_traffic(kernel: str, args, levels) -> float | None:
    """HBM bytes per launch of `kernel` measured with rocprofv3 PMC counters
    (tools/pmc.sh + tools/pmc_traffic.py: 2 x FETCH_SIZE + WRITE_SIZE, the gfx950
    correction of MI355X_MICROARCH.md) for this exact configuration, else None."""
    try:
        with open(PMC_TRAFFIC) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    cfg = {"rows": args.rows, "k": args.k, "levels": list(levels), "vcov": args.vcov}
    if t.get("config") != cfg or kernel not in t.get("kernels", {}):
        return None
    return float(t["kernels"][kernel]["bytes_per_launch"])


def cpu_baseline(args, levels, eng: Engine) -> dict:
    """CPU baseline: the C restatement of the reference alt_proj path (oracle/altproj_c.c,
    OpenMP over columns) on the host cores, over the first ``--cpu-rows`` rows of the very
    panel the GPU solved (copied back from the device)."""
    from oracle.altproj_c import fit_c

    threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", "16")), os.cpu_count() or 1, 16))
    cols, codes = eng.copy_inputs()
    n = min(args.cpu_rows, cols.shape[1])
    t0 = time.perf_counter()
    r = fit_c([c[:n] for c in cols], [c[:n] for c in codes], levels, vcov=args.vcov, threads=threads)
    dt = time.perf_counter() - t0
    whole = "the whole" if n == cols.shape[1] else f"the first {n:_} rows of the"
    return dict(value=n / dt / 1e6, unit="Mrows/s", cores=threads, kind="port",
                sample=f"{whole} {cols.shape[1]:_}-row panel (k={args.k}, levels={levels}, vcov={args.vcov}); "
                       f"oracle/altproj_c.c (C restatement of polars_impl.py alt_proj), {threads} OpenMP threads, "
                       f"{dt:.2f} s, iterations={r['iterations']}",
                iterations=int(r["iterations"]), seconds=round(dt, 3))


def main():
    args = parse()
    levels = [int(x) for x in args.levels.split(",")]
    d = HostGroup()
    eng = Engine(d.local)
    if d.world > 1:
        uid = Engine.unique_id() if d.rank == 0 else None
        uid = d.bcast_bytes(uid)
        eng.set_comm(uid, d.rank, d.world)
    beta = synth.betas(args.k)
    t0 = time.perf_counter()
    eng.synth_load(args.rows, args.k, levels, beta, seed=args.seed, row_offset=d.rank * args.rows)
    gen_s = time.perf_counter() - t0

    for _ in range(args.warmup):
        solve_step(eng, args.vcov)

    d.barrier()
    device_sync(eng)
    eng.profile(not args.no_prof)
    t0 = time.perf_counter()
    res = None
    for _ in range(args.steps):
        res = solve_step(eng, args.vcov)
    device_sync(eng)
    t1 = time.perf_counter()
    d.barrier()
    elapsed = d.max(t1 - t0)
    kstats = eng.kernel_stats()
    eng.profile(False)

    total_rows = args.rows * d.world
    value = total_rows * args.steps / elapsed / 1e6
    p = args.k + 1
    F = len(levels)
    T = res["iterations"]
    ab = algorithmic_bytes(args.rows, p, F, T, args.vcov.lower() == "hc1")
    # dominant kernel = most device time in the timed region
    dom = max(kstats.items(), key=lambda kv: kv[1][0]) if kstats else ("none", (0.0, 1))
    dom_name, (dom_ms, dom_launches) = dom
    per_launch_s = dom_ms / 1e3 / max(dom_launches, 1)
    dom_bytes = ab.get(dom_name)
    roofline = None
    if dom_bytes:
        achieved = dom_bytes / per_launch_s / 1e9
        roofline = {"bound": "hbm", "kernel": dom_name, "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS,
                    "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4),
                    "traffic": pmc_traffic(dom_name, args, levels),
                    "bytes_per_launch": dom_bytes, "avg_launch_ms": round(per_launch_s * 1e3, 4)}
        if roofline["traffic"] is not None:
            roofline["traffic_source"] = os.path.relpath(PMC_TRAFFIC, ROOT) + " (rocprofv3 PMC, same config)"
    cpu = None
    if d.rank == 0 and d.world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args, levels, eng)
    if d.rank == 0:
        line = {
            "metric": "Mrows/sec demean+solve, 50M x 2-HDFE (1e5/1e3 levels), k=10, HC1",
            "value": round(value, 2),
            "unit": "Mrows/s",
            "n_gpus": d.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (counter-based splitmix64 panel generated on device, seed 12345)",
            "config": {"workload": "configs[2]: 50M rows/GPU, 2 FE (1e5, 1e3 levels), k=10, HC1 SE",
                       "rows_per_gpu": args.rows, "total_rows": total_rows, "k": args.k, "levels": levels,
                       "vcov": args.vcov, "iterations": T, "parallelism": f"row-shard dp{d.world}"},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "kernels_ms": {k: [round(v[0] / args.steps, 4), v[1] // args.steps] for k, v in kstats.items()},
            "gen_s": round(gen_s, 3),
        }
        if args.verbose:
            line["beta"] = [float(x) for x in res["beta"]]
            line["se"] = [float(x) for x in res["se"]]
        print(json.dumps(line))
    eng.close()
    d.close()


if __name__ == "__main__":
    main()

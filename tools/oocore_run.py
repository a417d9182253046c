"""Out-of-core X at a size whose resident layout does not fit one MI355X.

    python tools/oocore_run.py --rows 2100000000 --k 10 --levels 100000,1000 --chunk 50000000
    python tools/oocore_run.py --rows 3000000000 --contexts 2 --chunk 50000000 --chunk2 70000000

The synthetic panel of bench.py (counter-based, seed 12345) with only the FE codes resident;
the columns are generated chunk by chunk on the device and streamed through pass 1 (group sums
+ raw Gram), the codes-only sweeps, the Gram from the tables and pass 2 (residual + HC1 meat).
Checks printed with the timing: the fit is the same under a second chunking (--chunk2), and
beta lies within a few SEs of the generating coefficients.  One JSON line on stdout.
``--contexts S``: the rows in S contexts of < 2^31 rows each on the device (rows [row0, row0 + n_r)
of the panel per context, lfe_synth_load_codes_at), joined in one in-process group (EmuGroup), as
hip_impl._out_of_core_split runs a fit of more rows than one context holds.
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


def fit(eng, n, k, L, beta, chunk, seed, row0=0):
    from leanfe_amd import inference
    from leanfe_amd._lib import NeedsStreamPass
    t = {}
    t0 = time.perf_counter()
    eng.synth_load_codes(n, k, L, seed=seed, row0=row0)
    eng.sync()
    t["codes_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    n_obs, dims, card = eng.drop_singletons()
    eng.sync()
    t["drop_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    eng.stream_synth_pass(1, k, L, beta, chunk_rows=chunk, seed=seed)
    eng.sync()
    t["pass1_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    it, _ = eng.demean(sorted(range(2), key=lambda i: card[i]), 1e-6, 50, check_from=3)
    try:
        G = eng.gram()
    except NeedsStreamPass:  # several contexts (ranks' raw tiles have their own shifts): the design-Gram pass
        G = eng.stream_synth_pass(3, k, L, beta, chunk_rows=chunk, seed=seed)[:(k + 2) ** 2].reshape(k + 2, k + 2)
    t["demean_gram_s"] = time.perf_counter() - t0
    XtX, Xty = inference.split_gram(G)
    bf, XtX_inv = inference.solve_normal(XtX, Xty)
    t0 = time.perf_counter()
    out = eng.stream_synth_pass(2, k, L, beta, chunk_rows=chunk, seed=seed, beta_full=bf)
    eng.sync()
    t["pass2_s"] = time.perf_counter() - t0
    df = n_obs - (k + 1) - (sum(dims) - 2)
    se = inference.se_hc1(XtX_inv[1:, 1:], out[4:4 + k * k].reshape(k, k), n_obs, df)
    return dict(beta=bf[1:], se=se, iterations=it, n_obs=n_obs, df_resid=df, rss=float(out[1]), t=t)


def fit_contexts(S, rows, k, L, beta, chunk, seed):
    """The fit on S contexts of one device (one thread each, one in-process group): rank 0's result."""
    import threading

    from leanfe_amd import dist
    from leanfe_amd._lib import EmuGroup, Engine
    if S == 1:
        with Engine(0) as eng:
            return fit(eng, rows, k, L, beta, chunk, seed)
    group, out, errs = EmuGroup(S), [None] * S, []

    def work(r):
        lo, hi = dist.shard_range(rows, r, S)
        try:
            with Engine(0) as eng:
                eng.set_emu(group, r)
                out[r] = fit(eng, hi - lo, k, L, beta, chunk, seed, row0=lo)
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            group.abort()

    ts = [threading.Thread(target=work, args=(r,)) for r in range(S)]
    for t_ in ts:
        t_.start()
    for t_ in ts:
        t_.join()
    if errs:
        raise errs[0]
    for r in range(1, S):  # every context returns the same global fit
        assert np.array_equal(out[r]["beta"], out[0]["beta"])
    return out[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_100_000_000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--levels", type=str, default="100000,1000")
    ap.add_argument("--chunk", type=int, default=50_000_000)
    ap.add_argument("--chunk2", type=int, default=0, help="second chunking for the invariance check (0: off)")
    ap.add_argument("--seed", type=int, default=12345)
    ap.add_argument("--contexts", type=int, default=1, help="contexts of < 2^31 rows on the device")
    a = ap.parse_args()
    from leanfe_amd import synth
    L = [int(x) for x in a.levels.split(",")]
    beta = synth.betas(a.k)
    r = fit_contexts(a.contexts, a.rows, a.k, L, beta, a.chunk, a.seed)
    free = total = None
    try:
        import torch
        free, total = torch.cuda.mem_get_info(0)
    except Exception:  # noqa: BLE001 - torch is plumbing only; the figure is optional
        pass
    line = dict(kind="out-of-core X (codes resident, columns streamed in chunks generated on the device)",
                rows=a.rows, contexts=a.contexts, k=a.k, levels=L, chunk_rows=a.chunk, iterations=r["iterations"], n_obs=r["n_obs"],
                x_bytes=a.rows * (a.k + 1) * 8, resident_layout_bytes_estimate=a.rows * (2 * 8 * (a.k + 1) + 30),
                hbm_total=total, hbm_free_after=free, times=r["t"],
                total_s=sum(r["t"].values()), mrows_s=a.rows / sum(r["t"].values()) / 1e6,
                beta=[float(x) for x in r["beta"]], se=[float(x) for x in r["se"]],
                max_abs_t_vs_generating_beta=float(np.max(np.abs((r["beta"] - beta) / r["se"]))))
    if a.chunk2:
        r2 = fit_contexts(a.contexts, a.rows, a.k, L, beta, a.chunk2, a.seed)
        line["chunk2"] = a.chunk2
        line["chunking_max_rel_beta"] = float(np.max(np.abs(r2["beta"] - r["beta"]) / np.abs(r["beta"])))
        line["chunking_max_rel_se"] = float(np.max(np.abs(r2["se"] - r["se"]) / np.abs(r["se"])))
        line["chunking_ints_equal"] = (r2["iterations"], r2["n_obs"], r2["df_resid"]) == (
            r["iterations"], r["n_obs"], r["df_resid"])
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()

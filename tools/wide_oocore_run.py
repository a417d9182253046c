"""A wide streamed fit without a resident design matrix, at a size where D could not be held
(VERDICT r5 item 7).

    python tools/wide_oocore_run.py --rows 1000000000 --k 100 --levels 100000,1000 \
        --chunk 20000000 --chunk2 32000000

The K-regressor synthetic panel (leanfe_amd/synth.py: counter-based, seed 12345) with only the FE
codes resident, in column blocks of engine contexts (block 0 = [y, x1..x62] with the stop test,
block 1 = [x63..xK] with block 0's number of sweeps), every column generated chunk by chunk on the
device (lfe_stream_synth_cols) three times: pass 1 of each block (group sums), pass A (each chunk's
[1_kept, y~, x~] from every block into one chunk buffer, lfe_stream_materialize_rows, then its Gram,
lfe_wide_gram_rows) and pass B (residual, statistics and HC1 meat, lfe_wide_resid_rows).  D of 1e9
rows x 102 columns would be 816 GB; the device holds the blocks' codes and effect tables plus
102 x chunk doubles.  The same steps as hip_impl._wide_fit_chunked with a synthetic source.

Checks printed with the timing: a second chunking (--chunk2) gives the same fit (relative 1e-13,
the chunk-order sums differ only in their grouping), and beta lies within a few SEs of the
generating coefficients.  tests/test_gpu_wide.py runs `wide_fit` at 150K rows against the oracle.
One JSON line on stdout.
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

PER = 63  # columns of one engine context (MAX_CONTEXT_COLS)


def wide_fit(n, K, L, beta, chunk, seed=12345, vcov="HC1", tol=1e-6, max_iter=50, device=0, say=None):
    """A chunked wide fit of y ~ x1..xK | fe1 + .. on rows [0, n) of the synthetic panel."""
    from leanfe_amd import inference
    from leanfe_amd._lib import Engine

    chunk = max(64, chunk // 64 * 64)
    spans, lo = [], 0  # (c_lo, pb): the block's global columns (0 = y, j = x_j)
    while lo < K + 1:
        spans.append((lo, min(PER, K + 1 - lo)))
        lo += spans[-1][1]
    P = K + 2
    t = {}
    engines, Dc, r = [], None, None
    eng = Engine(device)
    engines.append(eng)
    try:
        t0 = time.perf_counter()
        iterations = 0
        for b, (c_lo, pb) in enumerate(spans):
            e = eng if b == 0 else Engine(device)
            if b > 0:
                engines.append(e)
            e.synth_load_codes(n, pb - 1, L, seed=seed)
            n_obs, dims, card = e.drop_singletons()
            e.stream_begin(1)
            for r0 in range(0, n, chunk):
                e.stream_synth_cols(r0, min(chunk, n - r0), K, c_lo, L, beta, seed)
            e.stream_end()
            order = sorted(range(len(L)), key=lambda i: card[i])  # polars_impl.py:485
            if b == 0:
                iterations, _ = e.demean(order, tol, max_iter, check_from=3)
            else:
                e.demean(order, 0.0, iterations, check_from=3)
            e.sync()
            if say:
                say(f"block {b}: columns [{c_lo}, {c_lo + pb}) demeaned, {time.perf_counter() - t0:.1f} s")
        t["blocks_s"] = time.perf_counter() - t0
        df = n_obs - (K + 1) - (sum(dims) - len(L))
        Dc = eng.dev_alloc(P * chunk)
        r = eng.dev_alloc(chunk)
        eng.sync()

        def fill(row0, rows):
            col0 = 1
            for b, (c_lo, pb) in enumerate(spans):
                engines[b].stream_materialize_rows(Dc, chunk, col0, row0, ("synth", rows, K, c_lo, L, beta, seed),
                                                   0 if b == 0 else -1)
                col0 += pb

        t0 = time.perf_counter()
        G = np.zeros((P, P))
        for row0 in range(0, n, chunk):  # pass A
            rows = min(chunk, n - row0)
            fill(row0, rows)
            G += eng.wide_gram_rows(Dc, chunk, row0, rows, 0, P, mode=0)
        t["pass_a_s"] = time.perf_counter() - t0
        XtX, Xty = inference.split_gram(G)
        bf, XtX_inv = inference.solve_normal(XtX, Xty)
        coef = np.concatenate([[-bf[0], 1.0], -bf[1:]])
        t0 = time.perf_counter()
        stats, meat = np.zeros(4), np.zeros((K, K))
        for row0 in range(0, n, chunk):  # pass B
            rows = min(chunk, n - row0)
            fill(row0, rows)
            stats += eng.wide_resid_rows(Dc, chunk, row0, rows, coef, r)
            if vcov == "HC1":
                meat += eng.wide_gram_rows(Dc, chunk, row0, rows, 2, K, mode=3, r=r)
        eng.sync()
        t["pass_b_s"] = time.perf_counter() - t0
        rss_w, rss = stats[0], stats[1]
        if vcov == "HC1":
            se = inference.se_hc1(XtX_inv[1:, 1:], meat, n_obs, df)
        else:
            se = inference.se_iid(XtX_inv[1:, 1:], rss_w, df)
        return dict(beta=bf[1:], se=se, iterations=iterations, n_obs=n_obs, df_resid=df, rss=float(rss), t=t,
                    blocks=len(spans))
    finally:
        for ptr in (Dc, r):
            if ptr is not None:
                eng.dev_free(ptr)
        for e in engines:
            e.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000_000)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--levels", type=str, default="100000,1000")
    ap.add_argument("--chunk", type=int, default=20_000_000)
    ap.add_argument("--chunk2", type=int, default=0, help="second chunking for the invariance check (0: off)")
    ap.add_argument("--seed", type=int, default=12345)
    ap.add_argument("--vcov", default="HC1", choices=["HC1", "iid"])
    a = ap.parse_args()
    from leanfe_amd import synth
    L = [int(x) for x in a.levels.split(",")]
    beta = synth.betas(a.k)

    def say(m):
        print(m, file=sys.stderr, flush=True)

    r = wide_fit(a.rows, a.k, L, beta, a.chunk, a.seed, a.vcov, say=say)
    free = total = None
    try:
        import torch
        free, total = torch.cuda.mem_get_info(0)
    except Exception:  # noqa: BLE001 - torch is plumbing only; the figure is optional
        pass
    tot = sum(r["t"].values())
    line = dict(kind="wide fit without a resident D (codes resident, columns generated per chunk on the device)",
                rows=a.rows, k=a.k, levels=L, vcov=a.vcov, chunk_rows=a.chunk, column_blocks=r["blocks"],
                iterations=r["iterations"], n_obs=r["n_obs"], df_resid=r["df_resid"],
                resident_D_bytes_avoided=a.rows * (a.k + 2) * 8, hbm_total=total, hbm_free_after=free,
                times=r["t"], total_s=tot, mrows_s=a.rows / tot / 1e6,
                beta_head=[float(x) for x in r["beta"][:4]], se_head=[float(x) for x in r["se"][:4]],
                max_abs_t_vs_generating_beta=float(np.max(np.abs((r["beta"] - beta) / r["se"]))))
    if a.chunk2:
        r2 = wide_fit(a.rows, a.k, L, beta, a.chunk2, a.seed, a.vcov, say=say)
        line["chunk2"] = a.chunk2
        line["chunk2_total_s"] = sum(r2["t"].values())
        line["chunking_max_rel_beta"] = float(np.max(np.abs(r2["beta"] - r["beta"]) / np.abs(r["beta"])))
        line["chunking_max_rel_se"] = float(np.max(np.abs(r2["se"] - r["se"]) / np.abs(r["se"])))
        line["chunking_ints_equal"] = (r2["iterations"], r2["n_obs"], r2["df_resid"]) == (
            r["iterations"], r["n_obs"], r["df_resid"])
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()

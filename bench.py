#!/usr/bin/env python
"""Headline benchmark: Mrows/s of demean + solve at 50M rows x 2 HDFE (BASELINE.json).

Workloads (BASELINE.json ``configs``; ``--config``, default 3 = the headline):
  1  1M rows, FEs (2e4, 500), k = 3, IID
  2  10M rows, FEs (1e5, 1e3), k = 5, IID
  3  50M rows, FEs (1e5, 1e3), k = 10, HC1            <- metric of BASELINE.json
  4  50M rows, FEs (1e6, 1e5, 1e4), k = 10, two-way clustered SE on fe2 x fe3 (CGM)
  5  500M rows, FEs (1e5, 1e3), k = 10, IID
Synthetic counter-based panel (leanfe_amd/synth.py, seed 12345) generated on the device.
One "step" = one full regression on device-resident inputs exactly as ``leanfe_hip`` runs
it after the data hand-off: singleton drop -> alternating projections to convergence
(tol 1e-6, max_iter 50, check from it = 3) -> Gram (MFMA) -> Cholesky -> residual pass
(+ HC1 meat / cluster scores) -> SEs.  tests/test_gpu_configs.py runs ``solve_step`` on
the same workloads against the C restatement of the reference (oracle/altproj_c.c).

Multi-GPU: one process per GPU.  Under torchrun the rank comes from the environment;
``python bench.py --gpus N`` without it spawns N rank processes itself (before any GPU
call).  ``--scaling strong`` (default): ``--rows`` rows in total, sharded over the ranks;
``--scaling weak``: ``--rows`` rows per rank.  ``--shard owner`` (default for fits with two
or more FEs) gives each rank every row of a contiguous range of the primary FE's (most
levels) levels, so the primary FE's group tables stay rank-local and only the other FEs'
tables, the Gram and the SE statistics are all-reduced over RCCL (clustered scores go to
their owner ranks by cluster key); ``--shard rows`` shards contiguous row blocks (every
group table all-reduced).  Timing: W warm-up steps, barrier + device
sync, K timed steps, device sync + barrier; the max over ranks is reported.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
BASELINE_METRIC = "Mrows/sec demean+solve, 50M×2-HDFE; achieved HBM GB/s at 1/2/4/8 GPUs"

# BASELINE.json configs (index = config number): rows (total), levels, k, vcov, cluster FEs
CONFIGS = {
    1: dict(rows=1_000_000, levels=[20_000, 500], k=3, vcov="iid", cl=None),
    2: dict(rows=10_000_000, levels=[100_000, 1_000], k=5, vcov="iid", cl=None),
    3: dict(rows=50_000_000, levels=[100_000, 1_000], k=10, vcov="HC1", cl=None),
    4: dict(rows=50_000_000, levels=[1_000_000, 100_000, 10_000], k=10, vcov="cluster", cl=[1, 2]),
    5: dict(rows=500_000_000, levels=[100_000, 1_000], k=10, vcov="iid", cl=None),
}

# The reference's own benchmark panels (python/tests/create_data.py:143-194, formulas and cluster
# columns python/tests/reg_test.py:26-97): the only shapes BASELINE.md has timings for
# (benchmark_results132132.csv:2-7, benchmark_results3.csv:2-10, benchmark_results2.csv:27,29).
# FE 0 = firm_id, 1 = worker_id, 2 = city_id; k = 4 named regressors (+ 16 / 10 extra x's).
# The synthetic generator stands in for create_data.py's polars_ds draws (not importable here).
PRESETS = {
    "hdfe_base": dict(rows=15_000_000, levels=[10_000, 2_000], k=4, vcov="iid", cl=None),
    "hdfe_cluster1": dict(rows=15_000_000, levels=[10_000, 2_000], k=4, vcov="cluster", cl=[0]),
    "hdfe_cluster2": dict(rows=15_000_000, levels=[10_000, 2_000], k=4, vcov="cluster", cl=[0, 1]),
    "uhdfe_base": dict(rows=15_000_000, levels=[10_000, 2_000, 500], k=20, vcov="iid", cl=None),
    "uhdfe_cluster2": dict(rows=15_000_000, levels=[10_000, 2_000, 500], k=20, vcov="cluster", cl=[0, 1]),
    "mega_base": dict(rows=50_000_000, levels=[20_000, 4_000, 1_000], k=14, vcov="iid", cl=None),
    "mega_cluster1": dict(rows=50_000_000, levels=[20_000, 4_000, 1_000], k=14, vcov="cluster", cl=[0]),
    "mega_cluster2": dict(rows=50_000_000, levels=[20_000, 4_000, 1_000], k=14, vcov="cluster", cl=[0, 1]),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10, help="untimed steps (GPU clocks settle within ~0.1 s)")
    ap.add_argument("--config", type=int, default=3, choices=sorted(CONFIGS))
    ap.add_argument("--preset", type=str, default=None, choices=sorted(PRESETS),
                    help="one of the reference's own benchmark panels instead of a BASELINE config")
    ap.add_argument("--runs", type=int, default=5, help="timed runs the K steps are split into (value = median)")
    ap.add_argument("--rows", type=int, default=None, help="rows (total with --scaling strong, per GPU with weak)")
    ap.add_argument("--k", type=int, default=None)
    ap.add_argument("--levels", type=str, default=None)
    ap.add_argument("--vcov", type=str, default=None)
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong")
    ap.add_argument("--shard", choices=["auto", "owner", "rows"], default="auto")
    ap.add_argument("--seed", type=int, default=12345)
    ap.add_argument("--emulate-rank", type=str, default=None, metavar="R/N",
                    help="diagnostic: solve rank R's owner shard of an N-rank strong-scaled run alone on one "
                         "GPU (no collectives): the per-rank compute and fixed cost of the N-GPU run")
    ap.add_argument("--cpu-rows", type=int, default=50_000_000, help="CPU baseline sample (prefix rows)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-h2d", action="store_true")
    ap.add_argument("--no-prof", action="store_true", help="diagnostic: no per-kernel events (no roofline)")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--knob", action="append", default=[], metavar="NAME=VALUE",
                    help="A/B only: an engine test knob (lfe_test_set_knob); the engine reads no environment")
    ap.add_argument("--print-rank-env", action="store_true",
                    help="diagnostic: each rank prints its rank / world / device and exits (no GPU call)")
    a = ap.parse_args(argv)
    cfg = PRESETS[a.preset] if a.preset else CONFIGS[a.config]
    a.rows = cfg["rows"] if a.rows is None else a.rows
    a.k = cfg["k"] if a.k is None else a.k
    a.levels = list(cfg["levels"]) if a.levels is None else [int(x) for x in a.levels.split(",")]
    a.vcov = cfg["vcov"] if a.vcov is None else a.vcov
    a.cl = cfg["cl"] if a.vcov.lower() == "cluster" else None
    if a.vcov.lower() == "cluster" and a.cl is None:
        a.cl = list(range(1, len(a.levels)))[:2] or [0]
    return a


def is_headline(a) -> bool:
    return (a.rows, a.k, a.levels, a.vcov.lower()) == (50_000_000, 10, [100_000, 1_000], "hc1") \
        and (a.scaling == "strong" or a.gpus == 1) and not a.emulate_rank and not a.preset


def workload_label(a, world: int) -> str:
    per = "total" if a.scaling == "strong" else "per GPU"
    se = a.vcov if a.vcov.lower() != "cluster" else f"{len(a.cl)}-way clustered SE on " + " x ".join(
        f"fe{f + 1}" for f in a.cl)
    lv = ", ".join(f"{g:.0e}".replace("e+0", "e") for g in a.levels)
    name = f"reference panel {a.preset.upper()}" if a.preset else f"configs[{a.config - 1}]"
    return f"{name}: {a.rows / 1e6:g}M rows {per}, {len(a.levels)} FE ({lv} levels), k={a.k}, {se}"


def split_runs(steps: int, runs: int) -> list[int]:
    """The K timed steps as ``runs`` consecutive timed runs (sizes differ by at most one)."""
    runs = max(1, min(runs, steps))
    return [steps // runs + (1 if i < steps % runs else 0) for i in range(runs)]


# ---------------------------------------------------------------------------
# launcher (no GPU call, no engine import: the children initialise the GPU)
# ---------------------------------------------------------------------------

def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_envs(n: int, port: int, base: dict | None = None) -> list[dict]:
    """Environment of each of the n rank processes (torchrun's variables, local node)."""
    base = dict(os.environ if base is None else base)
    envs = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        envs.append(e)
    return envs


def spawn_ranks(n: int, argv: list[str], timeout: float | None = None) -> int:
    """Run this script as n rank processes; if one fails the others are ended.  Returns the
    first non-zero exit code (0 when all succeed)."""
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=e)
             for e in rank_envs(n, _free_port())]
    t0 = time.time()
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            if timeout is not None and time.time() - t0 > timeout:
                rc = 124
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return rc


# ---------------------------------------------------------------------------
# one step (the hip backend's hot path on device-resident data)
# ---------------------------------------------------------------------------

def device_sync(eng):
    eng.sync()


def solve_step(eng, vcov: str, n_cl: int = 0) -> dict:
    """One regression on the loaded shard, as ``leanfe_hip`` runs it (hip_impl.py, the same
    fallbacks: a second residual pass when r'r cancels in the Gram or the device Cholesky's beta
    drifted from the host solve): one lfe_fit call - drop, projections, Gram + device solve +
    residual pass, host solve and IID / HC1 SEs - then, clustered, the meats and the CGM sandwich."""
    from leanfe_amd import inference

    v = vcov.lower()
    r = eng.fit(v)
    n_obs, df_resid = r["n_obs"], r["df_resid"]
    ncl = None
    se = r["se"]
    if v == "cluster":
        Vb = r["xtx_inv"][1:, 1:]
        if n_cl == 1:
            meats, Gs = eng.cluster_meat()
            se, ncl = inference.se_cluster_oneway(Vb, meats[0], int(Gs[0]), n_obs, df_resid, True)
        else:
            subsets = inference.cluster_subsets(n_cl)
            meats, Gs = eng.cluster_meat_subsets(subsets)  # intersections formed on the device
            se, ncl = inference.se_cluster_multiway(Vb, list(meats), [int(g) for g in Gs], subsets, n_obs, df_resid,
                                                    True)
    return dict(n_obs=n_obs, iterations=r["iterations"], beta=r["beta_full"][1:], se=se, df_resid=df_resid,
                fe_dims=list(r["fe_dims"]), n_clusters=ncl, rss=float(r["stats"][1]),
                beta_dev_vs_host=r["beta_dev_vs_host"])


def load_shard(eng, a, rank: int, world: int, shard: str) -> dict:
    """Generate this rank's shard of the synthetic panel on the device; returns its geometry."""
    from leanfe_amd import dist, synth

    total = a.rows if a.scaling == "strong" else a.rows * world
    beta = synth.betas(a.k)
    if a.emulate_rank:
        rank, world = (int(x) for x in a.emulate_rank.split("/"))
        shard = "owner"
    if shard == "owner":
        # every row whose primary-FE code lies in this rank's level range (dist.owner_range)
        P = max(range(len(a.levels)), key=lambda f: a.levels[f])
        lo, hi = dist.owner_range(a.levels[P], rank, world)
        eng.synth_load_owned(total, a.k, a.levels, beta, P, lo, hi, seed=a.seed)
        return dict(total=total, local=eng.n, owner=(P, lo, hi))
    lo, hi = dist.shard_range(total, rank, world)
    eng.synth_load(hi - lo, a.k, a.levels, beta, seed=a.seed, row_offset=lo)
    return dict(total=total, local=hi - lo, rows=(lo, hi))


# ---------------------------------------------------------------------------
# measurement helpers
# ---------------------------------------------------------------------------

def algorithmic_bytes(n: int, p: int, F: int, clustered: bool = False, dense_cells: int = 0,
                      cell_bytes: int = 2, levels: list | None = None) -> dict:
    """HBM bytes each kernel must move per launch, n rows of the shard,
    p = 1 + k f64 data columns, F int32 code columns.  Kernels absent here move only group
    tables or scalars (latency-bound) and count as 0 in the step total.  The general sweeps'
    cross / check passes (F >= 3) read F - 1 code arrays from HBM; the effect
    rows they gather come from L2 / MALL-resident tables and are not HBM bytes.  With the dense
    two-FE cross terms (``dense_cells`` > 0, lfe_dense.hip) the table build reads both codes and
    writes two count tables of ``cell_bytes`` per cell (1: the exact i8 form, 2: u16), and each
    cross-term pass reads one of them; with three or more FEs on pair tables (lfe_dense3.hip) the
    projections read the tables instead of gathering rows.  With ``levels`` (unweighted, two or
    three FEs on the general sweeps) the segment layouts come from the sorted build (lfe_seg.hip):
    per FE a key pass, radix passes over the code bits above 9 (none for the primary) and a rank
    pass, so its bytes per launch are that build's total over its launches."""
    k = p - 1
    seg = n * (4 * F + 4 * F * (F - 1))  # codes -> every FE's other codes, segment order (block scatter)
    if levels and F in (2, 3) and not dense_cells:
        prim = max(range(F), key=lambda f: levels[f])
        passes = sum(0 if f == prim else max(0, -(-(max(1, (levels[f] - 1).bit_length()) - 9) // 8))
                     for f in range(F))
        total = n * (F * (4 * (F + 1) + 12) + 32 * passes + F * (12 + 4 * (F - 1) + 4))
        seg = total / (2 * F + 2 * passes + 1)
    cb = cell_bytes
    dense = {"layout_scatter": 8 * n + 2 * cb * dense_cells, "tp": cb * dense_cells, "tq": cb * dense_cells,
             "layout_base": 0} if dense_cells else {}
    if dense_cells and F >= 3:
        # pair-table sweeps (lfe_dense3.hip; dense_cells = i8 bytes of every ordered pair's table):
        # a projection reads its FE's tables once per 16-column group, a y-only check pass once; the
        # build partitions the kept rows' codes (P, a, partners: <= 20 B read, 8 B written per row)
        # per partition FE and counts each pair from it (8 B per row read, both tables written)
        npairs = F * (F - 1) // 2
        ncg = (p + 15) // 16
        dense = {"cross": dense_cells * ncg / F, "check": dense_cells / F, "layout_hist": 8 * n,
                 "layout_scatter": 28 * n, "seg_build": 8 * n + dense_cells / npairs}
    return {
        "part_hist": 4 * n,                          # primary codes
        "part_scatter": n * (2 * 8 * p + 2 * 4 * F),  # read + write X and codes
        "layout_hist": 8 * n,                        # both codes in layout order
        "layout_scatter": n * (8 + 4 + 2),           # both codes -> seg_q (int32) + run_h (uint16)
        "group_sums": n * (8 * p + 4 * F),           # X + codes (+ the raw Gram, MFMA)
        "tp": 4 * n,                                 # seg_q: the cross term of the primary FE
        "tq": 2 * n,                                 # run_h: the cross term of the secondary FE
        "gram_design": n * (8 * p + 4 * F),          # X + codes
        "gram_resid": n * (8 * p + 4 * F + (8 * k if clustered else 0)),  # X + codes (+ score rows)
        "seg_build": seg,
        "cross": 4 * n * (F - 1),                    # the other FEs' codes in segment order
        "check": 4 * n * (F - 1),
        **({"count": 4 * n} if F != 2 else {}),      # one FE's codes (two FEs: the layouts' histograms)
        # clustered SEs (lfe_cluster.hip): a sort launch is a digit histogram (8 B keys read) or a
        # scatter (key + row read and written, 24 B) - 16 B/row on average over the pairs; a sorted
        # subset's segmented sums read the sorted keys, segment flags and row index and gather the
        # score rows through it (8k + 16 B/row); a one-column subset's sort-free fixed-point sums
        # (k_clfix_stats, k_clfix_add) read the score rows, cluster codes and keep flags twice
        "cluster_sort": 16 * n,
        "cluster_scatter": n * (8 * k + 16),
        "cluster_fix": n * (16 * k + 16),
        **dense,
    }


def gather_bytes(n: int, p: int, F: int) -> dict:
    """Bytes the general sweeps gather per launch from L2 / MALL (effect rows of the other FEs, each
    row one 128-byte line of the padded copy; the check passes one 8-byte y value)."""
    return {"cross": n * (F - 1) * 128, "check": n * (F - 1) * 8}


def pmc_traffic(kernel: str, a, local_rows: int) -> tuple[float | None, str | None]:
    """HBM bytes per launch of ``kernel`` from the newest rocprofv3 PMC summary for this exact
    configuration (tools/pmc.sh + tools/pmc_traffic.py: 2 x FETCH_SIZE + WRITE_SIZE, the gfx950
    correction of MI355X_MICROARCH.md), else None.  Matched on the rows of the shard this process
    solved (an --emulate-rank shard is not the whole panel the PMC pass may have measured)."""
    import glob
    import re

    if a.knob:
        return None, None  # an A/B variant: the PMC passes measured the production path
    cfg = {"rows": local_rows, "k": a.k, "levels": list(a.levels), "vcov": a.vcov}
    rounds = glob.glob(os.path.join(ROOT, "profiles", "r[0-9]*", "pmc_traffic.json"))
    rounds.sort(key=lambda p: int(re.search(r"r(\d+)", os.path.basename(os.path.dirname(p))).group(1)), reverse=True)
    for path in rounds:
        try:
            with open(path) as f:
                t = json.load(f)
        except (OSError, ValueError):
            continue
        if t.get("config") == cfg and kernel in t.get("kernels", {}):
            return float(t["kernels"][kernel]["bytes_per_launch"]), os.path.relpath(path, ROOT)
    return None, None


def host_info(threads: int) -> dict:
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        nproc = int(subprocess.run(["nproc"], capture_output=True, text=True, check=True).stdout.strip())
    except (OSError, ValueError, subprocess.CalledProcessError):
        nproc = None
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    return dict(cores=threads, nproc=nproc, affinity_cpus=aff, os_cpu_count=os.cpu_count(), cpu_model=model,
                omp_num_threads=os.environ.get("OMP_NUM_THREADS"))


def cpu_baseline(a, cols, codes) -> dict:
    """The C restatement of the reference alt_proj path (oracle/altproj_c.c: row-parallel
    OpenMP, every host thread this process may use) on the first ``--cpu-rows`` rows of the
    very panel the GPU solved."""
    from oracle.altproj_c import default_threads, fit_c

    threads = default_threads()
    n = min(a.cpu_rows, cols.shape[1])
    cl = [codes[f][:n] for f in a.cl] if a.cl else None
    t0 = time.perf_counter()
    r = fit_c([c[:n] for c in cols], [c[:n] for c in codes], a.levels, vcov=a.vcov, threads=threads, cl_codes=cl,
              cl_levels=[a.levels[f] for f in a.cl] if a.cl else None)
    dt = time.perf_counter() - t0
    whole = "the whole" if n == cols.shape[1] else f"the first {n:_} rows of the"
    out = dict(value=round(n / dt / 1e6, 3), unit="Mrows/s", kind="port",
               sample=f"{whole} {cols.shape[1]:_}-row panel (k={a.k}, levels={a.levels}, vcov={a.vcov}); "
                      f"oracle/altproj_c.c (C restatement of polars_impl.py alt_proj + std_errors.py, row-parallel "
                      f"OpenMP), {threads} threads, {dt:.2f} s, iterations={r['iterations']}",
               iterations=int(r["iterations"]), seconds=round(dt, 3))
    out.update(host_info(threads))
    return out


def main(argv=None):
    a = parse(argv)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # not under torchrun: one process per GPU, spawned before anything touches the GPU
        sys.exit(spawn_ranks(a.gpus, sys.argv[1:] if argv is None else list(argv)))

    if a.print_rank_env:
        print(json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR")}),
              flush=True)
        return

    import numpy as np

    from leanfe_amd._lib import Engine, set_knob
    from leanfe_amd.dist import HostGroup

    for kv in a.knob:
        name, _, val = kv.partition("=")
        set_knob(name, val)

    d = HostGroup()
    if d.world != a.gpus:
        raise SystemExit(f"bench.py --gpus {a.gpus} but WORLD_SIZE={d.world}")
    shard = a.shard
    if shard == "auto":
        shard = "owner" if (len(a.levels) >= 2 and d.world > 1) else "rows"
    # LEANFE_BENCH_DEVICE (diagnostic): every rank on that one device, e.g. to run the RCCL path of
    # a multi-rank solve on a one-GPU box (RCCL must accept several ranks on one device)
    eng = Engine(int(os.environ.get("LEANFE_BENCH_DEVICE", d.local)))
    if d.world > 1:
        uid = Engine.unique_id() if d.rank == 0 else None
        uid = d.bcast_bytes(uid)
        eng.set_comm(uid, d.rank, d.world)
    t0 = time.perf_counter()
    geo = load_shard(eng, a, d.rank, d.world, shard)
    n_cl = len(a.cl) if a.cl else 0
    if n_cl:
        _, codes = eng.copy_inputs()
        eng.load_clusters([np.ascontiguousarray(codes[f]) for f in a.cl], [a.levels[f] for f in a.cl])
    gen_s = time.perf_counter() - t0

    for _ in range(a.warmup):
        solve_step(eng, a.vcov, n_cl)

    # the K timed steps as `runs` timed runs, each bracketed by barrier + device sync and timed as
    # the max over ranks; `value` is the median run's rate, the mean is kept
    res = None
    run_s = []
    sizes = split_runs(a.steps, a.runs)
    for m in sizes:
        d.barrier()
        device_sync(eng)
        t0 = time.perf_counter()
        for _ in range(m):
            res = solve_step(eng, a.vcov, n_cl)
        device_sync(eng)
        t1 = time.perf_counter()
        d.barrier()
        run_s.append(d.max(t1 - t0))
    elapsed = sum(run_s)
    per_step = sorted(s / m for s, m in zip(run_s, sizes))
    med_step = per_step[len(per_step) // 2] if len(per_step) % 2 else 0.5 * (
        per_step[len(per_step) // 2 - 1] + per_step[len(per_step) // 2])
    # per-kernel times from a second pass of the same steps with an event pair around every
    # launch (the events cost ~0.2 ms of host time per step, so they stay out of `value`)
    kstats = {}
    if not a.no_prof:
        eng.profile(True)
        for _ in range(a.steps):
            solve_step(eng, a.vcov, n_cl)
        kstats = eng.kernel_stats()
        eng.profile(False)

    total_rows = geo["total"] if not a.emulate_rank else geo["local"]
    value = total_rows / med_step / 1e6
    ms_step = med_step * 1e3
    value_mean = total_rows * a.steps / elapsed / 1e6
    p, F = a.k + 1, len(a.levels)
    cells = eng.dense_cells()
    cbytes = eng.dense_cell_bytes() if cells else 0
    ab = algorithmic_bytes(geo["local"], p, F, clustered=bool(a.cl), dense_cells=cells, cell_bytes=cbytes or 2,
                           levels=list(a.levels))
    # dominant kernel = most device time in the timed region (rank 0's shard)
    dom = max(kstats.items(), key=lambda kv: kv[1][0]) if kstats else ("none", (0.0, 1))
    dom_name, (dom_ms, dom_launches) = dom
    per_launch_s = dom_ms / 1e3 / max(dom_launches, 1)
    roofline = None
    if ab.get(dom_name):
        achieved = ab[dom_name] / per_launch_s / 1e9
        traffic, tsrc = pmc_traffic(dom_name, a, geo["local"])
        roofline = {"bound": "hbm", "kernel": dom_name, "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS,
                    "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic,
                    "bytes_per_launch": ab[dom_name], "avg_launch_ms": round(per_launch_s * 1e3, 4)}
        if tsrc:
            roofline["traffic_source"] = tsrc + " (rocprofv3 PMC, same config)"
        gb = gather_bytes(geo["local"], p, F).get(dom_name)
        if gb:  # the general sweeps: what the gathers move from L2 / MALL per launch
            roofline["gathered"] = {"bytes_per_launch": gb, "GBps": round(gb / per_launch_s / 1e9, 1),
                                    "source": "L2 / MALL (padded effect rows, 128 B each)"}
    # step-level roofline: every modelled kernel's algorithmic bytes x its launches per step,
    # over the measured wall time per step (rank 0's shard; all ranks move the same amount)
    step_bytes = sum(ab[k] * v[1] / a.steps for k, v in kstats.items() if k in ab)
    if roofline is not None and step_bytes:
        ach = step_bytes / (ms_step / 1e3) / 1e9
        kern_ms = sum(v[0] for v in kstats.values()) / a.steps
        roofline["step"] = {"bytes": int(step_bytes), "achieved": round(ach, 1), "frac": round(ach / PEAK_HBM_GBS, 4),
                            "kernel_ms": round(kern_ms, 4), "host_gap_ms": round(ms_step - kern_ms, 4),
                            "model": "sum over kernels of DESIGN.md §4 bytes/row x rows x launches per step"}
        # the traffic no design can avoid: X and the codes read once for the group sums (+ Gram), and
        # once more for the residual pass unless the SE come from the Gram (IID)
        passes = 1 if a.vcov.lower() == "iid" else 2
        cb = passes * geo["local"] * (8 * p + 4 * F)
        cach = cb / (ms_step / 1e3) / 1e9
        roofline["step"]["compulsory"] = {"bytes": int(cb), "achieved": round(cach, 1),
                                          "frac": round(cach / PEAK_HBM_GBS, 4),
                                          "model": f"{passes} pass(es) over X (8p B/row) + codes (4F B/row)"}

    extra = {}
    if d.rank == 0 and d.world == 1 and (not a.no_cpu or not a.no_h2d):
        cols, codes = eng.copy_inputs()
        if not a.no_cpu:
            extra["cpu_baseline"] = cpu_baseline(a, cols, codes)
        if not a.no_h2d:
            # PCIe-inclusive load of the same shard from pageable host memory (never `value`)
            t0 = time.perf_counter()
            eng.load(list(cols), list(codes), a.levels)
            eng.sync()
            h2d = time.perf_counter() - t0
            nbytes = cols.nbytes + codes.nbytes
            extra["h2d"] = {"seconds": round(h2d, 4), "GBps": round(nbytes / h2d / 1e9, 2), "bytes": int(nbytes),
                            "source": "pageable NumPy columns -> lfe_load (H2D + code validation)"}
        del cols, codes
    if d.rank == 0:
        headline = is_headline(a)
        line = {
            "metric": BASELINE_METRIC if headline else f"Mrows/sec demean+solve, {workload_label(a, d.world)}",
            "value": round(value, 2),
            "unit": "Mrows/s",
            "n_gpus": d.world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_step, 3),
            "statistic": f"median over {len(sizes)} timed runs of {'/'.join(map(str, sizes))} steps",
            "value_mean": round(value_mean, 2),
            "ms_per_step_mean": round(elapsed / a.steps * 1e3, 3),
            "runs_ms_per_step": [round(s / m * 1e3, 3) for s, m in zip(run_s, sizes)],
            "higher_is_better": True,
            "scaling": a.scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic (counter-based splitmix64 panel generated on device, seed {a.seed})",
            "config": {"workload": workload_label(a, d.world), "rows_total": total_rows,
                       "rows_rank0": geo["local"], "k": a.k, "levels": a.levels, "vcov": a.vcov,
                       "cluster_fes": a.cl, "iterations": res["iterations"],
                       "cross_terms": (f"dense count tables ({cells} cells, "
                                       + ("exact i8 x base-128 digits, v_mfma_i32_16x16x64_i8)" if cbytes == 1
                                          else "u16, v_mfma_f64_16x16x4f64)")) if cells else "row layouts",
                       "parallelism": f"dp{d.world} ({shard}-sharded rows, RCCL inside the engine)"
                       if not a.emulate_rank else f"rank {a.emulate_rank} owner shard solved alone (diagnostic)"},
            "roofline": roofline,
            "cpu_baseline": extra.get("cpu_baseline"),
            "h2d": extra.get("h2d"),
            "kernels_ms": {k: [round(v[0] / a.steps, 4), v[1] // a.steps] for k, v in kstats.items()},
            "gen_s": round(gen_s, 3),
            "beta_dev_vs_host": res["beta_dev_vs_host"],
        }
        if a.knob:
            line["knobs"] = list(a.knob)
        if a.verbose:
            line["beta"] = [float(x) for x in res["beta"]]
            line["se"] = [float(x) for x in res["se"]]
        print(json.dumps(line), flush=True)
    eng.close()
    d.close()


if __name__ == "__main__":
    main()

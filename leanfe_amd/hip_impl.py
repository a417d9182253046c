"""``backend="hip"``: the reference's ``leanfe_polars`` control flow
(python/leanfe/polars_impl.py:287-579) driving the gfx950 engine.

Host side: formula parsing, column selection, categorical -> int32 codes,
factor/interaction expansion and strategy choice (all cheap, O(n) or less).
Device side (``liblfe_hip.so`` through ctypes): singleton drop, alternating
projections to convergence, Gram, residuals and SE reductions.  Host again:
the (k+1)^2 Cholesky solve and k x k sandwich products (leanfe_amd.inference).
"""
from __future__ import annotations

import os
import time

import numpy as np

from . import dist, frame, inference
from ._lib import Engine
from .formula import parse_formula
from .result import LeanFEResult
from .strategy import DEFAULT_MAX_FE_LEVELS, determine_strategy

MAX_FE_LEVELS = DEFAULT_MAX_FE_LEVELS  # polars_impl.py:24
MAX_CONTEXT_COLS = 63  # columns one engine context holds (y + regressors + instruments); wider: _wide_fit
_VERBOSE = os.environ.get("LEANFE_HIP_VERBOSE", "0") not in ("", "0")  # log lines only
# Path switches for tests and A/B runs (the process environment selects no path):
#   out_of_core   default of leanfe_hip(out_of_core=None)
#   stream        a Parquet path streams into the engine batch by batch (False: read whole first)
#   stream_batch  rows per streamed Parquet batch
#   reshard       sharded two-FE fits move contiguous row blocks to owner ranks (lfe_reshard_owner)
#   context_rows  rows per engine context (None: 2^31 - 64, the int32 row-index cap)
#   phase_timing  the engine's per-phase device times in LeanFEResult.timings (HIP events: host time
#                 on the launch path; also on with LEANFE_HIP_VERBOSE)
#   wide_chunked  streamed wide IID / HC1 fits in row chunks without a resident D (False: D resident)
KNOBS = {"out_of_core": False, "stream": True, "stream_batch": 1 << 22, "reshard": True, "context_rows": None,
         "phase_timing": False, "wide_chunked": True}


def _default_device() -> int:
    return int(os.environ.get("LOCAL_RANK", os.environ.get("LEANFE_HIP_DEVICE", "0")))


def leanfe_hip(data, demean_tol: float = 1e-6, y_col: str | None = None, x_cols: list[str] | None = None,
               fe_cols: list[str] | None = None, formula: str | None = None, strategy: str = "auto",
               weights: str | None = None, max_iter: int = 50, vcov: str = "iid",
               cluster_cols: list[str] | None = None, ssc: bool = True, sample_frac: float | None = None,
               device: int | None = None, engine: Engine | None = None, quiet: bool = False,
               out_of_core: bool | None = None, chunk_rows: int = 1 << 22) -> LeanFEResult:
    """Fixed-effects OLS on the MI355X engine; arguments as ``leanfe_polars``.

    ``vcov`` accepts 'iid', 'HC1' (or 'hc1') and 'cluster'.  ``engine`` lets a
    caller reuse an ``Engine`` (e.g. one joined to an RCCL communicator with
    ``leanfe_amd.dist.attach``: every rank then passes its own row shard and
    gets the global fit; FE/cluster columns must then be global int codes).

    ``out_of_core`` (data larger than HBM; default: env ``LEANFE_HIP_OUT_OF_CORE``): only the FE
    codes (and weights, cluster codes) are loaded; the columns [y] + x + instruments are streamed
    in ``chunk_rows`` row chunks through the group sums, (if needed) the design Gram and the
    residual pass.  Any number of FEs and regressors, weights, IV, IID / HC1 /
    one-way and multi-way clustered SEs, one process or a sharded engine; factor and interaction
    terms are expanded chunk by chunk as the columns stream (frame.Expansion)."""
    t_start = time.perf_counter()
    say = (lambda *a: None) if quiet else print
    if formula is not None:
        y_col, x_cols, fe_cols, factor_vars, interactions, instruments = parse_formula(formula)
    elif y_col is None or x_cols is None or fe_cols is None:
        raise ValueError("Must provide either 'formula' or (y_col, x_cols, fe_cols)")
    else:
        factor_vars, interactions, instruments = [], [], []
    instruments = list(instruments or [])
    x_cols = list(x_cols)
    fe_cols = list(fe_cols) if fe_cols is not None else []
    v = vcov.lower()
    if v not in ("iid", "hc1", "cluster"):
        raise ValueError(f"Unknown vcov type: {vcov}")
    if v == "cluster" and cluster_cols is None:
        raise ValueError("cluster_cols required for vcov='cluster'")

    needed = [y_col] + x_cols + fe_cols + instruments
    for var, _ in factor_vars:
        needed.append(var)
    for var, fac, _ in interactions:
        needed += [var, fac]
    if cluster_cols is not None:
        needed += list(cluster_cols)
    if weights is not None:
        needed.append(weights)
    # a Parquet path streams: the FE / cluster / weight columns are read first (for the codes),
    # then [y] + x + instruments are decoded batch by batch while earlier batches upload
    # (pl.scan_parquet's role, polars_impl.py:341-343)
    if out_of_core is None:
        out_of_core = bool(KNOBS["out_of_core"])
    expand = bool(factor_vars or interactions)
    # (a resident fit expands factor / interaction terms on whole columns; an out-of-core fit per chunk)
    stream = (isinstance(data, str) and (out_of_core or not expand) and sample_frac is None
              and KNOBS["stream"])
    factor_src = [var for var, _ in factor_vars] + [fac for _, fac, _ in interactions]
    if stream:
        small = list(dict.fromkeys(fe_cols + list(cluster_cols or []) + ([weights] if weights else []) + factor_src))
        cols = frame.get_columns(data, small) if small else {}
        n_rows = frame.parquet_rows(data)
    else:
        cols = frame.get_columns(data, needed)

    plan, x_base = None, list(x_cols)
    sharded = engine is not None and dist.is_sharded(engine)
    # a row shard's categories are agreed over the ranks (every rank expands the same columns)
    unique = (lambda v: dist.agree_categories(engine, v)) if sharded else np.unique
    if out_of_core and expand and sample_frac is None:
        # planned on the whole factor columns, applied to each streamed chunk (polars_impl.py:342-365)
        plan = frame.Expansion(cols, interactions, factor_vars, unique)
        x_cols = x_cols + plan.names
    else:
        if interactions:
            x_cols = x_cols + frame.expand_interactions(cols, interactions, unique)
        if sample_frac is not None:
            n0 = len(cols[y_col])
            idx = np.sort(np.random.default_rng(42).choice(n0, size=int(round(n0 * sample_frac)), replace=False))
            cols = {c: np.asarray(a)[idx] for c, a in cols.items()}
        if factor_vars:
            x_cols = x_cols + frame.expand_factors(cols, factor_vars, unique)
    num_cols = [y_col] + x_cols + instruments  # the columns leanfe demeans (polars_impl.py:486)

    if len(num_cols) > MAX_CONTEXT_COLS:
        if sharded or strategy == "compress":
            raise ValueError(f"{len(num_cols)} columns: a fit wider than {MAX_CONTEXT_COLS} columns runs in one "
                             "process, with strategy alt_proj / demean")
        ooc = None
        if out_of_core:
            if not fe_cols or strategy not in ("auto", "alt_proj", "demean"):
                raise ValueError("out_of_core fits take one or more FEs and strategy 'alt_proj' (or 'demean' for "
                                 "one FE)")
            src = data if stream else cols
            n_oc = n_rows if stream else len(cols[y_col])
            if n_oc > context_rows():
                raise ValueError(f"{len(num_cols)} columns: a wide out-of-core fit takes at most {context_rows()} rows")
            ooc = dict(source=src, n_rows=n_oc, chunk_rows=int(chunk_rows), plan=plan, x_base=x_base)
        elif stream:  # a Parquet path read resident: the numeric columns too
            cols.update(frame.get_columns(data, [c for c in num_cols if c not in cols]))
        return _wide_fit(cols, y_col, x_cols, fe_cols, weights, cluster_cols, v, vcov, ssc, strategy, demean_tol,
                         max_iter, formula, t_start, say, engine, device, ooc, instruments)

    own_engine = engine is None
    eng = engine if engine is not None else Engine(_default_device() if device is None else device)
    if KNOBS["phase_timing"] or _VERBOSE:
        eng.phase_timing(True)
    try:
        # FE codes (polars_impl.py:118-139); sparse integer ids are factorized on the GPU
        codes, levels = [], []
        for fe in fe_cols:
            c, g = frame.factorize(cols[fe], global_codes=sharded, device=None if sharded else eng)
            codes.append(c)
            levels.append(g)
        levels = dist.agree_levels(eng, levels)
        if out_of_core:
            if not fe_cols or strategy not in ("auto", "alt_proj", "demean"):
                raise ValueError("out_of_core fits take one or more FEs and strategy 'alt_proj' (or 'demean' for "
                                 "one FE)")
            source = data if stream else cols
            n_rows_oc = n_rows if stream else len(cols[y_col])
            w_oc = None if weights is None else np.asarray(cols[weights], dtype=np.float64)
            args = (source, cols, n_rows_oc, y_col, x_cols, instruments, fe_cols, codes, levels, w_oc, cluster_cols,
                    v, vcov, ssc, demean_tol, max_iter, int(chunk_rows), formula, t_start, say)
            if not sharded and n_rows_oc > context_rows():
                # more rows than one context holds: contexts of < 2^31 rows on this device, joined in
                # one in-process group (the same collectives as row shards on several GPUs)
                dev = eng.device if own_engine else getattr(eng, "device", _default_device())
                return _out_of_core_split(dev, args, plan, x_base)
            return _out_of_core_fit(eng, *args, sharded, plan, x_base)
        w = None if weights is None else np.asarray(cols[weights], dtype=np.float64)
        # polars_impl.py:180: an all-ones instrument stops 2SLS from adding an intercept to Z.
        # Demeaned instruments cannot be all ones; without FEs they are the raw columns.
        z_ones = {z: not fe_cols for z in instruments}
        t0 = time.perf_counter()
        if stream:
            eng.load_begin(n_rows, len(num_cols), levels, weighted=w is not None)
            batch = int(KNOBS["stream_batch"])
            for row0, b in frame.stream_parquet(data, num_cols, batch_rows=batch):
                sl = slice(row0, row0 + len(b[y_col]))
                eng.load_rows(row0, [b[c] for c in num_cols], [c[sl] for c in codes], None if w is None else w[sl])
                for z in instruments:
                    z_ones[z] = z_ones[z] and bool(np.allclose(np.asarray(b[z], dtype=np.float64), 1.0))
            eng.load_finish()
            n_initial = n_rows
        else:
            Y = np.asarray(cols[y_col], dtype=np.float64)
            Xc = [np.asarray(cols[c], dtype=np.float64) for c in num_cols[1:]]
            for z in instruments:
                z_ones[z] = z_ones[z] and bool(np.allclose(np.asarray(cols[z], dtype=np.float64), 1.0))
            eng.load([Y] + Xc, codes, levels, w)
            n_initial = Y.size
        cl_loaded = None
        if v == "cluster" and strategy != "compress":
            # cluster columns load before the singleton drop: the partition moves them with the rows
            # (no gathers into the layout later), an owner re-shard moves them too, and a one-way
            # cluster on the primary FE is then summed inside the residual pass (lfe_gram.hip)
            cl_loaded = _load_clusters(eng, cols, cluster_cols, sharded)
        if (sharded and len(fe_cols) >= 2 and strategy in ("auto", "alt_proj")
                and KNOBS["reshard"]):
            # contiguous row blocks -> owner-sharded rows (lfe_reshard_owner): every rank then holds
            # all rows of a range of the primary FE's (most levels) levels, and a projection
            # all-reduces only the other FEs' tables - two FEs or more, weighted or not
            try:
                eng.reshard_owner(max(range(len(fe_cols)), key=lambda f: levels[f]))
            except (ValueError, MemoryError):
                # refused before any row moved, by a decision every rank takes alike from all-reduced
                # counts / memory flags (a rank would hold no rows or 2^31+ rows, or lacks device
                # memory for the staging copy): every rank keeps its contiguous block
                pass
        t_load = time.perf_counter() - t0
        n_obs, fe_dims, fe_card = eng.drop_singletons()
        fe_cardinality = dict(zip(fe_cols, fe_card))

        est_comp_ratio = None
        if strategy == "auto":
            # distinct (x, FE) rows / n over all loaded rows, exact (compress.py:187-253), on the
            # GPU; a row shard cannot see the other shards' rows, so sharded fits skip it
            if not sharded and n_initial:
                est_comp_ratio = eng.count_distinct_rows(len(x_cols)) / n_initial
            elif not sharded:
                est_comp_ratio = 1.0
            if not fe_cols:
                # polars_impl.py:385-390 ('compress' without FEs runs OLS here, the same estimates)
                inferred = "ols" if est_comp_ratio is None or est_comp_ratio >= 0.8 else "compress"
            elif len(fe_cols) == 1:
                inferred = "demean"
            else:
                inferred = determine_strategy(vcov, bool(instruments), fe_cardinality, max_fe_levels=MAX_FE_LEVELS,
                                              n_obs=n_initial, n_x_cols=len(x_cols),
                                              estimated_compression_ratio=est_comp_ratio)
                if sharded and inferred == "compress":
                    # compress groups one process's rows; a row shard runs the same fit by alt_proj
                    inferred = "alt_proj"
            say(f"Auto selection: Inferring {inferred} strategy. N = {n_initial:_}, "
                f"est. compression ratio: {est_comp_ratio}")
            strategy = inferred
        if strategy == "compress":
            if sharded:
                raise ValueError("strategy='compress' groups one process's rows; use alt_proj with a sharded engine")
            say("Using compresssion strategy...")
            return _compress_fit(eng, cols, x_cols, fe_cols, fe_card, cluster_cols, v, vcov, ssc, formula, t_start,
                                 t_load)

        if strategy == "demean":
            if len(fe_cols) != 1:
                raise ValueError("Strategy 'demean' requires exactly one FE column.")
            say("Using simple within-transform (demean) strategy for single FE...")
            iterations, _ = eng.demean([0], demean_tol, max_iter, check_from=0)
            absorbed_df = fe_dims[0] - 1
        elif strategy == "alt_proj":
            if not fe_cols:
                raise ValueError("Strategy 'alt_proj' requires FE-cols. "
                                 "Use strategy='ols' instead for OLS without FE.")
            say("Using FWL/alternating projections strategy...")
            if weights is None and not instruments:
                # projections, Gram, solve, residual pass and the IID / HC1 SEs in one engine call
                # (lfe_fit: the same steps as below without a return to Python between them)
                fit = eng.fit(v, demean_tol, max_iter, check_from=3, drop=False)
                return _fit_result(eng, fit, cols, x_cols, fe_cols, fe_dims, cluster_cols, v, vcov, sharded, ssc,
                                   cl_loaded, formula, est_comp_ratio, t_load, t_start)
            order = sorted(range(len(fe_cols)), key=lambda i: fe_card[i])  # polars_impl.py:485
            iterations, _ = eng.demean(order, demean_tol, max_iter, check_from=3)
            absorbed_df = sum(fe_dims) - len(fe_cols)
        elif strategy == "ols":
            if fe_cols:
                raise ValueError("Strategy 'ols' takes no fixed effects")
            say("Using simple OLS strategy (no fixed effects)...")
            iterations, _ = eng.demean([], demean_tol, max_iter, check_from=0)
            iterations, absorbed_df, fe_dims = 0, 0, None
        else:
            raise ValueError(f"Unknown strategy: {strategy}")

        k = len(x_cols)
        df_resid = n_obs - (k + 1) - absorbed_df
        if instruments:
            beta, se, n_clusters, rss, stats = _iv_fit(eng, cols, x_cols, instruments, cluster_cols, v,
                                                       any(z_ones.values()), sharded, n_obs, df_resid, ssc, cl_loaded)
            timings = dict(eng.timings(), load_s=t_load, total_s=time.perf_counter() - t_start)
            return LeanFEResult(coefs=dict(zip(x_cols, (float(b) for b in beta))),
                                std_errors=dict(zip(x_cols, (float(s) for s in se))), n_obs=n_obs,
                                iterations=iterations, vcov_type=vcov, is_iv=True,
                                n_instruments=len(instruments), n_clusters=n_clusters, df_resid=df_resid,
                                formula=formula, fe_cols=fe_cols, fe_dims=fe_dims, r_squared=None,
                                compression_ratio=est_comp_ratio, rss=rss, tss=None, backend="hip",
                                timings=timings)
        # IID without weights: the residual statistics follow from the Gram (no residual pass)
        gram_only = v == "iid" and weights is None
        # Gram + solve + residual pass; one host round trip when the fused path applies
        # (the residuals then use the device's Cholesky solve of the same Gram)
        fused = None if gram_only else eng.gram_resid(hc1=(v == "hc1"), keep_scores=(v == "cluster"))
        G = fused[0] if fused is not None else eng.gram()
        XtX, Xty = inference.split_gram(G)
        beta_full, XtX_inv = inference.solve_normal(XtX, Xty)  # polars_impl.py:212-226, host
        beta = beta_full[1:]
        Vb = XtX_inv[1:, 1:]
        stats = inference.stats_from_gram(G, beta_full) if gram_only else None
        meat = None
        if stats is not None:
            pass
        elif fused is not None and _beta_agrees(fused[1], beta_full):
            stats, meat = fused[2], fused[3]
        else:
            # no fused pass, or its device Cholesky beta drifted from the host solve the SEs
            # use (ill-conditioned Gram): the residual pass runs again with the host beta
            stats, meat = eng.resid(beta_full, hc1=(v == "hc1"), keep_scores=(v == "cluster"))
        rss_w, rss, sum_y, sum_y2 = stats
        n_clusters = None
        if v == "iid":
            se = inference.se_iid(Vb, rss_w, df_resid)
        elif v == "hc1":
            se = inference.se_hc1(Vb, meat, n_obs, df_resid)
        else:
            se, n_clusters = _cluster_se(eng, cols, cluster_cols, sharded, Vb, lambda M: M, n_obs, df_resid, ssc,
                                         cl_loaded)
        tss = sum_y2 - sum_y * sum_y / n_obs if n_obs else 0.0
        r_squared = 1 - rss / tss if tss > 0 else None
        timings = dict(eng.timings(), load_s=t_load, total_s=time.perf_counter() - t_start)
        if _VERBOSE:
            print(f"[leanfe_amd] iterations={iterations} device ms: {timings}")
    finally:
        if own_engine:
            eng.close()

    return LeanFEResult(coefs=dict(zip(x_cols, (float(b) for b in beta))),
                        std_errors=dict(zip(x_cols, (float(s) for s in se))), n_obs=n_obs,
                        iterations=iterations, vcov_type=vcov, is_iv=False, n_instruments=None,
                        n_clusters=n_clusters, df_resid=df_resid, formula=formula, fe_cols=fe_cols,
                        fe_dims=fe_dims, r_squared=r_squared, compression_ratio=est_comp_ratio,
                        rss=rss, tss=tss, backend="hip", timings=timings)


def _fit_result(eng, fit, cols, x_cols, fe_cols, fe_dims, cluster_cols, v, vcov, sharded, ssc, cl_loaded, formula,
                est_comp_ratio, t_load, t_start) -> LeanFEResult:
    """LeanFEResult of an lfe_fit call (Engine.fit): IID / HC1 SEs come with it, clustered ones from
    the kept score rows (std_errors.py:289-441)."""
    n_obs, df_resid = fit["n_obs"], fit["df_resid"]
    beta = fit["beta_full"][1:]
    rss_w, rss, sum_y, sum_y2 = fit["stats"]
    n_clusters = None
    if v == "cluster":
        se, n_clusters = _cluster_se(eng, cols, cluster_cols, sharded, fit["xtx_inv"][1:, 1:], lambda M: M, n_obs,
                                     df_resid, ssc, cl_loaded)
    else:
        se = fit["se"]
    tss = sum_y2 - sum_y * sum_y / n_obs if n_obs else 0.0
    r_squared = 1 - rss / tss if tss > 0 else None
    timings = dict(eng.timings(), load_s=t_load, total_s=time.perf_counter() - t_start)
    if _VERBOSE:
        print(f"[leanfe_amd] iterations={fit['iterations']} device ms: {timings}")
    return LeanFEResult(coefs=dict(zip(x_cols, (float(b) for b in beta))),
                        std_errors=dict(zip(x_cols, (float(s) for s in se))), n_obs=n_obs,
                        iterations=fit["iterations"], vcov_type=vcov, is_iv=False, n_instruments=None,
                        n_clusters=n_clusters, df_resid=df_resid, formula=formula, fe_cols=fe_cols,
                        fe_dims=fe_dims, r_squared=r_squared, compression_ratio=est_comp_ratio,
                        rss=rss, tss=tss, backend="hip", timings=timings)


def context_rows() -> int:
    """Rows one engine context holds (its row indices are int32; KNOBS["context_rows"] lowers
    it, e.g. for tests of the multi-context split at small sizes)."""
    cap = (1 << 31) - 64
    want = KNOBS["context_rows"]
    return max(1, min(cap, int(want if want is not None else cap)))


def _out_of_core_split(device, args, plan, x_base) -> LeanFEResult:
    """An out-of-core fit of more rows than one context holds: the rows are cut
    into S = ceil(n / context_rows()) contiguous blocks, each a context on the same device driven by
    its own thread and joined in an in-process group (EmuGroup), so that the fit runs the row-shard
    schedule of several GPUs - all-reduced group sums, cross terms, Gram and SE statistics, cluster
    scores to owner contexts - and every context returns the same global result.  FE codes are
    global already; cluster columns are factorized here over all rows."""
    import threading

    from ._lib import EmuGroup

    (source, cols, n_rows, y_col, x_cols, instruments, fe_cols, codes, levels, w, cluster_cols, v, vcov, ssc,
     demean_tol, max_iter, chunk_rows, formula, t_start, say) = args
    S = -(-n_rows // context_rows())
    say(f"{n_rows:_} rows: {S} engine contexts on device {device}")
    group = EmuGroup(S)
    cl = {c: frame.factorize(cols[c])[0] for c in (cluster_cols or [])}
    out, errs = [None] * S, []

    def work(r):
        lo, hi = dist.shard_range(n_rows, r, S)
        eng = None
        try:
            eng = Engine(device)
            eng.set_emu(group, r)
            eng.dist_group = ("local", group, r)
            sub = {c: np.asarray(a)[lo:hi] for c, a in cols.items()}
            sub.update({c: a[lo:hi] for c, a in cl.items()})
            src = source if isinstance(source, str) else sub
            out[r] = _out_of_core_fit(eng, src, sub, hi - lo, y_col, x_cols, instruments, fe_cols,
                                      [c[lo:hi] for c in codes], levels, None if w is None else w[lo:hi],
                                      cluster_cols, v, vcov, ssc, demean_tol, max_iter, chunk_rows, formula, t_start,
                                      say if r == 0 else (lambda *a_: None), True, plan, x_base, (lo, hi))
        except BaseException as e:  # noqa: BLE001 - the others must not wait for this member
            errs.append(e)
            group.abort()
        finally:
            if eng is not None:
                eng.close()

    threads = [threading.Thread(target=work, args=(r,)) for r in range(S)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errs:
        raise errs[0]
    return out[0]


def _stream_chunks(source, cols, n_rows, chunk_rows, y_col, x_cols, instruments, plan, x_base, row_range=None,
                   select=None):
    """(row0, columns) per row chunk of an out-of-core source (a Parquet path, re-read per pass, or
    in-memory arrays): [y] + x_cols + instruments, the factor / interaction columns of x_cols (after
    ``x_base``) formed from the chunk by ``plan``; ``select``: only these indices of that list, and
    only the source columns they need are read (a wide fit's column block)."""
    base = [y_col] + list(x_cols if plan is None else x_base)
    nb, nt = len(base), (len(plan.terms) if plan is not None else 0)
    sel = list(range(nb + nt + len(instruments))) if select is None else list(select)
    sb = [i for i in sel if i < nb]
    st = [i - nb for i in sel if nb <= i < nb + nt]
    sz = [i - nb - nt for i in sel if i >= nb + nt]
    need = [base[i] for i in sb] + [plan.terms[t][1] for t in st if plan.terms[t][1] is not None] + \
        [instruments[j] for j in sz]
    read = list(dict.fromkeys(need or [y_col]))
    pos = {i: j for j, i in enumerate(sb + [nb + t for t in st] + [nb + nt + z for z in sz])}

    def assemble(b, rows):
        out = [np.asarray(b[base[i]], dtype=np.float64) for i in sb]
        if st:
            out += plan.columns(cols, b, rows, which=st)
        out += [np.asarray(b[instruments[j]], dtype=np.float64) for j in sz]
        return [out[pos[i]] for i in sel]

    if isinstance(source, str):
        for row0, b in frame.stream_parquet(source, read, batch_rows=chunk_rows, row_range=row_range):
            yield row0, assemble(b, slice(row0, row0 + len(b[read[0]])))
    else:
        for r0 in range(0, n_rows, chunk_rows):
            b = {c: source[c][r0:r0 + chunk_rows] for c in read}
            yield r0, assemble(b, slice(r0, r0 + len(b[read[0]])))


def _out_of_core_fit(eng, source, cols, n_rows, y_col, x_cols, instruments, fe_cols, codes, levels, w, cluster_cols,
                     v, vcov, ssc, demean_tol, max_iter, chunk_rows, formula, t_start, say,
                     sharded=False, plan=None, x_base=None, row_range=None) -> LeanFEResult:
    """Out-of-core X (data larger than HBM): the FE codes (and weights, cluster codes) and their
    layouts stay on the GPU, the columns [y] + x (+ instruments) are streamed from host memory (or a
    Parquet file, re-read per pass) in row chunks through pass 1 (group sums S_f, W_f,
    polars_impl.py:491-508), the codes-only sweeps (any number of FEs), the Gram from the group
    tables (pass 3, the explicit design Gram of sqrt(w) [1, y~, x~], when that is unavailable),
    the host solve (:212-226; 2SLS for instruments, common.py:188-240) and pass 2 / 4 (residual,
    RSS, the HC1 meat and the cluster scores, :229, std_errors.py:183-602).  Same estimator, same
    stop rule and iterations as the resident fit.  A sharded engine streams this rank's rows; the
    group sums, Gram tiles and SE statistics are all-reduced, and the per-cluster score sums go to
    their owner ranks (lfe_stream.hip), so cluster columns must hold global codes (``row_range``: this
    context's rows of a Parquet source, _out_of_core_split).  ``plan``
    (frame.Expansion): the factor / interaction columns of x_cols (after ``x_base``) are formed
    per chunk from the whole factor columns in ``cols`` and the chunk's numeric columns."""
    from leanfe_amd._lib import NeedsStreamPass

    num_cols = [y_col] + list(x_cols) + list(instruments)
    p, k, mz = len(num_cols), len(x_cols), len(instruments)
    say("Using FWL/alternating projections strategy (out-of-core columns)...")

    def chunks():
        return _stream_chunks(source, cols, n_rows, chunk_rows, y_col, x_cols, instruments, plan, x_base, row_range)

    t0 = time.perf_counter()
    eng.load_codes(codes, levels, p, weights=w)  # a sharded engine: this rank's rows (global codes)
    subsets = None
    if v == "cluster":
        _load_clusters(eng, cols, cluster_cols, sharded)
        subsets = inference.cluster_subsets(len(cluster_cols))
    t_load = time.perf_counter() - t0
    n_obs, fe_dims, fe_card = eng.drop_singletons()
    eng.stream_pass(1, chunks())
    if len(fe_cols) == 1:
        iterations, _ = eng.demean([0], demean_tol, max_iter, check_from=0)  # polars_impl.py:437-465
    else:
        order = sorted(range(len(fe_cols)), key=lambda i: fe_card[i])  # polars_impl.py:485
        iterations, _ = eng.demean(order, demean_tol, max_iter, check_from=3)
    absorbed_df = sum(fe_dims) - len(fe_cols)
    df_resid = n_obs - (k + 1) - absorbed_df
    if subsets is not None:
        eng.stream_clusters([sum(1 << j for j in sub) for sub in subsets])
    try:
        G = eng.gram()
    except NeedsStreamPass:
        G = eng.stream_pass(3, chunks())[:(p + 1) ** 2].reshape(p + 1, p + 1)
    n_clusters = None
    if mz:
        iv = inference.IVSystem(G, k, mz, z_has_ones=False)  # demeaned instruments are never all ones
        out = eng.stream_pass(4, chunks(), iv.coef)
        stats, meat_u = out[:4], out[4:4 + p * p].reshape(p, p)
        Vb, to_meat = iv.XtX_inv, iv.xhat_meat
        if v == "iid":
            se = inference.se_iid(Vb, stats[0], df_resid)
        elif v == "hc1":
            se = inference.se_hc1(Vb, to_meat(meat_u), n_obs, df_resid)
        beta_full = iv.beta_full
    else:
        XtX, Xty = inference.split_gram(G)
        beta_full, XtX_inv = inference.solve_normal(XtX, Xty)  # host, polars_impl.py:212-226
        Vb, to_meat = XtX_inv[1:, 1:], (lambda M: M)
        # IID without weights: the residual statistics from the Gram unless r'r cancels there
        stats = inference.stats_from_gram(G, beta_full) if v == "iid" and w is None else None
        if stats is None:
            out = eng.stream_pass(2, chunks(), beta_full)
            stats, meat = out[:4], out[4:4 + k * k].reshape(k, k)
        if v == "iid":
            se = inference.se_iid(Vb, stats[0], df_resid)
        elif v == "hc1":
            se = inference.se_hc1(Vb, meat, n_obs, df_resid)
    if v == "cluster":
        ks = p if mz else k
        meats, Gs = eng.stream_cluster_meats(ks)
        if len(cluster_cols) == 1:
            se, n_clusters = inference.se_cluster_oneway(Vb, to_meat(meats[0]), int(Gs[0]), n_obs, df_resid, ssc)
        else:
            se, n_clusters = inference.se_cluster_multiway(Vb, [to_meat(M) for M in meats], [int(g) for g in Gs],
                                                           subsets, n_obs, df_resid, ssc)
    rss_w, rss, sum_y, sum_y2 = stats
    tss = sum_y2 - sum_y * sum_y / n_obs if n_obs else 0.0
    if mz:
        strip = len(beta_full) == k + 1
        beta = beta_full[1:] if strip else beta_full
        se = se[1:] if strip else se
    else:
        beta = beta_full[1:]
    timings = dict(eng.timings(), load_s=t_load, total_s=time.perf_counter() - t_start)
    return LeanFEResult(coefs=dict(zip(x_cols, (float(b) for b in beta))),
                        std_errors=dict(zip(x_cols, (float(s) for s in se))), n_obs=n_obs,
                        iterations=iterations, vcov_type=vcov, is_iv=bool(mz), n_instruments=mz or None,
                        n_clusters=n_clusters, df_resid=df_resid, formula=formula, fe_cols=fe_cols,
                        fe_dims=fe_dims, r_squared=None if mz else (1 - rss / tss if tss > 0 else None),
                        compression_ratio=None, rss=float(rss), tss=None if mz else tss, backend="hip",
                        timings=timings)


def _wide_fit_chunked(cols, y_col, x_cols, fe_cols, weights, v, vcov, strategy, demean_tol, max_iter, formula, t_start,
                      say, engine, device, ooc, instruments) -> LeanFEResult:
    """A streamed wide fit (IID / HC1) without a resident D: every column block stays an engine
    context (codes, layouts and its effect tables: ~22 B a row each), and the source is read twice
    more in row chunks - each chunk's [1_kept, y~, x~, z~] formed for all blocks into one chunk
    buffer (lfe_stream_materialize_rows), whose Gram (pass A) or residual, statistics and HC1 meat
    (pass B) are added in chunk order (lfe_wide_gram_rows, lfe_wide_resid_rows).  So the P n doubles
    of D and the context's 2^31-row cap on D's rows are gone: device memory is the blocks' codes plus
    P x chunk doubles (polars_impl.py:165-209 at any width; duckdb_impl.py:272-300 forms X'X out of
    core in one aggregation the same way)."""
    instruments = list(instruments)
    k, mz = len(x_cols), len(instruments)
    if mz and not fe_cols:
        raise ValueError("a wide IV fit takes one or more FEs (demeaned instruments are never all ones)")
    dcols = list(x_cols) + instruments
    P = 2 + len(dcols)
    w = None if weights is None else np.asarray(cols[weights], dtype=np.float64)
    n = ooc["n_rows"]
    chunk = max(64, int(ooc["chunk_rows"]) // 64 * 64)
    per = MAX_CONTEXT_COLS - (1 if w is not None else 0)
    blocks = [dcols[:per - 1]] + [dcols[j:j + per] for j in range(per - 1, len(dcols), per)]
    dev = _default_device() if device is None else device
    eng = engine if engine is not None else Engine(dev)
    engines = [eng]
    Dc = r = None

    def chunks(select=None):  # the source re-read in row chunks of `chunk` rows
        return _stream_chunks(ooc["source"], cols, n, chunk, y_col, x_cols, instruments, ooc["plan"], ooc["x_base"],
                              select=select)

    try:
        codes, levels = [], []
        for fe in fe_cols:
            c, g = frame.factorize(cols[fe], device=eng)
            codes.append(c)
            levels.append(g)
        if strategy == "auto":
            strategy = "demean" if len(fe_cols) == 1 else ("alt_proj" if fe_cols else "ols")
        if strategy == "demean" and len(fe_cols) != 1:
            raise ValueError("Strategy 'demean' requires exactly one FE column.")
        if strategy == "alt_proj" and not fe_cols:
            raise ValueError("Strategy 'alt_proj' requires FE-cols. Use strategy='ols' instead for OLS without FE.")
        if strategy == "ols" and fe_cols:
            raise ValueError("Strategy 'ols' takes no fixed effects")
        say(f"Wide fit: {k} regressors{f' and {mz} instruments' if mz else ''} in {len(blocks)} column blocks, "
            f"chunks of {chunk:_} rows (no resident D)")
        t0 = time.perf_counter()
        iterations = 0
        spans = []  # each block's columns within [y] + dcols
        lo = 0
        for b, xb in enumerate(blocks):
            e = eng if b == 0 else Engine(eng.device)
            if b > 0:
                engines.append(e)
            pb = len(xb) + (1 if b == 0 else 0)
            spans.append((lo, pb))
            e.load_codes(codes, levels, pb, weights=w)
            n_obs, fe_dims, fe_card = e.drop_singletons()
            e.stream_pass(1, chunks(list(range(lo, lo + pb))))
            if strategy == "demean":
                e.demean([0], demean_tol, max_iter, check_from=0)
                iterations = 1
            elif strategy == "alt_proj":
                order = sorted(range(len(fe_cols)), key=lambda i: fe_card[i])  # polars_impl.py:485
                if b == 0:
                    iterations, _ = e.demean(order, demean_tol, max_iter, check_from=3)
                else:  # the same sweeps as the first block: no stop test of its own
                    e.demean(order, 0.0, iterations, check_from=3)
            else:
                e.demean([], demean_tol, max_iter, check_from=0)
            lo += pb
        if strategy == "ols":
            iterations, absorbed_df, fe_dims = 0, 0, None
        elif strategy == "demean":
            absorbed_df = fe_dims[0] - 1
        else:
            absorbed_df = sum(fe_dims) - len(fe_cols)
        df_resid = n_obs - (k + 1) - absorbed_df
        Dc = eng.dev_alloc(P * chunk)
        r = eng.dev_alloc(chunk)
        eng.sync()

        def fill(row0, colsall):  # the chunk's [1_kept, y~, x~, z~] from every block
            col0 = 1
            for b, (lo_b, pb) in enumerate(spans):
                engines[b].stream_materialize_rows(Dc, chunk, col0, row0, colsall[lo_b:lo_b + pb], 0 if b == 0 else -1)
                col0 += pb
            return len(colsall[0])

        mode_g = 1 if w is not None else 0
        G = np.zeros((P, P))
        for row0, colsall in chunks():  # pass A: the Gram, chunk by chunk
            rows = fill(row0, colsall)
            G += eng.wide_gram_rows(Dc, chunk, row0, rows, 0, P, mode=mode_g)
        t_load = time.perf_counter() - t0
        if mz:  # 2SLS from the Gram of [1, y~, x~, z~] (common.py:188-287)
            iv = inference.IVSystem(G, k, mz, z_has_ones=False)
            beta_full, Vb, to_meat = iv.beta_full, iv.XtX_inv, iv.xhat_meat
            coef = np.concatenate([[-iv.coef[0], 1.0], -iv.coef[1:]])
            keep = [0] + list(range(2, P))
            c0, km = 0, P
        else:
            XtX, Xty = inference.split_gram(G)
            beta_full, XtX_inv = inference.solve_normal(XtX, Xty)  # polars_impl.py:212-226
            Vb, to_meat = XtX_inv[1:, 1:], (lambda M: M)
            coef = np.concatenate([[-beta_full[0], 1.0], -beta_full[1:]])
            keep = None
            c0, km = 2, k
        sub = (lambda M: M) if keep is None else (lambda M: M[np.ix_(keep, keep)])
        stats = np.zeros(4)
        meat = np.zeros((km, km))
        for row0, colsall in chunks():  # pass B: residuals, statistics, the HC1 meat
            rows = fill(row0, colsall)
            stats += eng.wide_resid_rows(Dc, chunk, row0, rows, coef, r)
            if v == "hc1":
                meat += eng.wide_gram_rows(Dc, chunk, row0, rows, c0, km, mode=2 if w is not None else 3, r=r)
        rss_w, rss, sum_y, sum_y2 = stats
        if v == "iid":
            se = inference.se_iid(Vb, rss_w, df_resid)
        else:
            se = inference.se_hc1(Vb, to_meat(sub(meat)), n_obs, df_resid)
        if mz:
            se = se[1:]
        tss = sum_y2 - sum_y * sum_y / n_obs if n_obs else 0.0
        timings = dict(eng.timings(), load_s=t_load, total_s=time.perf_counter() - t_start)
    finally:
        for ptr in (Dc, r):
            if ptr is not None:
                eng.dev_free(ptr)
        for e in engines[1:]:
            e.close()
        if engine is None:
            eng.close()
    return LeanFEResult(coefs=dict(zip(x_cols, (float(b_) for b_ in beta_full[1:]))),
                        std_errors=dict(zip(x_cols, (float(s_) for s_ in se))), n_obs=n_obs,
                        iterations=iterations, vcov_type=vcov, is_iv=bool(mz), n_instruments=mz or None,
                        n_clusters=None, df_resid=df_resid, formula=formula, fe_cols=fe_cols,
                        fe_dims=fe_dims, r_squared=None if mz else (1 - rss / tss if tss > 0 else None),
                        compression_ratio=None, rss=float(rss), tss=None if mz else tss, backend="hip",
                        timings=timings)


def _wide_fit(cols, y_col, x_cols, fe_cols, weights, cluster_cols, v, vcov, ssc, strategy, demean_tol, max_iter,
              formula, t_start, say, engine=None, device=None, ooc=None, instruments=()) -> LeanFEResult:
    """A fit of more than 63 columns (e.g. an event study's i(year) dummies, polars_impl.py:27-69,
    whose X'X the reference forms at any width, :165-209): the columns run in blocks of engine
    contexts - the first [y] + 62 regressors with the stop test, every later one 63 regressors
    with exactly the first block's number of sweeps (each column's projections are its own,
    :491-508) - and each block writes its demeaned columns into one device matrix D = [1_kept, y~,
    x~] (input row order, lfe_materialize).  The Gram, the residual, the HC1 meat and the cluster
    score sums then come from D (lfe_wide.hip), the solve and the sandwiches from the host as in
    the resident fit (inference.py, std_errors.py:183-441).  ``ooc`` (out-of-core source: the
    arguments of _stream_chunks): every block is a streamed context - group sums from one pass over
    its columns, codes-only sweeps, then a second pass writes its x~ into D (lfe_stream_materialize) -
    so the columns are never resident twice; D itself (P n doubles) stays on the device.
    ``instruments`` (IV / 2SLS, common.py:188-287): D = [1_kept, y~, x~, z~]; 2SLS from D's Gram
    (inference.IVSystem), the residual over u = [1, x~, z~] and its meats over u (D's column 1
    dropped), mapped to the X_hat space as in the resident fit (std_errors.py:448-602)."""
    if ooc is not None and v in ("iid", "hc1") and KNOBS["wide_chunked"]:
        return _wide_fit_chunked(cols, y_col, x_cols, fe_cols, weights, v, vcov, strategy, demean_tol, max_iter,
                                 formula, t_start, say, engine, device, ooc, instruments)
    instruments = list(instruments)
    k, mz = len(x_cols), len(instruments)
    if mz and not fe_cols:
        raise ValueError("a wide IV fit takes one or more FEs (demeaned instruments are never all ones)")
    dcols = list(x_cols) + instruments  # D's columns after [1, y~]
    P = 2 + len(dcols)
    w = None if weights is None else np.asarray(cols[weights], dtype=np.float64)
    y = None if ooc is not None else np.asarray(cols[y_col], dtype=np.float64)
    n = ooc["n_rows"] if ooc is not None else y.size
    ldD = (n + 63) // 64 * 64
    per = MAX_CONTEXT_COLS - (1 if ooc is not None and w is not None else 0)  # streamed weighted sums: p <= 62
    blocks = [dcols[:per - 1]] + [dcols[j:j + per] for j in range(per - 1, len(dcols), per)]
    dev = _default_device() if device is None else device
    eng = engine if engine is not None else Engine(dev)
    D = r = None
    try:
        codes, levels = [], []
        for fe in fe_cols:
            c, g = frame.factorize(cols[fe], device=eng)
            codes.append(c)
            levels.append(g)
        if strategy == "auto":
            strategy = "demean" if len(fe_cols) == 1 else ("alt_proj" if fe_cols else "ols")
        if strategy == "demean" and len(fe_cols) != 1:
            raise ValueError("Strategy 'demean' requires exactly one FE column.")
        if strategy == "alt_proj" and not fe_cols:
            raise ValueError("Strategy 'alt_proj' requires FE-cols. Use strategy='ols' instead for OLS without FE.")
        if strategy == "ols" and fe_cols:
            raise ValueError("Strategy 'ols' takes no fixed effects")
        say(f"Wide fit: {k} regressors{f' and {mz} instruments' if mz else ''} in {len(blocks)} column blocks")
        t0 = time.perf_counter()
        D = eng.dev_alloc(P * ldD)
        eng.sync()  # zero-filled before any block's context writes into it
        iterations = 0
        col0 = 1
        for b, xb in enumerate(blocks):
            e = eng if b == 0 else Engine(eng.device)
            try:
                pb = len(xb) + (1 if b == 0 else 0)
                if ooc is None:
                    colsb = ([y] if b == 0 else []) + [np.asarray(cols[c], dtype=np.float64) for c in xb]
                    e.load(colsb, codes, levels, w)
                else:
                    # the block's indices in [y] + x_cols: block 0 holds y and x[0:62], block b the next 63
                    lo = 0 if b == 0 else col0 - 1
                    sel = list(range(lo, lo + pb))

                    def chunks(sel=sel):
                        return _stream_chunks(ooc["source"], cols, n, ooc["chunk_rows"], y_col, x_cols, instruments,
                                              ooc["plan"], ooc["x_base"], select=sel)

                    e.load_codes(codes, levels, pb, weights=w)
                n_obs, fe_dims, fe_card = e.drop_singletons()
                if ooc is not None:
                    e.stream_pass(1, chunks())
                if strategy == "demean":
                    it, _ = e.demean([0], demean_tol, max_iter, check_from=0)
                    iterations = 1
                elif strategy == "alt_proj":
                    order = sorted(range(len(fe_cols)), key=lambda i: fe_card[i])  # polars_impl.py:485
                    if b == 0:
                        iterations, _ = e.demean(order, demean_tol, max_iter, check_from=3)
                    else:  # the same sweeps as the first block: no stop test of its own
                        e.demean(order, 0.0, iterations, check_from=3)
                else:
                    e.demean([], demean_tol, max_iter, check_from=0)
                if ooc is None:
                    e.materialize(D, ldD, 0, col0, 0 if b == 0 else -1)
                else:
                    e.stream_materialize(D, ldD, col0, chunks(), 0 if b == 0 else -1)
                col0 += pb
                e.sync()
            finally:
                if b > 0:
                    e.close()
        t_load = time.perf_counter() - t0
        if strategy == "ols":
            iterations, absorbed_df, fe_dims = 0, 0, None
        elif strategy == "demean":
            absorbed_df = fe_dims[0] - 1
        else:
            absorbed_df = sum(fe_dims) - len(fe_cols)
        df_resid = n_obs - (k + 1) - absorbed_df
        G = eng.wide_gram(D, ldD, 0, P, mode=1 if w is not None else 0)
        if mz:  # 2SLS from the Gram of [1, y~, x~, z~] (common.py:188-287)
            iv = inference.IVSystem(G, k, mz, z_has_ones=False)
            beta_full, Vb, to_meat = iv.beta_full, iv.XtX_inv, iv.xhat_meat
            coef = np.concatenate([[-iv.coef[0], 1.0], -iv.coef[1:]])  # r = y~ - u coef, u = [1, x~, z~]
            keep = [0] + list(range(2, P))  # u's columns in D (y~ dropped from the meats)
            c0, km = 0, P
        else:
            XtX, Xty = inference.split_gram(G)
            beta_full, XtX_inv = inference.solve_normal(XtX, Xty)  # polars_impl.py:212-226
            Vb, to_meat = XtX_inv[1:, 1:], (lambda M: M)
            coef = np.concatenate([[-beta_full[0], 1.0], -beta_full[1:]])
            keep = None
            c0, km = 2, k
        sub = (lambda M: M) if keep is None else (lambda M: M[np.ix_(keep, keep)])
        r = eng.dev_alloc(ldD)
        rss_w, rss, sum_y, sum_y2 = eng.wide_resid(D, ldD, coef, r)
        n_clusters = None
        if v == "iid":
            se = inference.se_iid(Vb, rss_w, df_resid)
        elif v == "hc1":
            meat = eng.wide_gram(D, ldD, c0, km, mode=2 if w is not None else 3, r=r)
            se = inference.se_hc1(Vb, to_meat(sub(meat)), n_obs, df_resid)
        else:
            _load_clusters(eng, cols, cluster_cols, False)
            subsets = inference.cluster_subsets(len(cluster_cols))
            meats, Gs = eng.wide_cluster_meats(D, ldD, c0, km, r, subsets)
            meats = [to_meat(sub(M)) for M in meats]
            if len(cluster_cols) == 1:
                se, n_clusters = inference.se_cluster_oneway(Vb, meats[0], int(Gs[0]), n_obs, df_resid, ssc)
            else:
                se, n_clusters = inference.se_cluster_multiway(Vb, list(meats), [int(g) for g in Gs], subsets, n_obs,
                                                               df_resid, ssc)
        if mz:  # the intercept's row of the IV covariance (polars_impl.py:238 slices it off)
            se = se[1:]
        tss = sum_y2 - sum_y * sum_y / n_obs if n_obs else 0.0
        timings = dict(eng.timings(), load_s=t_load, total_s=time.perf_counter() - t_start)
    finally:
        for ptr in (D, r):
            if ptr is not None:
                eng.dev_free(ptr)
        if engine is None:
            eng.close()
    return LeanFEResult(coefs=dict(zip(x_cols, (float(b_) for b_ in beta_full[1:]))),
                        std_errors=dict(zip(x_cols, (float(s_) for s_ in se))), n_obs=n_obs,
                        iterations=iterations, vcov_type=vcov, is_iv=bool(mz), n_instruments=mz or None,
                        n_clusters=n_clusters, df_resid=df_resid, formula=formula, fe_cols=fe_cols,
                        fe_dims=fe_dims, r_squared=None if mz else (1 - rss / tss if tss > 0 else None),
                        compression_ratio=None, rss=float(rss), tss=None if mz else tss, backend="hip",
                        timings=timings)


def _beta_agrees(beta_dev, beta_host, rtol: float = 1e-10) -> bool:
    """The fused residual pass used the device Cholesky's beta (lfe_gram_resid); its residuals,
    meats and scores stand for the host solve's (polars_impl.py:212-229) only while the two
    agree to far below the parity bar."""
    scale = max(float(np.max(np.abs(beta_host))), 1e-300)
    return bool(np.all(np.isfinite(beta_dev))) and float(np.max(np.abs(beta_dev - beta_host))) <= rtol * scale


def _load_clusters(eng, cols, cluster_cols, sharded):
    """Cluster columns -> dense codes on the device (in the loaded rows' order)."""
    cl_codes, cl_levels = [], []
    for c in cluster_cols:
        cc, gg = frame.factorize(cols[c], global_codes=sharded, device=None if sharded else eng)
        cl_codes.append(cc)
        cl_levels.append(gg)
    cl_levels = dist.agree_levels(eng, cl_levels)
    eng.load_clusters(cl_codes, cl_levels)
    return cl_levels


def _cluster_se(eng, cols, cluster_cols, sharded, Vb, to_meat, n_obs, df_resid, ssc, loaded=None):
    """One-way (std_errors.py:289-347) or CGM multi-way (:354-441) SEs from the device's
    score meats; ``to_meat`` maps a device meat to the estimator's space (identity for
    OLS, gamma' M_Z gamma for IV, :473-602).  ``loaded``: the cluster columns are on the
    device already (they moved with the rows of an owner re-shard)."""
    if loaded is None:
        _load_clusters(eng, cols, cluster_cols, sharded)
    if len(cluster_cols) == 1:
        meats, Gs = eng.cluster_meat()
        return inference.se_cluster_oneway(Vb, to_meat(meats[0]), int(Gs[0]), n_obs, df_resid, ssc)
    # intersections are formed and grouped on the device (std_errors.py:399-408)
    subsets = inference.cluster_subsets(len(cluster_cols))
    meats, Gs = eng.cluster_meat_subsets(subsets)
    return inference.se_cluster_multiway(Vb, [to_meat(M) for M in meats], [int(g) for g in Gs], subsets,
                                         n_obs, df_resid, ssc)


def _iv_fit(eng, cols, x_cols, instruments, cluster_cols, v, z_has_ones, sharded, n_obs, df_resid, ssc,
            cl_loaded=None):
    """IV/2SLS branch of ``_run_regression`` (polars_impl.py:176-200, 229, 254-270):
    the device Gram of [1, y~, x~, z~] -> host 2SLS (inference.IVSystem) -> one device
    residual pass r = y~ - X_hat beta_full with u = [1, x~, z~] meats / scores -> the
    reference's IV SEs (std_errors.py:448-602), intercept stripped."""
    k, m = len(x_cols), len(instruments)
    G = eng.gram()
    iv = inference.IVSystem(G, k, m, z_has_ones=z_has_ones)
    stats, meat_u = eng.resid_iv(iv.coef, meat=(v == "hc1"), keep_scores=(v == "cluster"))
    n_clusters = None
    XtX_inv = iv.XtX_inv
    if v == "iid":
        se = inference.se_iid(XtX_inv, stats[0], df_resid)
    elif v == "hc1":
        se = inference.se_hc1(XtX_inv, iv.xhat_meat(meat_u), n_obs, df_resid)
    else:
        se, n_clusters = _cluster_se(eng, cols, cluster_cols, sharded, XtX_inv, iv.xhat_meat, n_obs, df_resid, ssc,
                                     cl_loaded)
    strip = len(iv.beta_full) == k + 1
    beta = iv.beta_full[1:] if strip else iv.beta_full
    se = se[1:] if strip else se
    return beta, se, n_clusters, float(stats[1]), stats


def _compress_fit(eng, cols, x_cols, fe_cols, fe_card, cluster_cols, v, vcov, ssc, formula, t_start, t_load):
    """YOCO ``strategy='compress'`` (leanfe_compress_polars, compress.py:1049-1175) on the device.

    lfe_compress groups the loaded rows by (x, FE, cluster) into records (compress.py:282-358);
    the exact LSDV fit of the records (build_design_matrix + solve_wls, :503-747) is computed in
    its FWL form: weighted alternating projections of the records run to machine precision
    (stopping when the weighted group means no longer decrease), then the weighted Gram and the
    host solve give beta and the x block of the LSDV (X'WX)^-1.  The residual pass forms the
    grouped RSS (:754-811), the HC1 meat sum_g rss_g x~ x~' (:907-919) and the cluster scores
    x~_g e_g (:922-1042), whose x rows equal the reference's [X'WX]^-1 X' rows.
    """
    cl_codes = None
    if cluster_cols is not None:
        # polars_impl.py:407-416 passes cluster_cols whatever vcov is: they join the group key
        cl_codes, cl_levels = [], []
        for c in cluster_cols:
            cc, gg = frame.factorize(cols[c], device=eng)
            cl_codes.append(cc)
            cl_levels.append(gg)
        eng.load_clusters(cl_codes, cl_levels)
    n_obs = eng.n
    n_compressed = eng.compress()
    _, _, card = eng.drop_singletons()  # records mode: every record kept
    order = sorted(range(len(fe_cols)), key=lambda i: card[i])
    eng.demean(order, 0.0, 100_000, check_from=1)  # to the rounding floor (stall stop in the engine)
    k = len(x_cols)
    G = eng.gram()
    XtX, Xty = inference.split_gram(G)
    beta_full, XtX_inv = inference.solve_normal(XtX, Xty)
    Vb = XtX_inv[1:, 1:]
    fe_dims = tuple(int(c) for c in card) if fe_cols else None
    P = 1 + k + sum(int(c) - 1 for c in card)  # [1, x, dummies of every level but the first]
    df_resid = n_obs - P
    if fe_cols:
        stats, meat = eng.resid(beta_full, hc1=(v == "hc1"), keep_scores=(v == "cluster"))
    else:
        # no FE: x is not demeaned, so the reference's sandwich spans the intercept
        # (the full design's XtX_inv and meat, compress.py:907-919): u = [1, x] meats / scores
        stats, meat = eng.resid_iv(beta_full, meat=(v == "hc1"), keep_scores=(v == "cluster"))
        Vb = XtX_inv
    rss = float(stats[0])
    n_clusters = None
    if v == "iid":
        se = inference.se_iid(Vb, rss, df_resid)
    elif v == "hc1":
        se = inference.se_hc1(Vb, meat, n_obs, df_resid)
    else:
        if len(cluster_cols) == 1:
            meats, Gs = eng.cluster_meat()
            se, n_clusters = inference.se_cluster_oneway(Vb, meats[0], int(Gs[0]), n_obs, df_resid, ssc)
        else:
            subsets = inference.cluster_subsets(len(cluster_cols))
            meats, Gs = eng.cluster_meat_subsets(subsets)
            se, n_clusters = inference.se_cluster_multiway(Vb, list(meats), [int(g) for g in Gs], subsets, n_obs,
                                                           df_resid, ssc)
    beta = beta_full[1:]
    if not fe_cols:
        se = se[1:]
    timings = dict(eng.timings(), load_s=t_load, total_s=time.perf_counter() - t_start)
    return LeanFEResult(coefs=dict(zip(x_cols, (float(b) for b in beta))),
                        std_errors=dict(zip(x_cols, (float(s) for s in se))), n_obs=n_obs,
                        n_compressed=n_compressed, vcov_type=vcov, df_resid=df_resid, rss=rss,
                        n_clusters=n_clusters, fe_dims=fe_dims, formula=formula, fe_cols=fe_cols, backend="hip",
                        timings=timings)

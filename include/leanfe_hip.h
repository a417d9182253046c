/* leanfe_hip.h — C ABI of the MI355X (gfx950) fixed-effects demean + solve engine.
 *
 * This is the drop-in boundary for leanfe's `strategy='alt_proj'` / `'demean'`
 * hot path.  The reference has no FFI: its only seam is the backend string
 * dispatch in `leanfe()` (python/leanfe/leanfe.py:138-184).  Each entry point
 * below replaces one block of the reference's Polars backend, cited as
 * (reference file:line).  Python binds it with ctypes (leanfe_amd/_lib.py),
 * which releases the GIL for every call.
 *
 * Conventions
 *   - return 0 on success, a negative LFE_E* code on failure; lfe_last_error()
 *     (thread-local) describes the last failure.
 *   - all host buffers are caller-owned; outputs go to caller-provided buffers.
 *   - device memory is owned by the context and reused across calls.
 *   - one context is not thread-safe; use one per host thread.
 *   - non-convergence is not an error: *iterations_out == max_iter, as in the
 *     reference (polars_impl.py:526).
 */
#ifndef LEANFE_HIP_H
#define LEANFE_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lfe_ctx lfe_ctx;

enum {
  LFE_OK = 0,
  LFE_EINVAL = -1, /* bad argument (maps to ValueError) */
  LFE_EHIP = -2,   /* HIP runtime failure (RuntimeError) */
  LFE_ERCCL = -3,  /* RCCL failure (RuntimeError) */
  LFE_ENOMEM = -4, /* device allocation failure (MemoryError) */
  LFE_ESTATE = -5, /* call out of order (RuntimeError) */
  LFE_ENEEDPASS = -6 /* streamed X: lfe_gram needs the streamed design-Gram pass (lfe_stream_begin pass 3) */
};

enum { LFE_HOST = 0, LFE_DEVICE = 1 };

/* Context on one GPU (`device` = HIP ordinal).  Owns one HIP stream. */
int lfe_ctx_create(lfe_ctx** out, int device);
void lfe_ctx_destroy(lfe_ctx* ctx);

/* Multi-GPU: join an RCCL communicator (one process per GPU).  `unique_id` is
 * the 128-byte id from lfe_comm_unique_id() on rank 0, broadcast by the caller.
 * Every reduction below (counts, per-group partial sums, Gram, SE partials)
 * is then summed over the ranks' row shards. */
int lfe_comm_unique_id(void* out128);
int lfe_ctx_set_comm(lfe_ctx* ctx, const void* unique_id128, int rank, int world);

/* An in-process group of `world` contexts (each driven by its own host thread) whose
 * collectives go through host memory behind a barrier, in the same order as with RCCL: the
 * multi-rank paths tested on one GPU, and a fit of more rows than one context holds (< 2^31
 * rows per context) as several contexts on one device.  lfe_emu_abort (a member failed): every
 * collective waiting in the group, and every later one, returns LFE_ESTATE. */
typedef struct lfe_emu lfe_emu;
int lfe_emu_create(int world, lfe_emu** out);
void lfe_emu_destroy(lfe_emu* emu);
void lfe_emu_abort(lfe_emu* emu);
int lfe_ctx_set_emu(lfe_ctx* ctx, lfe_emu* emu, int rank);

/* Upload one row shard.  cols[0] = y, cols[1..p-1] = x (then instruments),
 * f64; fe_codes[f] = dense int32 codes in [0, n_levels[f]) (global across
 * shards); weights may be NULL.  `where` = LFE_HOST or LFE_DEVICE for the
 * source pointers.  Replaces the data handoff of polars_impl.py:324-356. */
int lfe_load(lfe_ctx* ctx, int64_t n, int p, const double* const* cols, int F,
             const int32_t* const* fe_codes, const int32_t* n_levels,
             const double* weights, int where);

/* Chunked upload for streaming ingest (the reference streams
 * Parquet with pl.scan_parquet, polars_impl.py:341-343).  lfe_load_begin sizes the shard
 * (n rows, p columns, F FEs with n_levels, weighted or not); lfe_load_rows copies rows
 * [row0, row0 + rows) of every column (and code array, and weights) from host memory
 * asynchronously, returning once the copies issued two calls earlier have completed, so
 * the caller keeps the host arrays of its last two calls alive and decodes the next chunk
 * while this one crosses PCIe; lfe_load_finish waits, validates the codes (as lfe_load)
 * and marks the shard loaded.  The calls must cover every row exactly once. */
int lfe_load_begin(lfe_ctx* ctx, int64_t n, int p, int F, const int32_t* n_levels, int weighted);
int lfe_load_rows(lfe_ctx* ctx, int64_t row0, int64_t rows, const double* const* cols,
                  const int32_t* const* fe_codes, const double* weights);
int lfe_load_finish(lfe_ctx* ctx);

/* Fill the context with rows [row_offset, row_offset+n) of the counter-based
 * synthetic panel (leanfe_amd/synth.py) directly on the device: p = 1 + k
 * columns, F = n_fe FE code arrays with n_levels[f] levels. */
int lfe_synth_load(lfe_ctx* ctx, int64_t n, int k, int n_fe, const int32_t* n_levels,
                   const double* beta, uint64_t seed, int64_t row_offset);

/* Owner-sharded rows (multi-GPU, SURVEY.md §8e "balanced by fe1 segment"): declare that
 * this rank holds EVERY row whose code of FE `fe` lies in [lo, hi) and no other row
 * (validated against the loaded codes; LFE_EINVAL otherwise).  When `fe` is the primary
 * FE (most levels) of a two-FE unweighted fit, the engine keeps that FE's counts, group
 * sums S and cross term T rank-local (no all-reduce of the G x p tables of
 * polars_impl.py:491-508's largest FE) and all-reduces only the other FE's tables, the
 * Gram and the SE statistics.  fe = -1 clears it; every lfe_load* clears it. */
int lfe_ctx_set_owner(lfe_ctx* ctx, int fe, int32_t lo, int32_t hi);

/* Owner re-shard (multi-GPU, after every rank loaded a contiguous block of rows with lfe_load):
 * rows move between the ranks so that rank r holds every row whose code of FE `fe` lies in
 * [lo_r, hi_r), the ranges cut where the running count of rows over the all-reduced level counts
 * crosses r N / world (equal rows per rank up to one level's rows).  X, the weights, every FE's
 * codes and the loaded cluster columns move (one grouped ncclSend / ncclRecv set per column);
 * on the receiving rank rows are ordered by (source rank, source row).  Then
 * lfe_ctx_set_owner(ctx, fe, lo_r, hi_r); *lo_out / *hi_out receive this rank's range.  Every
 * rank must call it (collective).  LFE_EINVAL (nothing moved) when a rank would hold no rows.
 * Replaces the caller-side routing by owner and the level-balanced ranges
 * of dist.owner_range. */
int lfe_reshard_owner(lfe_ctx* ctx, int fe, int32_t* lo_out, int32_t* hi_out);

/* The rows of the synthetic panel's rows [0, n_total) whose code of FE `owner_fe` lies in
 * [lo, hi), generated on the device in increasing row order (the same rows and values as
 * lfe_synth_load over the whole panel), then lfe_ctx_set_owner(ctx, owner_fe, lo, hi). */
int lfe_synth_load_owned(lfe_ctx* ctx, int64_t n_total, int k, int n_fe, const int32_t* n_levels,
                         const double* beta, uint64_t seed, int owner_fe, int32_t lo, int32_t hi);

/* Cluster code arrays for SEs, in the same row order as lfe_load (dense int32
 * codes, n_levels[j] each).  Subsets/intersections are passed as separate
 * arrays (std_errors.py:396-408). */
int lfe_load_clusters(lfe_ctx* ctx, int m, const int32_t* const* cl_codes,
                      const int32_t* cl_levels, int where);

/* YOCO compression (compress.py:282-358): group the loaded rows
 * by every regressor (columns 1..p-1, exact f64 values; -0.0 == 0.0, NaNs alike), FE
 * code and loaded cluster column, and replace them in the context by one record per
 * group: column 0 = _mean_y = _sum_y / _n, the key columns, weight _n = count (or
 * sum w), and the record's _sum_y / _sum_y_sq kept on the device.  *n_records_out =
 * number of records (n_compressed).  The context is then in records mode:
 *   - lfe_drop_singletons keeps every record (compress has no singleton drop);
 *     fe_card = fe_dims = levels present;
 *   - lfe_demean runs weighted projections and stops when the weighted group means of
 *     y~ are below tol or no longer decrease (20 checks without a new minimum): the
 *     FWL form of the exact LSDV solve (build_design_matrix + solve_wls, :503-747);
 *   - lfe_resid returns stats_out[0] = sum_g rss_g with rss_g = _sum_y_sq -
 *     2 fit_g _sum_y + _n fit_g^2 (compute_rss_grouped, :754-811), the HC1 meat
 *     sum_g rss_g x~_g x~_g' (:907-919) and scores x~_g e_g, e_g = _sum_y - _n fit_g
 *     (:1118-1124), fit_g = _mean_y - r_g; lfe_resid_iv likewise with u = [1, x]
 *     (records without FEs: the reference's meat spans the intercept, :907-919).
 * One process only. */
int lfe_compress(lfe_ctx* ctx, int64_t* n_records_out);

/* Single-pass singleton drop (polars_impl.py:477-482; :433-435 for 'demean'):
 * keep a row iff every FE's pre-filter group count is > 1.  Outputs the kept
 * row count (global over ranks), per-FE distinct levels among kept rows
 * (fe_dims, :531-534) and pre-filter cardinality (fe_card, :373).  Either
 * output pointer may be NULL. */
int lfe_drop_singletons(lfe_ctx* ctx, int64_t* n_kept, int32_t* fe_dims_out,
                        int32_t* fe_card_out);

/* Alternating projections (polars_impl.py:490-526): for it = 1..max_iter,
 * project every FE in `fe_order`; from it >= check_from stop when
 * max_f max_g |mean_g(y)| < tol (y only, unweighted).  check_from <= 0 means
 * a single projection pass ('demean', polars_impl.py:437-465). */
int lfe_demean(lfe_ctx* ctx, const int* fe_order, double tol, int max_iter, int check_from,
               int* iterations_out, double* last_check_out);

/* Gram of [1, y~, x~] (with sqrt(w) row scaling when weighted), p+1 columns,
 * row-major (p+1)x(p+1), column 0 = intercept, column 1 = y.  Replaces
 * XtX = X'X, Xty = X'Y of polars_impl.py:165-209. */
int lfe_gram(lfe_ctx* ctx, double* gram_out);

/* With beta_full = [intercept, beta_1..beta_k] (host Cholesky solve of the
 * Gram, polars_impl.py:212-225): residual r = y~ - [1, x~] beta_full
 * (:229) and stats_out[0..3] = {sum w r^2, sum r^2, sum y~, sum y~^2}
 * (std_errors.py:196-207, polars_impl.py:281-282).  If hc1_meat is non-NULL it
 * receives the k x k meat sum (w) r^2 x~ x~' (std_errors.py:240-264).
 * If keep_scores != 0 the per-row scores x~ r (w) are kept on the device for
 * lfe_cluster_meat. */
int lfe_resid(lfe_ctx* ctx, const double* beta_full, double* stats_out, double* hc1_meat,
              int keep_scores);

/* IV/2SLS residual pass (polars_impl.py:176-200, 229 with instruments loaded as the
 * columns after x; std_errors.py:448-602).  coef[p] = {c_0, c_1..c_{p-1}} over
 * u = [1, col_1..col_{p-1}] (the host's first stage folded into the second:
 * X_hat beta = Z (gamma beta), zero on the x columns); r = y~ - coef . u, stats_out
 * as lfe_resid; meat_out (p x p, may be NULL) = sum (w) r^2 u u' — the intercept
 * in slot 0, so X_hat' diag(r^2) X_hat = gamma' meat[Z, Z] gamma on the host.
 * keep_scores != 0 keeps u r (w), p wide, for lfe_cluster_meat*. */
int lfe_resid_iv(lfe_ctx* ctx, const double* coef, double* stats_out, double* meat_out, int keep_scores);

/* lfe_gram + solve + lfe_resid with one host round trip: the (p+1)^2 Gram as
 * lfe_gram, the beta_full[p] a one-thread device Cholesky solved from it (used
 * for the residuals; equal to the host's polars_impl.py:212-226 solve up to
 * rounding), then stats/HC1 meat/scores as lfe_resid.  Returns 1 and computes
 * nothing usable when the fused path does not apply (F != 2, weights, p > 11,
 * or X'X not positive definite): call lfe_gram and lfe_resid instead. */
int lfe_gram_resid(lfe_ctx* ctx, double* gram_out, double* beta_full_out, double* stats_out, double* hc1_meat,
                   int keep_scores);

/* One whole regression on the loaded shard in one call (no return to the caller between the
 * steps): [flags & LFE_FIT_DROP: lfe_drop_singletons], lfe_demean with the FEs ordered by
 * pre-filter cardinality (polars_impl.py:485), the Gram with the fused device solve + residual
 * pass (lfe_gram_resid; lfe_gram alone for IID), the host solve (:211-220: Cholesky, LU when X'X
 * is not positive definite) and the SEs: IID (std_errors.py:196-210) from the Gram's residual
 * statistics unless r'r cancels there, HC1 (:275-282).  vcov LFE_FIT_SCORES keeps the score rows
 * for lfe_cluster_meat*: se_out is then 0 and the caller forms the CGM sandwich.  Unweighted,
 * resident, no instruments (every column after y is a regressor): else LFE_EINVAL.
 * Outputs: ints_out[4 + 2F] = {n_obs, iterations, df_resid, fused pass used, fe_dims[F],
 * fe_card[F]}; gram_out (p+1)^2 as lfe_gram; beta_full_out[p]; xtx_inv_out p x p; stats_out[4]
 * as lfe_resid; meat_out k x k (HC1, k = p-1); se_out[k]; diag_out[2] (may be NULL) = {last stop
 * test, |beta_device - beta_host| / max|beta_host|}. */
#define LFE_FIT_IID 0
#define LFE_FIT_HC1 1
#define LFE_FIT_SCORES 2
#define LFE_FIT_DROP 1
int lfe_fit(lfe_ctx* ctx, int flags, double tol, int max_iter, int check_from, int vcov, int64_t* ints_out,
            double* gram_out, double* beta_full_out, double* xtx_inv_out, double* stats_out, double* meat_out,
            double* se_out, double* diag_out);

/* For each loaded cluster array j: S_c = sum_{i in c} u_i r_i (w_i);
 * meats_out[j] = S'S (k x k), G_out[j] = number of clusters present among the
 * kept rows (std_errors.py:317-336, compress.py:929-942 — the W_C'(X.e) SpMM).
 * u and k are those of the last residual pass that kept scores: u = x~, k = p-1
 * (lfe_resid, lfe_gram_resid), or u = [1, x~, z~], k = p (lfe_resid_iv,
 * std_errors.py:473-602). */
int lfe_cluster_meat(lfe_ctx* ctx, double* meats_out, int64_t* G_out);

/* Multi-way CGM subsets on the device (std_errors.py:354-441).  subset_masks[s]
 * selects loaded cluster columns (bit j = column j); its clusters are the distinct
 * tuples of those columns' codes among kept rows (the group_by of the intersection,
 * std_errors.py:399-408), formed and grouped on the device (mixed-radix key, radix
 * sort; no host factorization).  meats_out[s] = S'S, G_out[s] = number of clusters.
 * The product of the selected n_levels must be < 2^62 (and < 2^31 with a
 * communicator); otherwise LFE_EINVAL. */
int lfe_cluster_meat_subsets(lfe_ctx* ctx, int n_subsets, const int32_t* subset_masks, double* meats_out,
                             int64_t* G_out);

/* Host prep on the device.
 * Dense int32 codes of an integer id column in sorted-unique order (np.unique's
 * inverse; polars_impl.py:118-139 only needs group membership): n host int64 ids in,
 * n host codes out, *n_levels_out = number of distinct ids.  Needs no loaded data. */
int lfe_factorize_ids(lfe_ctx* ctx, int64_t n, const int64_t* ids, int32_t* codes_out, int32_t* n_levels_out);

/* Dense int32 codes of a string column (the String branch of _cats_to_int,
 * polars_impl.py:118-139: cast to Categorical, take the physical codes; only group
 * membership matters).  Arrow layout on the host: offsets [n + 1] int64 (offsets[0] = 0,
 * non-decreasing), string i = data[offsets[i], offsets[i + 1]) compared as bytes.  Codes are
 * numbered in the order of 64-bit string hashes, not lexicographically; equal-hash strings
 * are compared byte by byte, so the grouping is exact.  *n_levels_out = number of distinct
 * strings.  Needs no loaded data. */
int lfe_factorize_strings(lfe_ctx* ctx, int64_t n, const int64_t* offsets, const uint8_t* data, int32_t* codes_out,
                          int32_t* n_levels_out);

/* Exact number of distinct rows over the regressors x (loaded columns 1..n_x, not y
 * and not the instruments loaded after x; n_x < 0: every column 1..p-1) and the FE
 * codes, all loaded rows: the numerator of estimate_compression_ratio, whose key is
 * x_cols + fe_cols (compress.py:187-253, :249-250).  -0.0 == 0.0 and NaNs compare
 * equal.  One process only. */
int lfe_count_distinct_rows(lfe_ctx* ctx, int n_x, int64_t* n_distinct_out);

/* Debug/fixtures: copy the demeaned columns (kept rows, device order) to host. */
int lfe_copy_demeaned(lfe_ctx* ctx, double* const* cols_out, int64_t* n_out);

/* Debug/fixtures: copy the loaded inputs (p columns, F code arrays; input row
 * order) back to host buffers. */
int lfe_copy_inputs(lfe_ctx* ctx, double* const* cols_out, int32_t* const* codes_out);

/* Out-of-core X (data larger than HBM; SURVEY.md §8f rank 4, the role of scan_parquet /
 * DuckDB's disk-backed tables, polars_impl.py:341-343, duckdb_impl.py:417-452).  The FE codes
 * (and weights) stay resident with their layouts; the p data columns are streamed in row chunks
 * through the passes below, each a sequence of lfe_stream_rows calls covering rows [0, n)
 * exactly once between lfe_stream_begin and lfe_stream_end:
 *   pass 1 (after lfe_drop_singletons): the group sums S_f of polars_impl.py:491-508 (weighted:
 *          of w x, with W_f = sum w and the unweighted y sums of the stop test) and the raw Gram
 *          of the tables, two-limb fixed point per chunk, folded in chunk order;
 *   lfe_demean (any number of FEs, weighted or not), then lfe_gram (the Gram from the group
 *          tables; LFE_ENEEDPASS when it is unavailable - three or more FEs, weights - or fails
 *          its guard: then pass 3, the Gram of sqrt(w) [1, y~, x~], polars_impl.py:201-209);
 *   pass 2 (beta_full = [intercept, beta]): the residual (polars_impl.py:229), RSS / TSS and the
 *          HC1 meat (std_errors.py:217-282); pass 4 (the 2SLS coefficients of u = [1, x~, z~]):
 *          the IV residual and its meat over u (std_errors.py:448-602);
 *   clustered SEs: lfe_load_clusters (input order) and lfe_stream_clusters(subset masks) before
 *          pass 2 / 4, whose chunks then add their score rows into per-cluster sums; then
 *          lfe_stream_cluster_meats (std_errors.py:289-441).
 * p <= 63 (weighted: 62): up to p = 11 the passes run row per lane (16 x 16 tiles), wider fits on
 * the MFMA lane layout with 16 ceil((p + 1) / 16)-wide tiles.  A sharded engine (lfe_ctx_set_comm)
 * streams its own rows: the sums and every pass's tile are all-reduced, and the clustered score
 * sums go to their owner ranks by cluster key (cluster codes must then be global).
 * cols = p column pointers of `rows` doubles each (kind LFE_HOST / LFE_DEVICE).
 * lfe_stream_end's `out`: pass 2: stats[4] then the (p-1)^2 meat; pass 4: stats[4] then the p^2
 * meat; pass 3: the (p+1)^2 Gram; pass 1 and 5 (materialize): unused - pass 5 returns with D written
 * (the context's stream synchronized: another context's stream reads D next). */
int lfe_load_codes(lfe_ctx* ctx, int64_t n, int p, int F, const int32_t* const* fe_codes,
                   const int32_t* n_levels, const double* weights_or_null, int kind);
int lfe_stream_begin(lfe_ctx* ctx, int pass, const double* beta_full);
int lfe_stream_rows(lfe_ctx* ctx, int64_t row0, int64_t rows, const double* const* cols, int kind);
int lfe_stream_end(lfe_ctx* ctx, double* out);
/* Clustered SEs of a streamed fit: every subset (bit j = loaded cluster column j) factorized on the
 * device once (its intersection, std_errors.py:399-408); the residual passes then fill the
 * per-cluster score sums.  meats_out: n_subsets blocks of ks x ks (ks = p - 1, or p after pass 4);
 * G_out: clusters per subset (among kept rows). */
int lfe_stream_clusters(lfe_ctx* ctx, int n_subsets, const int32_t* masks);
int lfe_stream_cluster_meats(lfe_ctx* ctx, double* meats_out, int64_t* G_out);
/* Benchmark / test helpers: lfe_synth_load's panel with only the codes resident, and one chunk
 * of its columns generated on the device and streamed through the current pass. */
int lfe_synth_load_codes(lfe_ctx* ctx, int64_t n, int k, int n_fe, const int32_t* n_levels, uint64_t seed);
/* The same for rows [row0, row0 + n) of the panel (lfe_stream_synth_rows then generates rows
 * row0 + r): one context of several on one device, each under 2^31 rows, joined in a group
 * (a fit of more rows than one context holds). */
int lfe_synth_load_codes_at(lfe_ctx* ctx, int64_t n, int64_t row0, int k, int n_fe, const int32_t* n_levels,
                            uint64_t seed);
int lfe_stream_synth_rows(lfe_ctx* ctx, int64_t row0, int64_t rows, int k, const int32_t* n_levels,
                          const double* beta, uint64_t seed);

/* Whether the last group sums of the two-FE fast path accumulated exactly (int64
 * fixed point per column, so S does not depend on the order of the adds and a
 * repeated solve is bit-identical): *on = 1, else 0 (f64 atomic sums, or another
 * path).  Replaces nothing in the reference (Polars' group sums are serial). */
int lfe_exact_sums(lfe_ctx* ctx, int* on);

/* Cells of the count tables the last two-FE lfe_demean multiplied on the matrix cores (the dense
 * cross terms, buckets x primary groups per bucket x secondary levels rounded to 16), or 0 when it
 * took the row layouts (lfe_dense.hip).  A diagnostic for the byte model of bench.py; replaces
 * nothing in the reference. */
int lfe_dense_cells(lfe_ctx* ctx, int64_t* cells);
/* Bytes per cell of those tables as the passes read them: 1 for the exact i8 form (count tables
 * x base-128 digits of the effects on v_mfma_i32_16x16x64_i8), 2 for the u16 / f64-MFMA form. */
int lfe_dense_cell_bytes(lfe_ctx* ctx, int32_t* bytes);

/* Wide fits (more than 63 columns: the reference's X'X of any width, polars_impl.py:165-209).
 * A context holds at most 63 columns, so the columns run in blocks of contexts (each loads the
 * codes and its columns; blocks after the first demean with tol = 0 and max_iter = the first
 * block's iterations, so every column gets the same sweeps) and every block writes its demeaned
 * columns into one device matrix D [P][ldD] in input row order:
 *   lfe_dev_alloc / lfe_dev_free: a zero-filled device buffer of n_doubles (the caller frees it);
 *   lfe_materialize: the context's demeaned columns [first, p) into D's columns col0, col0 + 1, ...
 *     (0 on dropped rows) and, mask_col >= 0, the kept-row indicator (1 / 0) into column mask_col;
 *   lfe_stream_materialize: the same for a streamed (codes-only) context - it opens pass 5, whose
 *     chunks (lfe_stream_rows / lfe_stream_synth_rows, all p columns) write x~ into D's rows
 *     row0.. from column col0; lfe_stream_end (out may be null) closes it;
 * then on the block holding y, the weights and the cluster columns (input order, ldD >= its rows):
 *   lfe_wide_gram: out (P x P, host) = sum over rows of s_i D_i D_i' over D's columns [c0, c0 + P),
 *     s = 1 (mode 0), w (1), w r^2 (2), r^2 (3) - the Gram of [1, y~, x~] and the HC1 meat;
 *   lfe_wide_resid: r = D v over D's first P columns (v = [-b0, 1, -b], r: ldD device doubles),
 *     stats = [sum w r^2, sum r^2, sum y~, sum y~^2] over kept rows;
 *   lfe_wide_cluster_meats: per CGM subset (as lfe_cluster_meat_subsets) the meat S'S of the
 *     per-cluster sums of D's columns [c0, c0 + k) times r (w), and the cluster counts. */
int lfe_dev_alloc(lfe_ctx* ctx, int64_t n_doubles, double** dev_out);
int lfe_dev_free(lfe_ctx* ctx, double* dev);
int lfe_materialize(lfe_ctx* ctx, double* D, int64_t ldD, int first, int col0, int mask_col);
int lfe_stream_materialize(lfe_ctx* ctx, double* D, int64_t ldD, int col0, int mask_col);
/* Chunked wide fits (no resident D: the P n doubles of D cap a one-GPU fit near 3.5e8 rows at
 * k = 100): the same for the rows [row0, row0 + rows) only, into D rows 0 .. rows - 1 (one chunk
 * buffer for every column block); then lfe_wide_gram_rows / lfe_wide_resid_rows over that chunk
 * (weights offset by row0), whose Grams, meats and statistics the caller adds in chunk order. */
int lfe_stream_materialize_rows(lfe_ctx* ctx, double* D, int64_t ldD, int col0, int mask_col, int64_t row0,
                                int64_t rows);
int lfe_wide_gram_rows(lfe_ctx* ctx, const double* D, int64_t ldD, int64_t row0, int64_t rows, int c0, int P,
                       int mode, const double* r, double* out);
int lfe_wide_resid_rows(lfe_ctx* ctx, const double* D, int64_t ldD, int64_t row0, int64_t rows, int P,
                        const double* coef, double* r, double* stats);
/* A column block [c_lo, c_lo + p) of the K-regressor synthetic panel (column 0 = y, j = x_j; the
 * generator of lfe_synth_load for any K, beta[K]) generated on the device for rows [row0, + rows)
 * and streamed through the current pass (benchmarks and tests of wide streamed fits). */
int lfe_stream_synth_cols(lfe_ctx* ctx, int64_t row0, int64_t rows, int K, int c_lo, const int32_t* n_levels,
                          const double* beta, uint64_t seed);
int lfe_wide_gram(lfe_ctx* ctx, const double* D, int64_t ldD, int c0, int P, int mode, const double* r, double* out);
int lfe_wide_resid(lfe_ctx* ctx, const double* D, int64_t ldD, int P, const double* coef, double* r, double* stats);
int lfe_wide_cluster_meats(lfe_ctx* ctx, const double* D, int64_t ldD, int c0, int k, const double* r, int n_subsets,
                           const int32_t* masks, double* meats_out, int64_t* G_out);

/* Test-only switches of one context (0 clears them; production code never sets any).
 * LFE_TEST_SHORT_MEMORY: lfe_reshard_owner on this rank reports too little device memory for
 * its staging copy, so that the all-rank refusal can be tested (every rank keeps its rows). */
#define LFE_TEST_SHORT_MEMORY 1
/* LFE_TEST_CLUSTER_SORTED: one-column cluster subsets take the sorted path (keys, radix sort,
 * segmented sums) instead of the sort-free fixed-point sums.
 * LFE_TEST_CLUSTER_STATS: the sort-free sums take their quanta from a statistics pass over the
 * score rows instead of the residual pass's meat. */
#define LFE_TEST_CLUSTER_SORTED 2
#define LFE_TEST_CLUSTER_STATS 4
/* LFE_TEST_SEG_SCATTER: the row sweeps' segment layouts are built by the block scatter
 * (k_seg_scatter2) instead of the sorted build. */
#define LFE_TEST_SEG_SCATTER 8
int lfe_ctx_test_hooks(lfe_ctx* ctx, int flags);

/* Test / A-B knobs (no reference counterpart; tests and bench.py --knob only).  A process-wide
 * name -> value table: the engine never reads the environment, so only this call can move it off
 * its production kernel paths.  value NULL removes the knob; name "*" with value NULL removes all.
 * Names: LFE_DENSE ("0" never / "1" whenever the count tables fit), LFE_DN8 ("0": f64 dense passes),
 * LFE_DN_C8 / LFE_DN_C4 (table build counter width), LFE_SUMS_CG, LFE_TAB3, LFE_CL_FIX, LFE_CL_FUSED,
 * LFE_CL_STATS, LFE_CL_OWNER_MIN_SPAN, LFE_ROW_HASH_BITS / LFE_STR_HASH_BITS (short hashes force
 * collisions), LFE_K1_UNIT, LFE_SEG_SORTED, LFE_GRAM_GEN, ... (the A/B sizes are listed in DESIGN.md).
 * The diagnostics LFE_DN8_TIMING / LFE_SWEEP_TIMING print per-workgroup phase times to stderr. */
int lfe_test_set_knob(const char* name, const char* value);

/* Host helper (no reference counterpart; frame.factorize's dense-code test, polars_impl.py:118-139
 * casts FE columns to integer codes): min and max of n signed integers of `width` bytes (1, 2, 4
 * or 8) in one pass over up to 8 host threads. */
int lfe_int_range(const void* values, int64_t n, int width, int64_t* min_out, int64_t* max_out);

/* Wait for all work queued on the context's stream. */
int lfe_sync(lfe_ctx* ctx);

/* Rows of the loaded shard (input rows, before the singleton drop). */
int lfe_shard_rows(lfe_ctx* ctx, int64_t* n_out);

/* Per-phase device times (ms) of the last lfe_* calls, measured with HIP
 * events on the context's stream: [prep, demean, gram, resid, cluster, last_kernel].
 * Only while lfe_phase_timing(ctx, 1) is on (else zeros): every event record costs host time
 * on the launch path. */
int lfe_timings(lfe_ctx* ctx, double* out6);
int lfe_phase_timing(lfe_ctx* ctx, int enable);

/* Per-kernel HIP-event timing on the context's stream.  lfe_profile(ctx, 1)
 * resets and enables it (each launch is bracketed by an event pair; adds no
 * synchronisation); lfe_kernel_stats() synchronises, folds every pending
 * pair and returns, per kernel name, total milliseconds and launch count.
 * `names` receives n_out NUL-terminated names of at most 32 bytes each. */
int lfe_profile(lfe_ctx* ctx, int enable);
int lfe_kernel_stats(lfe_ctx* ctx, int max, char* names, double* total_ms, int64_t* launches, int* n_out);

const char* lfe_last_error(void);
const char* lfe_version(void);
/* Hash of the engine sources this library was built from (leanfe_amd/build.py source_hash();
 * the Python loader refuses a library whose hash differs from the checked-out sources). */
const char* lfe_build_hash(void);

#ifdef __cplusplus
}
#endif

#endif /* LEANFE_HIP_H */

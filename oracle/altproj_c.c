/* CPU ORACLE (C restatement) — TEST / BASELINE INFRASTRUCTURE ONLY.
 *
 * A direct C restatement of the reference Polars backend's alt_proj hot path,
 * in the reference's own form (each projection subtracts group means from all
 * p data columns), used as bench.py's multi-threaded CPU baseline and as the
 * full-size parity checker of tests/test_gpu_configs.py.  It is checked against
 * oracle/altproj.py (itself pinned to the reference's own functions) by
 * tests/test_oracle_c.py.  The product path (leanfe_amd) never links or calls it.
 *
 *   singleton drop, single pass on pre-filter counts .. polars_impl.py:477-482
 *   FE order (ascending cardinality, stable) ........... polars_impl.py:485
 *   projection c <- c - mean_g(c), unweighted .......... polars_impl.py:502-505
 *   loop + y-only stop test from it >= 3 ............... polars_impl.py:490-526
 *   fe_dims / absorbed_df / df_resid .................... polars_impl.py:531-537, :232
 *   Gram with intercept + Cholesky solve ................ polars_impl.py:165-226
 *   residual (unweighted), R^2 .......................... polars_impl.py:229, :281-283
 *   IID / HC1 SEs ....................................... std_errors.py:183-210, :217-282
 *   one-way cluster SE .................................. std_errors.py:289-347
 *   multi-way CGM (intersection group-by) ............... std_errors.py:354-441 (:399-408)
 *
 * Unweighted fits.  Parallelism is over ROWS on every pass: each thread owns a
 * static row range and a private group table (or Gram / meat partial); the
 * partials are merged in thread order, so a run is deterministic for a fixed
 * thread count (no atomics).  Cluster intersections are grouped by a counting
 * sort on the subset's widest column, then a sort of each bucket by the
 * mixed-radix key of the other columns (row index breaks ties).
 *
 * Build: gcc -O3 -fopenmp -shared -fPIC oracle/altproj_c.c -o oracle/_build/libaltproj.so -lm
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#else
static int omp_get_thread_num(void) { return 0; }
static int omp_get_num_threads(void) { return 1; }
static int omp_get_max_threads(void) { return 1; }
static void omp_set_num_threads(int t) { (void)t; }
#endif

#define MAXF 8
#define MAXCL 8

static int64_t lo_of(int64_t n, int t, int nt) { return n * t / nt; }

/* out[g] = sum over rows with code g of x (rows [0, n)); part: [T][G] scratch */
static void group_sums(const double* x, const int32_t* code, int64_t n, int32_t G, double* part, double* out) {
#pragma omp parallel
  {
    const int t = omp_get_thread_num(), nt = omp_get_num_threads();
    double* mine = part + (size_t)t * G;
    memset(mine, 0, sizeof(double) * (size_t)G);
    const int64_t lo = lo_of(n, t, nt), hi = lo_of(n, t + 1, nt);
    for (int64_t i = lo; i < hi; ++i) mine[code[i]] += x[i];
#pragma omp barrier
#pragma omp for schedule(static)
    for (int32_t g = 0; g < G; ++g) {
      double s = 0.0;
      for (int u = 0; u < nt; ++u) s += part[(size_t)u * G + g];
      out[g] = s;
    }
  }
}

/* c <- c - mean_g(c) over present groups (polars_impl.py:502-505) */
static void project_col(double* c, const int32_t* code, int64_t n, const double* inv_cnt, int32_t G, double* part,
                        double* mean) {
  group_sums(c, code, n, G, part, mean);
#pragma omp parallel for schedule(static)
  for (int32_t g = 0; g < G; ++g) mean[g] *= inv_cnt[g];
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) c[i] -= mean[code[i]];
}

/* cnt[g] = rows with code g; part: [T][G] int scratch */
static void group_counts(const int32_t* code, int64_t n, int32_t G, int32_t* part, int32_t* cnt) {
#pragma omp parallel
  {
    const int t = omp_get_thread_num(), nt = omp_get_num_threads();
    int32_t* mine = part + (size_t)t * G;
    memset(mine, 0, sizeof(int32_t) * (size_t)G);
    const int64_t lo = lo_of(n, t, nt), hi = lo_of(n, t + 1, nt);
    for (int64_t i = lo; i < hi; ++i) mine[code[i]]++;
#pragma omp barrier
#pragma omp for schedule(static)
    for (int32_t g = 0; g < G; ++g) {
      int32_t s = 0;
      for (int u = 0; u < nt; ++u) s += part[(size_t)u * G + g];
      cnt[g] = s;
    }
  }
}

static int cholesky_solve(int m, const double* A, double* L, const double* b, double* x, double* inv) {
  /* L L^T = A (row-major m x m); x = A^-1 b; inv = A^-1 (polars_impl.py:212-226) */
  memset(L, 0, sizeof(double) * m * m);
  for (int j = 0; j < m; ++j) {
    double s = A[j * m + j];
    for (int k = 0; k < j; ++k) s -= L[j * m + k] * L[j * m + k];
    if (!(s > 0.0)) return -1;
    L[j * m + j] = sqrt(s);
    for (int i = j + 1; i < m; ++i) {
      double t = A[i * m + j];
      for (int k = 0; k < j; ++k) t -= L[i * m + k] * L[j * m + k];
      L[i * m + j] = t / L[j * m + j];
    }
  }
  double* y = (double*)malloc(sizeof(double) * m);
  for (int col = -1; col < m; ++col) { /* col -1: solve for b; else unit vector e_col */
    for (int i = 0; i < m; ++i) {
      double t = col < 0 ? b[i] : (i == col ? 1.0 : 0.0);
      for (int k = 0; k < i; ++k) t -= L[i * m + k] * y[k];
      y[i] = t / L[i * m + i];
    }
    for (int i = m - 1; i >= 0; --i) {
      double t = y[i];
      for (int k = i + 1; k < m; ++k) t -= L[k * m + i] * (col < 0 ? x[k] : inv[k * m + col]);
      if (col < 0) x[i] = t / L[i * m + i];
      else inv[i * m + col] = t / L[i * m + i];
    }
  }
  free(y);
  return 0;
}

/* V += sign * Vb M Vb (k x k, row-major) */
static void sandwich_add(int k, const double* Vb, const double* M, double sign, double* V) {
  double* t = (double*)calloc((size_t)k * k, sizeof(double));
  for (int a = 0; a < k; ++a)
    for (int j = 0; j < k; ++j) {
      double s = 0.0;
      for (int i = 0; i < k; ++i) s += Vb[a * k + i] * M[i * k + j];
      t[a * k + j] = s;
    }
  for (int a = 0; a < k; ++a)
    for (int b = 0; b < k; ++b) {
      double s = 0.0;
      for (int j = 0; j < k; ++j) s += t[a * k + j] * Vb[j * k + b];
      V[a * k + b] += sign * s;
    }
  free(t);
}

/* ---- cluster meats (std_errors.py:289-347 one-way, :354-441 per CGM subset) ----
 * score rows u_i = x~_i r_i (k wide, kept rows).  meat = sum_c S_c S_c^T with
 * S_c = sum_{i in c} u_i; returns the number of clusters present. */

/* one column: dense S table [G][k]; thread t owns the row range t, partial meats merged in order */
static int64_t meat_oneway(int k, int64_t n, double* const* X, const double* r, const int32_t* code, int32_t G,
                           double* meat) {
  double* S = (double*)calloc((size_t)G * k, sizeof(double));
  char* present = (char*)calloc((size_t)G, 1);
  /* columns in parallel: each thread owns whole S columns (rows in order: deterministic) */
#pragma omp parallel for schedule(static)
  for (int j = 0; j < k; ++j) {
    const double* x = X[j + 1];
    for (int64_t i = 0; i < n; ++i) S[(size_t)code[i] * k + j] += x[i] * r[i];
  }
  for (int64_t i = 0; i < n; ++i) present[code[i]] = 1;
  int64_t Gp = 0;
  for (int32_t g = 0; g < G; ++g) Gp += present[g];
  const int T = omp_get_max_threads();
  double* part = (double*)calloc((size_t)T * k * k, sizeof(double));
#pragma omp parallel
  {
    const int t = omp_get_thread_num(), nt = omp_get_num_threads();
    double* mine = part + (size_t)t * k * k;
    const int64_t g0 = lo_of(G, t, nt), g1 = lo_of(G, t + 1, nt);
    for (int64_t g = g0; g < g1; ++g) {
      if (!present[g]) continue;
      const double* s = S + (size_t)g * k;
      for (int a = 0; a < k; ++a)
        for (int b = a; b < k; ++b) mine[a * k + b] += s[a] * s[b];
    }
  }
  memset(meat, 0, sizeof(double) * k * k);
  for (int t = 0; t < T; ++t)
    for (int a = 0; a < k; ++a)
      for (int b = a; b < k; ++b) meat[a * k + b] += part[(size_t)t * k * k + a * k + b];
  for (int a = 0; a < k; ++a)
    for (int b = 0; b < a; ++b) meat[a * k + b] = meat[b * k + a];
  free(part);
  free(present);
  free(S);
  return Gp;
}

typedef struct {
  uint64_t key;
  int64_t row;
} KeyRow;

static int cmp_keyrow(const void* a, const void* b) {
  const KeyRow* x = (const KeyRow*)a;
  const KeyRow* y = (const KeyRow*)b;
  if (x->key != y->key) return x->key < y->key ? -1 : 1;
  return x->row < y->row ? -1 : (x->row > y->row);
}

/* intersection of the columns in `cols` (>= 2): counting sort by the widest column, then each
 * bucket sorted by the mixed-radix key of the others (the group_by of std_errors.py:399-408) */
static int64_t meat_intersect(int k, int64_t n, double* const* X, const double* r, int nc, int32_t* const* cols,
                              const int32_t* levels, double* meat) {
  int wide = 0;
  for (int j = 1; j < nc; ++j)
    if (levels[j] > levels[wide]) wide = j;
  const int32_t Gw = levels[wide];
  const int32_t* cw = cols[wide];
  const int T = omp_get_max_threads();
  int32_t* cnt = (int32_t*)malloc(sizeof(int32_t) * (size_t)Gw);
  int32_t* ipart = (int32_t*)malloc(sizeof(int32_t) * (size_t)T * Gw);
  group_counts(cw, n, Gw, ipart, cnt);
  free(ipart);
  int64_t* off = (int64_t*)malloc(sizeof(int64_t) * ((size_t)Gw + 1));
  off[0] = 0;
  for (int32_t g = 0; g < Gw; ++g) off[g + 1] = off[g] + cnt[g];
  free(cnt);
  int64_t* cur = (int64_t*)malloc(sizeof(int64_t) * (size_t)Gw);
  memcpy(cur, off, sizeof(int64_t) * (size_t)Gw);
  KeyRow* kr = (KeyRow*)malloc(sizeof(KeyRow) * (size_t)(n > 0 ? n : 1));
  for (int64_t i = 0; i < n; ++i) { /* rows in order: buckets keep row order */
    uint64_t key = 0;
    for (int j = 0; j < nc; ++j)
      if (j != wide) key = key * (uint64_t)levels[j] + (uint64_t)cols[j][i];
    const int64_t d = cur[cw[i]]++;
    kr[d].key = key;
    kr[d].row = i;
  }
  free(cur);
  double* part = (double*)calloc((size_t)T * k * k, sizeof(double));
  int64_t* gpart = (int64_t*)calloc((size_t)T, sizeof(int64_t));
#pragma omp parallel
  {
    const int t = omp_get_thread_num(), nt = omp_get_num_threads();
    double* mine = part + (size_t)t * k * k;
    double* s = (double*)malloc(sizeof(double) * (k > 0 ? k : 1));
    int64_t Gt = 0;
    const int64_t b0 = lo_of(Gw, t, nt), b1 = lo_of(Gw, t + 1, nt);
    for (int64_t b = b0; b < b1; ++b) {
      const int64_t lo = off[b], hi = off[b + 1];
      if (hi <= lo) continue;
      if (hi - lo > 1) qsort(kr + lo, (size_t)(hi - lo), sizeof(KeyRow), cmp_keyrow);
      int64_t i = lo;
      while (i < hi) {
        const uint64_t key = kr[i].key;
        for (int a = 0; a < k; ++a) s[a] = 0.0;
        for (; i < hi && kr[i].key == key; ++i) {
          const int64_t row = kr[i].row;
          for (int a = 0; a < k; ++a) s[a] += X[a + 1][row] * r[row];
        }
        for (int a = 0; a < k; ++a)
          for (int c2 = a; c2 < k; ++c2) mine[a * k + c2] += s[a] * s[c2];
        ++Gt;
      }
    }
    gpart[t] = Gt;
    free(s);
  }
  memset(meat, 0, sizeof(double) * k * k);
  int64_t G = 0;
  for (int t = 0; t < T; ++t) {
    G += gpart[t];
    for (int a = 0; a < k; ++a)
      for (int b = a; b < k; ++b) meat[a * k + b] += part[(size_t)t * k * k + a * k + b];
  }
  for (int a = 0; a < k; ++a)
    for (int b = 0; b < a; ++b) meat[a * k + b] = meat[b * k + a];
  free(part);
  free(gpart);
  free(kr);
  free(off);
  return G;
}

/* cols: p column pointers (y first), n rows each; codes: F arrays of int32 in [0, levels[f]).
 * vcov: 0 IID, 1 HC1, 2 cluster (m cluster columns cl_codes / cl_levels, dense codes).
 * Outputs: beta[k], se[k] (k = p - 1), iterations, n_obs, df_resid, n_clusters[m] (cluster:
 * first-order counts), stats[4] = (rss, tss, r2, G_min), meats[(2^m - 1) k k] (or null; CGM
 * subsets in itertools.combinations order), G_sub[2^m - 1] (or null).  Returns 0, or -1 on a
 * singular Gram / bad input.  `threads` <= 0: OpenMP default. */
int lfe_oracle_fit(int64_t n, int p, const double* const* cols, int F, const int32_t* const* codes,
                   const int32_t* levels, int m, const int32_t* const* cl_codes, const int32_t* cl_levels, double tol,
                   int max_iter, int vcov, int ssc, int threads, double* beta, double* se, int32_t* iterations,
                   int64_t* n_obs_out, int64_t* df_resid_out, int64_t* n_clusters, double* stats, double* meats,
                   int64_t* G_sub) {
  if (n <= 0 || p < 1 || F < 0 || F > MAXF || m < 0 || m > MAXCL || (vcov == 2 && m < 1)) return -1;
  if (threads > 0) omp_set_num_threads(threads);
  const int T = omp_get_max_threads();
  const int k = p - 1;
  int32_t Gmax = 1;
  for (int f = 0; f < F; ++f) Gmax = levels[f] > Gmax ? levels[f] : Gmax;
  /* ---- single-pass singleton drop on pre-filter counts ---- */
  int32_t* cnt_pre[MAXF];
  int64_t card[MAXF];
  int32_t* ipart = (int32_t*)malloc(sizeof(int32_t) * (size_t)T * Gmax);
  for (int f = 0; f < F; ++f) {
    cnt_pre[f] = (int32_t*)malloc(sizeof(int32_t) * (size_t)levels[f]);
    group_counts(codes[f], n, levels[f], ipart, cnt_pre[f]);
    card[f] = 0;
    for (int32_t g = 0; g < levels[f]; ++g) card[f] += cnt_pre[f][g] > 0;
  }
  /* kept rows: per-thread counts, then ordered offsets (stable compaction) */
  int64_t* tk = (int64_t*)calloc((size_t)T + 1, sizeof(int64_t));
  int64_t* idx = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
  int64_t nk = 0;
#pragma omp parallel
  {
    const int t = omp_get_thread_num(), nt = omp_get_num_threads();
    const int64_t lo = lo_of(n, t, nt), hi = lo_of(n, t + 1, nt);
    int64_t c = 0;
    for (int64_t i = lo; i < hi; ++i) {
      int keep = 1;
      for (int f = 0; f < F; ++f) keep &= cnt_pre[f][codes[f][i]] > 1;
      c += keep;
    }
    tk[t + 1] = c;
#pragma omp barrier
#pragma omp single
    {
      for (int u = 0; u < nt; ++u) tk[u + 1] += tk[u];
      nk = tk[nt];
    }
    int64_t d = tk[t];
    for (int64_t i = lo; i < hi; ++i) {
      int keep = 1;
      for (int f = 0; f < F; ++f) keep &= cnt_pre[f][codes[f][i]] > 1;
      if (keep) idx[d++] = i;
    }
  }
  free(tk);
  /* compacted copies: p columns, F code arrays, m cluster columns */
  double** X = (double**)malloc(sizeof(double*) * p);
  int32_t* C[MAXF];
  int32_t* CL[MAXCL];
  const size_t nka = (size_t)(nk > 0 ? nk : 1);
  for (int j = 0; j < p; ++j) {
    X[j] = (double*)malloc(sizeof(double) * nka);
    const double* src = cols[j];
    double* dst = X[j];
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < nk; ++r) dst[r] = src[idx[r]];
  }
  for (int f = 0; f < F; ++f) {
    C[f] = (int32_t*)malloc(sizeof(int32_t) * nka);
    const int32_t* src = codes[f];
    int32_t* dst = C[f];
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < nk; ++r) dst[r] = src[idx[r]];
  }
  for (int j = 0; j < m; ++j) {
    CL[j] = (int32_t*)malloc(sizeof(int32_t) * nka);
    const int32_t* src = cl_codes[j];
    int32_t* dst = CL[j];
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < nk; ++r) dst[r] = src[idx[r]];
  }
  free(idx);
  double* inv_cnt[MAXF];
  int64_t dims_sum = 0;
  int32_t* cnt = (int32_t*)malloc(sizeof(int32_t) * (size_t)Gmax);
  for (int f = 0; f < F; ++f) {
    group_counts(C[f], nk, levels[f], ipart, cnt);
    inv_cnt[f] = (double*)malloc(sizeof(double) * (size_t)levels[f]);
    for (int32_t g = 0; g < levels[f]; ++g) {
      inv_cnt[f][g] = cnt[g] > 0 ? 1.0 / (double)cnt[g] : 0.0;
      dims_sum += cnt[g] > 0;
    }
    free(cnt_pre[f]);
  }
  free(cnt);
  free(ipart);
  /* ---- FE order: ascending pre-filter cardinality, stable ---- */
  int order[MAXF];
  for (int f = 0; f < F; ++f) order[f] = f;
  for (int a = 1; a < F; ++a)
    for (int b = a; b > 0 && card[order[b]] < card[order[b - 1]]; --b) {
      const int t = order[b];
      order[b] = order[b - 1];
      order[b - 1] = t;
    }
  /* ---- alternating projections (rows in parallel, one column at a time) ---- */
  double* part = (double*)malloc(sizeof(double) * (size_t)T * Gmax);
  double* mean = (double*)malloc(sizeof(double) * (size_t)Gmax);
  int it_done = 0;
  for (int it = 1; it <= max_iter && F > 0; ++it) {
    for (int q = 0; q < F; ++q)
      for (int j = 0; j < p; ++j) project_col(X[j], C[order[q]], nk, inv_cnt[order[q]], levels[order[q]], part, mean);
    it_done = it;
    if (it >= 3) { /* max over ALL FEs of |mean_g(y)|, y only, unweighted */
      double mx = 0.0;
      for (int f = 0; f < F; ++f) {
        group_sums(X[0], C[f], nk, levels[f], part, mean);
        for (int32_t g = 0; g < levels[f]; ++g)
          if (inv_cnt[f][g] > 0.0) {
            const double v = fabs(mean[g] * inv_cnt[f][g]);
            mx = (v > mx || isnan(v)) ? v : mx;
          }
      }
      if (mx < tol) break;
    }
  }
  free(part);
  free(mean);
  /* ---- Gram of v = [1, x~_1..x~_k, y~]: upper triangle, per-thread partials ---- */
  const int mm = k + 1;  /* [1, x] */
  const int w = mm + 1;  /* + y */
  double* gpart = (double*)calloc((size_t)T * w * w, sizeof(double));
#pragma omp parallel
  {
    const int t = omp_get_thread_num(), nt = omp_get_num_threads();
    double* mine = gpart + (size_t)t * w * w;
    double v[72];
    const int64_t lo = lo_of(nk, t, nt), hi = lo_of(nk, t + 1, nt);
    for (int64_t i = lo; i < hi; ++i) {
      v[0] = 1.0;
      for (int j = 1; j <= k; ++j) v[j] = X[j][i];
      v[mm] = X[0][i];
      for (int a = 0; a < w; ++a)
        for (int b = a; b < w; ++b) mine[a * w + b] += v[a] * v[b];
    }
  }
  double* Gm = (double*)calloc((size_t)mm * mm, sizeof(double));
  double* Xty = (double*)calloc((size_t)mm, sizeof(double));
  double syy = 0.0, sy = 0.0;
  for (int t = 0; t < T; ++t) {
    const double* g = gpart + (size_t)t * w * w;
    for (int a = 0; a < mm; ++a) {
      for (int b = a; b < mm; ++b) Gm[a * mm + b] += g[a * w + b];
      Xty[a] += g[a * w + mm];
    }
    syy += g[mm * w + mm];
    sy += g[0 * w + mm];
  }
  free(gpart);
  Gm[0] = (double)nk; /* the intercept count exactly */
  for (int a = 0; a < mm; ++a)
    for (int b = 0; b < a; ++b) Gm[a * mm + b] = Gm[b * mm + a];
  double* L = (double*)malloc(sizeof(double) * mm * mm);
  double* bf = (double*)malloc(sizeof(double) * mm);
  double* inv = (double*)malloc(sizeof(double) * mm * mm);
  int rc = cholesky_solve(mm, Gm, L, Xty, bf, inv);
  const int64_t df = nk - (int64_t)mm - (dims_sum - F);
  for (int j = 0; j < m; ++j) n_clusters[j] = 0;
  if (rc == 0) {
    /* residual r = y~ - [1, x~] beta_full; rss and the HC1 meat from per-thread partials */
    double* r = (double*)malloc(sizeof(double) * nka);
    double* mpart = (double*)calloc((size_t)T * (k * k + 1), sizeof(double));
#pragma omp parallel
    {
      const int t = omp_get_thread_num(), nt = omp_get_num_threads();
      double* mine = mpart + (size_t)t * (k * k + 1);
      const int64_t lo = lo_of(nk, t, nt), hi = lo_of(nk, t + 1, nt);
      double rss_t = 0.0;
      for (int64_t i = lo; i < hi; ++i) {
        double e = X[0][i] - bf[0];
        for (int j = 1; j < mm; ++j) e -= bf[j] * X[j][i];
        r[i] = e;
        rss_t += e * e;
        if (vcov == 1) {
          const double e2 = e * e;
          for (int a = 0; a < k; ++a) {
            const double xa = X[a + 1][i] * e2;
            for (int b = a; b < k; ++b) mine[1 + a * k + b] += xa * X[b + 1][i];
          }
        }
      }
      mine[0] = rss_t;
    }
    double rss = 0.0;
    double* meat = (double*)calloc((size_t)(k > 0 ? k : 1) * (k > 0 ? k : 1), sizeof(double));
    for (int t = 0; t < T; ++t) {
      rss += mpart[(size_t)t * (k * k + 1)];
      for (int a = 0; a < k; ++a)
        for (int b = a; b < k; ++b) meat[a * k + b] += mpart[(size_t)t * (k * k + 1) + 1 + a * k + b];
    }
    for (int a = 0; a < k; ++a)
      for (int b = 0; b < a; ++b) meat[a * k + b] = meat[b * k + a];
    free(mpart);
    double* Vb = (double*)malloc(sizeof(double) * (size_t)(k > 0 ? k * k : 1));
    for (int a = 0; a < k; ++a)
      for (int b = 0; b < k; ++b) Vb[a * k + b] = inv[(a + 1) * mm + (b + 1)];
    double* V = (double*)calloc((size_t)(k > 0 ? k * k : 1), sizeof(double));
    double gmin_out = 0.0;
    if (vcov == 0) {
      for (int a = 0; a < k; ++a) V[a * k + a] = Vb[a * k + a] * (rss / (double)df);
    } else if (vcov == 1) {
      sandwich_add(k, Vb, meat, (double)nk / (double)df, V);
    } else {
      /* every non-empty subset, by size, in itertools.combinations order (std_errors.py:392-425) */
      int nsub = 0;
      int64_t gmin = -1;
      double* M = (double*)malloc(sizeof(double) * (size_t)(k > 0 ? k * k : 1));
      for (int size = 1; size <= m; ++size) {
        int comb[MAXCL];
        for (int j = 0; j < size; ++j) comb[j] = j;
        for (;;) {
          int64_t G;
          if (size == 1) {
            G = meat_oneway(k, nk, X, r, CL[comb[0]], cl_levels[comb[0]], M);
            n_clusters[comb[0]] = G;
            if (gmin < 0 || G < gmin) gmin = G;
          } else {
            int32_t* sc[MAXCL];
            int32_t sl[MAXCL];
            for (int j = 0; j < size; ++j) {
              sc[j] = CL[comb[j]];
              sl[j] = cl_levels[comb[j]];
            }
            G = meat_intersect(k, nk, X, r, size, sc, sl, M);
          }
          if (meats) memcpy(meats + (size_t)nsub * k * k, M, sizeof(double) * k * k);
          if (G_sub) G_sub[nsub] = G;
          ++nsub;
          if (m == 1) {
            /* one-way (std_errors.py:335-342): G/(G-1) [* (n-1)/df], no guard for G = 1 */
            double adj = (double)G / (double)(G - 1);
            if (ssc) adj *= (double)(nk - 1) / (double)df;
            sandwich_add(k, Vb, M, adj, V);
            gmin_out = (double)G;
          } else if (G > 1) {
            sandwich_add(k, Vb, M, (size % 2 == 1) ? 1.0 : -1.0, V);
          }
          /* next combination */
          int j = size - 1;
          while (j >= 0 && comb[j] == m - size + j) --j;
          if (j < 0) break;
          comb[j]++;
          for (int u = j + 1; u < size; ++u) comb[u] = comb[u - 1] + 1;
        }
      }
      free(M);
      if (m > 1) {
        /* single G_min / (G_min - 1) only if G_min > 2 (std_errors.py:428-432), then ssc */
        double scale = 1.0;
        if (gmin > 2) scale *= (double)gmin / (double)(gmin - 1);
        if (ssc) scale *= (double)(nk - 1) / (double)df;
        for (int a = 0; a < k * k; ++a) V[a] *= scale;
        gmin_out = (double)gmin;
      }
    }
    for (int a = 0; a < k; ++a) {
      beta[a] = bf[a + 1];
      const double v = V[a * k + a];
      se[a] = sqrt(v > 0.0 ? v : 0.0);
    }
    if (stats) {
      const double tss = syy - sy * sy / (double)nk;
      stats[0] = rss;
      stats[1] = tss;
      stats[2] = tss > 0.0 ? 1.0 - rss / tss : NAN;
      stats[3] = gmin_out;
    }
    free(V);
    free(Vb);
    free(meat);
    free(r);
  }
  *iterations = it_done;
  *n_obs_out = nk;
  *df_resid_out = df;
  for (int j = 0; j < p; ++j) free(X[j]);
  free(X);
  for (int f = 0; f < F; ++f) {
    free(C[f]);
    free(inv_cnt[f]);
  }
  for (int j = 0; j < m; ++j) free(CL[j]);
  free(Gm);
  free(Xty);
  free(L);
  free(bf);
  free(inv);
  return rc;
}

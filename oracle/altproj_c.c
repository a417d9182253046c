/* CPU ORACLE (C restatement) — TEST / BASELINE INFRASTRUCTURE ONLY.
 *
 * A direct C restatement of the reference Polars backend's alt_proj hot path,
 * in the reference's own form (each projection subtracts group means from all
 * p data columns), used as bench.py's multi-threaded CPU baseline and checked
 * against oracle/altproj.py by tests/test_oracle_c.py.  The product path
 * (leanfe_amd) never links or calls it.
 *
 *   singleton drop, single pass on pre-filter counts .. polars_impl.py:477-482
 *   FE order (ascending cardinality, stable) ........... polars_impl.py:485
 *   projection c <- c - mean_g(c), unweighted .......... polars_impl.py:502-505
 *   loop + y-only stop test from it >= 3 ............... polars_impl.py:490-526
 *   fe_dims / absorbed_df / df_resid .................... polars_impl.py:531-537, :283
 *   Gram with intercept + Cholesky solve ................ polars_impl.py:165-226
 *   residual (unweighted) ............................... polars_impl.py:229
 *   IID / HC1 SEs ....................................... std_errors.py:183-210, :217-282
 *
 * Unweighted fits, IID or HC1 (the bench configurations).  OpenMP parallelism
 * is over columns (each thread owns whole columns: no atomics, deterministic).
 *
 * Build: gcc -O3 -fopenmp -shared -fPIC oracle/altproj_c.c -o oracle/_build/libaltproj.so -lm
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

/* group means of column c over codes (present groups only), subtract in place */
static void project_col(double* c, const int32_t* code, int64_t n, const double* inv_cnt, double* sum, int32_t G) {
  memset(sum, 0, sizeof(double) * (size_t)G);
  for (int64_t i = 0; i < n; ++i) sum[code[i]] += c[i];
  for (int32_t g = 0; g < G; ++g) sum[g] *= inv_cnt[g];
  for (int64_t i = 0; i < n; ++i) c[i] -= sum[code[i]];
}

static int cholesky_solve(int m, const double* A, double* L, const double* b, double* x, double* inv) {
  /* L L^T = A (row-major m x m); x = A^-1 b; inv = A^-1 (polars_impl.py:212-226) */
  memset(L, 0, sizeof(double) * m * m);
  for (int j = 0; j < m; ++j) {
    double s = A[j * m + j];
    for (int k = 0; k < j; ++k) s -= L[j * m + k] * L[j * m + k];
    if (s <= 0.0) return -1;
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

/* cols: p column pointers (y first), n rows each; codes: F arrays of int32 in [0, levels[f]).
 * Outputs: beta[k], se[k] (k = p - 1), iterations, n_obs, df_resid.  Returns 0, or -1 on a
 * singular Gram / bad input.  `threads` <= 0: OpenMP default. */
int lfe_oracle_fit(int64_t n, int p, const double* const* cols, int F, const int32_t* const* codes,
                   const int32_t* levels, double tol, int max_iter, int hc1, int threads, double* beta,
                   double* se, int32_t* iterations, int64_t* n_obs_out, int64_t* df_resid_out) {
  if (n <= 0 || p < 1 || F < 1 || F > 8) return -1;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
  const int k = p - 1;
  /* ---- single-pass singleton drop on pre-filter counts ---- */
  int32_t* cnt_pre[8];
  int64_t card[8];
  for (int f = 0; f < F; ++f) {
    cnt_pre[f] = (int32_t*)calloc((size_t)levels[f], sizeof(int32_t));
    for (int64_t i = 0; i < n; ++i) cnt_pre[f][codes[f][i]]++;
    card[f] = 0;
    for (int32_t g = 0; g < levels[f]; ++g) card[f] += cnt_pre[f][g] > 0;
  }
  int64_t nk = 0;
  int64_t* idx = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    int keep = 1;
    for (int f = 0; f < F; ++f) keep &= cnt_pre[f][codes[f][i]] > 1;
    if (keep) idx[nk++] = i;
  }
  /* compacted copies: p columns + F code arrays */
  double** X = (double**)malloc(sizeof(double*) * p);
  int32_t* C[8];
#pragma omp parallel for schedule(static)
  for (int j = 0; j < p; ++j) {
    X[j] = (double*)malloc(sizeof(double) * (size_t)(nk > 0 ? nk : 1));
    for (int64_t r = 0; r < nk; ++r) X[j][r] = cols[j][idx[r]];
  }
  double* inv_cnt[8];
  int64_t dims_sum = 0;
  for (int f = 0; f < F; ++f) {
    C[f] = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nk > 0 ? nk : 1));
    int32_t* cnt = (int32_t*)calloc((size_t)levels[f], sizeof(int32_t));
    for (int64_t r = 0; r < nk; ++r) {
      C[f][r] = codes[f][idx[r]];
      cnt[C[f][r]]++;
    }
    inv_cnt[f] = (double*)malloc(sizeof(double) * (size_t)levels[f]);
    for (int32_t g = 0; g < levels[f]; ++g) {
      inv_cnt[f][g] = cnt[g] > 0 ? 1.0 / (double)cnt[g] : 0.0;
      dims_sum += cnt[g] > 0;
    }
    free(cnt);
    free(cnt_pre[f]);
  }
  free(idx);
  /* ---- FE order: ascending pre-filter cardinality, stable ---- */
  int order[8];
  for (int f = 0; f < F; ++f) order[f] = f;
  for (int a = 1; a < F; ++a)
    for (int b = a; b > 0 && card[order[b]] < card[order[b - 1]]; --b) {
      const int t = order[b];
      order[b] = order[b - 1];
      order[b - 1] = t;
    }
  int32_t Gmax = 0;
  for (int f = 0; f < F; ++f) Gmax = levels[f] > Gmax ? levels[f] : Gmax;
  /* ---- alternating projections ---- */
  int it_done = 0;
  for (int it = 1; it <= max_iter; ++it) {
#pragma omp parallel
    {
      double* sum = (double*)malloc(sizeof(double) * (size_t)Gmax);
#pragma omp for schedule(dynamic, 1)
      for (int j = 0; j < p; ++j)
        for (int q = 0; q < F; ++q) project_col(X[j], C[order[q]], nk, inv_cnt[order[q]], sum, levels[order[q]]);
      free(sum);
    }
    it_done = it;
    if (it >= 3) { /* max over ALL FEs of |mean_g(y)|, y only, unweighted */
      double m = 0.0;
      double* sum = (double*)malloc(sizeof(double) * (size_t)Gmax);
      for (int f = 0; f < F; ++f) {
        memset(sum, 0, sizeof(double) * (size_t)levels[f]);
        for (int64_t r = 0; r < nk; ++r) sum[C[f][r]] += X[0][r];
        for (int32_t g = 0; g < levels[f]; ++g)
          if (inv_cnt[f][g] > 0.0) {
            const double v = fabs(sum[g] * inv_cnt[f][g]);
            m = (v > m || isnan(v)) ? v : m;
          }
      }
      free(sum);
      if (m < tol) break;
    }
  }
  /* ---- Gram of [1, x~] and X'y (columns: 0 = intercept, 1..k = x) ---- */
  const int m = k + 1;
  double* G = (double*)calloc((size_t)m * m, sizeof(double));
  double* Xty = (double*)calloc((size_t)m, sizeof(double));
#pragma omp parallel for schedule(dynamic, 1)
  for (int a = 0; a < m; ++a) {
    for (int b = a; b < m; ++b) {
      double s = 0.0;
      if (a == 0 && b == 0) s = (double)nk;
      else if (a == 0)
        for (int64_t r = 0; r < nk; ++r) s += X[b][r];
      else
        for (int64_t r = 0; r < nk; ++r) s += X[a][r] * X[b][r];
      G[a * m + b] = G[b * m + a] = s;
    }
    double t = 0.0;
    if (a == 0)
      for (int64_t r = 0; r < nk; ++r) t += X[0][r];
    else
      for (int64_t r = 0; r < nk; ++r) t += X[a][r] * X[0][r];
    Xty[a] = t;
  }
  double* L = (double*)malloc(sizeof(double) * m * m);
  double* bf = (double*)malloc(sizeof(double) * m);
  double* inv = (double*)malloc(sizeof(double) * m * m);
  int rc = cholesky_solve(m, G, L, Xty, bf, inv);
  const int64_t df = nk - (int64_t)m - (dims_sum - F);
  if (rc == 0) {
    /* residual r = y~ - [1, x~] beta_full */
    double* r = (double*)malloc(sizeof(double) * (size_t)(nk > 0 ? nk : 1));
    double rss = 0.0;
#pragma omp parallel for reduction(+ : rss) schedule(static)
    for (int64_t i = 0; i < nk; ++i) {
      double t = X[0][i] - bf[0];
      for (int j = 1; j < m; ++j) t -= bf[j] * X[j][i];
      r[i] = t;
      rss += t * t;
    }
    double* meat = (double*)calloc((size_t)k * k, sizeof(double));
    if (hc1) {
#pragma omp parallel for schedule(dynamic, 1)
      for (int a = 0; a < k; ++a)
        for (int b = a; b < k; ++b) {
          double s = 0.0;
          for (int64_t i = 0; i < nk; ++i) s += X[a + 1][i] * X[b + 1][i] * r[i] * r[i];
          meat[a * k + b] = meat[b * k + a] = s;
        }
    }
    for (int a = 0; a < k; ++a) {
      beta[a] = bf[a + 1];
      double v;
      if (!hc1) {
        v = inv[(a + 1) * m + (a + 1)] * (rss / (double)df);
      } else { /* (V meat V)_aa * n / df with V = XtX_inv[1:, 1:] */
        v = 0.0;
        for (int i = 0; i < k; ++i)
          for (int j = 0; j < k; ++j) v += inv[(a + 1) * m + (i + 1)] * meat[i * k + j] * inv[(j + 1) * m + (a + 1)];
        v *= (double)nk / (double)df;
      }
      se[a] = sqrt(v > 0.0 ? v : 0.0);
    }
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
  free(G);
  free(Xty);
  free(L);
  free(bf);
  free(inv);
  return rc;
}

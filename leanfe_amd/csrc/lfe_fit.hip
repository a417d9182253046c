// lfe_fit: one whole regression on the loaded shard in one C call (host code only).
//
// The hip backend's step is drop -> demean -> Gram (+ device Cholesky + residual pass) -> host
// solve -> SEs.  Driven from Python, every arrow is a return to the interpreter while the GPU
// waits (the 8-rank owner shard: ~10-15 us per arrow, ~40 us of NumPy on the 12 x 12 algebra after
// the last one).  lfe_fit runs the same C-ABI calls back to back and does the
// host algebra here:
//   - the order of the projections: FEs by pre-filter cardinality, ascending, stable
//     (polars_impl.py:485);
//   - the solve (polars_impl.py:211-220): Cholesky L of X'X, beta = L^-T L^-1 X'y and
//     (X'X)^-1 = L^-T L^-1 I; not positive definite: LU with partial pivoting (the reference's
//     np.linalg.solve / inv fallback);
//   - IID (std_errors.py:196-210) from the Gram's residual statistics
//     r'r = y'y - 2 b'X'y + b'X'X b when they do not cancel, HC1 (std_errors.py:275-282) from the
//     residual pass's meat;
//   - the residual pass reruns with the host beta when the device Cholesky's beta (used by the
//     fused pass) drifted from the host solve by more than 1e-10 relative.
// Clustered SEs keep the score rows (vcov = LFE_FIT_SCORES): the meats come from
// lfe_cluster_meat / lfe_cluster_meat_subsets and the CGM sandwich stays on the caller's side.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <numeric>
#include <string>
#include <vector>

#include "lfe_internal.h"

namespace lfe {

static int fail_code(int code, const char* msg) {
  set_error(msg);
  return code;
}

// Cholesky of the row-major m x m A into L (lower, row-major); false if A is not positive definite
static bool chol(int m, const double* A, double* L) {
  std::fill(L, L + (size_t)m * m, 0.0);
  for (int j = 0; j < m; ++j) {
    double d = A[(size_t)j * m + j];
    for (int k = 0; k < j; ++k) d -= L[(size_t)j * m + k] * L[(size_t)j * m + k];
    if (!(d > 0.0)) return false;
    const double ljj = std::sqrt(d);
    L[(size_t)j * m + j] = ljj;
    for (int i = j + 1; i < m; ++i) {
      double s = A[(size_t)i * m + j];
      for (int k = 0; k < j; ++k) s -= L[(size_t)i * m + k] * L[(size_t)j * m + k];
      L[(size_t)i * m + j] = s / ljj;
    }
  }
  return true;
}

// x = L^-T L^-1 b (forward, then back substitution)
static void chol_solve(int m, const double* L, const double* b, double* x) {
  std::vector<double> y(m);
  for (int i = 0; i < m; ++i) {
    double s = b[i];
    for (int k = 0; k < i; ++k) s -= L[(size_t)i * m + k] * y[k];
    y[i] = s / L[(size_t)i * m + i];
  }
  for (int i = m - 1; i >= 0; --i) {
    double s = y[i];
    for (int k = i + 1; k < m; ++k) s -= L[(size_t)k * m + i] * x[k];
    x[i] = s / L[(size_t)i * m + i];
  }
}

// LU with partial pivoting of A (row-major, in place) -> perm; false if singular
static bool lu(int m, double* A, std::vector<int>& perm) {
  perm.resize(m);
  std::iota(perm.begin(), perm.end(), 0);
  for (int j = 0; j < m; ++j) {
    int piv = j;
    for (int i = j + 1; i < m; ++i)
      if (std::fabs(A[(size_t)i * m + j]) > std::fabs(A[(size_t)piv * m + j])) piv = i;
    if (A[(size_t)piv * m + j] == 0.0) return false;
    if (piv != j) {
      for (int k = 0; k < m; ++k) std::swap(A[(size_t)j * m + k], A[(size_t)piv * m + k]);
      std::swap(perm[j], perm[piv]);
    }
    for (int i = j + 1; i < m; ++i) {
      const double f = A[(size_t)i * m + j] / A[(size_t)j * m + j];
      A[(size_t)i * m + j] = f;
      for (int k = j + 1; k < m; ++k) A[(size_t)i * m + k] -= f * A[(size_t)j * m + k];
    }
  }
  return true;
}

static void lu_solve(int m, const double* LU, const std::vector<int>& perm, const double* b, double* x) {
  std::vector<double> y(m);
  for (int i = 0; i < m; ++i) {
    double s = b[perm[i]];
    for (int k = 0; k < i; ++k) s -= LU[(size_t)i * m + k] * y[k];
    y[i] = s;
  }
  for (int i = m - 1; i >= 0; --i) {
    double s = y[i];
    for (int k = i + 1; k < m; ++k) s -= LU[(size_t)i * m + k] * x[k];
    x[i] = s / LU[(size_t)i * m + i];
  }
}

// beta and (X'X)^-1 of the m x m X'X and X'y (polars_impl.py:211-220)
static int host_solve(int m, const double* XtX, const double* Xty, double* beta, double* inv) {
  std::vector<double> L((size_t)m * m), e(m), col(m);
  auto fill_inv = [&](auto solve) {
    for (int j = 0; j < m; ++j) {
      std::fill(e.begin(), e.end(), 0.0);
      e[j] = 1.0;
      solve(e.data(), col.data());
      for (int i = 0; i < m; ++i) inv[(size_t)i * m + j] = col[i];
    }
  };
  if (chol(m, XtX, L.data())) {
    chol_solve(m, L.data(), Xty, beta);
    fill_inv([&](const double* b, double* x) { chol_solve(m, L.data(), b, x); });
    return LFE_OK;
  }
  std::vector<double> A(XtX, XtX + (size_t)m * m);
  std::vector<int> perm;
  if (!lu(m, A.data(), perm)) return fail_code(LFE_EINVAL, "X'X is singular");
  lu_solve(m, A.data(), perm, Xty, beta);
  fill_inv([&](const double* b, double* x) { lu_solve(m, A.data(), perm, b, x); });
  return LFE_OK;
}

}  // namespace lfe

using namespace lfe;

extern "C" int lfe_fit(lfe_ctx* c, int flags, double tol, int max_iter, int check_from, int vcov, int64_t* ints_out,
                       double* gram_out, double* beta_full_out, double* xtx_inv_out, double* stats_out,
                       double* meat_out, double* se_out, double* diag_out) {
  if (!c) return fail_code(LFE_EINVAL, "null context");
  if (!ints_out || !gram_out || !beta_full_out || !xtx_inv_out || !stats_out || !se_out)
    return fail_code(LFE_EINVAL, "null pointer");
  if (vcov < LFE_FIT_IID || vcov > LFE_FIT_SCORES) return fail_code(LFE_EINVAL, "unknown vcov");
  if (vcov == LFE_FIT_HC1 && !meat_out) return fail_code(LFE_EINVAL, "HC1 needs meat_out");
  if (c->w || c->records || c->F < 1 || c->p < 2 || c->sw.on)
    return fail_code(LFE_EINVAL, "lfe_fit: unweighted resident fits with fixed effects only");
  const int F = c->F, p = c->p, k = p - 1, D = p + 1;
  int64_t n_obs = 0;
  std::vector<int32_t> dims(F), card(F);
  if (flags & LFE_FIT_DROP) {
    LFE_TRY(lfe_drop_singletons(c, &n_obs, dims.data(), card.data()));
  } else {
    if (!c->prepared) return fail_code(LFE_ESTATE, "lfe_drop_singletons first (or LFE_FIT_DROP)");
    n_obs = c->n_kept;
    for (int f = 0; f < F; ++f) {
      dims[f] = c->fe[f].dims;
      card[f] = c->fe[f].card;
    }
  }
  std::vector<int> order(F);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return card[a] < card[b]; });
  int iterations = 0;
  double last = -1.0;
  LFE_TRY(lfe_demean(c, order.data(), tol, max_iter, check_from, &iterations, &last));

  std::vector<double> G((size_t)D * D), bdev(p, 0.0), meat((size_t)std::max(k, 1) * std::max(k, 1), 0.0);
  double stats[4] = {0.0, 0.0, 0.0, 0.0};
  bool have_stats = false, fused = false;
  if (vcov == LFE_FIT_IID) {
    LFE_TRY(lfe_gram(c, G.data()));
  } else {
    const int rc = lfe_gram_resid(c, G.data(), bdev.data(), stats, vcov == LFE_FIT_HC1 ? meat.data() : nullptr,
                                  vcov == LFE_FIT_SCORES);
    if (rc == 1) {
      LFE_TRY(lfe_gram(c, G.data()));
    } else {
      LFE_TRY(rc);
      fused = true;
    }
  }
  // X = [1, x]: Gram rows / columns 0, 2.. (column 1 is y)
  auto gi = [](int i) { return i == 0 ? 0 : i + 1; };
  std::vector<double> XtX((size_t)p * p), Xty(p), beta(p), inv((size_t)p * p);
  for (int i = 0; i < p; ++i) {
    Xty[i] = G[(size_t)gi(i) * D + 1];
    for (int j = 0; j < p; ++j) XtX[(size_t)i * p + j] = G[(size_t)gi(i) * D + gi(j)];
  }
  LFE_TRY(host_solve(p, XtX.data(), Xty.data(), beta.data(), inv.data()));
  double dbeta = 0.0;
  if (vcov == LFE_FIT_IID) {
    // r'r from the Gram (unweighted): y'y - 2 b'X'y + b'X'X b, unless it cancels
    const double yy = G[(size_t)1 * D + 1];
    double bXy = 0.0, bXXb = 0.0;
    for (int i = 0; i < p; ++i) {
      bXy += beta[i] * Xty[i];
      double t = 0.0;
      for (int j = 0; j < p; ++j) t += XtX[(size_t)i * p + j] * beta[j];
      bXXb += beta[i] * t;
    }
    const double rss = yy - 2.0 * bXy + bXXb;
    if (rss > 1e-4 * yy) {
      stats[0] = stats[1] = rss;
      stats[2] = G[1];
      stats[3] = yy;
      have_stats = true;
    }
  } else if (fused) {
    double scale = 0.0, dev = 0.0;
    bool finite = true;
    for (int i = 0; i < p; ++i) {
      scale = std::max(scale, std::fabs(beta[i]));
      finite = finite && std::isfinite(bdev[i]);
      dev = std::max(dev, std::fabs(bdev[i] - beta[i]));
    }
    scale = std::max(scale, 1e-300);
    if (finite && dev <= 1e-10 * scale) {
      have_stats = true;
      dbeta = dev / scale;
    }
  }
  if (!have_stats)  // no fused pass, its beta drifted, or r'r cancels in the Gram: the pass with the host beta
    LFE_TRY(lfe_resid(c, beta.data(), stats, vcov == LFE_FIT_HC1 ? meat.data() : nullptr, vcov == LFE_FIT_SCORES));
  int64_t absorbed = 0;
  for (int f = 0; f < F; ++f) absorbed += dims[f] - 1;
  const int64_t df = n_obs - (k + 1) - absorbed;
  // SEs of the k regressors: Vb = (X'X)^-1 without the intercept row / column
  for (int j = 0; j < k; ++j) {
    double v = 0.0;
    if (vcov == LFE_FIT_IID) {
      v = stats[0] / (double)df * inv[(size_t)(j + 1) * p + (j + 1)];
    } else if (vcov == LFE_FIT_HC1) {  // (n / df) diag(Vb M Vb)
      for (int a = 0; a < k; ++a) {
        double t = 0.0;
        for (int b = 0; b < k; ++b) t += meat[(size_t)a * k + b] * inv[(size_t)(b + 1) * p + (j + 1)];
        v += inv[(size_t)(j + 1) * p + (a + 1)] * t;
      }
      v *= (double)n_obs / (double)df;
    }
    se_out[j] = vcov == LFE_FIT_SCORES ? 0.0 : std::sqrt(std::max(v, 0.0));
  }
  ints_out[0] = n_obs;
  ints_out[1] = iterations;
  ints_out[2] = df;
  ints_out[3] = fused ? 1 : 0;
  for (int f = 0; f < F; ++f) {
    ints_out[4 + f] = dims[f];
    ints_out[4 + F + f] = card[f];
  }
  std::copy(G.begin(), G.end(), gram_out);
  std::copy(beta.begin(), beta.end(), beta_full_out);
  std::copy(inv.begin(), inv.end(), xtx_inv_out);
  std::copy(stats, stats + 4, stats_out);
  if (meat_out && vcov == LFE_FIT_HC1) std::copy(meat.begin(), meat.begin() + (size_t)k * k, meat_out);
  if (diag_out) {
    diag_out[0] = last;
    diag_out[1] = dbeta;
  }
  return LFE_OK;
}

// leanfe HIP engine — streaming kernels for the FWL / alternating-projections hot path.
//
// Algorithmic form ("alpha form").  The reference (polars_impl.py:490-508)
// overwrites every column with c - mean_g(c) per FE per sweep.  Here the
// columns are never rewritten: each FE f keeps a table alpha_f[G_f][p] of the
// group means it has subtracted so far, and the demeaned value of row i is
//     x~_i = x_i - sum_f alpha_f[g_f(i)]                              (1)
// Projecting FE f replaces alpha_f by the (weighted) group mean of the
// residual with alpha_f removed:
//     alpha_f[g] = (S_f[g] - T_f[g]) / W_f[g],
//     S_f[g] = sum_{i in g} w_i x_i          (constant, computed once)
//     T_f[g] = sum_{i in g} w_i sum_{f' != f} alpha_f'[g_f'(i)]       (2)
// which is exactly the Gauss-Seidel iterate of the reference in exact
// arithmetic (mean_g(c - alpha_f_old) = mean_g(c) - alpha_f_old).  A sweep
// therefore reads only FE codes, not the p data columns.
#include "lfe_internal.h"

namespace lfe {

#define GRID_STRIDE(i, n)                                                      \
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (n);   \
       i += (int64_t)gridDim.x * blockDim.x)

// ---------------------------------------------------------------------------
// counts, singleton drop (polars_impl.py:477-482)
// ---------------------------------------------------------------------------

__global__ void k_validate(const int32_t* __restrict__ code, int64_t n, int32_t G,
                           int32_t* __restrict__ flag) {
  GRID_STRIDE(i, n) {
    int32_t g = code[i];
    if (g < 0 || g >= G) atomicOr(flag, 1);
  }
}

__global__ void k_count_pre(const int32_t* __restrict__ code, int64_t n, int32_t* __restrict__ cnt) {
  GRID_STRIDE(i, n) atomicAdd(&cnt[code[i]], 1);
}

struct KeepArgs {
  int F;
  const int32_t* code[kMaxFE];
  const int32_t* cnt_pre[kMaxFE];
  int32_t* cnt[kMaxFE];
  double* W[kMaxFE];
};

__global__ void k_keep(KeepArgs a, int64_t n, const double* __restrict__ w,
                       uint8_t* __restrict__ keep) {
  GRID_STRIDE(i, n) {
    bool ok = true;
    for (int f = 0; f < a.F; ++f) ok = ok && (a.cnt_pre[f][a.code[f][i]] > 1);
    keep[i] = ok ? 1 : 0;
    if (ok) {
      const double wi = w ? w[i] : 1.0;
      for (int f = 0; f < a.F; ++f) {
        const int32_t g = a.code[f][i];
        atomicAdd(&a.cnt[f][g], 1);
        atomicAdd(&a.W[f][g], wi);
      }
    }
  }
}

__global__ void k_count_nonzero(const int32_t* __restrict__ cnt, int32_t G, int32_t* __restrict__ out) {
  int local = 0;
  for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x)
    local += cnt[g] > 0;
  // wave reduce then one atomic per wave
  for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off, 64);
  if ((threadIdx.x & 63) == 0 && local) atomicAdd(out, local);
}

// ---------------------------------------------------------------------------
// constant group sums S_f (all FEs in one pass over the data)
// ---------------------------------------------------------------------------

struct SumArgs {
  int F, p;
  const int32_t* code[kMaxFE];
  double* S[kMaxFE];
};

__global__ void k_group_sums(SumArgs a, const double* __restrict__ X, int64_t ld, int64_t n,
                             const double* __restrict__ w, const uint8_t* __restrict__ keep) {
  GRID_STRIDE(i, n) {
    if (!keep[i]) continue;
    const double wi = w ? w[i] : 1.0;
    int64_t base[kMaxFE];
    for (int f = 0; f < a.F; ++f) base[f] = (int64_t)a.code[f][i] * a.p;
    for (int c = 0; c < a.p; ++c) {
      const double v = w ? wi * X[c * ld + i] : X[c * ld + i];
      for (int f = 0; f < a.F; ++f) atomicAdd(&a.S[f][base[f] + c], v);
    }
  }
}

// ---------------------------------------------------------------------------
// one projection: cross term T_f (eq. 2) then alpha_f = (S_f - T_f) / W_f
// ---------------------------------------------------------------------------

__global__ void k_cross_sums(FeArgs a, int f, double* __restrict__ T, int64_t n,
                             const double* __restrict__ w, const uint8_t* __restrict__ keep) {
  GRID_STRIDE(i, n) {
    if (!keep[i]) continue;
    const double wi = w ? w[i] : 1.0;
    int64_t base[kMaxFE];
    for (int q = 0; q < a.F; ++q) base[q] = (int64_t)a.code[q][i] * a.p;
    const int64_t tb = base[f];
    for (int c = 0; c < a.p; ++c) {
      double v = 0.0;
      for (int q = 0; q < a.F; ++q)
        if (q != f) v += a.alpha[q][base[q] + c];
      atomicAdd(&T[tb + c], w ? wi * v : v);
    }
  }
}

__global__ void k_finalize(const double* __restrict__ S, const double* __restrict__ T,
                           const double* __restrict__ W, int32_t G, int p,
                           double* __restrict__ alpha) {
  const int64_t total = (int64_t)G * p;
  GRID_STRIDE(e, total) {
    const int64_t g = e / p;
    const double wg = W[g];
    alpha[e] = wg > 0.0 ? (S[e] - T[e]) / wg : 0.0;
  }
}

// ---------------------------------------------------------------------------
// convergence check (polars_impl.py:511-521): y only, unweighted, all FEs
// ---------------------------------------------------------------------------

struct CheckArgs {
  int F, p;
  const int32_t* code[kMaxFE];
  const double* alpha[kMaxFE];
  double* R[kMaxFE];
};

__global__ void k_check_sums(CheckArgs a, const double* __restrict__ y, int64_t n,
                             const uint8_t* __restrict__ keep) {
  GRID_STRIDE(i, n) {
    if (!keep[i]) continue;
    int32_t g[kMaxFE];
    double r = y[i];
    for (int f = 0; f < a.F; ++f) {
      g[f] = a.code[f][i];
      r -= a.alpha[f][(int64_t)g[f] * a.p];
    }
    for (int f = 0; f < a.F; ++f) atomicAdd(&a.R[f][g[f]], r);
  }
}

// max_g |R[g] / cnt[g]| over groups present; non-negative doubles order like
// their bit patterns, so an unsigned 64-bit atomicMax is an exact double max.
__global__ void k_check_max(const double* __restrict__ R, const int32_t* __restrict__ cnt, int32_t G,
                            unsigned long long* __restrict__ out) {
  double m = 0.0;
  for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x)
    if (cnt[g] > 0) m = fmax(m, fabs(R[g] / (double)cnt[g]));
  for (int off = 32; off > 0; off >>= 1) m = fmax(m, __shfl_down(m, off, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(out, (unsigned long long)__double_as_longlong(m));
}

// ---------------------------------------------------------------------------
// Gram on MFMA (v_mfma_f64_16x16x4_f64).  Rows are staged through LDS as a
// 64 x (16*NT) tile Z; each wave multiplies 16 of the tile's rows into NT(NT+1)/2
// 16x16 accumulators (pair (I,J), I <= J, holds Z_I' Z_J).  Operand map for
// 16x16x4 f64: lane l supplies A[i=l&15][k=l>>4] and B[k=l>>4][j=l&15], so with
// k = row-in-step both operands are Z[row0 + (l>>4)][16*I + (l&15)];
// the result map is D[(l>>4) + 4*r][l&15] (r = 0..3).
// ---------------------------------------------------------------------------

typedef double d4 __attribute__((ext_vector_type(4)));

enum { GRAM_DESIGN = 0, GRAM_RESID = 1, GRAM_TABLE = 2 };

struct GramArgs {
  FeArgs fa;
  const double* X;
  int64_t ld, n;
  const double* w;
  const uint8_t* keep;
  const double* beta;      // GRAM_RESID: beta_full [p] = {intercept, b_1..b_{p-1}}
  double* scores;          // GRAM_RESID: optional [p-1][ld] output x~ r (w)
  const double* table;     // GRAM_TABLE: row-major [n][tcols]
  int tcols;
};

constexpr int kTileRows = 64;

template <int NT>
struct GramShape {
  static constexpr int ZW = 16 * NT;
  static constexpr int ZS = ZW + ((NT % 2 == 0) ? 16 : 0);  // pad so lanes 16..31 hit the other 32 banks
  static constexpr int NP = NT * (NT + 1) / 2;
  static constexpr int LEN = NP * 256;
};

// demeaned value x~_c(i) (eq. 1)
__device__ __forceinline__ double demeaned(const FeArgs& a, const double* __restrict__ X, int64_t ld,
                                           int64_t i, int c, const int64_t* base) {
  double v = X[c * ld + i];
  for (int f = 0; f < a.F; ++f) v -= a.alpha[f][base[f] + c];
  return v;
}

template <int MODE, int NT>
__global__ __launch_bounds__(256) void k_gram(GramArgs a, double* __restrict__ partial, int64_t pstride) {
  using Sh = GramShape<NT>;
  __shared__ __attribute__((aligned(16))) double Z[kTileRows * Sh::ZS];
  __shared__ double rowscale[kTileRows];
  __shared__ double stat_red[4][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int p = a.fa.p;
  const int ncols = (MODE == GRAM_DESIGN) ? p + 1 : (MODE == GRAM_RESID ? p - 1 : a.tcols);
  const int64_t ntiles = (a.n + kTileRows - 1) / kTileRows;

  d4 acc[Sh::NP];
#pragma unroll
  for (int q = 0; q < Sh::NP; ++q) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
  double st_rss_w = 0, st_rss = 0, st_sy = 0, st_sy2 = 0;

  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int r = tid & 63;
    const int64_t i = tile * kTileRows + r;
    bool valid = i < a.n;
    if (MODE != GRAM_TABLE && valid) valid = a.keep[i] != 0;
    int64_t base[kMaxFE];
    if (MODE != GRAM_TABLE && valid)
      for (int f = 0; f < a.fa.F; ++f) base[f] = (int64_t)a.fa.code[f][i] * p;
    // ---- build the tile ----
    if (MODE == GRAM_DESIGN) {
      const double sw = (valid && a.w) ? sqrt(a.w[i]) : 1.0;
      for (int c = tid >> 6; c < Sh::ZW; c += 4) {
        double v = 0.0;
        if (valid && c < ncols) v = (c == 0) ? 1.0 : demeaned(a.fa, a.X, a.ld, i, c - 1, base);
        if (a.w) v *= sw;  // X_w = X * sqrt(w)  (polars_impl.py:202-203)
        Z[r * Sh::ZS + c] = v;
      }
    } else if (MODE == GRAM_RESID) {
      // stage x~ (cols 0..p-1, col 0 = y~), then residual per row, then scale
      for (int c = tid >> 6; c < Sh::ZW; c += 4)
        Z[r * Sh::ZS + c] = (valid && c < p) ? demeaned(a.fa, a.X, a.ld, i, c, base) : 0.0;
      __syncthreads();
      if (tid < kTileRows) {
        double s = 0.0;
        if (valid) {
          const double* zr = &Z[r * Sh::ZS];
          double fit = a.beta[0];
          for (int c = 1; c < p; ++c) fit += zr[c] * a.beta[c];
          const double yv = zr[0];
          const double res = yv - fit;  // resid = Y - X beta_full (polars_impl.py:229)
          const double wi = a.w ? a.w[i] : 1.0;
          st_rss_w += wi * res * res;
          st_rss += res * res;
          st_sy += yv;
          st_sy2 += yv * yv;
          s = a.w ? res * sqrt(wi) : res;
          if (a.scores) {
            const double sc = a.w ? res * wi : res;
            for (int c = 1; c < p; ++c) a.scores[(int64_t)(c - 1) * a.ld + i] = zr[c] * sc;
          }
        } else if (a.scores && i < a.n) {
          for (int c = 1; c < p; ++c) a.scores[(int64_t)(c - 1) * a.ld + i] = 0.0;
        }
        rowscale[r] = s;
      }
      __syncthreads();
      // shift left by one column (drop y~) and scale by r*sqrt(w)
      {
        double tmp[Sh::ZW / 4];
        int t = 0;
        for (int c = tid >> 6; c < Sh::ZW; c += 4, ++t)
          tmp[t] = (c < ncols) ? Z[r * Sh::ZS + c + 1] * rowscale[r] : 0.0;
        __syncthreads();
        t = 0;
        for (int c = tid >> 6; c < Sh::ZW; c += 4, ++t) Z[r * Sh::ZS + c] = tmp[t];
      }
    } else {  // GRAM_TABLE
      for (int c = tid >> 6; c < Sh::ZW; c += 4)
        Z[r * Sh::ZS + c] = (valid && c < ncols) ? a.table[i * a.tcols + c] : 0.0;
    }
    __syncthreads();
    // ---- MFMA over the tile: wave handles rows [16*wave, 16*wave+16) in 4 steps ----
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int row = wave * 16 + kk * 4 + (lane >> 4);
      double av[NT];
#pragma unroll
      for (int I = 0; I < NT; ++I) av[I] = Z[row * Sh::ZS + I * 16 + (lane & 15)];
      int q = 0;
#pragma unroll
      for (int I = 0; I < NT; ++I)
#pragma unroll
        for (int J = I; J < NT; ++J, ++q)
          acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[I], av[J], acc[q], 0, 0, 0);
    }
    __syncthreads();
  }

  // ---- reduce the 4 waves' accumulators through LDS (reuse Z) ----
  static_assert(Sh::LEN <= kTileRows * Sh::ZS, "LDS reuse");
  for (int wv = 0; wv < 4; ++wv) {
    if (wave == wv) {
#pragma unroll
      for (int q = 0; q < Sh::NP; ++q)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int e = q * 256 + ((lane >> 4) + 4 * rr) * 16 + (lane & 15);
          Z[e] = (wv == 0) ? acc[q][rr] : Z[e] + acc[q][rr];
        }
    }
    __syncthreads();
  }
  double* out = partial + (int64_t)blockIdx.x * pstride;
  for (int e = tid; e < Sh::LEN; e += 256) out[e] = Z[e];
  if (MODE == GRAM_RESID) {
    double v[4] = {st_rss_w, st_rss, st_sy, st_sy2};
#pragma unroll
    for (int s = 0; s < 4; ++s)
      for (int off = 32; off > 0; off >>= 1) v[s] += __shfl_down(v[s], off, 64);
    if (lane == 0)
      for (int s = 0; s < 4; ++s) stat_red[wave][s] = v[s];
    __syncthreads();
    if (tid < 4) out[Sh::LEN + tid] = stat_red[0][tid] + stat_red[1][tid] + stat_red[2][tid] + stat_red[3][tid];
  }
}

// fixed-order sum of per-block partials (deterministic for a fixed grid)
__global__ void k_reduce_partials(const double* __restrict__ partial, int nblocks, int64_t pstride, int len,
                                  double* __restrict__ out) {
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < len; e += gridDim.x * blockDim.x) {
    double s = 0.0;
    for (int b = 0; b < nblocks; ++b) s += partial[(int64_t)b * pstride + e];
    out[e] = s;
  }
}

// ---------------------------------------------------------------------------
// cluster scores S_c = sum_{i in c} x~_i r_i (w_i): the one-hot SpMM W_C'(X.e)
// (compress.py:929-936, std_errors.py:317-333)
// ---------------------------------------------------------------------------

__global__ void k_cluster_scatter(const int32_t* __restrict__ cl, const double* __restrict__ U, int64_t ld,
                                  int64_t n, int k, const uint8_t* __restrict__ keep,
                                  double* __restrict__ S, int32_t* __restrict__ present) {
  GRID_STRIDE(i, n) {
    if (!keep[i]) continue;
    const int64_t c = cl[i];
    present[c] = 1;
    for (int j = 0; j < k; ++j) atomicAdd(&S[c * k + j], U[(int64_t)j * ld + i]);
  }
}

__global__ void k_copy_demeaned(FeArgs a, const double* __restrict__ X, int64_t ld, int64_t n,
                                const uint8_t* __restrict__ keep, double* __restrict__ out) {
  GRID_STRIDE(i, n) {
    int64_t base[kMaxFE];
    for (int f = 0; f < a.F; ++f) base[f] = (int64_t)a.code[f][i] * a.p;
    for (int c = 0; c < a.p; ++c)
      out[(int64_t)c * n + i] = keep[i] ? demeaned(a, X, ld, i, c, base) : __builtin_nan("");
  }
}

// ===========================================================================
// launchers
// ===========================================================================

int launch_validate_codes(const int32_t* code, int64_t n, int32_t G, int32_t* flag, hipStream_t s) {
  if (n == 0) return LFE_OK;
  hipLaunchKernelGGL(k_validate, dim3(grid_for(n)), dim3(kBlock), 0, s, code, n, G, flag);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

int launch_count_pre(lfe_ctx* c) {
  for (auto& fe : c->fe) {
    LFE_HIP(hipMemsetAsync(fe.cnt_pre, 0, sizeof(int32_t) * fe.G, c->stream));
    if (c->n)
      {
        ProfScope _ps(c, K_COUNT_PRE);
        hipLaunchKernelGGL(k_count_pre, dim3(grid_for(c->n)), dim3(kBlock), 0, c->stream, fe.code, c->n,
                           fe.cnt_pre);
      }
    LFE_HIP(hipGetLastError());
  }
  return LFE_OK;
}

int launch_keep(lfe_ctx* c) {
  KeepArgs a{};
  a.F = c->F;
  for (int f = 0; f < c->F; ++f) {
    auto& fe = c->fe[f];
    LFE_HIP(hipMemsetAsync(fe.cnt, 0, sizeof(int32_t) * fe.G, c->stream));
    LFE_HIP(hipMemsetAsync(fe.W, 0, sizeof(double) * fe.G, c->stream));
    a.code[f] = fe.code;
    a.cnt_pre[f] = fe.cnt_pre;
    a.cnt[f] = fe.cnt;
    a.W[f] = fe.W;
  }
  if (c->n)
    {
      ProfScope _ps(c, K_KEEP);
      hipLaunchKernelGGL(k_keep, dim3(grid_for(c->n)), dim3(kBlock), 0, c->stream, a, c->n, c->w, c->keep);
    }
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

int launch_count_dims(lfe_ctx* c, int32_t* dims, int32_t* card) {
  const int F = c->F;
  LFE_TRY(ensure_iscratch(c, 2 * kMaxFE));
  LFE_HIP(hipMemsetAsync(c->iscratch, 0, sizeof(int32_t) * 2 * kMaxFE, c->stream));
  for (int f = 0; f < F; ++f) {
    auto& fe = c->fe[f];
    hipLaunchKernelGGL(k_count_nonzero, dim3(grid_for(fe.G)), dim3(kBlock), 0, c->stream, fe.cnt, fe.G,
                       c->iscratch + f);
    hipLaunchKernelGGL(k_count_nonzero, dim3(grid_for(fe.G)), dim3(kBlock), 0, c->stream, fe.cnt_pre, fe.G,
                       c->iscratch + kMaxFE + f);
  }
  LFE_HIP(hipGetLastError());
  int32_t h[2 * kMaxFE];
  LFE_HIP(hipMemcpyAsync(h, c->iscratch, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  LFE_HIP(hipStreamSynchronize(c->stream));
  for (int f = 0; f < F; ++f) {
    dims[f] = h[f];
    card[f] = h[kMaxFE + f];
  }
  return LFE_OK;
}

int launch_group_sums(lfe_ctx* c) {
  SumArgs a{};
  a.F = c->F;
  a.p = c->p;
  for (int f = 0; f < c->F; ++f) {
    auto& fe = c->fe[f];
    LFE_HIP(hipMemsetAsync(fe.S, 0, sizeof(double) * (size_t)fe.G * c->p, c->stream));
    a.code[f] = fe.code;
    a.S[f] = fe.S;
  }
  if (c->n && c->F)
    {
      ProfScope _ps(c, K_GROUP_SUMS);
      hipLaunchKernelGGL(k_group_sums, dim3(grid_for(c->n)), dim3(kBlock), 0, c->stream, a, c->X, c->ld, c->n,
                         c->w, c->keep);
    }
  LFE_HIP(hipGetLastError());
  for (int f = 0; f < c->F; ++f) LFE_TRY(allreduce_sum_f64(c, c->fe[f].S, (size_t)c->fe[f].G * c->p));
  return LFE_OK;
}

int launch_cross_sums(lfe_ctx* c, int f) {
  auto& fe = c->fe[f];
  LFE_HIP(hipMemsetAsync(fe.T, 0, sizeof(double) * (size_t)fe.G * c->p, c->stream));
  if (c->n && c->F > 1)
    {
      ProfScope _ps(c, K_CROSS_SUMS);
      hipLaunchKernelGGL(k_cross_sums, dim3(grid_for(c->n)), dim3(kBlock), 0, c->stream, fe_args(c), f, fe.T,
                         c->n, c->w, c->keep);
    }
  LFE_HIP(hipGetLastError());
  if (c->F > 1) LFE_TRY(allreduce_sum_f64(c, fe.T, (size_t)fe.G * c->p));
  return LFE_OK;
}

int launch_finalize(lfe_ctx* c, int f) {
  auto& fe = c->fe[f];
  const int64_t total = (int64_t)fe.G * c->p;
  {
    ProfScope _ps(c, K_FINALIZE);
    hipLaunchKernelGGL(k_finalize, dim3(grid_for(total)), dim3(kBlock), 0, c->stream, fe.S, fe.T, fe.W, fe.G,
                       c->p, fe.alpha);
  }
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

int launch_check(lfe_ctx* c, double* host_max) {
  CheckArgs a{};
  a.F = c->F;
  a.p = c->p;
  for (int f = 0; f < c->F; ++f) {
    auto& fe = c->fe[f];
    LFE_HIP(hipMemsetAsync(fe.R, 0, sizeof(double) * fe.G, c->stream));
    a.code[f] = fe.code;
    a.alpha[f] = fe.alpha;
    a.R[f] = fe.R;
  }
  if (c->n)
    {
      ProfScope _ps(c, K_CHECK_SUMS);
      hipLaunchKernelGGL(k_check_sums, dim3(grid_for(c->n)), dim3(kBlock), 0, c->stream, a, c->X, c->n, c->keep);
    }
  LFE_HIP(hipGetLastError());
  LFE_TRY(ensure_dred(c, 1));
  LFE_HIP(hipMemsetAsync(c->dred, 0, sizeof(double), c->stream));
  for (int f = 0; f < c->F; ++f) {
    auto& fe = c->fe[f];
    LFE_TRY(allreduce_sum_f64(c, fe.R, fe.G));
    {
      ProfScope _ps(c, K_CHECK_MAX);
      hipLaunchKernelGGL(k_check_max, dim3(grid_for(fe.G)), dim3(kBlock), 0, c->stream, fe.R, fe.cnt, fe.G,
                         reinterpret_cast<unsigned long long*>(c->dred));
    }
  }
  LFE_HIP(hipGetLastError());
  LFE_HIP(hipMemcpyAsync(host_max, c->dred, sizeof(double), hipMemcpyDeviceToHost, c->stream));
  LFE_HIP(hipStreamSynchronize(c->stream));
  return LFE_OK;
}

// Run k_gram<MODE, NT> over `rows` rows, reduce, all-reduce, copy `len+extra` values to host.
template <int MODE, int NT>
static int run_gram(lfe_ctx* c, GramArgs a, int64_t rows, double* host_out, int extra) {
  using Sh = GramShape<NT>;
  const int64_t ntiles = (rows + kTileRows - 1) / kTileRows;
  int nblocks = (int)std::min<int64_t>(std::max<int64_t>(ntiles, 1), 1024);
  const int64_t pstride = Sh::LEN + 4;
  LFE_TRY(ensure_scratch(c, (size_t)nblocks * pstride));
  LFE_TRY(ensure_dred(c, (size_t)pstride));
  a.n = rows;
  {
    ProfScope _ps(c, MODE == GRAM_DESIGN ? K_GRAM_DESIGN : (MODE == GRAM_RESID ? K_GRAM_RESID : K_GRAM_TABLE));
    hipLaunchKernelGGL((k_gram<MODE, NT>), dim3(nblocks), dim3(256), 0, c->stream, a, c->scratch, pstride);
  }
  LFE_HIP(hipGetLastError());
  const int len = Sh::LEN + extra;
  {
    ProfScope _ps(c, K_REDUCE);
    hipLaunchKernelGGL(k_reduce_partials, dim3((len + 255) / 256), dim3(256), 0, c->stream, c->scratch, nblocks,
                       pstride, len, c->dred);
  }
  LFE_HIP(hipGetLastError());
  LFE_TRY(allreduce_sum_f64(c, c->dred, len));
  LFE_HIP(hipMemcpyAsync(host_out, c->dred, sizeof(double) * len, hipMemcpyDeviceToHost, c->stream));
  LFE_HIP(hipStreamSynchronize(c->stream));
  return LFE_OK;
}

// tiles (I<=J) of 16x16 -> dense symmetric [ncols][ncols]
static void unpack_tiles(const double* tiles, int NT, int ncols, double* out) {
  int q = 0;
  for (int I = 0; I < NT; ++I)
    for (int J = I; J < NT; ++J, ++q)
      for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
          const int a = 16 * I + i, b = 16 * J + j;
          if (a < ncols && b < ncols) {
            const double v = tiles[q * 256 + i * 16 + j];
            out[a * ncols + b] = v;
            out[b * ncols + a] = v;
          }
        }
}

template <int MODE>
static int gram_dispatch(lfe_ctx* c, GramArgs a, int64_t rows, int ncols, double* dense_out, double* extra_out,
                         int extra, int tile_cols = -1) {
  // tile width must hold every staged column (GRAM_RESID stages p = ncols + 1)
  const int NT = ((tile_cols > ncols ? tile_cols : ncols) + 15) / 16;
  std::vector<double> h((size_t)10 * 256 + 4);
  int rc;
  switch (NT) {
    case 0:
    case 1: rc = run_gram<MODE, 1>(c, a, rows, h.data(), extra); break;
    case 2: rc = run_gram<MODE, 2>(c, a, rows, h.data(), extra); break;
    case 3: rc = run_gram<MODE, 3>(c, a, rows, h.data(), extra); break;
    case 4: rc = run_gram<MODE, 4>(c, a, rows, h.data(), extra); break;
    default: set_error("too many columns for the Gram kernel (max 64)"); return LFE_EINVAL;
  }
  if (rc) return rc;
  const int NTe = NT < 1 ? 1 : NT;
  if (dense_out) unpack_tiles(h.data(), NTe, ncols, dense_out);
  if (extra_out) {
    const int len = NTe * (NTe + 1) / 2 * 256;
    for (int s = 0; s < extra; ++s) extra_out[s] = h[len + s];
  }
  return LFE_OK;
}

static GramArgs base_args(lfe_ctx* c) {
  GramArgs a{};
  a.fa = fe_args(c);
  a.X = c->X;
  a.ld = c->ld;
  a.n = c->n;
  a.w = c->w;
  a.keep = c->keep;
  return a;
}

int launch_gram(lfe_ctx* c, double* host_gram) {
  GramArgs a = base_args(c);
  return gram_dispatch<GRAM_DESIGN>(c, a, c->n, c->p + 1, host_gram, nullptr, 0);
}

int launch_resid(lfe_ctx* c, const double* beta_full, double* stats, double* hc1, int keep_scores) {
  GramArgs a = base_args(c);
  LFE_HIP(hipMemcpyAsync(c->dbeta, beta_full, sizeof(double) * c->p, hipMemcpyHostToDevice, c->stream));
  a.beta = c->dbeta;
  a.scores = keep_scores ? c->scores : nullptr;
  const int k = c->p - 1;
  std::vector<double> meat((size_t)std::max(k, 1) * std::max(k, 1));
  int rc = gram_dispatch<GRAM_RESID>(c, a, c->n, k, meat.data(), stats, 4, c->p);
  if (rc) return rc;
  if (hc1)
    for (int e = 0; e < k * k; ++e) hc1[e] = meat[e];
  c->scores_valid = keep_scores != 0;
  return LFE_OK;
}

int launch_cluster(lfe_ctx* c, double* meats, int64_t* G_out) {
  const int k = c->p - 1;
  for (size_t j = 0; j < c->cl.size(); ++j) {
    const int32_t C = c->cl_levels[j];
    double* S = nullptr;
    int32_t* present = nullptr;
    LFE_HIP(hipMallocAsync(&S, sizeof(double) * (size_t)C * std::max(k, 1), c->stream));
    LFE_HIP(hipMallocAsync(&present, sizeof(int32_t) * (size_t)C + 16, c->stream));
    LFE_HIP(hipMemsetAsync(S, 0, sizeof(double) * (size_t)C * std::max(k, 1), c->stream));
    LFE_HIP(hipMemsetAsync(present, 0, sizeof(int32_t) * (size_t)C + 16, c->stream));
    if (c->n && k > 0)
      {
        ProfScope _ps(c, K_CLUSTER_SCATTER);
        hipLaunchKernelGGL(k_cluster_scatter, dim3(grid_for(c->n)), dim3(kBlock), 0, c->stream, c->cl[j], c->scores,
                           c->ld, c->n, k, c->keep, S, present);
      }
    LFE_HIP(hipGetLastError());
    LFE_TRY(allreduce_sum_f64(c, S, (size_t)C * k));
    LFE_TRY(allreduce_sum_i32(c, present, C));
    int32_t* cntG = present + C;  // 16 spare bytes
    hipLaunchKernelGGL(k_count_nonzero, dim3(grid_for(C)), dim3(kBlock), 0, c->stream, present, C, cntG);
    LFE_HIP(hipGetLastError());
    int32_t hG = 0;
    LFE_HIP(hipMemcpyAsync(&hG, cntG, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    GramArgs a{};
    a.table = S;
    a.tcols = k;
    int rc = LFE_OK;
    if (k > 0) {
      // the S table is replicated on every rank after the all-reduce: reduce its
      // Gram locally only (no second all-reduce)
      const int world = c->world;
      c->world = 1;
      rc = gram_dispatch<GRAM_TABLE>(c, a, C, k, meats + j * (size_t)k * k, nullptr, 0);
      c->world = world;
    }
    hipFreeAsync(S, c->stream);
    hipFreeAsync(present, c->stream);
    LFE_HIP(hipStreamSynchronize(c->stream));
    if (rc) return rc;
    G_out[j] = hG;
  }
  return LFE_OK;
}

int launch_copy_demeaned(lfe_ctx* c, double* dev_out) {
  if (c->n)
    hipLaunchKernelGGL(k_copy_demeaned, dim3(grid_for(c->n)), dim3(kBlock), 0, c->stream, fe_args(c), c->X, c->ld,
                       c->n, c->keep, dev_out);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

}  // namespace lfe

// leanfe HIP engine — Gram, residual/HC1 meat and cluster scores on MFMA.
//
//   Gram   X'X, X'y with X = [1, x~]          (polars_impl.py:165-209)
//   resid  r = y~ - X beta_full, sum w r^2, sum r^2, HC1 meat sum (w) r^2 x~ x~'
//                                              (polars_impl.py:229, 281-282; std_errors.py:196-264)
//   scores S_c = sum_{i in c} x~_i r_i (w_i) and meat S'S: the one-hot SpMM
//          W_C'(X.e)                           (std_errors.py:317-336, compress.py:929-942)
//
// Every row pass is thread-per-row: a thread loads its row's p columns
// (coalesced: consecutive threads, consecutive rows), subtracts the group
// effects (eq. 1 of lfe_sweep.hip; the primary FE's alpha slice for the item's
// bucket is staged in LDS, other FEs' tables are read through L2) and writes
// the row into a column-major LDS tile Z[16*NT][kTR + 2].  Each wave then
// multiplies 64 tile rows into NT(NT+1)/2 16x16 f64 accumulators with
// v_mfma_f64_16x16x4_f64: lane l supplies A[i=l&15][k=l>>4] = B[k][j=l&15]
// = Z[16*I + (l&15)][row0 + (l>>4)], result D[(l>>4) + 4r][l&15].
// The tile stride kTR + 2 doubles keeps both the row-wise writes and the
// 16-column MFMA operand reads bank-conflict free.
#include "lfe_internal.h"

#include <algorithm>

namespace lfe {

typedef double d4 __attribute__((ext_vector_type(4)));

enum { GRAM_DESIGN = 0, GRAM_RESID = 1, GRAM_TABLE = 2 };

constexpr int kTR = 256;          // tile rows (= threads per workgroup)
constexpr int kZST = kTR + 2;     // column stride of the LDS tile (doubles)

struct GramArgs {
  LayoutArgs la;
  const double* X;
  int64_t ld;
  const double* w;
  const double* beta;   // GRAM_RESID: beta_full [p] = {intercept, b_1..b_{p-1}}
  double* scores;       // GRAM_RESID: optional [p-1][ld] output x~ r (w)
  const double* table;  // GRAM_TABLE: row-major [rows][tcols]
  int64_t rows;         // GRAM_TABLE
  int tcols;
  int B;                // 1 << s
  int G_P;
  int stage;            // 1: the primary FE's alpha slice is staged in LDS per item
};

template <int NT>
struct GramShape {
  static constexpr int ZW = 16 * NT;
  static constexpr int NP = NT * (NT + 1) / 2;
  static constexpr int LEN = NP * 256;
};

// MFMA over one staged tile: wave w owns tile rows [64w, 64w + 64)
template <int NT>
__device__ __forceinline__ void tile_mfma(const double* Z, d4* acc, int wave, int lane) {
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) {
    const int row = wave * 64 + kk * 4 + (lane >> 4);
    double av[NT];
#pragma unroll
    for (int I = 0; I < NT; ++I) av[I] = Z[(I * 16 + (lane & 15)) * kZST + row];
    int q = 0;
#pragma unroll
    for (int I = 0; I < NT; ++I)
#pragma unroll
      for (int J = I; J < NT; ++J, ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[I], av[J], acc[q], 0, 0, 0);
  }
}

template <int MODE, int NT>
__global__ __launch_bounds__(kTR) void k_gram(GramArgs a, double* __restrict__ partial, int64_t pstride) {
  using Sh = GramShape<NT>;
  __shared__ __attribute__((aligned(16))) double Z[Sh::ZW * kZST];
  __shared__ double stat_red[4][4];
  extern __shared__ __attribute__((aligned(16))) double slice[];  // [B][p] alpha_P slice of the item's bucket
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int p = a.la.p, P = a.la.P;

  d4 acc[Sh::NP];
#pragma unroll
  for (int q = 0; q < Sh::NP; ++q) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
  double st[4] = {0.0, 0.0, 0.0, 0.0};  // sum w r^2, sum r^2, sum y~, sum y~^2

  if (MODE == GRAM_TABLE) {
    const int64_t ntiles = (a.rows + kTR - 1) / kTR;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
      const int64_t i = tile * kTR + tid;
      const bool valid = i < a.rows;
#pragma unroll
      for (int c = 0; c < Sh::ZW; ++c) Z[c * kZST + tid] = (valid && c < a.tcols) ? a.table[i * a.tcols + c] : 0.0;
      __syncthreads();
      tile_mfma<NT>(Z, acc, wave, lane);
      __syncthreads();
    }
  } else {
    const int nitems = a.la.n_items;
    for (int item = blockIdx.x; item < nitems; item += gridDim.x) {
      const int4 it = a.la.items[item];
      const int lo = it.x << a.la.s;
      __syncthreads();
      if (P >= 0 && a.stage)
        for (int j = tid; j < a.B * p; j += kTR) {
          const int g = lo + j / p;
          slice[j] = g < a.G_P ? a.la.alpha[P][(int64_t)g * p + (j % p)] : 0.0;
        }
      __syncthreads();
      for (int64_t r0 = it.y; r0 < it.z; r0 += kTR) {
        const int64_t i = r0 + tid;
        int32_t hP = 0;
        bool valid = i < it.z;
        if (valid && P >= 0) {
          hP = a.la.code[P][i];
          valid = hP >= 0;  // singleton-dropped rows contribute nothing
        }
        double xt[Sh::ZW];
#pragma unroll
        for (int c = 0; c < Sh::ZW; ++c) xt[c] = 0.0;
        if (valid) {
#pragma unroll
          for (int c = 0; c < Sh::ZW; ++c)
            if (c < p) xt[c] = a.X[(int64_t)c * a.ld + i];
          if (P >= 0) {
            const double* sl = a.stage ? &slice[(hP - lo) * p] : &a.la.alpha[P][(int64_t)hP * p];
#pragma unroll
            for (int c = 0; c < Sh::ZW; ++c)
              if (c < p) xt[c] -= sl[c];
          }
          for (int f = 0; f < a.la.F; ++f) {
            if (f == P) continue;
            const double* al = &a.la.alpha[f][(int64_t)a.la.code[f][i] * p];
#pragma unroll
            for (int c = 0; c < Sh::ZW; ++c)
              if (c < p) xt[c] -= al[c];
          }
        }
        if (MODE == GRAM_DESIGN) {
          // Z = sqrt(w) [1, y~, x~]   (X_w = X * sqrt(w), polars_impl.py:202-203)
          const double sw = (valid && a.w) ? sqrt(a.w[i]) : 1.0;
          Z[tid] = valid ? sw : 0.0;
#pragma unroll
          for (int c = 1; c < Sh::ZW; ++c) Z[c * kZST + tid] = (valid && c - 1 < p) ? (a.w ? xt[c - 1] * sw : xt[c - 1]) : 0.0;
        } else {
          // r = y~ - beta0 - sum_j beta_j x~_j  (unweighted residual, polars_impl.py:229)
          double scale = 0.0;
          if (valid) {
            double fit = a.beta[0];
#pragma unroll
            for (int c = 1; c < Sh::ZW; ++c)
              if (c < p) fit += xt[c] * a.beta[c];
            const double res = xt[0] - fit;
            const double wi = a.w ? a.w[i] : 1.0;
            st[0] += wi * res * res;
            st[1] += res * res;
            st[2] += xt[0];
            st[3] += xt[0] * xt[0];
            scale = a.w ? res * sqrt(wi) : res;
            if (a.scores) {
              const double sc = a.w ? res * wi : res;
#pragma unroll
              for (int c = 1; c < Sh::ZW; ++c)
                if (c < p) a.scores[(int64_t)(c - 1) * a.ld + i] = xt[c] * sc;
            }
          } else if (a.scores && i < it.z) {
#pragma unroll
            for (int c = 1; c < Sh::ZW; ++c)
              if (c < p) a.scores[(int64_t)(c - 1) * a.ld + i] = 0.0;
          }
          // HC1 meat rows: r sqrt(w) x~_j over the k = p-1 regressors
#pragma unroll
          for (int c = 0; c < Sh::ZW; ++c) Z[c * kZST + tid] = (c + 1 < p && c + 1 < Sh::ZW) ? xt[c + 1] * scale : 0.0;
        }
        __syncthreads();
        tile_mfma<NT>(Z, acc, wave, lane);
        __syncthreads();
      }
    }
  }

  // ---- reduce the 4 waves' accumulators through LDS (reuse Z) ----
  static_assert(Sh::LEN <= Sh::ZW * kZST, "LDS reuse");
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
  for (int e = tid; e < Sh::LEN; e += kTR) out[e] = Z[e];
  if (MODE == GRAM_RESID) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
      for (int off = 32; off > 0; off >>= 1) st[s] += __shfl_down(st[s], off, 64);
    if (lane == 0)
      for (int s = 0; s < 4; ++s) stat_red[wave][s] = st[s];
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

// cluster scores on the layout: S[cl[orig(i)]] += scores_i
__global__ void k_cluster_scatter(const int32_t* __restrict__ cl, const int32_t* __restrict__ orig,
                                  const int32_t* __restrict__ codeP, const double* __restrict__ U, int64_t ld,
                                  int64_t n, int k, double* __restrict__ S, int32_t* __restrict__ present) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (codeP && codeP[i] < 0) continue;
    const int64_t c = cl[orig ? orig[i] : i];
    present[c] = 1;
    for (int j = 0; j < k; ++j) atomicAdd(&S[c * k + j], U[(int64_t)j * ld + i]);
  }
}

__global__ void k_count_nonzero(const int32_t* __restrict__ cnt, int32_t G, int32_t* __restrict__ out) {
  int local = 0;
  for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x) local += cnt[g] > 0;
  for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off, 64);
  if ((threadIdx.x & 63) == 0 && local) atomicAdd(out, local);
}

__global__ void k_validate(const int32_t* __restrict__ code, int64_t n, int32_t G, int32_t* __restrict__ flag) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t g = code[i];
    if (g < 0 || g >= G) atomicOr(flag, 1);
  }
}

__global__ void k_copy_demeaned(LayoutArgs la, const double* __restrict__ X, int64_t ld, int64_t n,
                                const int32_t* __restrict__ orig, double* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t o = orig ? orig[i] : i;
    const bool dropped = la.P >= 0 && la.code[la.P][i] < 0;
    for (int c = 0; c < la.p; ++c) {
      double v = X[(int64_t)c * ld + i];
      if (!dropped)
        for (int f = 0; f < la.F; ++f) v -= la.alpha[f][(int64_t)la.code[f][i] * la.p + c];
      out[(int64_t)c * n + o] = dropped ? __builtin_nan("") : v;
    }
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

template <int MODE, int NT>
static int run_gram(lfe_ctx* c, GramArgs a, double* host_out, int extra) {
  using Sh = GramShape<NT>;
  int nblocks;
  if (MODE == GRAM_TABLE) {
    const int64_t ntiles = (a.rows + kTR - 1) / kTR;
    nblocks = (int)std::min<int64_t>(std::max<int64_t>(ntiles, 1), 1024);
  } else {
    nblocks = std::max(1, std::min(c->L.n_items, 1024));
  }
  const int64_t pstride = Sh::LEN + 4;
  LFE_TRY(ensure_scratch(c, (size_t)nblocks * pstride));
  LFE_TRY(ensure_dred(c, (size_t)pstride));
  // stage the alpha_P slice in LDS when it fits beside the tile (<= 160 KB per CU, 1+ workgroups)
  const size_t zbytes = sizeof(double) * Sh::ZW * kZST + 128;
  const size_t sbytes = sizeof(double) * (size_t)a.B * a.la.p;
  a.stage = (MODE != GRAM_TABLE && a.la.P >= 0 && zbytes + sbytes <= 150 * 1024) ? 1 : 0;
  const size_t dyn = a.stage ? sbytes : 0;
  {
    ProfScope _ps(c, MODE == GRAM_DESIGN ? K_GRAM_DESIGN : (MODE == GRAM_RESID ? K_GRAM_RESID : K_GRAM_TABLE));
    if (dyn > 0)  // dynamic LDS above 64 KB must be opted in
      LFE_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gram<MODE, NT>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn));
    hipLaunchKernelGGL((k_gram<MODE, NT>), dim3(nblocks), dim3(kTR), dyn, c->stream, a, c->scratch, pstride);
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

// ncols = Gram width; tile_cols = columns a row staging needs (>= ncols)
template <int MODE>
static int gram_dispatch(lfe_ctx* c, GramArgs a, int ncols, int tile_cols, double* dense_out, double* extra_out,
                         int extra) {
  const int NT = (std::max(std::max(ncols, tile_cols), 1) + 15) / 16;
  std::vector<double> h((size_t)10 * 256 + 4);
  int rc;
  switch (NT) {
    case 1: rc = run_gram<MODE, 1>(c, a, h.data(), extra); break;
    case 2: rc = run_gram<MODE, 2>(c, a, h.data(), extra); break;
    case 3: rc = run_gram<MODE, 3>(c, a, h.data(), extra); break;
    case 4: rc = run_gram<MODE, 4>(c, a, h.data(), extra); break;
    default: set_error("too many columns for the Gram kernel (max 64)"); return LFE_EINVAL;
  }
  if (rc) return rc;
  if (dense_out) unpack_tiles(h.data(), NT, ncols, dense_out);
  if (extra_out) {
    const int len = NT * (NT + 1) / 2 * 256;
    for (int s = 0; s < extra; ++s) extra_out[s] = h[len + s];
  }
  return LFE_OK;
}

static GramArgs base_args(lfe_ctx* c) {
  GramArgs a{};
  a.la = layout_args(c);
  a.X = c->L.X;
  a.ld = c->ld;
  a.w = c->L.w;
  a.B = 1 << c->L.s;
  a.G_P = c->L.P >= 0 ? c->fe[c->L.P].G : 0;
  return a;
}

int launch_gram(lfe_ctx* c, double* host_gram) {
  GramArgs a = base_args(c);
  return gram_dispatch<GRAM_DESIGN>(c, a, c->p + 1, c->p + 1, host_gram, nullptr, 0);
}

int launch_resid(lfe_ctx* c, const double* beta_full, double* stats, double* hc1, int keep_scores) {
  GramArgs a = base_args(c);
  LFE_HIP(hipMemcpyAsync(c->dbeta, beta_full, sizeof(double) * c->p, hipMemcpyHostToDevice, c->stream));
  a.beta = c->dbeta;
  a.scores = keep_scores ? c->scores : nullptr;
  const int k = c->p - 1;
  std::vector<double> meat((size_t)std::max(k, 1) * std::max(k, 1));
  const int rc = gram_dispatch<GRAM_RESID>(c, a, k, c->p, meat.data(), stats, 4);
  if (rc) return rc;
  if (hc1)
    for (int e = 0; e < k * k; ++e) hc1[e] = meat[e];
  c->scores_valid = keep_scores != 0;
  return LFE_OK;
}

int launch_cluster(lfe_ctx* c, double* meats, int64_t* G_out) {
  const int k = c->p - 1;
  const int32_t* codeP = c->L.P >= 0 ? c->L.code[c->L.P] : nullptr;
  for (size_t j = 0; j < c->cl.size(); ++j) {
    const int32_t C = c->cl_levels[j];
    const size_t tab = (size_t)C * std::max(k, 1);
    LFE_TRY(ensure_cluster_ws(c, tab, (size_t)C + 4));
    double* S = c->clS;
    int32_t* present = c->clP;
    int32_t* cntG = present + C;
    LFE_HIP(hipMemsetAsync(S, 0, sizeof(double) * tab, c->stream));
    LFE_HIP(hipMemsetAsync(present, 0, sizeof(int32_t) * ((size_t)C + 4), c->stream));
    if (c->n && k > 0) {
      ProfScope _ps(c, K_CLUSTER_SCATTER);
      hipLaunchKernelGGL(k_cluster_scatter, dim3(grid_for(c->n)), dim3(kBlock), 0, c->stream, c->cl[j], c->L.orig,
                         codeP, c->scores, c->ld, c->n, k, S, present);
    }
    LFE_HIP(hipGetLastError());
    LFE_TRY(allreduce_sum_f64(c, S, (size_t)C * k));
    LFE_TRY(allreduce_sum_i32(c, present, C));
    hipLaunchKernelGGL(k_count_nonzero, dim3(grid_for(C)), dim3(kBlock), 0, c->stream, present, C, cntG);
    LFE_HIP(hipGetLastError());
    int32_t hG = 0;
    LFE_HIP(hipMemcpyAsync(&hG, cntG, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    LFE_HIP(hipStreamSynchronize(c->stream));
    G_out[j] = hG;
    if (k > 0) {
      GramArgs a{};
      a.table = S;
      a.rows = C;
      a.tcols = k;
      // the S table is replicated on every rank after the all-reduce: its Gram
      // is reduced locally only (no second all-reduce)
      const int world = c->world;
      c->world = 1;
      const int rc = gram_dispatch<GRAM_TABLE>(c, a, k, k, meats + j * (size_t)k * k, nullptr, 0);
      c->world = world;
      if (rc) return rc;
    }
  }
  return LFE_OK;
}

int launch_copy_demeaned(lfe_ctx* c, double* dev_out) {
  if (c->n)
    hipLaunchKernelGGL(k_copy_demeaned, dim3(grid_for(c->n)), dim3(kBlock), 0, c->stream, layout_args(c), c->L.X,
                       c->ld, c->n, c->L.orig, dev_out);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

}  // namespace lfe

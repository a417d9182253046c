// leanfe HIP engine — fits wider than one context (p > 63 columns: y, regressors, instruments).
//
// The reference forms X'X of [1, X_dm] whatever its width (polars_impl.py:165-209) and the SE
// meats from the same columns (std_errors.py:183-441).  A context holds at most 63 columns (its
// kernels keep a row's columns in registers or 16-column MFMA slots), so a wide fit runs as column
// blocks, one context per block: each loads the FE codes and its columns and demeans them - every
// column's projections are its own (polars_impl.py:491-508), and the blocks after the first run
// exactly the first block's number of sweeps - then writes its demeaned columns into one device
// matrix D [P][ld] in input row order (lfe_materialize; column 0 the kept-row indicator, then y~,
// then the regressors; 0 on dropped rows).  The solve's products are then dense ones:
//   Gram   D' D (weighted: D' diag(w) D)              k_wide_syrk
//   r      D v, v = [-b0, 1, -b]                       k_wide_resid (+ RSS, sums of y~)
//   HC1    D_x' diag(w r^2) D_x                        k_wide_syrk
//   CGM    per-cluster sums of x~ r (w) in two-limb fixed point over per-row cluster ids (a
//          one-column subset's codes, an intersection's sorted segments), then S' S
// k_wide_syrk: one 64 x 64 output tile pair (ti <= tj) per workgroup and row range, four waves of
// 16 output rows each on v_mfma_f64_16x16x4f64 (lane (kq, c): 4 consecutive rows of one column,
// the layout of lfe_gram.hip's raw Gram); the row ranges' partial tiles are added in range order.
#include "lfe_internal.h"

#include <algorithm>
#include <string>
#include <vector>

namespace lfe {

static int fail(int code, const char* msg) {
  set_error(msg);
  return code;
}

template <typename T>
static int walloc(T** p, size_t elems) {
  const hipError_t e = hipMalloc(reinterpret_cast<void**>(p), sizeof(T) * std::max<size_t>(elems, 1));
  if (e != hipSuccess) {
    *p = nullptr;
    set_error(std::string("hipMalloc: ") + hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? LFE_ENOMEM : LFE_EHIP;
  }
  return LFE_OK;
}

typedef double d4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// demeaned columns -> D (input row order)
// ---------------------------------------------------------------------------
__global__ void k_materialize(LayoutArgs la, const double* __restrict__ X, int64_t ld, int64_t n,
                              const int32_t* __restrict__ orig, double* __restrict__ D, int64_t ldD, int first,
                              int col0, int mask_col) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t o = orig ? orig[i] : i;
    const bool dropped = la.P >= 0 && la.code[la.P][i] < 0;
    if (mask_col >= 0) D[(int64_t)mask_col * ldD + o] = dropped ? 0.0 : 1.0;
    for (int c = first; c < la.p; ++c) {
      double v = 0.0;
      if (!dropped) {
        v = X[(int64_t)c * ld + i];
        for (int f = 0; f < la.F; ++f) v -= la.alpha[f][(int64_t)la.code[f][i] * la.p + c];
      }
      D[(int64_t)(col0 + c - first) * ldD + o] = v;
    }
  }
}

// streamed X (pass 5): a chunk's x~ = x - sum_f alpha_f[g_f] (the keep test of the streamed passes,
// lfe_gram.hip k_stream_rows) into D's rows row0.. (the chunk is in input order already)
struct StreamMatArgs {
  const double* X;
  int64_t ld, rows;
  int p, F;
  const int32_t* code[kMaxFE];
  const int32_t* cnt_pre[kMaxFE];
  const double* alpha[kMaxFE];
  double* D;
  int64_t ldD;
  int col0, mask_col;
};

__global__ void k_stream_materialize(StreamMatArgs a) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.rows; i += (int64_t)gridDim.x * blockDim.x) {
    bool keep = true;
    for (int f = 0; f < a.F; ++f) keep = keep && a.cnt_pre[f][a.code[f][i]] > 1;
    if (a.mask_col >= 0) a.D[(int64_t)a.mask_col * a.ldD + i] = keep ? 1.0 : 0.0;
    for (int c = 0; c < a.p; ++c) {
      double v = 0.0;
      if (keep) {
        v = a.X[(int64_t)c * a.ld + i];
        for (int f = 0; f < a.F; ++f) v -= a.alpha[f][(int64_t)a.code[f][i] * a.p + c];
      }
      a.D[(int64_t)(a.col0 + c) * a.ldD + i] = v;
    }
  }
}

int stream_materialize_chunk(lfe_ctx* c, const double* X, int64_t ld, int64_t row0, int64_t rows) {
  const auto& w = c->sw;
  StreamMatArgs a{};
  a.X = X;
  a.ld = ld;
  a.rows = rows;
  a.p = c->p;
  a.F = c->F;
  for (int f = 0; f < c->F; ++f) {
    a.code[f] = c->fe[f].code + row0;
    a.cnt_pre[f] = c->fe[f].cnt_pre;
    a.alpha[f] = c->fe[f].alpha;
  }
  if (row0 < w.mbase || (w.mrows >= 0 && row0 + rows > w.mbase + w.mrows) || row0 - w.mbase + rows > w.mld)
    return fail(LFE_EINVAL, "rows outside the materialized range");
  a.D = w.mD + (row0 - w.mbase);
  a.ldD = w.mld;
  a.col0 = w.mcol0;
  a.mask_col = w.mmask;
  if (rows > 0) hipLaunchKernelGGL(k_stream_materialize, dim3(grid_for(rows)), dim3(kBlock), 0, c->stream, a);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

// ---------------------------------------------------------------------------
// A' diag(s) A over the rows, tiles of 64 x 64
// ---------------------------------------------------------------------------
constexpr int kWT = 64;  // tile side
struct SyrkArgs {
  const double* A;
  int64_t cs, rs;      // element (row i, column c) at A[c cs + i rs]; rs == 1: 32-byte row quads
  int64_t n;           // rows
  int P;               // columns
  const double* w;     // row weights (mode 1, 2), null: 1
  const double* r;     // residuals (mode 2, 3)
  int mode;            // row scale: 0 1, 1 w, 2 w r^2, 3 r^2
  int nt, nsplit;      // tiles per side, row ranges
  double* partial;     // [pairs][nsplit][kWT * kWT]
};

__device__ __forceinline__ void tile_of_pair(int pair, int nt, int& ti, int& tj) {
  ti = 0;
  while (pair >= nt - ti) {
    pair -= nt - ti;
    ++ti;
  }
  tj = ti + pair;
}

template <bool ROWQ>  // ROWQ: rs == 1, a lane's 4 rows of a column are one 32-byte load
__global__ __launch_bounds__(256) void k_wide_syrk(SyrkArgs a) {
  const int pair = blockIdx.x / a.nsplit, split = blockIdx.x - pair * a.nsplit;
  int ti, tj;
  tile_of_pair(pair, a.nt, ti, tj);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, kq = lane >> 4, c = lane & 15;
  const int ca = ti * kWT + wave * 16 + c;
  const bool va = ca < a.P;
  const double* pa = a.A + (int64_t)(va ? ca : 0) * a.cs;
  const double* pb[4];
  bool vb[4];
#pragma unroll
  for (int jb = 0; jb < 4; ++jb) {
    const int cb = tj * kWT + jb * 16 + c;
    vb[jb] = cb < a.P;
    pb[jb] = a.A + (int64_t)(vb[jb] ? cb : 0) * a.cs;
  }
  const int64_t n16 = (a.n + 15) / 16;
  const int64_t r0 = n16 * split / a.nsplit * 16, r1 = n16 * (split + 1) / a.nsplit * 16;
  d4 acc[4];
#pragma unroll
  for (int jb = 0; jb < 4; ++jb) acc[jb] = d4{0.0, 0.0, 0.0, 0.0};
  for (int64_t rb = r0 + 4 * kq; rb < r1; rb += 16) {
    double av[4], bv[4][4];
    if (ROWQ) {  // rows past n (A's padding, or a previous chunk's rows in a chunk buffer) count 0
      const d4 x = *reinterpret_cast<const d4*>(pa + rb);
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const d4 y = *reinterpret_cast<const d4*>(pb[jb] + rb);
#pragma unroll
        for (int s = 0; s < 4; ++s) bv[jb][s] = vb[jb] ? y[s] : 0.0;
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) av[s] = (va && rb + s < a.n) ? x[s] : 0.0;
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int64_t i = rb + s;
        const bool in = i < a.n;
        av[s] = (in && va) ? pa[i * a.rs] : 0.0;
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) bv[jb][s] = (in && vb[jb]) ? pb[jb][i * a.rs] : 0.0;
      }
    }
    if (a.mode) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int64_t i = rb + s;
        const bool in = i < a.n;
        double sc = 0.0;
        if (in) {
          sc = (a.mode == 1 || a.mode == 2) && a.w ? a.w[i] : 1.0;
          if (a.mode >= 2) sc *= a.r[i] * a.r[i];
        }
        av[s] *= sc;
      }
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) acc[jb] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s], bv[jb][s], acc[jb], 0, 0, 0);
  }
  // D of the MFMA: lane (kq, c) register rr holds output row kq + 4 rr, column c of its 16 x 16 block
  double* out = a.partial + (int64_t)blockIdx.x * kWT * kWT;
#pragma unroll
  for (int jb = 0; jb < 4; ++jb)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) out[(wave * 16 + kq + 4 * rr) * kWT + jb * 16 + c] = acc[jb][rr];
}

// tiles[pair][e] = the row ranges' partial tiles added in range order
__global__ void k_wide_reduce(const double* __restrict__ partial, int npairs, int nsplit, double* __restrict__ tiles) {
  const int64_t m = (int64_t)npairs * kWT * kWT;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < m; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t pair = t / (kWT * kWT), e = t - pair * kWT * kWT;
    double s = 0.0;
    for (int sp = 0; sp < nsplit; ++sp) s += partial[(pair * nsplit + sp) * kWT * kWT + e];
    tiles[t] = s;
  }
}

// out (host, P x P, row-major) = A' diag(s) A
int wide_syrk(lfe_ctx* c, const double* A, int64_t cs, int64_t rs, int64_t n, int P, int mode, const double* w,
              const double* r, double* out) {
  if (P <= 0) return LFE_OK;
  const int nt = (P + kWT - 1) / kWT, npairs = nt * (nt + 1) / 2;
  const int64_t n16 = std::max<int64_t>(1, (n + 15) / 16);
  // row ranges: ~4 workgroups per CU in all, each range >= 4096 rows
  const int nsplit = (int)std::max<int64_t>(1, std::min<int64_t>(n16 / 256, (4 * (int64_t)c->n_cu + npairs - 1) / npairs));
  double* part = nullptr;
  double* tiles = nullptr;
  LFE_TRY(walloc(&part, (size_t)npairs * nsplit * kWT * kWT));
  int rc = walloc(&tiles, (size_t)npairs * kWT * kWT);
  std::vector<double> h((size_t)npairs * kWT * kWT);
  if (rc == LFE_OK) {
    SyrkArgs a{};
    a.A = A;
    a.cs = cs;
    a.rs = rs;
    a.n = n;
    a.P = P;
    a.w = w;
    a.r = r;
    a.mode = mode;
    a.nt = nt;
    a.nsplit = nsplit;
    a.partial = part;
    {
      ProfScope _ps(c, K_GRAM_DESIGN);
      // the 32-byte row quads need rows up to the next multiple of 16 inside A's padded columns
      if (rs == 1 && cs >= (n + 15) / 16 * 16 && cs % 4 == 0)
        hipLaunchKernelGGL(k_wide_syrk<true>, dim3((unsigned)(npairs * nsplit)), dim3(256), 0, c->stream, a);
      else
        hipLaunchKernelGGL(k_wide_syrk<false>, dim3((unsigned)(npairs * nsplit)), dim3(256), 0, c->stream, a);
      hipLaunchKernelGGL(k_wide_reduce, dim3(grid_for((int64_t)npairs * kWT * kWT)), dim3(kBlock), 0, c->stream, part,
                         npairs, nsplit, tiles);
    }
    hipError_t e = hipGetLastError();
    if (e == hipSuccess)
      e = hipMemcpyAsync(h.data(), tiles, sizeof(double) * h.size(), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
      set_error(std::string("wide syrk: ") + hipGetErrorString(e));
      rc = LFE_EHIP;
    }
  }
  dfree_any(part);
  dfree_any(tiles);
  if (rc != LFE_OK) return rc;
  for (int pair = 0, ti = 0; ti < nt; ++ti)
    for (int tj = ti; tj < nt; ++tj, ++pair)
      for (int i = 0; i < kWT; ++i)
        for (int j = 0; j < kWT; ++j) {
          const int gi = ti * kWT + i, gj = tj * kWT + j;
          if (gi >= P || gj >= P) continue;
          const double v = h[((size_t)pair * kWT + i) * kWT + j];
          out[(size_t)gi * P + gj] = v;
          out[(size_t)gj * P + gi] = v;
        }
  return LFE_OK;
}

// ---------------------------------------------------------------------------
// residual r = D v, statistics
// ---------------------------------------------------------------------------
constexpr int kWrMaxP = 4096;
__global__ __launch_bounds__(256) void k_wide_resid(const double* __restrict__ D, int64_t ldD, int64_t n, int P,
                                                    const double* __restrict__ v, const double* __restrict__ w,
                                                    double* __restrict__ r, double* __restrict__ partial) {
  extern __shared__ double vs[];
  __shared__ double red[4][4];
  for (int j = threadIdx.x; j < P; j += blockDim.x) vs[j] = v[j];
  __syncthreads();
  double st[4] = {0.0, 0.0, 0.0, 0.0};  // sum w r^2, sum r^2, sum y~, sum y~^2 over kept rows
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    double s = 0.0;
    for (int c = 0; c < P; ++c) s = __builtin_fma(D[(int64_t)c * ldD + i], vs[c], s);
    r[i] = s;
    if (D[i] != 0.0) {
      const double rr = s * s, y = D[ldD + i];
      st[0] += (w ? w[i] : 1.0) * rr;
      st[1] += rr;
      st[2] += y;
      st[3] += y * y;
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const auto addop = [](double x, double y) { return x + y; };
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const double t = wave_reduce63(st[e], 0.0, addop);
    if (lane == 63) red[wave][e] = t;
  }
  __syncthreads();
  if (threadIdx.x < 4)
    partial[(int64_t)blockIdx.x * 4 + threadIdx.x] =
        ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
}

__global__ void k_wide_stats(const double* __restrict__ partial, int nblk, double* __restrict__ out) {
  if (threadIdx.x >= 4) return;
  double s = 0.0;
  for (int b = 0; b < nblk; ++b) s += partial[(int64_t)b * 4 + threadIdx.x];
  out[threadIdx.x] = s;
}

// ---------------------------------------------------------------------------
// cluster score sums over per-row cluster ids: two-limb fixed point (lfe_cluster.hip's form)
// ---------------------------------------------------------------------------
constexpr int kWcChunk = 8192;
constexpr int kWcCols = 64;  // score columns per fixed-point pass (the statistics head and quanta table width)
struct WideScoreArgs {
  const double* D;
  int64_t ldD, n;
  int c0, k;           // score columns: D's [c0, c0 + k) times e = r (w) (one pass: k <= kWcCols)
  const double* r;
  const double* w;
  const int32_t* cid;  // cluster id of every row (-1: not in any cluster)
};

__device__ __forceinline__ double wide_score(const WideScoreArgs& a, int64_t i, int c) {
  const double e = a.r[i] * (a.w ? a.w[i] : 1.0);
  return a.D[(int64_t)(a.c0 + c) * a.ldD + i] * e;
}

__global__ __launch_bounds__(256) void k_wc_stats(WideScoreArgs a, int nchunks, int32_t* __restrict__ cnt,
                                                  double* __restrict__ st) {
  __shared__ double ws[2][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t i0 = (int64_t)blockIdx.x * kWcChunk, i1 = min(a.n, i0 + kWcChunk);
  if (cnt)  // the first column pass counts the rows per cluster
    for (int64_t i = i0 + tid; i < i1; i += 256)
      if (a.cid[i] >= 0) atomicAdd(&cnt[a.cid[i]], 1);
  const auto fmaxop = [](double x, double y) { return fmax(x, y); };
  const auto addop = [](double x, double y) { return x + y; };
  for (int c = 0; c < a.k; ++c) {
    double m = 0.0, q = 0.0;
    for (int64_t i = i0 + tid; i < i1; i += 256) {
      if (a.cid[i] < 0) continue;
      const double v = wide_score(a, i, c);
      m = fmax(m, fabs(v));
      q = __builtin_fma(v, v, q);
    }
    m = wave_reduce63(m, 0.0, fmaxop);
    q = wave_reduce63(q, 0.0, addop);
    if (lane == 63) {
      ws[0][wave] = m;
      ws[1][wave] = q;
    }
    __syncthreads();
    if (tid == 0) {
      const double mm = fmax(fmax(ws[0][0], ws[0][1]), fmax(ws[0][2], ws[0][3]));
      st[kColStatHead + (int64_t)c * nchunks + blockIdx.x] = ((ws[1][0] + ws[1][1]) + ws[1][2]) + ws[1][3];
      atomicMax(reinterpret_cast<unsigned long long*>(st) + c, (unsigned long long)__double_as_longlong(mm));
    }
    __syncthreads();
  }
}

__global__ void k_wc_count(const int32_t* __restrict__ cnt, int32_t G, int32_t* __restrict__ out) {
  int32_t nz = 0, mx = 0;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < G; g += (int64_t)gridDim.x * blockDim.x) {
    nz += cnt[g] > 0 ? 1 : 0;
    mx = max(mx, cnt[g]);
  }
  if (nz) atomicAdd(&out[0], nz);
  if (mx) atomicMax(&out[1], mx);
}

// entry (cluster g, column c) at S[g k + c] (row-major: the fixed-point conversion's column is e % k)
__global__ void k_wc_add(WideScoreArgs a, const double* __restrict__ fq, unsigned long long* __restrict__ S,
                         double* __restrict__ hi) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t g = a.cid[i];
    if (g < 0) continue;
    for (int c = 0; c < a.k; ++c) {
      double hh;
      const unsigned long long xi = fix_split(wide_score(a, i, c), fix_col(fq, c), hh);
      const int64_t t = (int64_t)g * a.k + c;
      if (xi) atomicAdd(&S[t], xi);
      if (hh != 0.0) atomicAdd(&hi[t], hh);
    }
  }
}

}  // namespace lfe

using namespace lfe;

#define LFE_WCTX(c)                                    \
  do {                                                 \
    if (!(c)) return fail(LFE_EINVAL, "null context"); \
    LFE_HIP(hipSetDevice((c)->device));                \
  } while (0)

extern "C" {

int lfe_dev_alloc(lfe_ctx* c, int64_t n_doubles, double** out) {
  LFE_WCTX(c);
  if (!out || n_doubles < 0) return fail(LFE_EINVAL, "bad arguments");
  double* p = nullptr;
  LFE_TRY(walloc(&p, (size_t)std::max<int64_t>(n_doubles, 1)));
  const hipError_t e = hipMemsetAsync(p, 0, sizeof(double) * (size_t)std::max<int64_t>(n_doubles, 1), c->stream);
  if (e != hipSuccess) {
    dfree_any(p);
    LFE_HIP(e);
  }
  *out = p;
  return LFE_OK;
}

int lfe_dev_free(lfe_ctx* c, double* p) {
  LFE_WCTX(c);
  LFE_HIP(hipStreamSynchronize(c->stream));
  dfree_any(p);
  return LFE_OK;
}

int lfe_materialize(lfe_ctx* c, double* D, int64_t ldD, int first, int col0, int mask_col) {
  LFE_WCTX(c);
  if (c->sw.on) return fail(LFE_ESTATE, "not available with streamed X");
  if (!c->demeaned) return fail(LFE_ESTATE, "lfe_demean first");
  if (!D || ldD < c->n || first < 0 || first > c->p || col0 < 0) return fail(LFE_EINVAL, "bad arguments");
  LFE_TRY(ensure_layout_orig(c));
  if (c->n)
    hipLaunchKernelGGL(k_materialize, dim3(grid_for(c->n)), dim3(kBlock), 0, c->stream, layout_args(c), c->L.X, c->ld,
                       c->n, c->L.orig, D, ldD, first, col0, mask_col);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

int lfe_stream_materialize_rows(lfe_ctx* c, double* D, int64_t ldD, int col0, int mask_col, int64_t row0,
                                int64_t rows) {
  LFE_WCTX(c);
  auto& w = c->sw;
  if (!w.on) return fail(LFE_ESTATE, "lfe_stream_materialize_rows: the context holds resident columns");
  if (!c->demeaned) return fail(LFE_ESTATE, "lfe_demean first");
  if (w.pass != 0) return fail(LFE_ESTATE, "a streamed pass is open (lfe_stream_end first)");
  if (!D || row0 < 0 || rows < 0 || row0 + rows > c->n || ldD < rows || col0 < 0) return fail(LFE_EINVAL, "bad arguments");
  w.mD = D;
  w.mld = ldD;
  w.mcol0 = col0;
  w.mmask = mask_col;
  w.mbase = row0;
  w.mrows = rows;
  w.pass = 5;
  w.rows_done = 0;
  return LFE_OK;
}

int lfe_stream_materialize(lfe_ctx* c, double* D, int64_t ldD, int col0, int mask_col) {
  LFE_WCTX(c);
  auto& w = c->sw;
  if (!w.on) return fail(LFE_ESTATE, "lfe_stream_materialize: the context holds resident columns (lfe_materialize)");
  if (!c->demeaned) return fail(LFE_ESTATE, "lfe_demean first");
  if (w.pass != 0) return fail(LFE_ESTATE, "a streamed pass is open (lfe_stream_end first)");
  if (!D || ldD < c->n || col0 < 0) return fail(LFE_EINVAL, "bad arguments");
  w.mD = D;
  w.mld = ldD;
  w.mcol0 = col0;
  w.mmask = mask_col;
  w.mbase = 0;
  w.mrows = -1;
  w.pass = 5;
  w.rows_done = 0;
  return LFE_OK;
}

int lfe_wide_gram_rows(lfe_ctx* c, const double* D, int64_t ldD, int64_t row0, int64_t rows, int c0, int P, int mode,
                       const double* r, double* out) {
  LFE_WCTX(c);
  if (!D || !out || P < 1 || c0 < 0 || row0 < 0 || rows < 0 || row0 + rows > c->n || ldD < rows || mode < 0 ||
      mode > 3 || (mode >= 2 && !r))
    return fail(LFE_EINVAL, "bad arguments");
  if (c->world > 1) return fail(LFE_EINVAL, "wide fits run in one process");
  return wide_syrk(c, D + (int64_t)c0 * ldD, ldD, 1, rows, P, mode, c->w ? c->w + row0 : nullptr, r, out);
}

int lfe_wide_gram(lfe_ctx* c, const double* D, int64_t ldD, int c0, int P, int mode, const double* r, double* out) {
  if (!c) return fail(LFE_EINVAL, "null context");
  return lfe_wide_gram_rows(c, D, ldD, 0, c->n, c0, P, mode, r, out);
}

int lfe_wide_resid(lfe_ctx* c, const double* D, int64_t ldD, int P, const double* coef, double* r, double* stats) {
  if (!c) return fail(LFE_EINVAL, "null context");
  return lfe_wide_resid_rows(c, D, ldD, 0, c->n, P, coef, r, stats);
}

int lfe_wide_resid_rows(lfe_ctx* c, const double* D, int64_t ldD, int64_t row0, int64_t rows, int P,
                        const double* coef, double* r, double* stats) {
  LFE_WCTX(c);
  if (!D || !coef || !r || !stats || P < 2 || P > kWrMaxP || row0 < 0 || rows < 0 || row0 + rows > c->n || ldD < rows)
    return fail(LFE_EINVAL, "bad arguments");
  const double* wr = c->w ? c->w + row0 : nullptr;
  double* v = nullptr;
  double* part = nullptr;
  const int nblk = (int)std::max<int64_t>(1, std::min<int64_t>((rows + 255) / 256, 4 * (int64_t)c->n_cu));
  LFE_TRY(walloc(&v, (size_t)P + 4));
  int rc = walloc(&part, (size_t)nblk * 4 + 4);
  if (rc == LFE_OK) {
    hipError_t e = hipMemcpyAsync(v, coef, sizeof(double) * P, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) {
      ProfScope _ps(c, K_GRAM_RESID);
      hipLaunchKernelGGL(k_wide_resid, dim3(nblk), dim3(256), sizeof(double) * P, c->stream, D, ldD, rows, P, v, wr,
                         r, part);
      hipLaunchKernelGGL(k_wide_stats, dim3(1), dim3(64), 0, c->stream, part, nblk, part + (size_t)nblk * 4);
      e = hipGetLastError();
    }
    if (e == hipSuccess)
      e = hipMemcpyAsync(stats, part + (size_t)nblk * 4, sizeof(double) * 4, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
      set_error(std::string("wide resid: ") + hipGetErrorString(e));
      rc = LFE_EHIP;
    }
  }
  dfree_any(v);
  dfree_any(part);
  return rc;
}

// per subset: cluster ids (cluster_ids_input, lfe_cluster.hip), S[g][c] = sum over g's rows of
// x~_c r (w) in two-limb fixed point, meat = S'S (k x k), G = clusters holding kept rows
int lfe_wide_cluster_meats(lfe_ctx* c, const double* D, int64_t ldD, int c0, int k, const double* r, int n_subsets,
                           const int32_t* masks, double* meats_out, int64_t* G_out) {
  LFE_WCTX(c);
  if (!D || !r || (n_subsets > 0 && (!masks || !meats_out || !G_out)) || k < 1 || ldD < c->n)
    return fail(LFE_EINVAL, "bad arguments");
  if (c->world > 1) return fail(LFE_EINVAL, "wide fits run in one process");
  const int m = (int)c->cl.size();
  for (int s = 0; s < n_subsets; ++s)
    if (masks[s] <= 0 || masks[s] >= (1 << m)) return fail(LFE_EINVAL, "subset mask must select loaded cluster columns");
  const int64_t n = c->n;
  int32_t* cid = nullptr;
  double* full = nullptr;  // k > kWcCols: the [G][k] table assembled from the column passes
  size_t full_cap = 0;
  LFE_TRY(walloc(&cid, (size_t)std::max<int64_t>(n, 1)));
  int rc = LFE_OK;
  auto hip_ok = [&rc](hipError_t e, const char* what) {  // the fills below: errors into rc, as the rest
    if (e != hipSuccess && rc == LFE_OK) {
      set_error(std::string(what) + ": " + hipGetErrorString(e));
      rc = e == hipErrorOutOfMemory ? LFE_ENOMEM : LFE_EHIP;
    }
  };
  for (int s = 0; s < n_subsets && rc == LFE_OK; ++s) {
    int32_t G = 0;
    rc = cluster_ids_input(c, masks[s], D, cid, &G);  // D's column 0: the kept rows
    if (rc != LFE_OK) break;
    auto& W = c->clw;
    const int nch = (int)std::max<int64_t>(1, (n + kWcChunk - 1) / kWcChunk);
    const int kg_max = std::min(k, kWcCols);
    const size_t tab = (size_t)std::max(G, 1) * kg_max;
    rc = ensure_f64(c, W.fixst, W.fixst_cap, (size_t)kColStatHead + (size_t)kg_max * nch);
    if (rc == LFE_OK) rc = ensure_f64(c, W.fixq, W.fixq_cap, (size_t)kFqRows * kFqCols);
    if (rc == LFE_OK) rc = ensure_cluster_ws(c, tab, (size_t)G + 4);
    if (rc == LFE_OK) rc = ensure_f64(c, W.srec, W.srec_cap, tab);
    if (rc == LFE_OK && k > kWcCols && (size_t)std::max(G, 1) * k > full_cap) {
      (void)hipStreamSynchronize(c->stream);  // an earlier subset's table may still be read
      dfree_any(full);
      full = nullptr;
      full_cap = (size_t)std::max(G, 1) * k;
      rc = walloc(&full, full_cap);
    }
    if (rc != LFE_OK) break;
    int32_t* cnt = c->clP;
    int32_t* cm = c->clP + G;
    hip_ok(hipMemsetAsync(cnt, 0, sizeof(int32_t) * ((size_t)G + 4), c->stream), "memset of the counts");
    // columns in passes of <= 64 (one quanta table each); a wider table is assembled in `full`
    for (int cb = 0; cb < k && rc == LFE_OK; cb += kWcCols) {
      const int kg = std::min(kWcCols, k - cb);
      hip_ok(hipMemsetAsync(W.fixst, 0, sizeof(double) * kColStatHead, c->stream), "memset of fixst");
      hip_ok(hipMemsetAsync(c->clS, 0, sizeof(double) * (size_t)std::max(G, 1) * kg, c->stream), "memset of clS");
      hip_ok(hipMemsetAsync(W.srec, 0, sizeof(double) * (size_t)std::max(G, 1) * kg, c->stream), "memset of srec");
      if (rc != LFE_OK) break;
      WideScoreArgs a{D, ldD, n, c0 + cb, kg, r, c->w, cid};
      {
        ProfScope _ps(c, K_CLUSTER_SCATTER);
        if (n > 0)
          hipLaunchKernelGGL(k_wc_stats, dim3(nch), dim3(256), 0, c->stream, a, nch, cb == 0 ? cnt : nullptr, W.fixst);
        if (cb == 0) hipLaunchKernelGGL(k_wc_count, dim3(grid_for(G, 256, 1024)), dim3(256), 0, c->stream, cnt, G, cm);
      }
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) {
        set_error(std::string("wide cluster sums: ") + hipGetErrorString(e));
        rc = LFE_EHIP;
        break;
      }
      rc = launch_fix_quanta(c, W.fixst, nch, std::max<int64_t>(n, 1), cm + 1, 1, W.fixq, kg);
      if (rc != LFE_OK) break;
      if (n > 0) {
        ProfScope _ps(c, K_CLUSTER_SCATTER);
        hipLaunchKernelGGL(k_wc_add, dim3(grid_for(n, 256, 8192)), dim3(256), 0, c->stream, a, W.fixq,
                           reinterpret_cast<unsigned long long*>(W.srec), c->clS);
      }
      rc = launch_fix_convert(c, W.srec, c->clS, (int64_t)G * kg, kg, W.fixq);
      if (rc == LFE_OK && full && G > 0) {  // [G][kg] -> columns cb.. of the [G][k] table
        const hipError_t e2 = hipMemcpy2DAsync(full + cb, sizeof(double) * k, W.srec, sizeof(double) * kg,
                                               sizeof(double) * kg, (size_t)G, hipMemcpyDeviceToDevice, c->stream);
        if (e2 != hipSuccess) rc = fail(LFE_EHIP, "wide cluster sums: hipMemcpy2DAsync");
      }
    }
    if (rc != LFE_OK) break;
    int32_t hG = 0;
    rc = d2h_sync(c, &hG, cm, sizeof(int32_t));
    if (rc != LFE_OK) break;
    G_out[s] = hG;
    // S' S of the row-major [G][k] table: element (row g, column j) at S[j + g k]
    rc = wide_syrk(c, full ? full : W.srec, 1, k, G, k, 0, nullptr, nullptr, meats_out + (size_t)s * k * k);
  }
  (void)hipStreamSynchronize(c->stream);
  dfree_any(cid);
  dfree_any(full);
  return rc;
}

}  // extern "C"

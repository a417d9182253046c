// leanfe HIP engine — the alternating-projections sweep (polars_impl.py:490-526).
//
// Algorithmic form ("alpha form").  The reference overwrites every column with
// c - mean_g(c) per FE per sweep (polars_impl.py:502-508).  Here the columns
// are never rewritten: each FE f keeps a table alpha_f[G_f][p] of the group
// means subtracted so far, the demeaned row is
//     x~_i = x_i - sum_f alpha_f[g_f(i)]                                  (1)
// and projecting FE f sets
//     alpha_f[g] = (S_f[g] - T_f[g]) / W_f[g]
//     S_f[g] = sum_{i in g} w_i x_i                 (constant: one data pass)
//     T_f[g] = sum_{i in g} w_i sum_{f'!=f} alpha_f'[g_f'(i)]           (2)
// the Gauss-Seidel iterate of the reference in exact arithmetic
// (mean_g(c - alpha_f_old) = mean_g(c) - alpha_f_old).  A projection reads FE
// codes only (4 B per row per FE), not the 8p data bytes.
//
// This file holds the constant sums: S_f (all p columns, lane-layout kernel in
// lfe_fast.hip) and, for weighted fits, W_f = sum w and the unweighted y sums
// Sy_f the stop test uses.  The cross terms T_f are in lfe_iter.hip (two FEs)
// and lfe_seg.hip (general case).
//
// Kernel shape (W_f, Sy_f): one workgroup per work item range.  Target tables
// live in LDS — a 2^s-group slice for the primary FE (rows of an item share one
// bucket), the whole table for small FEs — accumulated with ds_add_f64 and
// flushed to HBM once per item (slice) or per workgroup (table).  FE tables too
// large for LDS fall back to global f64 atomics.
#include "lfe_internal.h"

#include <algorithm>

namespace lfe {

enum { SRC_WEIGHT = 1, SRC_Y = 2 };

struct SweepArgs {
  LayoutArgs la;
  const double* X;   // y column (SRC_Y)
  const double* w;
  int src;           // value source
  int G[kMaxFE];
  double* out[kMaxFE];  // output tables [G] (nullptr: not a target)
  int lds_off[kMaxFE];  // LDS table offset (doubles), -1 = global atomics
  int lds_doubles;
  const double* fq;     // quanta of the two-limb sums (k_fix_quanta of k_col_stats_w)
  int fcol;             // the quanta's column of this source (p: weights, p + 1: y)
  double* hi[kMaxFE];   // coarse limbs [G] per FE
};

__global__ __launch_bounds__(kSweepThreads) void k_sweep_sums(SweepArgs a) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int tid = threadIdx.x;
  const int P = a.la.P, s = a.la.s;
  const int B = 1 << s;
  typedef unsigned long long u64;
  // two-limb fixed point (lfe_internal.h): integer adds commute, so the tables do not depend on
  // the order of the adds; outliers' coarse limbs go to the global hi tables
  const FixCol fc = fix_col(a.fq, a.fcol);
  auto add = [&](double* dst, double* hdst, double v) {
    double h;
    atomicAdd(reinterpret_cast<u64*>(dst), fix_split(v, fc, h));
    if (h != 0.0) atomicAdd(hdst, h);
  };
  auto nonzero = [&](const double* src) { return *reinterpret_cast<const u64*>(src) != 0ull; };
  auto flush_add = [&](double* dst, const double* src) {
    atomicAdd(reinterpret_cast<u64*>(dst), *reinterpret_cast<const u64*>(src));
  };

  // zero the non-slice LDS tables once per workgroup
  for (int f = 0; f < a.la.F; ++f)
    if (a.out[f] && a.lds_off[f] >= 0 && f != P)
      for (int j = tid; j < a.G[f]; j += blockDim.x) lds[a.lds_off[f] + j] = 0.0;

  for (int item = blockIdx.x; item < a.la.n_items; item += gridDim.x) {
    const int4 it = a.la.items[item];
    const int lo = it.x << s;
    __syncthreads();
    if (P >= 0 && a.out[P] && a.lds_off[P] >= 0)
      for (int j = tid; j < B; j += blockDim.x) lds[a.lds_off[P] + j] = 0.0;
    __syncthreads();
    for (int64_t i = it.y + tid; i < it.z; i += blockDim.x) {
      const int32_t hP = P >= 0 ? a.la.code[P][i] : 0;
      if (hP < 0) continue;  // dropped row (singleton filter)
      const double v = a.src == SRC_WEIGHT ? a.w[i] : a.X[i];
      for (int f = 0; f < a.la.F; ++f) {
        if (!a.out[f]) continue;
        const int64_t g = (f == P) ? (int64_t)(hP - lo) : (int64_t)a.la.code[f][i];
        const int64_t gg = (f == P) ? (int64_t)hP : g;
        if (a.lds_off[f] >= 0) add(&lds[a.lds_off[f] + g], &a.hi[f][gg], v);
        else add(&a.out[f][gg], &a.hi[f][gg], v);
      }
    }
    __syncthreads();
    // flush the primary slice of this item
    if (P >= 0 && a.out[P] && a.lds_off[P] >= 0)
      for (int j = tid; j < B; j += blockDim.x) {
        const int g = lo + j;
        if (nonzero(&lds[a.lds_off[P] + j]) && g < a.G[P]) flush_add(&a.out[P][g], &lds[a.lds_off[P] + j]);
      }
  }
  __syncthreads();
  // flush whole tables of the other FEs
  for (int f = 0; f < a.la.F; ++f)
    if (a.out[f] && a.lds_off[f] >= 0 && f != P)
      for (int j = tid; j < a.G[f]; j += blockDim.x) {
        if (nonzero(&lds[a.lds_off[f] + j])) flush_add(&a.out[f][j], &lds[a.lds_off[f] + j]);
      }
}

// two-limb one-column tables (fine limbs int64 bits in T, coarse limbs in hi, cleared) -> double
__global__ void k_fix_convert1(double* __restrict__ T, double* __restrict__ hi, int64_t m,
                               const double* __restrict__ fq, int col) {
  const bool big = fq[FQ_BIG * kFqCols + col] != 0.0;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
    double h = 0.0;
    if (big) {
      h = hi[e];
      if (h != 0.0) hi[e] = 0.0;
    }
    T[e] = fix_value((unsigned long long)__double_as_longlong(T[e]), h, fq, col);
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------

LayoutArgs layout_args(const lfe_ctx* c) {
  LayoutArgs a{};
  a.F = c->F;
  a.p = c->p;
  a.P = c->L.P;
  a.s = c->L.s;
  for (int f = 0; f < c->F; ++f) {
    a.code[f] = c->L.code[f];
    a.alpha[f] = c->fe[f].alpha;
  }
  a.items = reinterpret_cast<const int4*>(c->items_d);
  a.n_items = c->L.n_items;
  return a;
}

// one-column sums into the LDS-resident tables that fit (largest to global first)
static int run_sums(lfe_ctx* c, SweepArgs a) {
  const int P = c->L.P;
  const int B = 1 << c->L.s;
  bool in_lds[kMaxFE];
  for (int f = 0; f < c->F; ++f) in_lds[f] = a.out[f] != nullptr;
  const int64_t budget = kLdsBudget / 8;  // doubles
  for (;;) {
    int64_t rows = 0;
    for (int f = 0; f < c->F; ++f)
      if (in_lds[f]) rows += (f == P) ? B : c->fe[f].G;
    if (rows <= budget) break;
    int big = -1;
    for (int f = 0; f < c->F; ++f)
      if (in_lds[f] && (big < 0 || ((f == P) ? B : c->fe[f].G) > ((big == P) ? B : c->fe[big].G))) big = f;
    in_lds[big] = false;
  }
  int off = 0;
  for (int f = 0; f < c->F; ++f) {
    a.lds_off[f] = -1;
    if (in_lds[f]) {
      a.lds_off[f] = off;
      off += (f == P) ? B : c->fe[f].G;
    }
  }
  a.lds_doubles = off;
  const int grid = std::max(1, std::min(c->L.n_items, 512));
  {
    ProfScope _ps(c, K_GROUP_SUMS);
    hipLaunchKernelGGL(k_sweep_sums, dim3(grid), dim3(kSweepThreads), sizeof(double) * off, c->stream, a);
  }
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

int sweep_group_sums(lfe_ctx* c) {
  if (c->F == 0) return LFE_OK;
  // S_f: all p columns (weighted by w), lane-layout kernel (lfe_fast.hip)
  LFE_TRY(sums4(c));
  if (c->L.w) {
    // W_f = sum w and Sy_f = unweighted sum of y (the stop test is unweighted)
    SweepArgs a{};
    a.la = layout_args(c);
    a.X = c->L.X;
    a.w = c->L.w;
    for (int f = 0; f < c->F; ++f) {
      a.G[f] = c->fe[f].G;
      a.hi[f] = c->fe[f].hi;
    }
    // two-limb fixed point like S, with the quanta sums4 formed from the weighted statistics
    // (columns p: w, p + 1: y); W and Sy share the coarse-limb tables, one after the other
    a.fq = c->fixq;
    for (int pass = 0; pass < 2; ++pass) {
      for (int f = 0; f < c->F; ++f) {
        double* out = pass == 0 ? c->fe[f].W : c->fe[f].Sy;
        LFE_HIP(hipMemsetAsync(out, 0, sizeof(double) * c->fe[f].G, c->stream));
        a.out[f] = out;
      }
      a.fcol = c->p + pass;
      a.src = pass == 0 ? SRC_WEIGHT : SRC_Y;
      LFE_TRY(hi_begin(c));
      LFE_TRY(run_sums(c, a));
      for (int f = 0; f < c->F; ++f)
        hipLaunchKernelGGL(k_fix_convert1, dim3(grid_for(c->fe[f].G)), dim3(kBlock), 0, c->stream, a.out[f],
                           c->fe[f].hi, (int64_t)c->fe[f].G, c->fixq, a.fcol);
      LFE_HIP(hipGetLastError());
      hi_end(c);
    }
    for (int f = 0; f < c->F; ++f) {
      if (c->owner_on && f == c->L.P) continue;  // owner-sharded: the primary FE's are complete
      LFE_TRY(allreduce_sum_f64(c, c->fe[f].W, c->fe[f].G));
      LFE_TRY(allreduce_sum_f64(c, c->fe[f].Sy, c->fe[f].G));
    }
  }
  return LFE_OK;
}

}  // namespace lfe

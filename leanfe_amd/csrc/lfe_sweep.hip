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
// Kernel shape: one workgroup per (work item range, column group).  Target
// tables live in LDS — a 2^s-group slice for the primary FE (rows of an item
// share one bucket), the whole table for small FEs — accumulated with
// ds_add_f64 and flushed to HBM once per item (slice) or per workgroup
// (table).  FE tables too large for LDS fall back to global f64 atomics.
#include "lfe_internal.h"

#include <algorithm>

namespace lfe {

enum { SW_SUMS = 0, SW_CROSS = 1 };
enum { SRC_X = 0, SRC_WEIGHT = 1, SRC_Y = 2 };

struct SweepArgs {
  LayoutArgs la;
  const double* X;
  int64_t ld;
  const double* w;
  int c0, W;       // column groups: workgroup (x, y) handles [c0 + y*W, c0 + y*W + W) & < ncols
  int ncols;
  int src;         // SUMS value source
  int weighted;    // CROSS: scale the cross term by w_i
  int target;      // CROSS: target FE
  int G[kMaxFE];
  double* out[kMaxFE];  // output tables (nullptr: not a target)
  int ostride;          // output row stride (p or 1)
  int lds_off[kMaxFE];  // LDS table offset (doubles), -1 = global atomics
  int stage_off;        // CROSS, target != P: LDS offset of the staged alpha_P slice (-1: none)
  int lds_doubles;
};

template <int MODE>
__global__ __launch_bounds__(kSweepThreads) void k_sweep(SweepArgs a) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int tid = threadIdx.x;
  const int P = a.la.P, s = a.la.s, p = a.la.p;
  const int B = 1 << s;
  // column group of this workgroup: [c0, c0 + W) ; LDS tables use the full stride a.W
  const int c0 = a.c0 + blockIdx.y * a.W;
  const int W = min(a.W, a.ncols - c0);
  const int Ws = a.W;

  // zero the non-slice LDS tables once per workgroup
  for (int f = 0; f < a.la.F; ++f)
    if (a.out[f] && a.lds_off[f] >= 0 && f != P)
      for (int j = tid; j < a.G[f] * Ws; j += blockDim.x) lds[a.lds_off[f] + j] = 0.0;

  for (int item = blockIdx.x; item < a.la.n_items; item += gridDim.x) {
    const int4 it = a.la.items[item];
    const int lo = it.x << s;
    __syncthreads();
    if (P >= 0) {
      if (a.out[P] && a.lds_off[P] >= 0)
        for (int j = tid; j < B * Ws; j += blockDim.x) lds[a.lds_off[P] + j] = 0.0;
      if (MODE == SW_CROSS && a.stage_off >= 0)
        for (int j = tid; j < B * Ws; j += blockDim.x) {
          const int g = lo + j / Ws, cc = j % Ws;
          lds[a.stage_off + j] = (g < a.G[P] && cc < W) ? a.la.alpha[P][(int64_t)g * p + c0 + cc] : 0.0;
        }
    }
    __syncthreads();
    for (int64_t i = it.y + tid; i < it.z; i += blockDim.x) {
      const int32_t hP = P >= 0 ? a.la.code[P][i] : 0;
      if (hP < 0) continue;  // dropped row (singleton filter)
      double v[kMaxGroupCols];
      if (MODE == SW_SUMS) {
        const double wi = a.w ? a.w[i] : 1.0;
#pragma unroll
        for (int cc = 0; cc < kMaxGroupCols; ++cc) {
          if (cc < W) {
            double x;
            if (a.src == SRC_WEIGHT) x = wi;
            else if (a.src == SRC_Y) x = a.X[i];
            else x = a.w ? wi * a.X[(int64_t)(c0 + cc) * a.ld + i] : a.X[(int64_t)(c0 + cc) * a.ld + i];
            v[cc] = x;
          }
        }
        for (int f = 0; f < a.la.F; ++f) {
          if (!a.out[f]) continue;
          const int64_t g = (f == P) ? (int64_t)(hP - lo) : (int64_t)a.la.code[f][i];
          if (a.lds_off[f] >= 0) {
            double* t = &lds[a.lds_off[f] + g * Ws];
#pragma unroll
            for (int cc = 0; cc < kMaxGroupCols; ++cc)
              if (cc < W) atomicAdd(&t[cc], v[cc]);
          } else {
            const int64_t gg = (f == P) ? (int64_t)hP : g;
            double* t = &a.out[f][gg * a.ostride + c0];
#pragma unroll
            for (int cc = 0; cc < kMaxGroupCols; ++cc)
              if (cc < W) atomicAdd(&t[cc], v[cc]);
          }
        }
      } else {
        const int t = a.target;
#pragma unroll
        for (int cc = 0; cc < kMaxGroupCols; ++cc) v[cc] = 0.0;
        for (int f = 0; f < a.la.F; ++f) {
          if (f == t) continue;
          if (f == P && a.stage_off >= 0) {
            const double* sl = &lds[a.stage_off + (int64_t)(hP - lo) * Ws];
#pragma unroll
            for (int cc = 0; cc < kMaxGroupCols; ++cc)
              if (cc < W) v[cc] += sl[cc];
          } else {
            const int64_t g = (f == P) ? (int64_t)hP : (int64_t)a.la.code[f][i];
            const double* al = &a.la.alpha[f][g * p + c0];
#pragma unroll
            for (int cc = 0; cc < kMaxGroupCols; ++cc)
              if (cc < W) v[cc] += al[cc];
          }
        }
        if (a.weighted && a.w) {
          const double wi = a.w[i];
#pragma unroll
          for (int cc = 0; cc < kMaxGroupCols; ++cc) v[cc] *= wi;
        }
        const int64_t g = (t == P) ? (int64_t)(hP - lo) : (int64_t)a.la.code[t][i];
        if (a.lds_off[t] >= 0) {
          double* tt = &lds[a.lds_off[t] + g * Ws];
#pragma unroll
          for (int cc = 0; cc < kMaxGroupCols; ++cc)
            if (cc < W) atomicAdd(&tt[cc], v[cc]);
        } else {
          const int64_t gg = (t == P) ? (int64_t)hP : g;
          double* tt = &a.out[t][gg * a.ostride + c0];
#pragma unroll
          for (int cc = 0; cc < kMaxGroupCols; ++cc)
            if (cc < W) atomicAdd(&tt[cc], v[cc]);
        }
      }
    }
    __syncthreads();
    // flush the primary slice of this item
    if (P >= 0 && a.out[P] && a.lds_off[P] >= 0)
      for (int j = tid; j < B * Ws; j += blockDim.x) {
        const double val = lds[a.lds_off[P] + j];
        const int g = lo + j / Ws, cc = j % Ws;
        if (val != 0.0 && g < a.G[P] && cc < W) atomicAdd(&a.out[P][(int64_t)g * a.ostride + c0 + cc], val);
      }
  }
  __syncthreads();
  // flush whole tables of the other FEs
  for (int f = 0; f < a.la.F; ++f)
    if (a.out[f] && a.lds_off[f] >= 0 && f != P)
      for (int j = tid; j < a.G[f] * Ws; j += blockDim.x) {
        const double val = lds[a.lds_off[f] + j];
        const int cc = j % Ws;
        if (val != 0.0 && cc < W) atomicAdd(&a.out[f][(int64_t)(j / Ws) * a.ostride + c0 + cc], val);
      }
}

// alpha_f = (S_f - T_f) / W_f   (weighted: W = sum w; else W = kept count)
__global__ void k_finalize(const double* __restrict__ S, const double* __restrict__ T, const double* __restrict__ Wsum,
                           const int32_t* __restrict__ cnt, int32_t G, int p, double* __restrict__ alpha) {
  const int64_t total = (int64_t)G * p;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t g = e / p;
    const double den = Wsum ? Wsum[g] : (double)cnt[g];
    alpha[e] = den > 0.0 ? (S[e] - (T ? T[e] : 0.0)) / den : 0.0;
  }
}

// check (polars_impl.py:512-521): for every group present,
//   mean_g(y~) = (Sy[g] - cnt[g] alpha[g][0] - R[g]) / cnt[g]
// max |.| -> out (non-negative doubles order like their bit patterns)
__global__ void k_check_max(const double* __restrict__ Sy, int sy_stride, const double* __restrict__ R,
                            const double* __restrict__ alpha, int p, const int32_t* __restrict__ cnt, int32_t G,
                            unsigned long long* __restrict__ out) {
  double m = 0.0;
  for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x) {
    const int32_t n = cnt[g];
    if (n > 0) {
      const double r = Sy[(int64_t)g * sy_stride] - (double)n * alpha[(int64_t)g * p] - (R ? R[g] : 0.0);
      m = fmax(m, fabs(r / (double)n));
    }
  }
  for (int off = 32; off > 0; off >>= 1) m = fmax(m, __shfl_down(m, off, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(out, (unsigned long long)__double_as_longlong(m));
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

// Pick the column-group width W and which target tables live in LDS.
// lds_rows[f] = rows of FE f's LDS table (slice 2^s for P); returns W >= 1.
static int plan_lds(const lfe_ctx* c, const bool* target, int stage_rows, int ncols, int* lds_off, int* lds_doubles,
                    int* W_out) {
  const int P = c->L.P;
  const int B = 1 << c->L.s;
  bool in_lds[kMaxFE];
  for (int f = 0; f < c->F; ++f) in_lds[f] = target[f];
  const int budget = kLdsBudget / 8;  // doubles
  for (;;) {
    int64_t rows = stage_rows;
    for (int f = 0; f < c->F; ++f)
      if (in_lds[f]) rows += (f == P) ? B : c->fe[f].G;
    int W = rows > 0 ? (int)std::min<int64_t>(budget / std::max<int64_t>(rows, 1), kMaxGroupCols) : kMaxGroupCols;
    W = std::min(W, ncols);
    if (W >= 1) {
      const int ng = (ncols + W - 1) / W;
      W = (ncols + ng - 1) / ng;  // equalise groups
      int off = 0;
      for (int f = 0; f < c->F; ++f) {
        lds_off[f] = -1;
        if (in_lds[f]) {
          lds_off[f] = off;
          off += ((f == P) ? B : c->fe[f].G) * W;
        }
      }
      *lds_doubles = off + stage_rows * W;
      *W_out = W;
      return off;  // stage offset
    }
    // drop the largest non-primary LDS table to global atomics
    int big = -1;
    for (int f = 0; f < c->F; ++f)
      if (in_lds[f] && f != P && (big < 0 || c->fe[f].G > c->fe[big].G)) big = f;
    if (big < 0) {  // only the slice left and it does not fit: shrink is impossible, go global
      for (int f = 0; f < c->F; ++f) in_lds[f] = false;
    } else {
      in_lds[big] = false;
    }
  }
}

template <int MODE>
static int run_sweep(lfe_ctx* c, SweepArgs a, int ncols, const bool* target, bool stage_alphaP, int kid) {
  const int B = 1 << c->L.s;
  int lds_off[kMaxFE], lds_doubles = 0, W = 1;
  const int stage_rows = (MODE == SW_CROSS && stage_alphaP) ? B : 0;
  const int stage_off = plan_lds(c, target, stage_rows, ncols, lds_off, &lds_doubles, &W);
  for (int f = 0; f < c->F; ++f) a.lds_off[f] = lds_off[f];
  a.stage_off = stage_rows ? stage_off : -1;
  a.W = W;
  a.lds_doubles = lds_doubles;
  const int ng = (ncols + W - 1) / W;
  // persistent-ish grid: about two resident 64 KB-LDS workgroups per CU in total
  const int per_group = std::max(1, std::min(c->L.n_items, 512 / ng));
  a.c0 = 0;
  a.ncols = ncols;
  {
    ProfScope _ps(c, kid);
    hipLaunchKernelGGL((k_sweep<MODE>), dim3(per_group, ng), dim3(kSweepThreads), sizeof(double) * lds_doubles,
                       c->stream, a);
  }
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

static SweepArgs sweep_base(lfe_ctx* c) {
  SweepArgs a{};
  a.la = layout_args(c);
  a.X = c->L.X;
  a.ld = c->ld;
  a.w = c->L.w;
  for (int f = 0; f < c->F; ++f) {
    a.G[f] = c->fe[f].G;
    a.out[f] = nullptr;
  }
  return a;
}

int sweep_group_sums(lfe_ctx* c) {
  if (c->F == 0) return LFE_OK;
  bool target[kMaxFE];
  for (int f = 0; f < c->F; ++f) target[f] = true;
  SweepArgs a = sweep_base(c);
  // S_f: all p columns (weighted by w), lane-layout kernel (lfe_fast.hip)
  LFE_TRY(sums4(c));
  if (c->L.w) {
    // W_f = sum w and Sy_f = unweighted sum of y (the stop test is unweighted)
    for (int f = 0; f < c->F; ++f) {
      LFE_HIP(hipMemsetAsync(c->fe[f].W, 0, sizeof(double) * c->fe[f].G, c->stream));
      a.out[f] = c->fe[f].W;
    }
    a.src = SRC_WEIGHT;
    a.ostride = 1;
    LFE_TRY(run_sweep<SW_SUMS>(c, a, 1, target, false, K_GROUP_SUMS));
    for (int f = 0; f < c->F; ++f) {
      LFE_HIP(hipMemsetAsync(c->fe[f].Sy, 0, sizeof(double) * c->fe[f].G, c->stream));
      a.out[f] = c->fe[f].Sy;
    }
    a.src = SRC_Y;
    LFE_TRY(run_sweep<SW_SUMS>(c, a, 1, target, false, K_GROUP_SUMS));
    for (int f = 0; f < c->F; ++f) {
      LFE_TRY(allreduce_sum_f64(c, c->fe[f].W, c->fe[f].G));
      LFE_TRY(allreduce_sum_f64(c, c->fe[f].Sy, c->fe[f].G));
    }
  }
  return LFE_OK;
}

int sweep_project(lfe_ctx* c, int f) {
  auto& fe = c->fe[f];
  const bool cross = c->F > 1;
  if (cross) {
    LFE_HIP(hipMemsetAsync(fe.T, 0, sizeof(double) * (size_t)fe.G * c->p, c->stream));
    bool target[kMaxFE] = {false};
    target[f] = true;
    SweepArgs a = sweep_base(c);
    a.out[f] = fe.T;
    a.ostride = c->p;
    a.target = f;
    a.weighted = c->L.w != nullptr;
    LFE_TRY(run_sweep<SW_CROSS>(c, a, c->p, target, f != c->L.P && c->L.P >= 0, K_CROSS));
    LFE_TRY(allreduce_sum_f64(c, fe.T, (size_t)fe.G * c->p));
  }
  ProfScope _ps(c, K_FINALIZE);
  hipLaunchKernelGGL(k_finalize, dim3(grid_for((int64_t)fe.G * c->p)), dim3(kBlock), 0, c->stream, fe.S,
                     cross ? fe.T : nullptr, c->L.w ? fe.W : nullptr, fe.cnt, fe.G, c->p, fe.alpha);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

int sweep_check(lfe_ctx* c, double* host_max) {
  LFE_TRY(ensure_dred(c, 1));
  LFE_HIP(hipMemsetAsync(c->dred, 0, sizeof(double), c->stream));
  for (int f = 0; f < c->F; ++f) {
    auto& fe = c->fe[f];
    const bool cross = c->F > 1;
    if (cross) {
      LFE_HIP(hipMemsetAsync(fe.R, 0, sizeof(double) * fe.G, c->stream));
      bool target[kMaxFE] = {false};
      target[f] = true;
      SweepArgs a = sweep_base(c);
      a.out[f] = fe.R;
      a.ostride = 1;
      a.target = f;
      a.weighted = 0;  // the reference's check is unweighted (polars_impl.py:513)
      LFE_TRY(run_sweep<SW_CROSS>(c, a, 1, target, f != c->L.P && c->L.P >= 0, K_CHECK));
      LFE_TRY(allreduce_sum_f64(c, fe.R, fe.G));
    }
    ProfScope _ps(c, K_CHECK_MAX);
    const double* Sy = c->L.w ? fe.Sy : fe.S;
    hipLaunchKernelGGL(k_check_max, dim3(grid_for(fe.G)), dim3(kBlock), 0, c->stream, Sy, c->L.w ? 1 : c->p,
                       cross ? fe.R : nullptr, fe.alpha, c->p, fe.cnt, fe.G,
                       reinterpret_cast<unsigned long long*>(c->dred));
  }
  LFE_HIP(hipGetLastError());
  LFE_TRY(d2h_sync(c, host_max, c->dred, sizeof(double)));
  return LFE_OK;
}

}  // namespace lfe

// leanfe HIP engine — fast paths of the demeaning loop (polars_impl.py:490-526).
//
// 1. k_sums4: the constant group sums S_f = sum_{i in g} w_i x_i in the
//    MFMA-native lane layout of lfe_gram.hip (lane = (row quad, column)): a
//    lane loads 4 consecutive rows of one column as a 32-byte vector and
//    adds them into LDS tables whose 16 lanes of a row hit 16 consecutive
//    doubles (primary FE: the 2^s-group slice of the item's bucket; small FEs:
//    whole tables).
//
// 2. Segment layout + fused iteration (two FEs, unweighted — the headline
//    case).  Kept rows are counting-sorted by the primary code h into
//    contiguous segments; only the secondary code q of each row is stored
//    (4 B/row).  One sweep (order [Q, P]) then is a single codes-only pass:
//        per segment h (one wavefront):
//          T_P[h]   = sum_{i in h} alpha_Q[q_i]          wave-local reduction, no atomics
//          alpha_P[h] = (S_P[h] - T_P[h]) / n_h           projection of P (eq. 2)
//          T_Q'[q_i] += alpha_P[h]  for i in h            LDS ds_add_f64 into the next Q cross term
//    followed by alpha_Q' = (S_Q - T_Q') / n_Q.  The stop test after the sweep
//    (max_g |mean_g(y~)|, y only, polars_impl.py:511-521) is exactly
//    |alpha_Q' - alpha_Q| on the y column for Q, and 0 for the just-projected
//    P (the reference sees rounding noise ~1e-17 there), so it is free.
//    Multi-GPU splits the kernel at the two cross terms (RCCL all-reduce of
//    T_P and T_Q between the halves).
#include "lfe_internal.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>

namespace lfe {

typedef double d4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ d4 ld4(const double* p) { return *reinterpret_cast<const d4*>(p); }

// ===========================================================================
// 1. group sums
// ===========================================================================

constexpr int kSumThreads = 512;

struct Sums4Args {
  LayoutArgs la;
  const double* X;
  int64_t ld;
  const double* w;
  int G[kMaxFE];
  double* S[kMaxFE];
  int tab_off[kMaxFE];  // LDS offset (doubles) of a non-primary table, -1: global atomics
  int B, G_P;
  int slice;            // 1: primary slice accumulated in LDS at offset 0
  int nq;               // number of non-primary FEs and their indices
  int qf[kMaxFE];
};

// FQ: max non-primary FEs held in registers; GU: 16-row groups loaded before use;
// NT: 16-column slots per lane (p <= 16 NT); TH: threads per workgroup
template <int FQ, int GU, int NT, int TH>
__global__ __launch_bounds__(TH) void k_sums4(Sums4Args a) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int nwv = TH / 64;
  const int kq = lane >> 4, c = lane & 15;
  const int p = a.la.p, P = a.la.P, F = a.la.F;
  const int nq = a.nq < FQ ? a.nq : FQ;
  for (int f = 0; f < F; ++f)
    if (f != P && a.tab_off[f] >= 0)
      for (int j = tid; j < a.G[f] * p; j += TH) lds[a.tab_off[f] + j] = 0.0;
  // primary slice [B][p] of the current bucket: flushed to S_P (and zeroed) on a
  // bucket change; a block owns a contiguous range of items
  auto flush = [&](int b) {
    const int lo = b << a.la.s;
    for (int j = tid; j < a.B * p; j += TH) {
      const double val = lds[j];
      const int g = lo + j / p;
      if (val != 0.0 && g < a.G_P) atomicAdd(&a.S[P][(int64_t)g * p + (j % p)], val);
      lds[j] = 0.0;
    }
  };
  if (a.slice)
    for (int j = tid; j < a.B * p; j += TH) lds[j] = 0.0;
  const int i0 = (int)((int64_t)blockIdx.x * a.la.n_items / gridDim.x);
  const int i1 = (int)((int64_t)(blockIdx.x + 1) * a.la.n_items / gridDim.x);
  int cur = -1;
  for (int item = i0; item < i1; ++item) {
    const int4 it = a.la.items[item];
    const int lo = it.x << a.la.s;
    if (a.slice && it.x != cur) {
      __syncthreads();
      if (cur >= 0) flush(cur);
      __syncthreads();
      cur = it.x;
    }
    const int64_t g0 = it.y >> 4, g1 = ((int64_t)it.z + 15) >> 4;
    for (int64_t gb = g0 + (int64_t)wave * GU; gb < g1; gb += nwv * GU) {
      int4 hq[GU], cq[GU][FQ];
      d4 xv[GU][NT], wv[GU];
      int64_t rb[GU];
#pragma unroll
      for (int u = 0; u < GU; ++u) {  // issue every load of GU groups first
        const int64_t gi = gb + u;
        const bool live = gi < g1;
        rb[u] = gi * 16 + kq * 4;
        hq[u] = !live ? int4{-1, -1, -1, -1}
                      : (P >= 0 ? *reinterpret_cast<const int4*>(a.la.code[P] + rb[u]) : int4{0, 0, 0, 0});
#pragma unroll
        for (int q = 0; q < FQ; ++q)
          cq[u][q] = (q < nq && live) ? *reinterpret_cast<const int4*>(a.la.code[a.qf[q]] + rb[u]) : int4{0, 0, 0, 0};
#pragma unroll
        for (int I = 0; I < NT; ++I)
          xv[u][I] = (16 * I + c < p && live) ? ld4(a.X + (int64_t)(16 * I + c) * a.ld + rb[u]) : d4{0.0, 0.0, 0.0, 0.0};
        wv[u] = (a.w && live) ? ld4(a.w + rb[u]) : d4{1.0, 1.0, 1.0, 1.0};
      }
#pragma unroll
      for (int u = 0; u < GU; ++u) {
        const int hv[4] = {hq[u].x, hq[u].y, hq[u].z, hq[u].w};
        bool valid[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) valid[s] = rb[u] + s >= it.y && rb[u] + s < it.z && hv[s] >= 0;
#pragma unroll
        for (int I = 0; I < NT; ++I) {
          const int col = 16 * I + c;
          if (col >= p) continue;
          d4 v = xv[u][I];
          if (a.w) v *= wv[u];  // sum of (c * w), polars_impl.py:496
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            if (!valid[s]) continue;
            if (P >= 0) {
              if (a.slice) atomicAdd(&lds[(hv[s] - lo) * p + col], v[s]);
              else atomicAdd(&a.S[P][(int64_t)hv[s] * p + col], v[s]);
            }
#pragma unroll
            for (int q = 0; q < FQ; ++q) {
              if (q >= nq) continue;
              const int f = a.qf[q];
              const int g = (&cq[u][q].x)[s];
              if (a.tab_off[f] >= 0) atomicAdd(&lds[a.tab_off[f] + g * p + col], v[s]);
              else atomicAdd(&a.S[f][(int64_t)g * p + col], v[s]);
            }
          }
        }
      }
    }
  }
  __syncthreads();
  if (a.slice && cur >= 0) flush(cur);
  for (int f = 0; f < F; ++f)
    if (f != P && a.tab_off[f] >= 0)
      for (int j = tid; j < a.G[f] * p; j += TH) {
        const double val = lds[a.tab_off[f] + j];
        if (val != 0.0) atomicAdd(&a.S[f][j], val);
      }
}

int sums4(lfe_ctx* c) {
  Sums4Args a{};
  a.la = layout_args(c);
  a.X = c->L.X;
  a.ld = c->ld;
  a.w = c->L.w;
  a.B = 1 << c->L.s;
  const int P = c->L.P, p = c->p;
  a.G_P = P >= 0 ? c->fe[P].G : 0;
  size_t off = 0;
  a.slice = (P >= 0 && (size_t)a.B * p * 8 <= 64 * 1024) ? 1 : 0;
  if (a.slice) off = (size_t)a.B * p;
  const size_t budget = 150 * 1024 / 8;
  for (int f = 0; f < c->F; ++f) {
    a.G[f] = c->fe[f].G;
    a.S[f] = c->fe[f].S;
    a.tab_off[f] = -1;
    if (f != P && off + (size_t)c->fe[f].G * p <= budget) {
      a.tab_off[f] = (int)off;
      off += (size_t)c->fe[f].G * p;
    }
    LFE_HIP(hipMemsetAsync(c->fe[f].S, 0, sizeof(double) * (size_t)c->fe[f].G * p, c->stream));
  }
  a.nq = 0;
  for (int f = 0; f < c->F; ++f)
    if (f != P) a.qf[a.nq++] = f;
  const size_t lds = off * 8;
  const int NT = (p + 15) / 16;
  const void* fn = nullptr;
#define SUMS4_FN(FQ, GU, NT_, TH_) reinterpret_cast<const void*>(&k_sums4<FQ, GU, NT_, TH_>)
  static const int gu_env = [] {
    const char* e = getenv("LFE_SUMS_GU");  // tuning override
    return e ? atoi(e) : 0;
  }();
  int threads = kSumThreads;
  if (a.nq <= 1 && NT == 1) {
    // the 2-FE case: one workgroup per CU (LDS), so 16 waves of <= 128 VGPRs (GU 2)
    threads = gu_env == 4 ? kSumThreads : 1024;
    fn = gu_env == 4 ? SUMS4_FN(1, 4, 1, kSumThreads) : SUMS4_FN(1, 2, 1, 1024);
  } else if (a.nq <= 1) {
    fn = NT == 2 ? SUMS4_FN(1, 2, 2, kSumThreads) : NT == 3 ? SUMS4_FN(1, 2, 3, kSumThreads)
                                                    : SUMS4_FN(1, 2, 4, kSumThreads);
  } else {
    fn = NT == 1   ? SUMS4_FN(7, 1, 1, kSumThreads)
         : NT == 2 ? SUMS4_FN(7, 1, 2, kSumThreads)
         : NT == 3 ? SUMS4_FN(7, 1, 3, kSumThreads)
                   : SUMS4_FN(7, 1, 4, kSumThreads);
  }
#undef SUMS4_FN
  LFE_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)std::max<size_t>(lds, 1)));
  const int nblocks = std::max(1, std::min(c->L.n_items, resident_blocks(c, fn, threads, lds)));
  {
    ProfScope _ps(c, K_GROUP_SUMS);
    void* args[] = {&a};
    LFE_HIP(hipLaunchKernel(fn, dim3(nblocks), dim3(threads), args, lds, c->stream));
  }
  LFE_HIP(hipGetLastError());
  for (int f = 0; f < c->F; ++f) LFE_TRY(allreduce_sum_f64(c, c->fe[f].S, (size_t)c->fe[f].G * p));
  return LFE_OK;
}

// ===========================================================================
// 2. segment layout
// ===========================================================================

// per work item: counts of kept rows of each primary group of its bucket
__global__ __launch_bounds__(256) void k_seg_hist(const int4* __restrict__ items, const int32_t* __restrict__ code,
                                                  int s, int32_t* __restrict__ itemcnt) {
  extern __shared__ int32_t h[];
  const int4 it = items[blockIdx.x];
  const int B = 1 << s, lo = it.x << s;
  for (int j = threadIdx.x; j < B; j += blockDim.x) h[j] = 0;
  __syncthreads();
  for (int64_t i = it.y + threadIdx.x; i < it.z; i += blockDim.x) {
    const int32_t g = code[i];
    if (g >= 0) atomicAdd(&h[g - lo], 1);
  }
  __syncthreads();
  for (int j = threadIdx.x; j < B; j += blockDim.x) itemcnt[(int64_t)blockIdx.x * B + j] = h[j];
}

// per (bucket, group): exclusive scan over the bucket's items; local group size -> cnt
__global__ void k_seg_base(const int32_t* __restrict__ bitems, int nb, int s, int32_t G_P,
                           int32_t* __restrict__ itemcnt, int32_t* __restrict__ cnt) {
  const int B = 1 << s;
  const int64_t total = (int64_t)nb * B;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(e / B), j = (int)(e % B);
    int32_t run = 0;
    for (int i = bitems[b]; i < bitems[b + 1]; ++i) {
      const int32_t t = itemcnt[(int64_t)i * B + j];
      itemcnt[(int64_t)i * B + j] = run;
      run += t;
    }
    const int64_t g = ((int64_t)b << s) + j;
    if (g < G_P) cnt[g] = run;
  }
}

// Counting sort of an item's kept rows by primary group, sub-chunk by sub-chunk
// (per-wave cursors, as in the partition scatter), writing the secondary code
// of each row to its segment slot in runs.
constexpr int kSegThreads = 512;
constexpr int kSegWaves = kSegThreads / 64;
constexpr int kSegPer = 8;
constexpr int kSegRows = kSegThreads * kSegPer;

__global__ __launch_bounds__(kSegThreads) void k_seg_scatter(const int4* __restrict__ items,
                                                             const int32_t* __restrict__ codeP,
                                                             const int32_t* __restrict__ codeQ, int s,
                                                             const int32_t* __restrict__ seg_off,
                                                             const int32_t* __restrict__ itembase, int32_t G_P,
                                                             int32_t* __restrict__ seg_q) {
  extern __shared__ int32_t sm[];
  const int B = 1 << s;
  int32_t* cur = sm;                     // [waves][B]
  int32_t* run = cur + kSegWaves * B;    // [B] next free slot of each group
  int32_t* tot = run + B;                // [B]
  int32_t* delta = tot + B;              // [B]
  int32_t* stage = delta + B;            // [kSegRows]
  int32_t* sb = stage + kSegRows;        // [kSegRows]
  __shared__ int32_t wsum[kSegWaves];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int4 it = items[blockIdx.x];
  const int lo = it.x << s;
  for (int j = tid; j < B; j += kSegThreads) {
    const int64_t g = (int64_t)lo + j;
    run[j] = (g < G_P ? seg_off[g] : 0) + itembase[(int64_t)blockIdx.x * B + j];
  }
  for (int64_t r0 = it.y; r0 < it.z; r0 += kSegRows) {
    const int64_t r1 = min((int64_t)it.z, r0 + kSegRows);
    const int64_t wbase = r0 + (int64_t)wave * kSegPer * 64;
    __syncthreads();
    for (int j = tid; j < kSegWaves * B; j += kSegThreads) cur[j] = 0;
    __syncthreads();
    int32_t key[kSegPer], q[kSegPer];
#pragma unroll
    for (int k = 0; k < kSegPer; ++k) {
      const int64_t i = wbase + k * 64 + lane;
      key[k] = -1;
      if (i < r1) {
        const int32_t g = codeP[i];
        if (g >= 0) {
          key[k] = g - lo;
          q[k] = codeQ[i];
          atomicAdd(&cur[wave * B + key[k]], 1);
        }
      }
    }
    __syncthreads();
    for (int j = tid; j < B; j += kSegThreads) {
      int32_t t = 0;
      for (int w2 = 0; w2 < kSegWaves; ++w2) {
        const int32_t hh = cur[w2 * B + j];
        cur[w2 * B + j] = t;
        t += hh;
      }
      tot[j] = t;
    }
    __syncthreads();
    {  // exclusive scan of tot over groups
      const int per = (B + kSegThreads - 1) / kSegThreads;
      const int b0 = tid * per;
      int32_t sum = 0;
      for (int k = 0; k < per; ++k)
        if (b0 + k < B) sum += tot[b0 + k];
      int32_t x = sum;
      for (int off = 1; off < 64; off <<= 1) {
        const int32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
      }
      if (lane == 63) wsum[wave] = x;
      __syncthreads();
      int32_t wofs = 0;
      for (int w2 = 0; w2 < wave; ++w2) wofs += wsum[w2];
      int32_t acc = x - sum + wofs;
      __syncthreads();
      for (int k = 0; k < per; ++k)
        if (b0 + k < B) {
          const int32_t t = tot[b0 + k];
          tot[b0 + k] = acc;  // local offset
          acc += t;
        }
    }
    __syncthreads();
    int32_t local_total = 0;
    for (int j = tid; j < B; j += kSegThreads) {
      const int32_t boff = tot[j];
      delta[j] = run[j] - boff;
      for (int w2 = 0; w2 < kSegWaves; ++w2) cur[w2 * B + j] += boff;
    }
    (void)local_total;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSegPer; ++k)
      if (key[k] >= 0) {
        const int32_t pos = atomicAdd(&cur[wave * B + key[k]], 1);
        stage[pos] = q[k];
        sb[pos] = key[k];
      }
    __syncthreads();
    // number of kept rows in this sub-chunk = sum of group totals
    const int32_t nk = (B > 0) ? (cur[(kSegWaves - 1) * B + (B - 1)]) : 0;  // end of the last group
    for (int j = tid; j < nk; j += kSegThreads) seg_q[delta[sb[j]] + j] = stage[j];
    __syncthreads();
    // advance the running slots: new run = delta + local end of each group
    for (int j = tid; j < B; j += kSegThreads) run[j] = delta[j] + cur[(kSegWaves - 1) * B + j];
  }
}

// first primary group of each work unit of ~U kept rows
__global__ void k_unit_bounds(const int32_t* __restrict__ seg_off, int32_t G_P, int64_t U, int n_units,
                              int32_t* __restrict__ units) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k <= n_units; k += gridDim.x * blockDim.x) {
    if (k == n_units) {
      units[k] = G_P;
      continue;
    }
    const int64_t target = (int64_t)k * U;
    int lo = 0, hi = G_P;  // first h with seg_off[h] >= target
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (seg_off[mid] < target) lo = mid + 1;
      else hi = mid;
    }
    units[k] = lo;
  }
}

int build_segments(lfe_ctx* c, int Q) {
  auto& L = c->L;
  const int P = L.P;
  const int B = 1 << L.s;
  const int32_t G_P = c->fe[P].G;
  LFE_TRY(ensure_i32(c, c->seg_aux, c->seg_aux_cap, (size_t)L.n_items * B));
  LFE_TRY(ensure_i32(c, c->seg_off, c->seg_off_cap, (size_t)G_P + 1));
  LFE_TRY(ensure_i32(c, c->seg_q, c->seg_q_cap, (size_t)c->ld));
  const int4* items = reinterpret_cast<const int4*>(c->items_d);
  {
    ProfScope _ps(c, K_MISC);
    hipLaunchKernelGGL(k_seg_hist, dim3(L.n_items), dim3(256), sizeof(int32_t) * B, c->stream, items, L.code[P], L.s,
                       c->seg_aux);
    LFE_HIP(hipMemsetAsync(c->seg_off, 0, sizeof(int32_t) * ((size_t)G_P + 1), c->stream));
    hipLaunchKernelGGL(k_seg_base, dim3(grid_for((int64_t)L.nb * B)), dim3(kBlock), 0, c->stream, c->bitems_d, L.nb,
                       L.s, G_P, c->seg_aux, c->seg_off);
    LFE_HIP(hipGetLastError());
  }
  LFE_TRY(exclusive_scan(c, c->seg_off, (int64_t)G_P + 1));
  {
    ProfScope _ps(c, K_MISC);
    const size_t lds = sizeof(int32_t) * ((size_t)kSegWaves * B + 3 * (size_t)B + 2 * (size_t)kSegRows);
    if (lds > 64 * 1024)
      LFE_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_seg_scatter),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(k_seg_scatter, dim3(L.n_items), dim3(kSegThreads), lds, c->stream, items, L.code[P],
                       L.code[Q], L.s, c->seg_off, c->seg_aux, G_P, c->seg_q);
    LFE_HIP(hipGetLastError());
  }
  // work units of ~2048 kept rows (whole segments)
  const int64_t U = 2048;
  const int64_t nk_local = c->n;  // upper bound on local kept rows
  c->n_units = (int)std::max<int64_t>(1, (nk_local + U - 1) / U);
  LFE_TRY(ensure_i32(c, c->seg_units, c->seg_units_cap, (size_t)c->n_units + 1));
  hipLaunchKernelGGL(k_unit_bounds, dim3(grid_for(c->n_units + 1)), dim3(kBlock), 0, c->stream, c->seg_off, G_P, U,
                     c->n_units, c->seg_units);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

// ===========================================================================
// 3. fused iteration
// ===========================================================================

constexpr int kIterThreads = 1024;
constexpr int kIterMaxW = 8;
constexpr int kIterK = 12;  // secondary codes per lane held in registers (segments <= 768 rows)
constexpr int kIterLds = 150 * 1024;  // LDS bytes for the two secondary tables

enum { IT_FUSED = 0, IT_REDUCE = 1, IT_SCATTER = 2 };

struct IterArgs {
  const int32_t* seg_off;
  const int32_t* seg_q;
  const int32_t* units;
  int n_units;
  int32_t G_P, G_Q;
  int p, c0, W;
  const double* alphaQ;  // [G_Q][p] current secondary effects (gather source)
  const double* S_P;     // [G_P][p]
  double* alphaP;        // [G_P][p] out (FUSED) / in (SCATTER)
  double* T_P;           // [G_P][p] out (REDUCE)
  double* T_Q;           // [G_Q][p] next secondary cross term (accumulated)
  int mode;
};

__global__ __launch_bounds__(kIterThreads) void k_iter(IterArgs a) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int W = a.W;
  // rows of the LDS tables are padded to an odd number of doubles (WS): with an
  // even stride the random secondary codes of a wavefront would fall on a few
  // banks only (a stride of 8 doubles: 16-way conflicts)
  const int WS = W | 1;
  double* aQ = lds;                        // [G_Q][WS] staged alpha_Q columns
  double* tQ = lds + (int64_t)a.G_Q * WS;  // [G_Q][WS] T_Q accumulation
  const int tid = threadIdx.x, lane = tid & 63;
  if (a.mode != IT_SCATTER)
    for (int j = tid; j < a.G_Q * W; j += kIterThreads)
      aQ[(j / W) * WS + (j % W)] = a.alphaQ[(int64_t)(j / W) * a.p + a.c0 + (j % W)];
  if (a.mode != IT_REDUCE)
    for (int j = tid; j < a.G_Q * WS; j += kIterThreads) tQ[j] = 0.0;
  __syncthreads();
  const int nwaves = gridDim.x * (kIterThreads / 64);
  // The secondary codes of a segment are held in registers (kIterK per lane:
  // segments up to 64 kIterK rows; longer ones finish in a plain loop) and the
  // next segment's codes are loaded while this one runs on LDS, so a segment
  // costs one exposed global latency at most.
  int qn[kIterK];
  int nr0 = 0, nr1 = 0;
  auto load_seg = [&](int h) {
    nr0 = a.seg_off[h];
    nr1 = a.seg_off[h + 1];
#pragma unroll
    for (int k = 0; k < kIterK; ++k) {
      const int32_t r = nr0 + lane + 64 * k;
      qn[k] = r < nr1 ? a.seg_q[r] : -1;
    }
  };
  for (int u = blockIdx.x * (kIterThreads / 64) + (tid >> 6); u < a.n_units; u += nwaves) {
    const int h0 = a.units[u], h1 = a.units[u + 1];
    if (h0 < h1) load_seg(h0);
    for (int h = h0; h < h1; ++h) {
      int qc[kIterK];
#pragma unroll
      for (int k = 0; k < kIterK; ++k) qc[k] = qn[k];
      const int32_t r0 = nr0, r1 = nr1;
      const int32_t n = r1 - r0;
      if (h + 1 < h1) load_seg(h + 1);
      const int32_t rtail = r0 + 64 * kIterK + lane;  // rows beyond the register window
      double ap[kIterMaxW];
      if (a.mode != IT_SCATTER) {
        double acc[kIterMaxW];
#pragma unroll
        for (int cc = 0; cc < kIterMaxW; ++cc) acc[cc] = 0.0;
#pragma unroll
        for (int k = 0; k < kIterK; ++k) {
          if (qc[k] < 0) continue;
          const double* src = &aQ[qc[k] * WS];
#pragma unroll
          for (int cc = 0; cc < kIterMaxW; ++cc)
            if (cc < W) acc[cc] += src[cc];
        }
        for (int32_t r = rtail; r < r1; r += 64) {
          const double* src = &aQ[a.seg_q[r] * WS];
#pragma unroll
          for (int cc = 0; cc < kIterMaxW; ++cc)
            if (cc < W) acc[cc] += src[cc];
        }
#pragma unroll
        for (int cc = 0; cc < kIterMaxW; ++cc)
#pragma unroll
          for (int off = 32; off > 0; off >>= 1) acc[cc] += __shfl_xor(acc[cc], off, 64);
        if (a.mode == IT_REDUCE) {
#pragma unroll
          for (int cc = 0; cc < kIterMaxW; ++cc)
            if (cc < W && lane == cc) a.T_P[(int64_t)h * a.p + a.c0 + cc] = acc[cc];
          continue;
        }
#pragma unroll
        for (int cc = 0; cc < kIterMaxW; ++cc) {
          ap[cc] = 0.0;
          if (cc < W && n > 0) ap[cc] = (a.S_P[(int64_t)h * a.p + a.c0 + cc] - acc[cc]) / (double)n;
          if (cc < W && lane == cc) a.alphaP[(int64_t)h * a.p + a.c0 + cc] = ap[cc];
        }
      } else {
#pragma unroll
        for (int cc = 0; cc < kIterMaxW; ++cc) ap[cc] = cc < W ? a.alphaP[(int64_t)h * a.p + a.c0 + cc] : 0.0;
      }
#pragma unroll
      for (int k = 0; k < kIterK; ++k) {
        if (qc[k] < 0) continue;
        double* dst = &tQ[qc[k] * WS];
#pragma unroll
        for (int cc = 0; cc < kIterMaxW; ++cc)
          if (cc < W) atomicAdd(&dst[cc], ap[cc]);
      }
      for (int32_t r = rtail; r < r1; r += 64) {
        double* dst = &tQ[a.seg_q[r] * WS];
#pragma unroll
        for (int cc = 0; cc < kIterMaxW; ++cc)
          if (cc < W) atomicAdd(&dst[cc], ap[cc]);
      }
    }
  }
  if (a.mode == IT_REDUCE) return;
  __syncthreads();
  for (int j = tid; j < a.G_Q * W; j += kIterThreads) {
    const double v = tQ[(j / W) * WS + (j % W)];
    if (v != 0.0) atomicAdd(&a.T_Q[(int64_t)(j / W) * a.p + a.c0 + (j % W)], v);
  }
}

// alpha_new = (S - T) / cnt; check = max_g |alpha_new[g][0] - alpha_cur[g][0]| over groups present
// (= |mean_g(y~)| after the sweep); NaN propagates (a NaN panel never converges).
__global__ void k_fin_check(const double* __restrict__ S, const double* __restrict__ T,
                            const int32_t* __restrict__ cnt, int32_t G, int p, const double* __restrict__ cur,
                            double* __restrict__ out, unsigned long long* __restrict__ check) {
  double m = 0.0;
  const int64_t total = (int64_t)G * p;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t g = e / p;
    const int32_t n = cnt[g];
    const double v = n > 0 ? (S[e] - (T ? T[e] : 0.0)) / (double)n : 0.0;
    out[e] = v;
    if (check && n > 0 && e % p == 0) {
      const double d = fabs(v - cur[e]);
      m = (isnan(d) || isnan(m)) ? __builtin_nan("") : fmax(m, d);
    }
  }
  if (!check) return;
  for (int off = 32; off > 0; off >>= 1) {
    const double o = __shfl_down(m, off, 64);
    m = (isnan(o) || isnan(m)) ? __builtin_nan("") : fmax(m, o);
  }
  if ((threadIdx.x & 63) == 0) atomicMax(check, (unsigned long long)__double_as_longlong(fabs(m)));
}

static int fin_check(lfe_ctx* c, int f, const double* T, const double* cur, double* out, bool check) {
  auto& fe = c->fe[f];
  ProfScope _ps(c, K_FINALIZE);
  hipLaunchKernelGGL(k_fin_check, dim3(grid_for((int64_t)fe.G * c->p)), dim3(kBlock), 0, c->stream, fe.S, T, fe.cnt,
                     fe.G, c->p, cur, out, check ? reinterpret_cast<unsigned long long*>(c->dred) : nullptr);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

bool fast_path_ok(const lfe_ctx* c, const std::vector<int>& order) {
  if (c->F != 2 || c->L.w || c->L.P < 0 || !c->L.permuted) return false;
  if (order.back() != c->L.P) return false;
  const int Q = 1 - c->L.P;
  return (int64_t)c->fe[Q].G * 2 * 8 <= kIterLds;  // W >= 1 columns of alpha_Q and T_Q in LDS
}

int demean_fast(lfe_ctx* c, double tol, int max_iter, int check_from, int* iterations_out, double* last_out) {
  const int P = c->L.P, Q = 1 - P, p = c->p;
  auto& fp = c->fe[P];
  auto& fq = c->fe[Q];
  LFE_TRY(build_segments(c, Q));
  LFE_TRY(ensure_f64(c, c->alpha_spare, c->alpha_spare_cap, (size_t)fq.G * p));
  LFE_TRY(ensure_dred(c, 1));
  // column groups: 2 * G_Q * (W | 1) doubles of LDS (odd row stride, see k_iter)
  const int64_t wmax = (kIterLds / 16) / std::max<int32_t>(fq.G, 1);  // max odd-padded stride
  int W = (int)std::min<int64_t>(kIterMaxW, wmax);
  if ((W | 1) > wmax) --W;
  W = std::max(1, std::min(W, p));
  const int ng = (p + W - 1) / W;
  W = (p + ng - 1) / ng;
  const size_t lds = sizeof(double) * 2 * (size_t)fq.G * (W | 1);
  LFE_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_iter), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)std::max<size_t>(lds, 1)));
  const int nblocks = std::max(1, std::min(256, (c->n_units + 15) / 16));
  // iteration 1's Q projection: alpha_P = 0 -> alpha_Q = S_Q / n_Q
  LFE_HIP(hipMemsetAsync(fp.alpha, 0, sizeof(double) * (size_t)fp.G * p, c->stream));
  LFE_TRY(fin_check(c, Q, nullptr, nullptr, fq.alpha, false));
  int iterations = 0;
  double last = -1.0;
  for (int it = 1; it <= max_iter; ++it) {
    LFE_HIP(hipMemsetAsync(fq.T, 0, sizeof(double) * (size_t)fq.G * p, c->stream));
    IterArgs a{};
    a.seg_off = c->seg_off;
    a.seg_q = c->seg_q;
    a.units = c->seg_units;
    a.n_units = c->n_units;
    a.G_P = fp.G;
    a.G_Q = fq.G;
    a.p = p;
    a.alphaQ = fq.alpha;
    a.S_P = fp.S;
    a.alphaP = fp.alpha;
    a.T_P = fp.T;
    a.T_Q = fq.T;
    if (c->world == 1) {
      a.mode = IT_FUSED;
      for (int g = 0; g < ng; ++g) {
        a.c0 = g * W;
        a.W = std::min(W, p - a.c0);
        ProfScope _ps(c, K_CROSS);
        hipLaunchKernelGGL(k_iter, dim3(nblocks), dim3(kIterThreads), lds, c->stream, a);
      }
    } else {
      a.mode = IT_REDUCE;
      for (int g = 0; g < ng; ++g) {
        a.c0 = g * W;
        a.W = std::min(W, p - a.c0);
        ProfScope _ps(c, K_CROSS);
        hipLaunchKernelGGL(k_iter, dim3(nblocks), dim3(kIterThreads), lds, c->stream, a);
      }
      LFE_TRY(allreduce_sum_f64(c, fp.T, (size_t)fp.G * p));
      LFE_TRY(fin_check(c, P, fp.T, nullptr, fp.alpha, false));
      a.mode = IT_SCATTER;
      for (int g = 0; g < ng; ++g) {
        a.c0 = g * W;
        a.W = std::min(W, p - a.c0);
        ProfScope _ps(c, K_CROSS);
        hipLaunchKernelGGL(k_iter, dim3(nblocks), dim3(kIterThreads), lds, c->stream, a);
      }
    }
    LFE_HIP(hipGetLastError());
    LFE_TRY(allreduce_sum_f64(c, fq.T, (size_t)fq.G * p));
    iterations = it;
    const bool check = it >= check_from;
    if (!check && it == max_iter) break;
    if (check) LFE_HIP(hipMemsetAsync(c->dred, 0, sizeof(double), c->stream));
    LFE_TRY(fin_check(c, Q, fq.T, fq.alpha, c->alpha_spare, check));
    if (check) {
      LFE_HIP(hipMemcpyAsync(&last, c->dred, sizeof(double), hipMemcpyDeviceToHost, c->stream));
      LFE_HIP(hipStreamSynchronize(c->stream));
      if (last < tol) break;  // converged after sweep `it`: keep alpha_Q of this sweep
    }
    if (it == max_iter) break;
    std::swap(fq.alpha, c->alpha_spare);
  }
  *iterations_out = iterations;
  *last_out = last;
  return LFE_OK;
}

}  // namespace lfe

// leanfe HIP engine — alternating projections, general case (polars_impl.py:490-526):
// three or more FEs, weighted fits, and two-FE fits whose secondary table does not
// fit in LDS (the unweighted two-FE case with a small secondary FE runs lfe_iter.hip).
//
// alpha form (see lfe_sweep.hip): projecting FE f sets
//     alpha_f[g] = (S_f[g] - T_f[g]) / W_f[g]
//     T_f[g]     = sum_{i in g} w_i sum_{f' != f} alpha_f'[g_f'(i)]
// so a projection reads FE codes and gathers alpha rows; it never touches X.
//
// Segment layouts.  For every FE f the kept rows are counting-sorted by g_f
// (seg_off_f[g] .. seg_off_f[g+1]) and, in that order, the codes of the other
// FEs (and w) are stored.  T_f is then a segmented sum of gathered alpha rows:
// no atomics, except where a segment crosses a work-unit boundary (2048-row
// units, so one huge group cannot serialize a wave).  The gathers hit the
// alpha tables in L2 / MALL (88 MB for 1e6 levels at p = 11).
//
// Lane layout as in lfe_iter.hip: lane = row quad kq (4 rows) x column c (16
// columns per slot, NT slots), a wave walks its unit in 16-row groups.
//
// Stop test (polars_impl.py:511-521): after sweep `it`, max_f max_g |mean_g(y~)|.
//   - last FE in the order: mean_g(y~) = (Sy - n alpha - T)/n with the T it was
//     just projected with;
//   - first FE: the same with T' = the next sweep's first cross term (computed
//     now, reused as that projection when the loop continues);
//   - middle FEs: one y-only cross pass each.
// Weighted fits check with unweighted sums (polars_impl.py:513), so they run
// y-only passes for every FE.
#include "lfe_internal.h"

#include <algorithm>
#include <cstdlib>

namespace lfe {

constexpr int kSegUnit = 2048;   // rows per work unit (multiple of 16)
constexpr int kSegThreads = 256;

// ---------------------------------------------------------------------------
// layout build
// ---------------------------------------------------------------------------

// local kept counts (multi-rank; world == 1 copies the kept counts instead)
__global__ __launch_bounds__(256) void k_seg_hist(const int32_t* __restrict__ keep, const int32_t* __restrict__ code,
                                                  int64_t n, int32_t* __restrict__ hist) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (keep[i] >= 0) atomicAdd(&hist[code[i]], 1);
}

struct SegScatterArgs {
  int F;
  int64_t n, ld;
  const int32_t* keep;          // layout codes of P (-1: dropped row)
  const int32_t* code[kMaxFE];  // layout order
  const double* w;              // layout order, or null
  int32_t* cur[kMaxFE];         // per FE cursor (starts at seg_off)
  int32_t* oc[kMaxFE];          // per FE: F-1 arrays of other codes, stride ld
  double* ws[kMaxFE];           // per FE weights in segment order (null: unweighted)
};

// every kept row goes to one slot of every FE's layout (unstable: the order
// within a segment follows the cursor atomics; sums are order-independent up to
// rounding, as with the reduction trees elsewhere)
__global__ __launch_bounds__(256) void k_seg_scatter(SegScatterArgs a) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
    if (a.keep[i] < 0) continue;
    int32_t g[kMaxFE];
    for (int f = 0; f < a.F; ++f) g[f] = a.code[f][i];
    const double wi = a.w ? a.w[i] : 0.0;
    for (int f = 0; f < a.F; ++f) {
      const int64_t pos = atomicAdd(&a.cur[f][g[f]], 1);
      int j = 0;
      for (int f2 = 0; f2 < a.F; ++f2)
        if (f2 != f) a.oc[f][(int64_t)(j++) * a.ld + pos] = g[f2];
      if (a.ws[f]) a.ws[f][pos] = wi;
    }
  }
}

// Block-aggregated variant: a workgroup takes kSegBlkRows consecutive layout rows.  For every FE
// whose codes in the block fall in a range of at most kSegLocalBins (the whole code range of a
// small FE; the primary FE's few buckets in the bucket-sorted layout) it counts the block's rows
// per code in LDS, reserves each code's slots with ONE returning global add, and ranks its rows in
// LDS; the other FEs keep one returning global add per row.  The slots of a (block, code) pair are
// consecutive, so the block's stores of the other codes land in short contiguous pieces.  (The
// order within a pair follows LDS atomics: unstable, as k_seg_scatter; the cross terms' two-limb
// sums do not depend on it.)
constexpr int kSegBlkRows = 32768;
constexpr int kSegBlkThreads = 1024;
constexpr int kSegLocalBins = 24576;  // LDS bins over all local FEs (96 KB)

struct SegScatter2Args {
  SegScatterArgs s;
  int32_t G[kMaxFE];
  int P;  // the bucketed primary FE (its codes are sorted by bucket in layout order), or -1
};

__global__ __launch_bounds__(kSegBlkThreads) void k_seg_scatter2(SegScatter2Args A) {
  const SegScatterArgs& a = A.s;
  __shared__ int32_t bins[kSegLocalBins];
  __shared__ int32_t klo[kMaxFE], kw[kMaxFE], boff[kMaxFE + 1];
  __shared__ int32_t pmin, pmax;
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * kSegBlkRows, r1 = min(a.n, r0 + kSegBlkRows);
  if (tid == 0) {
    pmin = 0x7fffffff;
    pmax = -1;
  }
  __syncthreads();
  // the primary FE's code range in this block (kept rows)
  if (A.P >= 0) {
    int32_t mn = 0x7fffffff, mx = -1;
    for (int64_t i = r0 + tid; i < r1; i += kSegBlkThreads) {
      if (a.keep[i] < 0) continue;
      const int32_t g = a.code[A.P][i];
      mn = min(mn, g);
      mx = max(mx, g);
    }
    for (int off = 32; off > 0; off >>= 1) {
      mn = min(mn, __shfl_xor(mn, off, 64));
      mx = max(mx, __shfl_xor(mx, off, 64));
    }
    if ((tid & 63) == 0) {
      atomicMin(&pmin, mn);
      atomicMax(&pmax, mx);
    }
  }
  __syncthreads();
  if (tid == 0) {  // which FEs are ranked in LDS, and where their bins live
    int used = 0;
    for (int f = 0; f < a.F; ++f) {
      int lo = 0, w = A.G[f];
      if (f == A.P) {
        lo = pmax >= 0 ? pmin : 0;
        w = pmax >= 0 ? pmax - pmin + 1 : 0;
      }
      const bool local = w <= kSegLocalBins - used;
      klo[f] = lo;
      kw[f] = local ? w : -1;
      boff[f] = used;
      if (local) used += w;
    }
    boff[a.F] = used;
  }
  __syncthreads();
  for (int j = tid; j < boff[a.F]; j += kSegBlkThreads) bins[j] = 0;
  __syncthreads();
  for (int64_t i = r0 + tid; i < r1; i += kSegBlkThreads) {
    if (a.keep[i] < 0) continue;
    for (int f = 0; f < a.F; ++f)
      if (kw[f] >= 0) atomicAdd(&bins[boff[f] + a.code[f][i] - klo[f]], 1);
  }
  __syncthreads();
  // one returning global add per (local FE, code present): the first slot of the block's rows
  for (int f = 0; f < a.F; ++f) {
    if (kw[f] < 0) continue;
    for (int j = tid; j < kw[f]; j += kSegBlkThreads) {
      const int32_t cnt = bins[boff[f] + j];
      if (cnt > 0) bins[boff[f] + j] = atomicAdd(&a.cur[f][klo[f] + j], cnt);
    }
  }
  __syncthreads();
  for (int64_t i = r0 + tid; i < r1; i += kSegBlkThreads) {
    if (a.keep[i] < 0) continue;
    int32_t g[kMaxFE];
    for (int f = 0; f < a.F; ++f) g[f] = a.code[f][i];
    const double wi = a.w ? a.w[i] : 0.0;
    for (int f = 0; f < a.F; ++f) {
      const int64_t pos = kw[f] >= 0 ? atomicAdd(&bins[boff[f] + g[f] - klo[f]], 1) : atomicAdd(&a.cur[f][g[f]], 1);
      int j = 0;
      for (int f2 = 0; f2 < a.F; ++f2)
        if (f2 != f) a.oc[f][(int64_t)(j++) * a.ld + pos] = g[f2];
      if (a.ws[f]) a.ws[f][pos] = wi;
    }
  }
}

// Sorted build (unweighted, two or three FEs), one FE f at a time: k_seg_keys writes every row's
// key (g_f in the low word - bit 31 marks a dropped row - and the first other FE's code in the high
// word) and the second other FE's code as the row slot; stable radix passes order them by the bits
// of g_f above the lowest `shift` (coarse buckets of at most 2^9 codes; none for the primary FE, whose
// layout order already is by buckets of 2^s codes); k_seg_rank then sorts each block of 8192 rows by
// code in LDS, reserves each code's slots with one returning global add and stores the block's rows
// code run by code run.  (k_seg_scatter2 instead takes a returning global add per row for an FE too
// wide for its LDS bins - config 4's 1e5-level FE - and stores runs of a few rows per code.
// Measured on config 4: the layouts' build 6.46 ms, of which the 1e5-level FE 3.0 ms, the 1e4-level
// FE 2.0 ms, the primary 1.7 ms; round 5.)
// key = g_f | a << bf | b << (bf + ba) (a, b: the other FEs' codes, bit 63: a dropped row), row
// slot = the layout row (the segment order's row permutation, for the cluster sums)
struct SegKeyArgs {
  const int32_t* keep;
  const int32_t* code;
  const int32_t* oa;
  const int32_t* ob;  // null: two FEs
  int64_t n;
  int bf, ba;
  uint64_t* keys;
  int32_t* rows;
};
__global__ void k_seg_keys(SegKeyArgs a) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t k = (uint64_t)(uint32_t)a.code[i] & ((1ull << a.bf) - 1);
    k |= (uint64_t)(uint32_t)a.oa[i] << a.bf;
    if (a.ob) k |= (uint64_t)(uint32_t)a.ob[i] << (a.bf + a.ba);
    if (a.keep[i] < 0) k |= 1ull << 63;
    a.keys[i] = k;
    a.rows[i] = (int32_t)i;
  }
}

constexpr int kRankThreads = 1024;
constexpr int kRankPer = 8;
constexpr int kRankRows = kRankThreads * kRankPer;  // rows per block
constexpr int kRankBins = 4096;                     // code range of a block ranked in LDS

struct SegRankArgs {
  const uint64_t* keys;  // ordered by the coarse bucket of g_f
  const int32_t* rows;
  int64_t n, ld;
  int bf, ba, bb;
  int32_t* cur;   // FE f's cursors (from seg_off)
  int32_t* oc;    // FE f's other codes [no][ld]
  int32_t* perm;  // FE f's layout row of every position
  int no;
};

__global__ __launch_bounds__(kRankThreads) void k_seg_rank(SegRankArgs a) {
  __shared__ int32_t st[kRankBins];  // counts, then the codes' starts in the block's sorted rows
  __shared__ int32_t gb[kRankBins];  // the codes' first global slots
  __shared__ int3 stage[kRankRows];  // the block's (other codes, layout row), sorted by g_f
  __shared__ int32_t wsum[kRankThreads / 64];
  __shared__ int32_t smin, smax;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * kRankRows;
  const uint64_t mf = (1ull << a.bf) - 1, ma = (1ull << a.ba) - 1, mb = (1ull << a.bb) - 1;
  if (tid == 0) {
    smin = 0x7fffffff;
    smax = -1;
  }
  uint64_t key[kRankPer];
  int32_t row[kRankPer];
  int32_t mn = 0x7fffffff, mx = -1;
#pragma unroll
  for (int s = 0; s < kRankPer; ++s) {
    const int64_t i = r0 + s * kRankThreads + tid;
    key[s] = i < a.n ? a.keys[i] : 1ull << 63;
    row[s] = i < a.n ? a.rows[i] : 0;
    if (!(key[s] >> 63)) {
      const int32_t g = (int32_t)(key[s] & mf);
      mn = min(mn, g);
      mx = max(mx, g);
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    mn = min(mn, __shfl_xor(mn, off, 64));
    mx = max(mx, __shfl_xor(mx, off, 64));
  }
  __syncthreads();
  if (lane == 0) {
    atomicMin(&smin, mn);
    atomicMax(&smax, mx);
  }
  __syncthreads();
  const int32_t lo = smin, w = smax >= smin ? smax - smin + 1 : 0;
  auto put = [&](int64_t pos, uint64_t k, int32_t r) {
    a.oc[pos] = (int32_t)((k >> a.bf) & ma);
    if (a.no > 1) a.oc[a.ld + pos] = (int32_t)((k >> (a.bf + a.ba)) & mb);
    a.perm[pos] = r;
  };
  if (w > kRankBins) {  // block-uniform: codes too spread for the LDS bins - one global add per row
#pragma unroll
    for (int s = 0; s < kRankPer; ++s)
      if (!(key[s] >> 63)) put(atomicAdd(&a.cur[(int32_t)(key[s] & mf)], 1), key[s], row[s]);
    return;
  }
  for (int j = tid; j < w; j += kRankThreads) st[j] = 0;
  __syncthreads();
  int rk[kRankPer];
#pragma unroll
  for (int s = 0; s < kRankPer; ++s) rk[s] = (key[s] >> 63) ? -1 : atomicAdd(&st[(int32_t)(key[s] & mf) - lo], 1);
  __syncthreads();
  // each code's slots (one returning global add), then the exclusive scan of the counts: thread t
  // takes codes 4t .. 4t + 3
  int v[4], sum = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int j = 4 * tid + q;
    v[q] = j < w ? st[j] : 0;
    if (v[q] > 0) gb[j] = atomicAdd(&a.cur[lo + j], v[q]);
    sum += v[q];
  }
  int x = sum;
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  int before = 0;
  for (int w2 = 0; w2 < wave; ++w2) before += wsum[w2];
  int run = before + x - sum;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int j = 4 * tid + q;
    if (j < w) st[j] = run;
    run += v[q];
  }
  int kept = 0;
  for (int w2 = 0; w2 < kRankThreads / 64; ++w2) kept += wsum[w2];
  __syncthreads();
#pragma unroll
  for (int s = 0; s < kRankPer; ++s)
    if (rk[s] >= 0) {
      const uint64_t k = key[s];
      stage[st[(int32_t)(k & mf) - lo] + rk[s]] =
          int3{(int32_t)((k >> a.bf) & ma), (int32_t)((k >> (a.bf + a.ba)) & mb), row[s]};
    }
  __syncthreads();
  // consecutive threads store consecutive rows of a code's run
  for (int q = tid; q < kept; q += kRankThreads) {
    int j = 0;  // the last code whose start is <= q (empty codes share the next one's start)
    for (int step = kRankBins / 2; step > 0; step >>= 1)
      if (j + step < w && st[j + step] <= q) j += step;
    const int64_t pos = (int64_t)gb[j] + (q - st[j]);
    const int3 e = stage[q];
    a.oc[pos] = e.x;
    if (a.no > 1) a.oc[a.ld + pos] = e.y;
    a.perm[pos] = e.z;
  }
}

// ufirst[u] = the segment holding row u * kSegUnit
__global__ void k_seg_units(const int32_t* __restrict__ seg_off, int32_t G, int32_t* __restrict__ ufirst) {
  for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x) {
    const int32_t a = seg_off[g], b = seg_off[g + 1];
    for (int32_t u = (a + kSegUnit - 1) / kSegUnit; (int64_t)u * kSegUnit < b; ++u) ufirst[u] = g;
  }
}

// ---------------------------------------------------------------------------
// cross term
// ---------------------------------------------------------------------------

struct SegCrossArgs {
  const int32_t* seg_off;            // [G + 1]
  const int32_t* ufirst;             // [n_units]
  int n_units;
  const int32_t* oc[kMaxFE - 1];     // other FEs' codes, segment order
  const double* alpha[kMaxFE - 1];   // their tables [G'][p]
  const double* ws;                  // weights in segment order (WT)
  int p;                             // alpha row stride
  int pc;                            // columns computed: p, or 1 (y only)
  int G;
  double* T;                         // [G][pc], zeroed before the launch
  const double* xq;                  // two-limb sums (lfe_internal.h): quanta; null: f64 (chain) sums
  double* Thi;                       // two-limb sums: coarse limbs [G][pc] (clean on entry)
  double* chain;                     // f64 sums: [2][n_units][pc] cut segments' parts (k_seg_chain)
};

// two-limb cross terms: a row's value v (the sum of the other FEs' effects) enters T as its fine
// limb in int64 and its coarse limb (outliers only) as an integer-valued f64, so T does not depend
// on the order of the segment layout's rows nor on which partial sum lands first
__device__ __forceinline__ long long seg_quad_sum_i64(long long v) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

__device__ __forceinline__ double seg_quad_sum(double v) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

// groups gathered per step (register budget: codes UNR*NO int4, values UNR*4*NT f64)
template <int NT, int NO>
constexpr int seg_unroll() {
  return NT >= 3 ? 1 : (NT == 2 ? (NO <= 2 ? 2 : 1) : (NO <= 2 ? 4 : (NO <= 4 ? 2 : 1)));
}

template <int NT, int NO, bool WT>
__global__ __launch_bounds__(kSegThreads) void k_seg_cross(SegCrossArgs a) {
  constexpr int UNR = seg_unroll<NT, NO>();
  const int lane = threadIdx.x & 63;
  const int kq = lane >> 4, c = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * (kSegThreads / 64) + (threadIdx.x >> 6)));
  const int nwaves = gridDim.x * (kSegThreads / 64);
  const int p = a.p, pc = a.pc, G = a.G;
  int cl[NT];
#pragma unroll
  for (int I = 0; I < NT; ++I) cl[I] = 16 * I + c < pc ? 16 * I + c : 0;
  const int32_t kept = a.seg_off[G];
  const bool ex = a.xq != nullptr;  // wave-uniform
  FixCol fcs[NT];
#pragma unroll
  for (int I = 0; I < NT; ++I) fcs[I] = ex ? fix_col(a.xq, cl[I]) : FixCol{};
  for (int u = wv; u < a.n_units; u += nwaves) {
    const int lo = u * kSegUnit;
    if (lo >= kept) break;
    const int hi = min(lo + kSegUnit, kept);
    int h = a.ufirst[u];
    int r0 = a.seg_off[h], r1 = a.seg_off[h + 1];
    bool part = r0 < lo;  // segment h began in an earlier unit
    bool done = false;
    double acc[NT];  // f64 sums, or the coarse limbs of the two-limb sums
    long long iacc[NT];
#pragma unroll
    for (int I = 0; I < NT; ++I) {
      acc[I] = 0.0;
      iacc[I] = 0;
    }
    // the fine limb of v (column slot I); its coarse limb joins acc[I] (integer-valued: exact)
    auto fx = [&](double v, int I) -> long long {
      double hh;
      const long long lo = (long long)fix_split(v, fcs[I], hh);
      acc[I] += hh;
      return lo;
    };
    // mode 0: segment h lies in this unit (store); 1: its part in this unit, begun in an earlier
    // unit; 2: its first part, continued in the next unit
    auto finalize = [&](int mode) {
#pragma unroll
      for (int I = 0; I < NT; ++I) {
        const int col = 16 * I + c;
        double* d = a.T + (int64_t)h * pc + col;
        if (ex) {  // integer adds commute: a cut segment's partials may land in any order
          const long long t = seg_quad_sum_i64(iacc[I]);
          const double th = seg_quad_sum(acc[I]);  // integer-valued coarse limbs: exact in any order
          if (kq == 0 && col < pc) {
            double* dh = a.Thi + (int64_t)h * pc + col;
            if (mode) {
              atomicAdd(reinterpret_cast<unsigned long long*>(d), (unsigned long long)t);
              if (th != 0.0) atomicAdd(dh, th);
            } else {
              *reinterpret_cast<long long*>(d) = t;
              if (th != 0.0) *dh = th;
            }
          }
        } else {
          const double t = seg_quad_sum(acc[I]);
          if (kq == 0 && col < pc) {
            if (mode == 0) *d = t;
            else if (a.chain) a.chain[((int64_t)(mode - 1) * a.n_units + u) * pc + col] = t;  // k_seg_chain adds
            else atomicAdd(d, t);
          }
        }
        acc[I] = 0.0;
        iacc[I] = 0;
      }
    };
    // pipeline: a batch's codes are loaded two batches ahead and its gathers one batch ahead (ping-pong
    // register sets, no copies): the batch being summed waits on nothing
    constexpr int UG = UNR > 1 ? UNR / 2 : 1;  // groups per batch
    auto load_codes = [&](int gs0, int4 (&cv)[UG][NO]) {
#pragma unroll
      for (int U = 0; U < UG; ++U) {
        const int rb = min(gs0 + 16 * U, hi - 1) & ~15;  // a group past the unit reloads a valid one
#pragma unroll
        for (int j = 0; j < NO; ++j) cv[U][j] = *reinterpret_cast<const int4*>(a.oc[j] + rb + 4 * kq);
      }
    };
    auto gather = [&](int gs0, const int4 (&cv)[UG][NO], double (&gv)[UG][NO][4][NT]) {
#pragma unroll
      for (int U = 0; U < UG; ++U) {
        const int rb = gs0 + 16 * U + 4 * kq;
        const bool gin = gs0 + 16 * U < hi;
#pragma unroll
        for (int j = 0; j < NO; ++j) {
          const int4 v = cv[U][j];
          const int cd[4] = {gin && rb + 0 < hi ? v.x : 0, gin && rb + 1 < hi ? v.y : 0,
                             gin && rb + 2 < hi ? v.z : 0, gin && rb + 3 < hi ? v.w : 0};
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const double* al = a.alpha[j] + (uint64_t)(uint32_t)cd[s] * (uint32_t)p;
#pragma unroll
            for (int I = 0; I < NT; ++I) gv[U][j][s][I] = al[cl[I]];
          }
        }
      }
    };
    auto batch = [&](int gs0, const double (&gv)[UG][NO][4][NT]) {
#pragma unroll
      for (int U = 0; U < UG; ++U) {
        const int gs = gs0 + 16 * U, ge = gs + 16;
        if (gs >= hi || done) break;
        const int rb = gs + 4 * kq;
        double val[4][NT];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          double ws = rb + s < hi ? 1.0 : 0.0;
          if (WT) ws = rb + s < hi ? a.ws[rb + s] : 0.0;
#pragma unroll
          for (int I = 0; I < NT; ++I) {
            double t = gv[U][0][s][I];
#pragma unroll
            for (int j = 1; j < NO; ++j) t += gv[U][j][s][I];
            val[s][I] = t * ws;
          }
        }
        while (true) {
          if (r0 <= gs && r1 >= ge) {  // the whole group lies in segment h
            if (ex) {
#pragma unroll
              for (int I = 0; I < NT; ++I)
                iacc[I] += (fx(val[0][I], I) + fx(val[1][I], I)) + (fx(val[2][I], I) + fx(val[3][I], I));
            } else {
#pragma unroll
              for (int I = 0; I < NT; ++I) acc[I] += (val[0][I] + val[1][I]) + (val[2][I] + val[3][I]);
            }
          } else {
#pragma unroll
            for (int s = 0; s < 4; ++s) {
              const int row = rb + s;
              const bool in = row >= r0 && row < r1;
#pragma unroll
              for (int I = 0; I < NT; ++I) {
                if (ex) iacc[I] += in ? fx(val[s][I], I) : 0ll;
                else acc[I] += in ? val[s][I] : 0.0;
              }
            }
          }
          if (r1 > ge) break;  // segment h continues in the next group
          finalize(part ? 1 : 0);  // r1 <= ge <= hi: segment h ends in this unit
          part = false;
          do {  // next non-empty segment
            ++h;
            r0 = r1;
            if (h >= G) break;
            r1 = a.seg_off[h + 1];
          } while (r1 == r0);
          if (h >= G || r0 >= hi) {
            done = true;
            break;
          }
          if (r0 >= ge) break;
        }
      }
    };
    constexpr int B = 16 * UG;  // rows per batch
    int4 cva[UG][NO], cvb[UG][NO];
    double gva[UG][NO][4][NT], gvb[UG][NO][4][NT];
    load_codes(lo, cva);
    load_codes(lo + B, cvb);
    gather(lo, cva, gva);
    for (int gs0 = lo; gs0 < hi && !done;) {
      load_codes(gs0 + 2 * B, cva);  // batch + 2
      gather(gs0 + B, cvb, gvb);     // batch + 1
      batch(gs0, gva);
      gs0 += B;
      if (gs0 >= hi || done) break;
      load_codes(gs0 + 2 * B, cvb);
      gather(gs0 + B, cva, gva);
      batch(gs0, gvb);
      gs0 += B;
    }
    // segment h continues past the unit: partial sum
    if (!done && h < G && r0 < hi && r1 > hi) finalize(part ? 1 : 2);
  }
}

// f64 segmented sums in a fixed order: a segment cut by unit edges is its first part
// (chain[1][u0], the unit it begins in) plus its part in every following unit (chain[0][u]),
// added in unit order (f64 atomics would add three or more parts in any order).  One thread per
// (unit, column) whose last segment continues into the next unit.
__global__ void k_seg_chain(const int32_t* __restrict__ seg_off, const int32_t* __restrict__ ufirst, int32_t G,
                            int n_units, int pc, const double* __restrict__ chain, double* __restrict__ T) {
  const int32_t kept = seg_off[G];
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < (int64_t)n_units * pc;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int u = (int)(e / pc), col = (int)(e % pc);
    const int64_t nxt = (int64_t)(u + 1) * kSegUnit;  // first row of unit u + 1
    if (u + 1 >= n_units || nxt >= kept) continue;
    const int h = ufirst[u + 1];  // the segment holding row nxt
    const int32_t s0 = seg_off[h];
    if (s0 >= nxt || s0 < (int64_t)u * kSegUnit) continue;  // not cut at nxt, or begun before unit u
    const int ue = (int)((seg_off[h + 1] - 1) / kSegUnit);
    double t = chain[((int64_t)n_units + u) * pc + col];
    for (int v = u + 1; v <= ue; ++v) t += chain[(int64_t)v * pc + col];
    T[(int64_t)h * pc + col] = t;
  }
}

int launch_seg_chain(lfe_ctx* c, const int32_t* seg_off, const int32_t* ufirst, int32_t G, int n_units, int pc,
                     double* T) {
  hipLaunchKernelGGL(k_seg_chain, dim3(grid_for((int64_t)n_units * pc)), dim3(kBlock), 0, c->stream, seg_off, ufirst,
                     G, n_units, pc, c->chain, T);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

// Statistics of an effect table for the cross terms' quanta: column max |alpha| (u64 bits, atomicMax)
// and, per block, sum_g cnt[g] alpha[g][c]^2 (col 63: sum_g cnt[g]) into slots [kAstatBlocks][64], so
// that rms over rows of alpha_f[g_f(i)] is formed in a fixed order (k_cross_quanta).  Block b takes
// the groups [b G / nb, (b + 1) G / nb); a wave reads 64 / L groups per step (L lanes per group, lane
// c of a group column c), four steps in flight, and the lanes of one column are combined over fixed
// shuffles, then the waves in order.
template <int L>
__global__ __launch_bounds__(256) void k_alpha_stats(const double* __restrict__ alpha, const int32_t* __restrict__ cnt,
                                                     int32_t G, int p, unsigned long long* __restrict__ amax,
                                                     double* __restrict__ slots) {
  constexpr int GPW = 64 / L;  // groups per wave step
  __shared__ double ss[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane / L, c = lane % L;
  const int64_t g0 = (int64_t)G * blockIdx.x / gridDim.x, g1 = (int64_t)G * (blockIdx.x + 1) / gridDim.x;
  double m = 0.0, sq = 0.0, nn = 0.0;
  const int64_t stride = 4 * GPW;
  int64_t g = g0 + wave * GPW + sub;
  for (; g + 3 * stride < g1; g += 4 * stride) {
    double v[4], ng[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t gu = g + u * stride;
      ng[u] = (double)cnt[gu];
      v[u] = c < p ? alpha[gu * p + c] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      nn += ng[u];
      m = fmax(m, fabs(v[u]));  // (fmax drops a NaN; the squares keep it)
      sq = __builtin_fma(ng[u] * v[u], v[u], sq);
    }
  }
  for (; g < g1; g += stride) {
    const double ng = (double)cnt[g];
    const double v = c < p ? alpha[g * p + c] : 0.0;
    nn += ng;
    m = fmax(m, fabs(v));
    sq = __builtin_fma(ng * v, v, sq);
  }
  // combine the GPW groups of the wave: lanes c, c + L, c + 2L, ... (fixed order)
#pragma unroll
  for (int off = L; off < 64; off <<= 1) {
    sq += __shfl_xor(sq, off, 64);
    nn += __shfl_xor(nn, off, 64);
    m = fmax(m, __shfl_xor(m, off, 64));
  }
  if (lane < L) ss[wave][lane] = sq;
  if (lane == 0) ss[wave][63] = nn;
  if (lane < L && c < p && m > 0.0) atomicMax(&amax[c], (unsigned long long)__double_as_longlong(m));
  __syncthreads();
  if (wave == 0) {
    const bool live = lane < L || lane == 63;
    const double t = live ? ((ss[0][lane] + ss[1][lane]) + ss[2][lane]) + ss[3][lane] : 0.0;
    slots[(int64_t)blockIdx.x * 64 + lane] = t;
  }
}

static int alpha_stat_blocks(int32_t G) { return (int)std::max<int64_t>(1, std::min<int64_t>(kAstatBlocks, (G + 63) / 64)); }

// Quanta of FE f's cross term (fix_quanta_col): a row's value is bounded by M = sum over the other
// FEs of their column max |alpha|, its typical size by the sum of their rms over rows; a sum adds
// at most N = the largest kept group of f.  Weighted (wfq != null): a row adds w v, so M and the
// rms are scaled by the weight column's max and rms (the weighted quanta of sums4, column wcol).
struct CrossQArgs {
  const unsigned long long* amax;  // [kMaxFE][kMaxCols]
  const double* astat;             // [kMaxFE][kAstatBlocks][64]
  int nblk[kMaxFE];
  int F, f, pc;
  const int32_t* cmax;
  const double* wfq;
  int wcol;
  double* xq;
};
// one block of 1024 threads: wave w sums the slots of blocks b = w, w + 16, ... (lane = column, lane
// 63 the counts), then lane col adds the 16 wave partials in order (a fixed order; the slots of
// up to kAstatBlocks blocks were one thread's serial loop, ~0.15 ms per launch)
__global__ __launch_bounds__(1024) void k_cross_quanta(CrossQArgs a) {
  __shared__ double part[16][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double rms = 0.0;
  for (int j = 0; j < a.F; ++j) {
    if (j == a.f) continue;
    const double* sl = a.astat + (int64_t)j * kAstatBlocks * 64;
    double t = 0.0;
    for (int b = wave; b < a.nblk[j]; b += 16) t += sl[b * 64 + lane];
    part[wave][lane] = t;
    __syncthreads();
    if (wave == 0) {
      double sq = 0.0, nn = 0.0;
      for (int w = 0; w < 16; ++w) {
        sq += part[w][lane];
        nn += part[w][63];
      }
      rms += nn > 0.0 ? sqrt(sq / nn) : 0.0;
    }
    __syncthreads();
  }
  const int col = lane;
  if (wave != 0 || col >= a.pc) return;
  double M = 0.0;
  for (int j = 0; j < a.F; ++j)
    if (j != a.f) M += __longlong_as_double((long long)a.amax[j * kMaxCols + col]);
  if (a.wfq) {
    M *= a.wfq[FQ_MAX * kFqCols + a.wcol];
    rms *= a.wfq[FQ_RMS * kFqCols + a.wcol];
  }
  fix_quanta_col(M, rms, (double)max(1, a.cmax[a.f]), a.xq, col);
}

// two-limb cross term (fine limbs int64 bits in T, coarse limbs in Thi, cleared) -> double
__global__ void k_cross_convert(double* __restrict__ T, double* __restrict__ Thi, int64_t m, int pc,
                                const double* __restrict__ xq) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % pc);
    double h = 0.0;
    if (xq[FQ_BIG * kFqCols + c] != 0.0) {
      h = Thi[e];
      if (h != 0.0) Thi[e] = 0.0;
    }
    T[e] = fix_value((unsigned long long)__double_as_longlong(T[e]), h, xq, c);
  }
}

// alpha_f = (S_f - T_f) / W_f   (weighted: W = sum w; else W = kept count), also into the
// line-aligned gather copy alpha_g (row pitch ap) and the dense y column alpha_y
__global__ void k_finalize(const double* __restrict__ S, const double* __restrict__ T, const double* __restrict__ Wsum,
                           const int32_t* __restrict__ cnt, int32_t G, int p, double* __restrict__ alpha,
                           double* __restrict__ alpha_g, int ap, double* __restrict__ alpha_y) {
  // one thread per (group, slot of the padded row): every line of alpha_g is written whole (the
  // pad slots as 0), so no partially written line has to be merged
  const int q = alpha_g ? ap : p;
  const int64_t total = (int64_t)G * q;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t g = t / q;
    const int cc = (int)(t - g * q);
    double v = 0.0;
    if (cc < p) {
      const int64_t e = g * p + cc;
      const double den = Wsum ? Wsum[g] : (double)cnt[g];
      v = den > 0.0 ? (S[e] - (T ? T[e] : 0.0)) / den : 0.0;
      alpha[e] = v;
      if (alpha_y && cc == 0) alpha_y[g] = v;
    }
    if (alpha_g) alpha_g[t] = v;
  }
}

// stop test (polars_impl.py:512-521): for every group present,
//   mean_g(y~) = (Sy[g] - cnt[g] alpha[g][0] - R[g]) / cnt[g]
// max |.| -> out (non-negative doubles order like their bit patterns)
// YOCO records (Wsum != null): the weighted mean, (S_y - W alpha - R) / W
__global__ void k_check_max(const double* __restrict__ Sy, int sy_stride, const double* __restrict__ R, int r_stride,
                            const double* __restrict__ alpha, int p, const int32_t* __restrict__ cnt,
                            const double* __restrict__ Wsum, int32_t G, unsigned long long* __restrict__ out) {
  double m = 0.0;
  for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x) {
    const int32_t n = cnt[g];
    if (n > 0) {
      const double den = Wsum ? Wsum[g] : (double)n;
      const double r =
          Sy[(int64_t)g * sy_stride] - den * alpha[(int64_t)g * p] - (R ? R[(int64_t)g * r_stride] : 0.0);
      if (den > 0.0) m = fmax(m, fabs(r / den));
    }
  }
  for (int off = 32; off > 0; off >>= 1) m = fmax(m, __shfl_down(m, off, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(out, (unsigned long long)__double_as_longlong(m));
}

// ---------------------------------------------------------------------------
// the stop test's y-only cross term, one row per lane
// ---------------------------------------------------------------------------
// R_f[g] = sum_{i in g} sum_{f' != f} alpha_f'[g_f'(i)][y] (unweighted, polars_impl.py:512-521).
// k_seg_cross would run it with 16 lanes per row doing the same work for one column; here a lane
// takes one position of the segment layout, gathers the other FEs' y effects from the dense y
// copies (alpha_y), splits the value into two-limb fixed point, and the lanes of one segment run
// are summed over a shuffle scan; the run's last lane adds it to R (int64 fine limbs, integer-valued
// f64 coarse limbs: the adds commute, so R does not depend on their order).  A wave takes 4 x 64
// consecutive positions per step.
struct SegCheckArgs {
  const int32_t* seg_off;  // [G + 1]
  const int32_t* ufirst;   // [n_units] the segment holding each unit's first position
  int n_units;
  int32_t G;
  const int32_t* oc[kMaxFE - 1];
  const double* ay[kMaxFE - 1];
  int no;
  const double* xq;        // quanta (column 0)
  unsigned long long* R;   // [G] fine limbs (zeroed)
  double* Rhi;             // [G] coarse limbs (clean)
};

__global__ __launch_bounds__(256) void k_seg_check(SegCheckArgs a) {
  const int lane = threadIdx.x & 63;
  const int32_t kept = a.seg_off[a.G];
  const FixCol fc = fix_col(a.xq, 0);
  const int nwaves = gridDim.x * 4;
  // a wave walks whole units of kSegUnit positions from the unit's first segment (ufirst), carrying
  // the segment from step to step (a binary search over seg_off per 256 positions cost ~20 dependent
  // loads each at 1e6 segments)
  for (int uu = blockIdx.x * 4 + (threadIdx.x >> 6); uu < a.n_units; uu += nwaves) {
    const int64_t u0 = (int64_t)uu * kSegUnit;
    if (u0 >= kept) break;
    const int64_t u1 = min((int64_t)kept, u0 + kSegUnit);
    int h = __builtin_amdgcn_readfirstlane(a.ufirst[uu]);
    for (int64_t base = u0; base < u1; base += 256) {
      double y[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {  // every gather of the step in flight together
        const int64_t q = base + u * 64 + lane;
        double v = 0.0;
        if (q < kept)
          for (int j = 0; j < a.no; ++j) v += a.ay[j][a.oc[j][q]];
        y[u] = v;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t q = base + u * 64 + lane;
        const bool in = q < kept;
        int hl = h;  // this lane's segment: h, or a few after it
        if (in)
          while (a.seg_off[hl + 1] <= q) ++hl;
        double hh = 0.0;
        long long lo_i = in ? (long long)fix_split(y[u], fc, hh) : 0ll;
        if (!in) hl = 0x7fffffff;
        // segmented inclusive scan over the lanes (segment ids do not decrease)
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const int oh = __shfl_up(hl, off, 64);
          const long long ol = __shfl_up(lo_i, off, 64);
          const double oH = __shfl_up(hh, off, 64);
          if (lane >= off && oh == hl) {
            lo_i += ol;
            hh += oH;
          }
        }
        const int nh = __shfl_down(hl, 1, 64);
        if (in && (lane == 63 || nh != hl)) {  // the last lane of its run
          atomicAdd(&a.R[hl], (unsigned long long)lo_i);
          if (hh != 0.0) atomicAdd(&a.Rhi[hl], hh);
        }
        h = __shfl(hl, 63, 64);  // the next 64 positions start in the last lane's segment (or later)
        if (h == 0x7fffffff) h = a.G - 1;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------

using CrossFn = void (*)(SegCrossArgs);

template <int NT, int NO>
static CrossFn cross_fn_nt(bool wt) {
  return wt ? &k_seg_cross<NT, NO, true> : &k_seg_cross<NT, NO, false>;
}
template <int NO>
static CrossFn cross_fn_no(int nt, bool wt) {
  switch (nt) {
    case 1: return cross_fn_nt<1, NO>(wt);
    case 2: return cross_fn_nt<2, NO>(wt);
    case 3: return cross_fn_nt<3, NO>(wt);
    default: return cross_fn_nt<4, NO>(wt);
  }
}
static CrossFn cross_fn(int nt, int no, bool wt) {
  switch (no) {
    case 1: return cross_fn_no<1>(nt, wt);
    case 2: return cross_fn_no<2>(nt, wt);
    case 3: return cross_fn_no<3>(nt, wt);
    case 4: return cross_fn_no<4>(nt, wt);
    case 5: return cross_fn_no<5>(nt, wt);
    case 6: return cross_fn_no<6>(nt, wt);
    default: return cross_fn_no<7>(nt, wt);
  }
}

static int n_units_of(const lfe_ctx* c) { return (int)((c->n + kSegUnit - 1) / kSegUnit); }

int seg_build(lfe_ctx* c) {
  if (c->seg_ready || c->F < 2) return LFE_OK;
  const auto& L = c->L;
  const int64_t n = c->n;
  const bool weighted = L.w != nullptr;
  const int nu = std::max(n_units_of(c), 1);
  SegScatterArgs a{};
  a.F = c->F;
  a.n = n;
  a.ld = c->ld;
  a.keep = L.code[L.P];
  a.w = L.w;
  for (int f = 0; f < c->F; ++f) {
    auto& fe = c->fe[f];
    LFE_TRY(ensure_i32(c, fe.seg_off, fe.seg_off_cap, (size_t)fe.G + 1));
    LFE_TRY(ensure_i32(c, fe.seg_cur, fe.seg_cur_cap, (size_t)fe.G));
    LFE_TRY(ensure_i32(c, fe.oc, fe.oc_cap, (size_t)(c->F - 1) * c->ld));
    LFE_TRY(ensure_i32(c, fe.ufirst, fe.ufirst_cap, (size_t)nu));
    if (weighted) LFE_TRY(ensure_f64(c, fe.ws, fe.ws_cap, (size_t)c->ld));
    LFE_HIP(hipMemsetAsync(fe.seg_off + fe.G, 0, sizeof(int32_t), c->stream));
    if (c->world == 1) {
      LFE_HIP(hipMemcpyAsync(fe.seg_off, fe.cnt, sizeof(int32_t) * fe.G, hipMemcpyDeviceToDevice, c->stream));
    } else {
      LFE_HIP(hipMemsetAsync(fe.seg_off, 0, sizeof(int32_t) * fe.G, c->stream));
      if (n > 0) {
        ProfScope _ps(c, K_SEG_BUILD);
        hipLaunchKernelGGL(k_seg_hist, dim3(grid_for(n, 256, 8192)), dim3(256), 0, c->stream, a.keep, L.code[f], n,
                           fe.seg_off);
      }
      LFE_HIP(hipGetLastError());
    }
    LFE_TRY(exclusive_scan(c, fe.seg_off, (int64_t)fe.G + 1));
    LFE_HIP(hipMemcpyAsync(fe.seg_cur, fe.seg_off, sizeof(int32_t) * fe.G, hipMemcpyDeviceToDevice, c->stream));
    a.code[f] = L.code[f];
    a.cur[f] = fe.seg_cur;
    a.oc[f] = fe.oc;
    a.ws[f] = weighted ? fe.ws : nullptr;
  }
  const int sorted_env = [] {  // "0": k_seg_scatter2 for every fit (A/B)
    const char* e = knob("LFE_SEG_SORTED");
    return e ? atoi(e) : 1;
  }();
  // the sorted build: unweighted, two or three FEs, its workspace (24 bytes a row) at most 6 GB
  const bool sorted0 = sorted_env != 0 && !(c->test_hooks & LFE_TEST_SEG_SCATTER) && !weighted && (c->F == 2 || c->F == 3) && n > 0 &&
                      c->ld <= (int64_t)1 << 28 && knob("LFE_SEG_SCATTER_ROWS") == nullptr;
  int bits[kMaxFE] = {}, bsum = 0;  // code bits of every FE (at least 1): the packed keys need <= 63
  for (int f = 0; f < c->F; ++f) {
    bits[f] = std::max(1, bit_length((uint64_t)std::max(c->fe[f].G - 1, 0)));
    bsum += bits[f];
  }
  const bool sorted = sorted0 && bsum <= 63;
  for (auto& fe : c->fe) fe.perm_ok = false;
  if (sorted) {
    LFE_TRY(ensure_sort_ws(c, (size_t)c->ld));
    for (auto& fe : c->fe) LFE_TRY(ensure_i32(c, fe.perm, fe.perm_cap, (size_t)c->ld));
    auto& W = c->clw;
    for (int f = 0; f < c->F; ++f) {
      const int32_t* other[2] = {nullptr, nullptr};
      int of[2] = {0, 0}, j = 0;
      for (int f2 = 0; f2 < c->F; ++f2)
        if (f2 != f) {
          of[j] = f2;
          other[j++] = L.code[f2];
        }
      SegKeyArgs ka{};
      ka.keep = a.keep;
      ka.code = L.code[f];
      ka.oa = other[0];
      ka.ob = other[1];
      ka.n = n;
      ka.bf = bits[f];
      ka.ba = bits[of[0]];
      ka.keys = W.keys[0];
      ka.rows = W.rows[0];
      {
        ProfScope _ps(c, K_SEG_BUILD);
        hipLaunchKernelGGL(k_seg_keys, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, ka);
      }
      LFE_HIP(hipGetLastError());
      // coarse buckets of at most 2^9 codes: the primary FE's layout buckets (2^s codes), else the
      // radix passes over the code's bits above the lowest `shift` (8 bits a pass)
      int cur = 0;
      if (!(f == L.P && L.permuted && L.s <= 9)) {
        const int passes = bits[f] > 9 ? (bits[f] - 9 + 7) / 8 : 0;
        for (int q = 0; q < passes; ++q) {
          LFE_TRY(radix_pass(c, n, bits[f] - 8 * (passes - q), cur, K_SEG_BUILD));
          cur = 1 - cur;
        }
      }
      SegRankArgs r{};
      r.keys = W.keys[cur];
      r.rows = W.rows[cur];
      r.n = n;
      r.ld = c->ld;
      r.bf = bits[f];
      r.ba = bits[of[0]];
      r.bb = c->F > 2 ? bits[of[1]] : 0;
      r.cur = c->fe[f].seg_cur;
      r.oc = c->fe[f].oc;
      r.perm = c->fe[f].perm;
      r.no = c->F - 1;
      {
        ProfScope _ps(c, K_SEG_BUILD);
        hipLaunchKernelGGL(k_seg_rank, dim3((unsigned)((n + kRankRows - 1) / kRankRows)), dim3(kRankThreads), 0,
                           c->stream, r);
      }
      LFE_HIP(hipGetLastError());
      c->fe[f].perm_ok = true;
    }
  }
  {
    ProfScope _ps(c, K_SEG_BUILD);
    if (sorted) {
      // (built above)
    } else if (n > 0 && knob("LFE_SEG_SCATTER_ROWS") == nullptr) {  // (env: the per-row kernel, A/B only)
      SegScatter2Args a2{};
      a2.s = a;
      for (int f = 0; f < c->F; ++f) a2.G[f] = c->fe[f].G;
      a2.P = L.permuted ? L.P : -1;
      hipLaunchKernelGGL(k_seg_scatter2, dim3((unsigned)((n + kSegBlkRows - 1) / kSegBlkRows)), dim3(kSegBlkThreads),
                         0, c->stream, a2);
    } else if (n > 0) {
      hipLaunchKernelGGL(k_seg_scatter, dim3(grid_for(n, 256, 8192)), dim3(256), 0, c->stream, a);
    }
    LFE_HIP(hipGetLastError());
    for (int f = 0; f < c->F; ++f) {
      auto& fe = c->fe[f];
      hipLaunchKernelGGL(k_seg_units, dim3(grid_for(fe.G)), dim3(kBlock), 0, c->stream, fe.seg_off, fe.G, fe.ufirst);
    }
    LFE_HIP(hipGetLastError());
  }
  c->seg_ready = true;
  return LFE_OK;
}

// T (all columns, weighted as the fit) or R (y only, unweighted) of FE f, summed over ranks
static int seg_cross(lfe_ctx* c, int f, bool y_only, int kid) {
  auto& fe = c->fe[f];
  const int pc = y_only ? 1 : c->p;
  double* out = y_only ? fe.R : fe.T;
  LFE_HIP(hipMemsetAsync(out, 0, sizeof(double) * (size_t)fe.G * pc, c->stream));
  SegCrossArgs a{};
  a.seg_off = fe.seg_off;
  a.ufirst = fe.ufirst;
  a.n_units = n_units_of(c);
  int j = 0;
  for (int f2 = 0; f2 < c->F; ++f2)
    if (f2 != f) {
      a.oc[j] = fe.oc + (size_t)j * c->ld;
      a.alpha[j] = y_only ? c->fe[f2].alpha_y : c->fe[f2].alpha_g;
      ++j;
    }
  const bool wt = (!y_only || c->records) && c->L.w != nullptr;  // the check is unweighted, except for records
  a.ws = wt ? fe.ws : nullptr;
  a.p = y_only ? 1 : alpha_pitch(c->p);  // the gather copies' row pitch
  a.pc = pc;
  a.G = fe.G;
  a.T = out;
  // two-limb fixed-point cross terms: bit-reproducible whatever the order of the segment layout's
  // rows (ranked by global cursor atomics) and of the cut segments' adds
  {
    LFE_TRY(ensure_f64(c, c->xq, c->xq_cap, (size_t)kFqRows * kFqCols));
    CrossQArgs q{};
    q.amax = reinterpret_cast<const unsigned long long*>(c->amax);
    q.astat = c->astat;
    for (int j = 0; j < c->F; ++j) q.nblk[j] = alpha_stat_blocks(c->fe[j].G);
    q.F = c->F;
    q.f = f;
    q.pc = pc;
    q.cmax = c->iscratch + kIscratchCmax;
    q.wfq = wt ? c->fixq : nullptr;  // sums4's weighted quanta: column p is w
    q.wcol = c->p;
    q.xq = c->xq;
    hipLaunchKernelGGL(k_cross_quanta, dim3(1), dim3(1024), 0, c->stream, q);
    LFE_HIP(hipGetLastError());
    a.xq = c->xq;
    a.Thi = fe.hi;
  }
  LFE_TRY(hi_begin(c));
  if (y_only && !wt) {  // the unweighted check term: one row per lane (k_seg_check)
    SegCheckArgs k{};
    k.seg_off = fe.seg_off;
    k.ufirst = a.ufirst;
    k.n_units = a.n_units;
    k.G = fe.G;
    for (int j2 = 0; j2 < c->F - 1; ++j2) {
      k.oc[j2] = a.oc[j2];
      k.ay[j2] = a.alpha[j2];
    }
    k.no = c->F - 1;
    k.xq = c->xq;
    k.R = reinterpret_cast<unsigned long long*>(out);
    k.Rhi = fe.hi;
    const int64_t n_kept = c->n;  // an upper bound on the kept positions (the kernel reads seg_off[G])
    if (n_kept > 0 && fe.G > 0 && a.n_units > 0) {
      ProfScope _ps(c, kid);
      hipLaunchKernelGGL(k_seg_check, dim3((unsigned)((a.n_units + 3) / 4)), dim3(256), 0, c->stream, k);
    }
    LFE_HIP(hipGetLastError());
  } else if (a.n_units > 0) {
    const int nt = (pc + 15) / 16;
    CrossFn fn = cross_fn(nt, c->F - 1, wt);
    const int waves_per_block = kSegThreads / 64;
    const int grid = (a.n_units + waves_per_block - 1) / waves_per_block;
    ProfScope _ps(c, kid);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(kSegThreads), 0, c->stream, a);
  }
  LFE_HIP(hipGetLastError());
  {
    const int64_t m = (int64_t)fe.G * pc;
    hipLaunchKernelGGL(k_cross_convert, dim3(grid_for(m)), dim3(kBlock), 0, c->stream, out, fe.hi, m, pc, c->xq);
    LFE_HIP(hipGetLastError());
  }
  hi_end(c);
  // owner-sharded rows: the primary FE's cross term is complete on its owner rank (its other
  // levels have no rows here and are never read); every other FE's is summed over the ranks
  if (c->owner_on && f == c->L.P) return LFE_OK;
  return allreduce_sum_f64(c, out, (size_t)fe.G * pc);
}

// out[h][0, cols) = sum over positions q in [seg_off[h], seg_off[h + 1]) of
// table[rows[q]][0, cols) (row stride `stride`); positions [0, seg_off[G]), at
// most n_pos.  `ufirst` holds ceil(n_pos / kSegUnit) ints.  The cluster score
// sums (lfe_cluster.hip) are this with rows = the cluster-sorted row indices.
int seg_gather_sum(lfe_ctx* c, const int32_t* seg_off, int32_t G, int32_t* ufirst, int64_t n_pos,
                   const int32_t* rows, const double* table, int stride, int cols, double* out, int kid) {
  LFE_HIP(hipMemsetAsync(out, 0, sizeof(double) * (size_t)G * cols, c->stream));
  const int n_units = (int)((n_pos + kSegUnit - 1) / kSegUnit);
  if (G == 0 || n_units == 0 || cols < 1) return LFE_OK;
  hipLaunchKernelGGL(k_seg_units, dim3(grid_for(G)), dim3(kBlock), 0, c->stream, seg_off, G, ufirst);
  SegCrossArgs a{};
  a.seg_off = seg_off;
  a.ufirst = ufirst;
  a.n_units = n_units;
  a.oc[0] = rows;
  a.alpha[0] = table;
  a.p = stride;
  a.pc = cols;
  a.G = G;
  a.T = out;
  LFE_TRY(ensure_f64(c, c->chain, c->chain_cap, (size_t)2 * n_units * cols));
  a.chain = c->chain;
  CrossFn fn = cross_fn((cols + 15) / 16, 1, false);
  const int grid = (n_units + kSegThreads / 64 - 1) / (kSegThreads / 64);
  {
    ProfScope _ps(c, kid);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(kSegThreads), 0, c->stream, a);
  }
  LFE_HIP(hipGetLastError());
  return launch_seg_chain(c, seg_off, ufirst, G, n_units, cols, out);
}

// Cluster score sums of a column that repeats FE f (lfe_cluster.hip): S[g][0, cols) = the sum over
// f's segment g of table[perm[q]][0, cols) (row stride cols), two-limb with quanta xq - fine limbs
// as int64 bits in S, coarse limbs in Shi, both zeroed by the caller - so exact whatever the order
// of a segment's rows (the sorted build ranks them by LDS atomics).  Needs the sorted build's perm.
// kid < 0: no timing scope of its own (the caller's is open)
int seg_score_sums(lfe_ctx* c, int f, const double* table, int cols, const double* xq, double* S, double* Shi,
                   int kid) {
  auto& fe = c->fe[f];
  if (!c->seg_ready || !fe.perm_ok || cols < 1 || cols > 64) {
    set_error("seg_score_sums: no segment permutation for this FE");
    return LFE_ESTATE;
  }
  SegCrossArgs a{};
  a.seg_off = fe.seg_off;
  a.ufirst = fe.ufirst;
  a.n_units = n_units_of(c);
  a.oc[0] = fe.perm;
  a.alpha[0] = table;
  a.p = cols;
  a.pc = cols;
  a.G = fe.G;
  a.T = S;
  a.xq = xq;
  a.Thi = Shi;
  if (a.n_units > 0 && fe.G > 0) {
    CrossFn fn = cross_fn((cols + 15) / 16, 1, false);
    const int waves_per_block = kSegThreads / 64;
    if (kid >= 0) {
      ProfScope _ps(c, kid);
      hipLaunchKernelGGL(fn, dim3((a.n_units + waves_per_block - 1) / waves_per_block), dim3(kSegThreads), 0, c->stream,
                         a);
    } else {  // (inside the caller's scope)
      hipLaunchKernelGGL(fn, dim3((a.n_units + waves_per_block - 1) / waves_per_block), dim3(kSegThreads), 0, c->stream,
                         a);
    }
  }
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

int seg_units_needed(int64_t n_pos) { return (int)std::max<int64_t>((n_pos + kSegUnit - 1) / kSegUnit, 1); }

static int seg_finalize(lfe_ctx* c, int f) {
  auto& fe = c->fe[f];
  const bool cross = c->F > 1;
  ProfScope _ps(c, K_FINALIZE);
  hipLaunchKernelGGL(k_finalize, dim3(grid_for((int64_t)fe.G * (cross ? alpha_pitch(c->p) : c->p))), dim3(kBlock), 0,
                     c->stream, fe.S,
                     cross ? fe.T : nullptr, c->L.w ? fe.W : nullptr, fe.cnt, fe.G, c->p, fe.alpha,
                     cross ? fe.alpha_g : nullptr, alpha_pitch(c->p), cross ? fe.alpha_y : nullptr);
  LFE_HIP(hipGetLastError());
  if (cross) {  // the statistics of the new effects (the other FEs' cross-term quanta)
    unsigned long long* am = reinterpret_cast<unsigned long long*>(c->amax) + (size_t)f * kMaxCols;
    LFE_HIP(hipMemsetAsync(am, 0, sizeof(double) * c->p, c->stream));
    double* slots = c->astat + (size_t)f * kAstatBlocks * 64;
    const dim3 grid(alpha_stat_blocks(fe.G));
    if (c->p <= 8) hipLaunchKernelGGL(k_alpha_stats<8>, grid, dim3(256), 0, c->stream, fe.alpha, fe.cnt, fe.G, c->p, am, slots);
    else if (c->p <= 16) hipLaunchKernelGGL(k_alpha_stats<16>, grid, dim3(256), 0, c->stream, fe.alpha, fe.cnt, fe.G, c->p, am, slots);
    else if (c->p <= 32) hipLaunchKernelGGL(k_alpha_stats<32>, grid, dim3(256), 0, c->stream, fe.alpha, fe.cnt, fe.G, c->p, am, slots);
    else hipLaunchKernelGGL(k_alpha_stats<64>, grid, dim3(256), 0, c->stream, fe.alpha, fe.cnt, fe.G, c->p, am, slots);
    LFE_HIP(hipGetLastError());
  }
  return LFE_OK;
}

// max_g |mean_g(y~)| of FE f given its check cross term R (stride r_stride, null: none)
// max_g |alpha[g][0]| (the y column of an effect table) into *out as u64 bits (atomicMax)
__global__ void k_y_absmax(const double* __restrict__ alpha, int32_t G, int p, unsigned long long* __restrict__ out) {
  double m = 0.0;
  for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x)
    m = fmax(m, fabs(alpha[(int64_t)g * p]));
  for (int off = 32; off > 0; off >>= 1) m = fmax(m, __shfl_down(m, off, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(out, (unsigned long long)__double_as_longlong(m));
}

static int seg_check_max(lfe_ctx* c, int f, const double* R, int r_stride) {
  auto& fe = c->fe[f];
  ProfScope _ps(c, K_CHECK_MAX);
  const bool unw = c->L.w && !c->records;  // weighted fit, unweighted check (polars_impl.py:513)
  const double* Sy = unw ? fe.Sy : fe.S;
  hipLaunchKernelGGL(k_check_max, dim3(grid_for(fe.G)), dim3(kBlock), 0, c->stream, Sy, unw ? 1 : c->p, R,
                     r_stride, fe.alpha, c->p, fe.cnt, (c->L.w && c->records) ? fe.W : nullptr, fe.G,
                     reinterpret_cast<unsigned long long*>(c->dred));
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

int demean_generic(lfe_ctx* c, const std::vector<int>& order, double tol, int max_iter, int check_from,
                   int* iterations_out, double* last_out) {
  // every effect table starts at zero (lfe_demean): so do the exact cross terms' column bounds
  LFE_TRY(ensure_f64(c, c->amax, c->amax_cap, (size_t)kMaxFE * kMaxCols));
  LFE_HIP(hipMemsetAsync(c->amax, 0, sizeof(double) * kMaxFE * kMaxCols, c->stream));
  LFE_TRY(ensure_f64(c, c->astat, c->astat_cap, (size_t)kMaxFE * kAstatBlocks * 64));
  if (c->F > 1)  // the line-aligned gather copies of the effects, zero like the tables
    for (auto& fe : c->fe) {
      const size_t m = (size_t)fe.G * alpha_pitch(c->p);
      LFE_TRY(ensure_f64(c, fe.alpha_g, fe.alpha_g_cap, m));
      LFE_HIP(hipMemsetAsync(fe.alpha_g, 0, sizeof(double) * m, c->stream));
      LFE_TRY(ensure_f64(c, fe.alpha_y, fe.alpha_y_cap, (size_t)fe.G));
      LFE_HIP(hipMemsetAsync(fe.alpha_y, 0, sizeof(double) * fe.G, c->stream));
    }
  LFE_HIP(hipMemsetAsync(c->astat, 0, sizeof(double) * kMaxFE * kAstatBlocks * 64, c->stream));
  const int F = c->F;
  const bool cross = F > 1;
  if (cross) LFE_TRY(seg_build(c));
  // T of the first FE doubles as its check term (unweighted fits, and YOCO records whose check is weighted)
  const bool reuse = cross && (c->L.w == nullptr || c->records);
  auto project = [&](int f) -> int {
    if (cross) LFE_TRY(seg_cross(c, f, false, K_CROSS));
    return seg_finalize(c, f);
  };
  int iterations = 0;
  double last = -1.0;
  if (check_from <= 0) {
    // single within-transform pass ('demean' strategy, polars_impl.py:437-465)
    for (int f : order) LFE_TRY(project(f));
    iterations = 1;
  } else {
    bool first_ready = false;  // T of order[0] already holds the next projection's cross term
    constexpr int kStall = 20;
    constexpr double kRecRel = 0x1p-46;  // 64 ulps of y's scale
    double best = 1e300, yscale = 0.0;
    int stall = 0;
    for (int it = 1; it <= max_iter; ++it) {
      for (size_t k = 0; k < order.size(); ++k) {
        if (k == 0 && first_ready) LFE_TRY(seg_finalize(c, order[0]));
        else LFE_TRY(project(order[k]));
      }
      first_ready = false;
      iterations = it;
      if (it < check_from) continue;
      LFE_TRY(ensure_dred(c, 2));
      LFE_HIP(hipMemsetAsync(c->dred, 0, sizeof(double) * 2, c->stream));
      const bool scale_now = c->records && it == check_from;
      if (scale_now) {  // y's scale: the largest group effect of the first FE after this sweep
        const int f0 = order[0];
        hipLaunchKernelGGL(k_y_absmax, dim3(grid_for(c->fe[f0].G)), dim3(kBlock), 0, c->stream, c->fe[f0].alpha,
                           c->fe[f0].G, c->p, reinterpret_cast<unsigned long long*>(c->dred + 1));
        LFE_HIP(hipGetLastError());
      }
      for (size_t k = 0; k < order.size(); ++k) {
        const int f = order[k];
        if (!cross) {
          LFE_TRY(seg_check_max(c, f, nullptr, 1));
        } else if (reuse && k == order.size() - 1) {
          LFE_TRY(seg_check_max(c, f, c->fe[f].T, c->p));
        } else if (reuse && k == 0) {
          LFE_TRY(seg_cross(c, f, false, K_CROSS));
          LFE_TRY(seg_check_max(c, f, c->fe[f].T, c->p));
          first_ready = true;
        } else {
          LFE_TRY(seg_cross(c, f, true, K_CHECK));
          LFE_TRY(seg_check_max(c, f, c->fe[f].R, 1));
        }
      }
      // owner-sharded rows: each rank's check covers its own primary levels; the max over ranks
      if (c->owner_on) LFE_TRY(allreduce_max_u64(c, reinterpret_cast<uint64_t*>(c->dred), 1));
      double chk[2] = {0.0, 0.0};
      LFE_TRY(d2h_sync(c, chk, c->dred, sizeof(double) * (scale_now ? 2 : 1)));
      last = chk[0];
      if (scale_now) yscale = chk[1];
      if (last < tol) break;
      if (c->records) {
        // records are solved to machine precision: stop once the largest group mean of y~ is
        // within kRecRel of y's scale (a scale-relative floor, so slowly converging records
        // stop as soon as they are there), or once the check has not reached a new minimum
        // for kStall checks (it only moves at rounding level from there)
        if (last <= kRecRel * yscale) break;
        if (last < best) {
          best = last;
          stall = 0;
        } else if (++stall >= kStall) {
          break;
        }
      }
    }
  }
  *iterations_out = iterations;
  *last_out = last;
  return LFE_OK;
}

}  // namespace lfe

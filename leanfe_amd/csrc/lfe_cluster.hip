// leanfe HIP engine — cluster scores and the CGM meats (std_errors.py:289-441,
// compress.py:817-851: the one-hot SpMM W_C'(X (.) e)).
//
// For a cluster subset s (bit j = loaded cluster column j) the clusters are the
// distinct tuples of the selected columns' codes among kept rows
// (std_errors.py:399-408 groups by the intersection).  On the device:
//   1. key_i = mixed-radix code of the tuple (span = prod of levels < 2^62);
//      dropped rows get key = span, which sorts last;
//   2. stable LSD radix sort of (key, row) pairs (lfe_keys.hip);
//   3. segments = runs of equal keys (flags + scan), G = their number;
//   4. S_c = segmented gather-sum of the row-major score rows x~_i r_i (w_i)
//      (seg_gather_sum, the general-sweep kernel of lfe_seg.hip);
//   5. meat = S'S (table Gram, lfe_gram.hip).
// No hash table and no f64 atomics, whatever the number of clusters (config 4:
// fe2 x fe3 has 48.8M clusters for 50M rows).
//
// Multi-rank: clusters span row shards; keys are global (codes are global).  Few
// clusters (key table <= 64 MB): the local clusters' sums (steps 2-4) are put into a
// key-indexed S table (one store per cluster, no atomics) and all-reduced.
// Otherwise owner-partitioned (owner_meat): local sums per cluster are sent to
// the rank owner(key) by an all-to-all, merged there, and only the k x k meats
// and the cluster counts are all-reduced.
#include "lfe_internal.h"

#include <cmath>
#include <cstring>

#include <algorithm>

namespace lfe {

static int fail(int code, const char* msg) {
  set_error(msg);
  return code;
}

// cluster code of every layout row (input-order array gathered through orig)
__global__ void k_cl_layout(const int32_t* __restrict__ cl, const int32_t* __restrict__ orig, int64_t n,
                            int32_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = cl[orig ? orig[i] : i];
}

struct KeyArgs {
  int m;
  const int32_t* code[kMaxCl];  // layout order
  uint64_t mult[kMaxCl];
  const int32_t* keep;          // layout codes of P (-1: dropped), or null
  int64_t n;
  uint64_t drop;                // key of dropped rows (= span)
  uint64_t* keys;
  int32_t* rows;
  // pj >= 0: column pj repeats the layout's primary FE (rows in order of its buckets of 2^ps codes):
  // its code g enters as (g mod 2^ps) mult[pj] + (g >> ps) << pshift, so the sort needs only the
  // bits below pshift (equal low parts keep the bucket order: equal keys stay contiguous)
  int pj, ps, pshift;
};

__global__ void k_cl_keys(KeyArgs a) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t key = 0;
    for (int j = 0; j < a.m; ++j) {
      const uint64_t g = (uint32_t)a.code[j][i];
      key += j == a.pj ? (g & ((1ull << a.ps) - 1)) * a.mult[j] + ((g >> a.ps) << a.pshift) : g * a.mult[j];
    }
    a.keys[i] = (a.keep && a.keep[i] < 0) ? a.drop : key;
    a.rows[i] = (int32_t)i;
  }
}

__device__ __forceinline__ bool cl_head(const uint64_t* K, int64_t i, uint64_t drop) {
  return K[i] != drop && (i == 0 || K[i] != K[i - 1]);
}

__global__ void k_cl_heads(const uint64_t* __restrict__ K, int64_t n, uint64_t drop, int32_t* __restrict__ flag) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    flag[i] = cl_head(K, i, drop) ? 1 : 0;
}

// seg_off[segment index] = first position; seg_off[G] = number of kept positions
__global__ void k_cl_segoff(const uint64_t* __restrict__ K, const int32_t* __restrict__ scan, int64_t n,
                            uint64_t drop, int32_t* __restrict__ seg_off) {
  const int32_t G = scan[n];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (cl_head(K, i, drop)) seg_off[scan[i]] = (int32_t)i;
    if (K[i] != drop && (i + 1 == n || K[i + 1] == drop)) seg_off[G] = (int32_t)(i + 1);
  }
}

// Short segments (a few rows per cluster): one sorted position per lane, its
// score row gathered into registers, a segmented inclusive scan across the
// wave (segment ids are non-decreasing), and the last lane of each segment
// stores S[h]; a segment cut by wave edges leaves its part of each wave in chain
// ([2][nv / 64][k]: [1] its first part, [0] the parts in the following waves), which
// k_seg_rows_chain adds in wave order.
template <int KM>
__global__ __launch_bounds__(256) void k_seg_rows(const uint64_t* __restrict__ K, const int32_t* __restrict__ scan,
                                                  const int32_t* __restrict__ R, int64_t nv, uint64_t drop,
                                                  const double* __restrict__ U, int k, double* __restrict__ S,
                                                  double* __restrict__ chain) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x / 64);
  for (int64_t wb = ((int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)) * 64; wb < nv; wb += nwaves * 64) {
    const int64_t q = wb + lane;
    const bool in = q < nv;
    int32_t h = 0x7fffffff;
    double v[KM];
#pragma unroll
    for (int j = 0; j < KM; ++j) v[j] = 0.0;
    if (in) {
      const bool head = q == 0 || K[q] != K[q - 1];
      h = scan[q] + (head ? 0 : -1);
      const double* u = U + (int64_t)R[q] * k;
#pragma unroll
      for (int j = 0; j < KM; ++j)
        if (j < k) v[j] = u[j];
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int32_t oh = __shfl_up(h, off, 64);
      const bool add = lane >= off && oh == h;
#pragma unroll
      for (int j = 0; j < KM; ++j) {
        const double o = __shfl_up(v[j], off, 64);
        if (add) v[j] += o;
      }
    }
    const int32_t nh = __shfl_down(h, 1, 64);
    const int32_t h0 = __shfl(h, 0, 64);
    const bool last = in && (lane == 63 || q + 1 == nv || nh != h);
    if (!last) continue;
    // complete inside this wave: starts after lane 0's segment, or lane 0 opens it
    const bool starts_here = h != h0 || wb == 0 || K[wb] != K[wb - 1];
    const bool ends_here = lane < 63 || q + 1 == nv || K[q + 1] != K[q];
    double* dst = S + (int64_t)h * k;
    if (starts_here && ends_here) {
#pragma unroll
      for (int j = 0; j < KM; ++j)
        if (j < k) dst[j] = v[j];
    } else {
      const int64_t nwb = (nv + 63) >> 6;
      double* part = chain + ((starts_here ? nwb : 0) + (wb >> 6)) * k;
#pragma unroll
      for (int j = 0; j < KM; ++j)
        if (j < k) part[j] = v[j];
    }
  }
}

// the segments cut by wave edges, their parts added in wave order: one thread per (wave w, column)
// whose last segment continues into wave w + 1 and began in wave w
__global__ void k_seg_rows_chain(const uint64_t* __restrict__ K, const int32_t* __restrict__ scan,
                                 const int32_t* __restrict__ seg_off, int64_t nv, int k,
                                 const double* __restrict__ chain, double* __restrict__ S) {
  const int64_t nwb = (nv + 63) >> 6;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nwb * k; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t w = e / k;
    const int j = (int)(e % k);
    const int64_t q = (w + 1) * 64;  // first position of wave w + 1
    if (q >= nv || K[q] != K[q - 1]) continue;  // no segment continues across this edge
    const int32_t h = scan[q] - 1;
    if (seg_off[h] < w * 64) continue;  // begun before wave w: a chain that starts earlier
    const int64_t we = (seg_off[h + 1] - 1) >> 6;
    double t = chain[(nwb + w) * k + j];
    for (int64_t v = w + 1; v <= we; ++v) t += chain[v * k + j];
    S[(int64_t)h * k + j] = t;
  }
}

// multi-rank dense form (span < 2^31): the local cluster h (sorted keys, segment offsets) goes to
// row key(h) of the zeroed key-indexed table; every key occurs once, so no two stores meet
__global__ void k_cl_dense_put(const uint64_t* __restrict__ K, const int32_t* __restrict__ seg_off, int32_t G,
                               const double* __restrict__ Sloc, int k, double* __restrict__ S,
                               int32_t* __restrict__ present) {
  const int kk = k > 0 ? k : 1;  // k = 0: presence only
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < (int64_t)G * kk;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t h = e / kk;
    const int j = (int)(e % kk);
    const uint64_t key = K[seg_off[h]];
    if (j == 0) present[key] = 1;
    if (j < k) S[key * k + j] = Sloc[h * k + j];
  }
}

__global__ __launch_bounds__(256) void k_count_nonzero(const int32_t* __restrict__ cnt, int32_t G,
                                                       int32_t* __restrict__ out) {
  __shared__ int32_t ws[4];
  int local = 0;
  for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x) local += cnt[g] > 0;
  for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = local;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = ws[0] + ws[1] + ws[2] + ws[3];
    if (t) atomicAdd(out, t);  // one add per block
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------


// Clusters of sorted (key, row) pairs [0, n) (dropped rows carry key = drop and sort
// last): segment offsets in W.seg_off, S[h] = sum of the rows' records (row-major
// [.][k] `table`) in c->clS; *G_out clusters.
// segments of sorted keys: head flags -> scan (clw.flag) -> offsets (clw.seg_off); *G_out clusters,
// *nv_out kept positions (dropped rows carry key = drop and sort last)
static int group_segments(lfe_ctx* c, int64_t n, uint64_t drop, const uint64_t* K, int32_t* G_out,
                          int32_t* nv_out) {
  auto& W = c->clw;
  LFE_TRY(ensure_i32(c, W.seg_off, W.seg_off_cap, (size_t)n + 1));
  LFE_TRY(ensure_i32(c, W.ufirst, W.ufirst_cap, (size_t)seg_units_needed(n)));
  LFE_HIP(hipMemsetAsync(W.flag + n, 0, sizeof(int32_t), c->stream));
  LFE_HIP(hipMemsetAsync(W.seg_off, 0, sizeof(int32_t), c->stream));
  if (n > 0) {
    ProfScope _ps(c, K_CLUSTER_SORT);
    hipLaunchKernelGGL(k_cl_heads, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, K, n, drop, W.flag);
  }
  LFE_HIP(hipGetLastError());
  LFE_TRY(exclusive_scan(c, W.flag, n + 1));
  if (n > 0) {
    ProfScope _ps(c, K_CLUSTER_SORT);
    hipLaunchKernelGGL(k_cl_segoff, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, K, W.flag, n, drop,
                       W.seg_off);
  }
  LFE_HIP(hipGetLastError());
  int32_t G = 0;
  LFE_TRY(d2h_sync(c, &G, W.flag + n, sizeof(int32_t)));
  *G_out = G;
  int32_t nv = 0;
  if (G > 0) LFE_TRY(d2h_sync(c, &nv, W.seg_off + G, sizeof(int32_t)));
  *nv_out = nv;
  return LFE_OK;
}

static int group_sums(lfe_ctx* c, int64_t n, uint64_t drop, const uint64_t* K, const int32_t* R, const double* table,
                      int k, int32_t G, int32_t nv);

int group_sorted(lfe_ctx* c, int64_t n, uint64_t drop, const uint64_t* K, const int32_t* R,
                        const double* table, int k, int32_t* G_out) {
  int32_t G = 0, nv = 0;
  LFE_TRY(group_segments(c, n, drop, K, &G, &nv));
  *G_out = G;
  if (k == 0) return LFE_OK;
  return group_sums(c, n, drop, K, R, table, k, G, nv);
}

// S[h] = sum of the rows' records of cluster h (c->clS), the segments formed by group_segments
static int group_sums(lfe_ctx* c, int64_t n, uint64_t drop, const uint64_t* K, const int32_t* R, const double* table,
                      int k, int32_t G, int32_t nv) {
  auto& W = c->clw;
  LFE_TRY(ensure_cluster_ws(c, (size_t)std::max(G, 1) * k, 4));
  if (k <= 16 && G > 0 && (int64_t)nv < 8 * (int64_t)G) {
    // short clusters (mean < 8 rows): row-per-lane segmented scan
    LFE_HIP(hipMemsetAsync(c->clS, 0, sizeof(double) * (size_t)G * k, c->stream));
    const int64_t nwb = ((int64_t)nv + 63) / 64;
    LFE_TRY(ensure_f64(c, c->chain, c->chain_cap, (size_t)2 * nwb * k));
    double* chain = c->chain;
    const int grid = grid_for(((int64_t)nv + 63) / 64 * 64, 256, 8192);
    ProfScope _ps(c, K_CLUSTER_SCATTER);
    if (k <= 4)
      hipLaunchKernelGGL(k_seg_rows<4>, dim3(grid), dim3(256), 0, c->stream, K, W.flag, R, (int64_t)nv, drop, table,
                         k, c->clS, chain);
    else if (k <= 8)
      hipLaunchKernelGGL(k_seg_rows<8>, dim3(grid), dim3(256), 0, c->stream, K, W.flag, R, (int64_t)nv, drop, table,
                         k, c->clS, chain);
    else if (k <= 12)
      hipLaunchKernelGGL(k_seg_rows<12>, dim3(grid), dim3(256), 0, c->stream, K, W.flag, R, (int64_t)nv, drop,
                         table, k, c->clS, chain);
    else
      hipLaunchKernelGGL(k_seg_rows<16>, dim3(grid), dim3(256), 0, c->stream, K, W.flag, R, (int64_t)nv, drop,
                         table, k, c->clS, chain);
    LFE_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_seg_rows_chain, dim3(grid_for(nwb * k)), dim3(kBlock), 0, c->stream, K, W.flag, W.seg_off,
                       (int64_t)nv, k, chain, c->clS);
  } else {
    LFE_TRY(seg_gather_sum(c, W.seg_off, G, W.ufirst, n, R, table, k, k, c->clS, K_CLUSTER_SCATTER));
  }
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

// Mostly-singleton subsets (e.g. config 4's fe2 x fe3: 48.8M clusters over 50M rows): with D the
// residual pass's sum of s s' over all kept rows, sum_c S_c S_c' = D + sum over clusters of two or
// more rows of (S_c S_c' - sum_{i in c} s_i s_i'), so only those clusters' rows are gathered.
// len2[h] = the rows of cluster h if it has two or more, else 0; one2[h] = 1 for such a cluster
__global__ void k_multi_mark(const int32_t* __restrict__ seg_off, int32_t G, int32_t* __restrict__ len2,
                             int32_t* __restrict__ one2) {
  for (int64_t h = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; h < G; h += (int64_t)gridDim.x * blockDim.x) {
    const int32_t len = seg_off[h + 1] - seg_off[h];
    len2[h] = len >= 2 ? len : 0;
    one2[h] = len >= 2 ? 1 : 0;
  }
}

// the multi-row clusters' rows and offsets, compacted (scans of k_multi_mark's arrays)
__global__ void k_multi_compact(const int32_t* __restrict__ seg_off, int32_t G, const int32_t* __restrict__ pos2,
                                const int32_t* __restrict__ idx2, const int32_t* __restrict__ R,
                                int32_t* __restrict__ seg2, int32_t* __restrict__ r2) {
  for (int64_t h = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; h < G; h += (int64_t)gridDim.x * blockDim.x) {
    const int32_t a = seg_off[h], len = seg_off[h + 1] - a;
    if (len < 2) continue;
    const int32_t q = pos2[h];
    seg2[idx2[h]] = q;
    for (int32_t j = 0; j < len; ++j) r2[q + j] = R[a + j];
  }
}

// t2[j] = the score row of r2[j]; s2[h] = the sum of its cluster's rows, in row order
__global__ void k_multi_rows(const int32_t* __restrict__ r2, int64_t N2, const double* __restrict__ U, int k,
                             double* __restrict__ t2) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < N2 * k; e += (int64_t)gridDim.x * blockDim.x)
    t2[e] = U[(int64_t)r2[e / k] * k + (e % k)];
}
__global__ void k_multi_sums(const int32_t* __restrict__ seg2, int32_t G2, const double* __restrict__ t2, int k,
                             double* __restrict__ s2) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < (int64_t)G2 * k;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t h = e / k;
    const int j = (int)(e % k);
    double t = 0.0;
    for (int32_t q = seg2[h]; q < seg2[h + 1]; ++q) t += t2[(int64_t)q * k + j];
    s2[e] = t;
  }
}

// s2[h] = the sum of cluster h's score rows U[r2[q]], q in [seg2[h], seg2[h+1]), in row order: a
// 16-lane group per cluster, lane j column j (k <= 16); two rows' loads in flight per step
__global__ __launch_bounds__(256) void k_multi_sums16(const int32_t* __restrict__ seg2, int32_t G2,
                                                      const int32_t* __restrict__ r2, const double* __restrict__ U,
                                                      int k, double* __restrict__ s2) {
  const int c = threadIdx.x & 15;
  const int cc = c < k ? c : 0;
  for (int64_t h = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4; h < G2;
       h += ((int64_t)gridDim.x * blockDim.x) >> 4) {
    const int32_t a = seg2[h], b = seg2[h + 1];
    double s = 0.0;
    int32_t q = a;
    for (; q + 1 < b; q += 2) {
      const int32_t i0 = r2[q], i1 = r2[q + 1];
      const double v0 = U[(int64_t)i0 * k + cc], v1 = U[(int64_t)i1 * k + cc];
      s += v0;
      s += v1;
    }
    if (q < b) s += U[(int64_t)r2[q] * k + cc];
    if (c < k) s2[h * k + c] = s;
  }
}

static int singleton_meat(lfe_ctx* c, const int32_t* R, int32_t G, int k, double* meat) {
  auto& W = c->clw;
  LFE_TRY(ensure_i32(c, W.off2, W.off2_cap, (size_t)G + 1));
  LFE_TRY(ensure_i32(c, W.idx2, W.idx2_cap, (size_t)G + 1));
  LFE_HIP(hipMemsetAsync(W.off2 + G, 0, sizeof(int32_t), c->stream));
  LFE_HIP(hipMemsetAsync(W.idx2 + G, 0, sizeof(int32_t), c->stream));
  {
    ProfScope _ps(c, K_CLUSTER_SCATTER);
    hipLaunchKernelGGL(k_multi_mark, dim3(grid_for(G, kBlock, 8192)), dim3(kBlock), 0, c->stream, W.seg_off, G,
                       W.off2, W.idx2);
  }
  LFE_HIP(hipGetLastError());
  LFE_TRY(exclusive_scan2(c, W.off2, (int64_t)G + 1, W.idx2, (int64_t)G + 1));
  int32_t n2[2] = {0, 0};
  LFE_TRY(d2h_sync(c, &n2[0], W.off2 + G, sizeof(int32_t)));
  LFE_TRY(d2h_sync(c, &n2[1], W.idx2 + G, sizeof(int32_t)));
  const int32_t N2 = n2[0], G2 = n2[1];
  std::vector<double> A((size_t)k * k, 0.0), B((size_t)k * k, 0.0);
  if (G2 > 0) {
    LFE_TRY(ensure_i32(c, W.seg2, W.seg2_cap, (size_t)G2 + 1));
    LFE_TRY(ensure_i32(c, W.r2, W.r2_cap, (size_t)N2));
    // 8 <= k <= 16: the clusters' sums by a 16-lane group each, straight from the score rows, and the
    // rows' Gram through the row index (no gathered copy t2: MEGA_CLUSTER2 25.9 -> 25.3 ms); narrower
    // rows keep the copy (k = 4, HDFE_CLUSTER2: the indexed Gram's 32-byte gathers cost 0.13 ms more
    // than copy + Gram); LFE_CL_MULTI_GATHER: the copy always
    const bool direct = k >= 8 && k <= 16 && knob("LFE_CL_MULTI_GATHER") == nullptr;
    if (!direct) LFE_TRY(ensure_f64(c, W.t2, W.t2_cap, (size_t)N2 * k));
    LFE_TRY(ensure_f64(c, W.s2, W.s2_cap, (size_t)G2 * k));
    LFE_TRY(h2d_small(c, W.seg2 + G2, &N2, sizeof(int32_t)));
    {
      ProfScope _ps(c, K_CLUSTER_SCATTER);
      hipLaunchKernelGGL(k_multi_compact, dim3(grid_for(G, kBlock, 8192)), dim3(kBlock), 0, c->stream, W.seg_off, G,
                         W.off2, W.idx2, R, W.seg2, W.r2);
      if (direct) {
        hipLaunchKernelGGL(k_multi_sums16, dim3(grid_for((int64_t)G2 * 16, 256, 8192)), dim3(256), 0, c->stream,
                           W.seg2, G2, W.r2, c->scores, k, W.s2);
      } else {
        hipLaunchKernelGGL(k_multi_rows, dim3(grid_for((int64_t)N2 * k, kBlock, 8192)), dim3(kBlock), 0, c->stream,
                           W.r2, (int64_t)N2, c->scores, k, W.t2);
        hipLaunchKernelGGL(k_multi_sums, dim3(grid_for((int64_t)G2 * k, kBlock, 8192)), dim3(kBlock), 0, c->stream,
                           W.seg2, G2, W.t2, k, W.s2);
      }
    }
    LFE_HIP(hipGetLastError());
    LFE_TRY(launch_table_gram(c, W.s2, G2, k, A.data()));
    if (direct) LFE_TRY(launch_table_gram(c, c->scores, N2, k, B.data(), W.r2));
    else LFE_TRY(launch_table_gram(c, W.t2, N2, k, B.data()));
  }
  for (int e = 0; e < k * k; ++e) meat[e] = c->score_meat[e] + (A[e] - B[e]);
  return LFE_OK;
}

__device__ __forceinline__ int cl_owner(uint64_t key, int world) {
  key ^= key >> 33;
  key *= 0xff51afd7ed558ccdull;
  key ^= key >> 33;
  return (int)(key % (uint64_t)world);
}

// the key of cluster h: K[seg_off[h]] over sorted row keys, or K[h] when K holds one key per cluster
__device__ __forceinline__ uint64_t cl_key(const uint64_t* K, const int32_t* seg_off, int h) {
  return seg_off ? K[seg_off[h]] : K[h];
}

__global__ void k_cl_owner_count(const uint64_t* __restrict__ K, const int32_t* __restrict__ seg_off, int32_t G,
                                 int world, int32_t* __restrict__ cnt) {
  for (int h = blockIdx.x * blockDim.x + threadIdx.x; h < G; h += gridDim.x * blockDim.x)
    atomicAdd(&cnt[cl_owner(cl_key(K, seg_off, h), world)], 1);
}

// send record of cluster h: its key and S[h][0, k), grouped by owner rank
__global__ void k_cl_owner_scatter(const uint64_t* __restrict__ K, const int32_t* __restrict__ seg_off,
                                   const double* __restrict__ S, int32_t G, int k, int world,
                                   int32_t* __restrict__ cursor, uint64_t* __restrict__ skey,
                                   double* __restrict__ srec) {
  for (int h = blockIdx.x * blockDim.x + threadIdx.x; h < G; h += gridDim.x * blockDim.x) {
    const uint64_t key = cl_key(K, seg_off, h);
    const int32_t pos = atomicAdd(&cursor[cl_owner(key, world)], 1);
    skey[pos] = key;
    for (int j = 0; j < k; ++j) srec[(int64_t)pos * k + j] = S[(int64_t)h * k + j];
  }
}

__global__ void k_iota_pairs(const uint64_t* __restrict__ kin, int64_t n, uint64_t* __restrict__ keys,
                             int32_t* __restrict__ rows) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    keys[i] = kin[i];
    rows[i] = (int32_t)i;
  }
}

// Owner-partitioned reduction of the local cluster sums: cluster h's
// record (its key and row S[h][0, k)) goes to rank owner(key); every owner merges what it received
// by key, forms S'S of its clusters, and only the k x k meats and cluster counts are all-reduced.
// Cluster h's key is K[seg_off[h]] (sorted row keys) or, with seg_off null, K[h].
int owner_meat(lfe_ctx* c, const uint64_t* K, const int32_t* seg_off, const double* S, int32_t G, int k,
               uint64_t span, double* meat, int64_t* G_out) {
  auto& W = c->clw;
  const int world = c->world, rank = c->rank;
  LFE_TRY(ensure_u64(c, W.skey, W.skey_cap, (size_t)std::max(G, 1)));
  LFE_TRY(ensure_f64(c, W.srec, W.srec_cap, (size_t)std::max(G, 1) * k));
  LFE_TRY(ensure_i32(c, W.ocnt, W.ocnt_cap, (size_t)world * world + 2 * world));
  int32_t* cnt = W.ocnt;               // [world] my records per owner, then cursors
  int32_t* cur = W.ocnt + world;       // [world]
  int32_t* mat = W.ocnt + 2 * world;   // [world][world] records from rank r to rank q
  LFE_HIP(hipMemsetAsync(cnt, 0, sizeof(int32_t) * world, c->stream));
  if (G > 0)
    hipLaunchKernelGGL(k_cl_owner_count, dim3(grid_for(G)), dim3(kBlock), 0, c->stream, K, seg_off, G, world, cnt);
  LFE_HIP(hipGetLastError());
  std::vector<int32_t> mine(world), offs(world);
  LFE_TRY(d2h_sync(c, mine.data(), cnt, sizeof(int32_t) * world));
  for (int q = 0, run = 0; q < world; ++q) {
    offs[q] = run;
    run += mine[q];
  }
  LFE_TRY(h2d_small(c, cur, offs.data(), sizeof(int32_t) * world));
  if (G > 0)
    hipLaunchKernelGGL(k_cl_owner_scatter, dim3(grid_for(G)), dim3(kBlock), 0, c->stream, K, seg_off, S, G, k,
                       world, cur, W.skey, W.srec);
  LFE_HIP(hipGetLastError());
  // who sends how much to whom
  std::vector<int32_t> hm((size_t)world * world, 0);
  for (int q = 0; q < world; ++q) hm[(size_t)rank * world + q] = mine[q];
  LFE_HIP(hipMemsetAsync(mat, 0, sizeof(int32_t) * world * world, c->stream));
  LFE_TRY(h2d_small(c, mat + (size_t)rank * world, mine.data(), sizeof(int32_t) * world));
  LFE_TRY(allreduce_sum_i32(c, mat, (size_t)world * world));
  LFE_TRY(d2h_sync(c, hm.data(), mat, sizeof(int32_t) * world * world));
  std::vector<size_t> so(world), sb(world), ro(world), rb(world), so8(world), sb8(world), ro8(world), rb8(world);
  int64_t R = 0;
  for (int q = 0; q < world; ++q) {
    const int64_t from_q = hm[(size_t)q * world + rank];
    so[q] = (size_t)offs[q] * k * sizeof(double);
    sb[q] = (size_t)mine[q] * k * sizeof(double);
    so8[q] = (size_t)offs[q] * sizeof(uint64_t);
    sb8[q] = (size_t)mine[q] * sizeof(uint64_t);
    ro[q] = (size_t)R * k * sizeof(double);
    rb[q] = (size_t)from_q * k * sizeof(double);
    ro8[q] = (size_t)R * sizeof(uint64_t);
    rb8[q] = (size_t)from_q * sizeof(uint64_t);
    R += from_q;
  }
  LFE_TRY(ensure_u64(c, W.rkey, W.rkey_cap, (size_t)std::max<int64_t>(R, 1)));
  LFE_TRY(ensure_f64(c, W.rrec, W.rrec_cap, (size_t)std::max<int64_t>(R, 1) * k));
  LFE_TRY(alltoallv_bytes(c, reinterpret_cast<const char*>(W.skey), so8.data(), sb8.data(),
                          reinterpret_cast<char*>(W.rkey), ro8.data(), rb8.data()));
  LFE_TRY(alltoallv_bytes(c, reinterpret_cast<const char*>(W.srec), so.data(), sb.data(),
                          reinterpret_cast<char*>(W.rrec), ro.data(), rb.data()));
  // merge the received partial sums of this rank's clusters
  LFE_TRY(ensure_sort_ws(c, (size_t)R));
  if (R > 0)
    hipLaunchKernelGGL(k_iota_pairs, dim3(grid_for(R, kBlock, 8192)), dim3(kBlock), 0, c->stream, W.rkey, R,
                       W.keys[0], W.rows[0]);
  LFE_HIP(hipGetLastError());
  int buf = 0;
  if (R > 0) LFE_TRY(radix_sort(c, R, bit_length(span), &buf));
  int32_t Gown = 0;
  LFE_TRY(group_sorted(c, R, span, W.keys[buf], W.rows[buf], W.rrec, k, &Gown));
  // this rank's clusters only: the table Gram is reduced locally, then the meats summed
  std::vector<double> part((size_t)k * k, 0.0);
  if (Gown > 0) {
    c->world = 1;
    const int rc = launch_table_gram(c, c->clS, Gown, k, part.data());
    c->world = world;
    if (rc) return rc;
  }
  LFE_TRY(ensure_dred(c, (size_t)k * k + 1));
  std::vector<double> packed(part);
  packed.push_back((double)Gown);
  LFE_TRY(h2d_small(c, c->dred, packed.data(), sizeof(double) * packed.size()));
  LFE_TRY(allreduce_sum_f64(c, c->dred, packed.size()));
  LFE_TRY(d2h_sync(c, packed.data(), c->dred, sizeof(double) * packed.size()));
  for (int e = 0; e < k * k; ++e) meat[e] = packed[e];
  *G_out = (int64_t)packed[(size_t)k * k];
  return LFE_OK;
}

// ---------------------------------------------------------------------------
// Per-row cluster ids in input row order (the wide fits of lfe_wide.hip)
// ---------------------------------------------------------------------------
__global__ void k_cid_one(const int32_t* __restrict__ code, const double* __restrict__ kept, int64_t n,
                          int32_t* __restrict__ cid) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    cid[i] = kept[i] != 0.0 ? code[i] : -1;
}

__global__ void k_cid_keys(KeyArgs a, const double* __restrict__ kept) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t key = 0;
    for (int j = 0; j < a.m; ++j) key += (uint64_t)(uint32_t)a.code[j][i] * a.mult[j];
    a.keys[i] = kept[i] != 0.0 ? key : a.drop;
    a.rows[i] = (int32_t)i;
  }
}

// sorted position j -> its segment's index (heads before j, minus one unless j heads a segment)
__global__ void k_cid_scatter(const uint64_t* __restrict__ K, const int32_t* __restrict__ R,
                              const int32_t* __restrict__ scan, int64_t n, uint64_t drop, int32_t* __restrict__ cid) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x)
    cid[R[j]] = K[j] == drop ? -1 : scan[j] - (cl_head(K, j, drop) ? 0 : 1);
}

int cluster_ids_input(lfe_ctx* c, int mask, const double* kept, int32_t* cid, int32_t* G_out) {
  const int64_t n = c->n;
  auto& W = c->clw;
  if (__builtin_popcount((unsigned)mask) == 1) {
    const int j = __builtin_ctz((unsigned)mask);
    if (n > 0)
      hipLaunchKernelGGL(k_cid_one, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, c->cl[j], kept, n,
                         cid);
    LFE_HIP(hipGetLastError());
    *G_out = c->cl_levels[j];
    return LFE_OK;
  }
  KeyArgs ka{};
  uint64_t span = 1;
  for (int j = 0; j < (int)c->cl.size(); ++j) {
    if (!(mask >> j & 1)) continue;
    if (ka.m == kMaxCl) return fail(LFE_EINVAL, "too many cluster columns in one subset");
    const uint64_t g = (uint64_t)c->cl_levels[j];
    if (span > ((1ull << 62) / g)) return fail(LFE_EINVAL, "cluster intersection span exceeds 2^62");
    ka.code[ka.m] = c->cl[j];
    ka.mult[ka.m] = span;
    ++ka.m;
    span *= g;
  }
  LFE_TRY(ensure_sort_ws(c, (size_t)c->ld));
  ka.n = n;
  ka.drop = span;
  ka.keys = W.keys[0];
  ka.rows = W.rows[0];
  if (n > 0) hipLaunchKernelGGL(k_cid_keys, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, ka, kept);
  LFE_HIP(hipGetLastError());
  int buf = 0;
  if (n > 0) LFE_TRY(radix_sort(c, n, bit_length(span), &buf));
  int32_t G = 0, nv = 0;
  LFE_TRY(group_segments(c, n, span, W.keys[buf], &G, &nv));
  if (n > 0)
    hipLaunchKernelGGL(k_cid_scatter, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, W.keys[buf],
                       W.rows[buf], W.flag, n, span, cid);
  LFE_HIP(hipGetLastError());
  *G_out = G;
  return LFE_OK;
}

// ---------------------------------------------------------------------------
// One cluster column: per-cluster score sums in two-limb fixed point, no sort
// ---------------------------------------------------------------------------
// A one-column subset's clusters are that column's codes, so S_c = sum of the score rows of c's kept
// rows can be formed the way the group sums S_f are (lfe_fast.hip): every score value enters its
// cluster's entry as a fine limb (int64 global adds) and, beyond the column's typical range, a
// coarse limb (integer-valued f64 adds) - exact in any order, so the meat repeats bit for bit
// without ordering the rows.  It replaces the key build, the radix sort and the segmented sums of
// the sorted path (std_errors.py:317-333 groups by the column).
constexpr int kClFixChunk = 8192;

// the score columns' statistics in the colstat form of lfe_fast.hip (max |s_c| bits by u64
// atomicMax; the chunk's sum of s_c^2 in fixed order) and the clusters' kept-row counts.  Thread t
// reads column t % k of rows t / k, t / k + R, ... (R = 256 / k rows per step): the row-major score
// rows are read in contiguous runs, each thread's sums in row order, then the R partials of a
// column in thread order.
__global__ __launch_bounds__(256) void k_clfix_stats(const int32_t* __restrict__ code, const int32_t* __restrict__ keep,
                                                     int64_t n, const double* __restrict__ U, int k, int nchunks,
                                                     int32_t* __restrict__ cnt, double* __restrict__ st) {
  __shared__ double wm[256], wq[256];
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * kClFixChunk, r1 = min(n, r0 + kClFixChunk);
  if (cnt)
    for (int64_t i = r0 + tid; i < r1; i += 256)
      if (!keep || keep[i] >= 0) atomicAdd(&cnt[code[i]], 1);
  const int R = 256 / k, c = tid % k, ro = tid / k;
  double m = 0.0, q = 0.0;
  if (ro < R) {
    // branch-free (a dropped row adds 0 to both), four rows in flight per thread
#pragma unroll 4
    for (int64_t i = r0 + ro; i < r1; i += R) {
      const double u = U[i * k + c];
      const double v = (!keep || keep[i] >= 0) ? u : 0.0;
      m = fmax(m, fabs(v));
      q = __builtin_fma(v, v, q);
    }
  }
  wm[tid] = m;
  wq[tid] = q;
  __syncthreads();
  if (tid < k) {
    double M = 0.0, Q = 0.0;
    for (int j = 0; j < R; ++j) {
      M = fmax(M, wm[tid + j * k]);
      Q += wq[tid + j * k];
    }
    st[kColStatHead + (int64_t)tid * nchunks + blockIdx.x] = Q;
    atomicMax(reinterpret_cast<unsigned long long*>(st) + tid, (unsigned long long)__double_as_longlong(M));
  }
}

// kept rows per cluster of a small table: per-workgroup LDS counts, then one global add per
// nonzero count (integer adds: any order)
__global__ __launch_bounds__(1024) void k_clfix_hist(const int32_t* __restrict__ code, const int32_t* __restrict__ keep,
                                                     int64_t n, int32_t G, int32_t* __restrict__ cnt) {
  extern __shared__ int32_t h[];
  for (int j = threadIdx.x; j < G; j += 1024) h[j] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 1024)
    if (!keep || keep[i] >= 0) atomicAdd(&h[code[i]], 1);
  __syncthreads();
  for (int j = threadIdx.x; j < G; j += 1024)
    if (h[j]) atomicAdd(&cnt[j], h[j]);
}

// the statistics head from the residual pass's meat, passed by value (no host-to-device copy to
// wait for): max |s_c| bits (an assumed bound) and one chunk's sum of s_c^2 per column
struct ClMeatStats {
  double M[64];
  double d[64];
  int k;
};
__global__ void k_clfix_meat_stats(ClMeatStats a, double* __restrict__ st) {
  for (int e = threadIdx.x; e < a.k; e += blockDim.x) {
    st[e] = a.M[e];  // as u64 bits: the same bits as a double >= 0
    st[kColStatHead + e] = a.d[e];
  }
}

// every column may carry coarse limbs (the adds split them, the conversion adds them back)
__global__ void k_fq_all_big(double* __restrict__ fq, int k) {
  for (int e = threadIdx.x; e < k; e += blockDim.x) fq[FQ_BIG * kFqCols + e] = 1.0;
}

// out[0] = clusters with kept rows, out[1] = the largest cluster (integer atomics: any order)
__global__ void k_clfix_count(const int32_t* __restrict__ cnt, int32_t G, int32_t* __restrict__ out) {
  int32_t nz = 0, mx = 0;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < G; g += (int64_t)gridDim.x * blockDim.x) {
    nz += cnt[g] > 0 ? 1 : 0;
    mx = max(mx, cnt[g]);
  }
  if (nz) atomicAdd(&out[0], nz);
  if (mx) atomicMax(&out[1], mx);
}

// every kept score value into its cluster's entry, fine limbs first into an LDS window of the
// table: the whole [G][k] table (a small G), or - the cluster column being the layout's primary FE -
// the [B][k] slice of the work item's bucket (items run bucket by bucket, like the group sums of
// lfe_fast.hip).  A window goes out by int64 global adds of its nonzero entries when the bucket
// changes and at the end; coarse limbs (outliers) go to the global f64 table directly.
constexpr int kClFixThreads = 1024;
constexpr size_t kClFixLds = 96 * 1024;
struct ClFixAdd {
  const int32_t* code;  // cluster codes (layout order)
  const int32_t* keep;  // the primary FE's codes (< 0: dropped row), or null
  const double* U;      // [n][k] score rows (layout order)
  const double* fq;
  const int4* items;
  unsigned long long* S;  // [G][k] fine limbs
  double* hi;             // [G][k] coarse limbs
  int n_items, k, s, win, G;
  int bucketed;
  // quanta from the residual pass's meat (no statistics pass): every value may carry a coarse
  // limb, and one whose coarse limb could make a cluster's f64 sum inexact raises *oflag (the
  // caller then redoes the subset with the statistics pass)
  const int32_t* cmax;  // [1]: the largest cluster's kept rows
  int32_t* oflag;       // null: quanta from the statistics pass
};

template <bool CHECK>  // CHECK: meat quanta (a.oflag set), every coarse limb checked against the bound
__global__ __launch_bounds__(kClFixThreads) void k_clfix_add(ClFixAdd a) {
  typedef unsigned long long u64;
  extern __shared__ u64 t[];  // [win][k]
  const int tid = threadIdx.x, k = a.k;
  const int wk = a.win * k;
  const int R = kClFixThreads / k, cc = tid % k, ro = tid / k;
  const FixCol fc = fix_col(a.fq, cc);
  // (meat quanta: every column flagged big) N (|h| + 1) < 2^51 keeps the f64 sums of h exact
  const double hlim = CHECK ? 0x1p51 / (double)max(*a.cmax, 1) - 1.0 : 0.0;
  bool over = false;
  for (int j = tid; j < wk; j += kClFixThreads) t[j] = 0ull;
  const int i0 = (int)((int64_t)a.n_items * blockIdx.x / gridDim.x);
  const int i1 = (int)((int64_t)a.n_items * (blockIdx.x + 1) / gridDim.x);
  int cur = -1;
  auto flush = [&](int lo) {
    for (int j = tid; j < wk; j += kClFixThreads) {
      const u64 v = t[j];
      if (v != 0ull && lo + j / k < a.G) atomicAdd(&a.S[(int64_t)lo * k + j], v);
      t[j] = 0ull;
    }
  };
  for (int item = i0; item < i1; ++item) {
    const int4 it = a.items[item];
    const int lo = a.bucketed ? it.x << a.s : 0;
    if (lo != cur) {
      __syncthreads();
      if (cur >= 0) flush(cur);
      __syncthreads();
      cur = lo;
    }
    if (ro < R) {  // thread (row ro, column cc): R rows of k contiguous values per step, two in flight
      int i = it.y + ro;
      for (; i + R < it.z; i += 2 * R) {
        const int i2 = i + R;
        const bool k1 = !a.keep || a.keep[i] >= 0, k2 = !a.keep || a.keep[i2] >= 0;
        const int g1 = a.code[i], g2 = a.code[i2];
        const double u1 = a.U[(int64_t)i * k + cc], u2 = a.U[(int64_t)i2 * k + cc];
        double h1, h2;
        const u64 x1 = fix_split(u1, fc, h1), x2 = fix_split(u2, fc, h2);
        if (k1 && x1) atomicAdd(&t[(g1 - lo) * k + cc], x1);
        if (k2 && x2) atomicAdd(&t[(g2 - lo) * k + cc], x2);
        if (k1 && h1 != 0.0) atomicAdd(&a.hi[(int64_t)g1 * k + cc], h1);
        if (k2 && h2 != 0.0) atomicAdd(&a.hi[(int64_t)g2 * k + cc], h2);
        if (CHECK) over |= (k1 & !(fabs(h1) <= hlim)) | (k2 & !(fabs(h2) <= hlim));  // branch-free
      }
      if (i < it.z && (!a.keep || a.keep[i] >= 0)) {
        const int g = a.code[i];
        double hh;
        const u64 xi = fix_split(a.U[(int64_t)i * k + cc], fc, hh);
        if (xi) atomicAdd(&t[(g - lo) * k + cc], xi);
        if (hh != 0.0) atomicAdd(&a.hi[(int64_t)g * k + cc], hh);
        if (CHECK) over |= !(fabs(hh) <= hlim);
      }
    }
  }
  __syncthreads();
  if (cur >= 0) flush(cur);
  if (CHECK && __any(over) && (tid & 63) == 0) a.oflag[0] = 1;
}

// flag[0] = 1 when some row's code in a differs from its code in p (rows with p < 0 are skipped)
__global__ void k_cl_same(const int32_t* __restrict__ a, const int32_t* __restrict__ p, int64_t n,
                          int32_t* __restrict__ flag) {
  bool diff = false;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    diff = diff || (p[i] >= 0 && a[i] != p[i]);
  if (__any(diff) && (threadIdx.x & 63) == 0) flag[0] = 1;
}

static bool clfix_on() {
  const bool on = [] {
    const char* e = knob("LFE_CL_FIX");  // "0": the sorted path for one-column subsets too (A/B, tests)
    return !(e && e[0] == '0');
  }();
  return on;
}

// meat and cluster count of the one-column subset j by the fixed-point sums (S: [G][k], then S'S);
// win / bucketed: the LDS window of k_clfix_add
// Owner-sharded ranks hold every row of a range of the primary FE's levels: a subset with a cluster
// column that repeats that FE (lfe_load_clusters compared them, every rank agreeing) has each of its
// clusters on one rank, so its sums - sort-free or sorted, bucket keys included - need no exchange:
// every rank forms S'S of its own clusters and the k x k meat and the cluster count are summed over
// ranks.  Returns that column, or -1.
static int owner_col(const lfe_ctx* c, int mask) {
  if (!(c->world > 1 && c->owner_on && c->L.P >= 0 && c->L.permuted)) return -1;
  for (int j = 0; j < (int)c->cl.size(); ++j)
    if ((mask >> j & 1) && j < (int)c->cl_fe.size() && c->cl_fe[j] == c->L.P &&
        c->cl_levels[j] == c->fe[c->L.P].G)
      return j;
  return -1;
}

// an integer summed over ranks (exact in f64 below 2^53)
static int sum_over_ranks(lfe_ctx* c, int64_t v, int64_t* out) {
  if (c->world <= 1) {
    *out = v;
    return LFE_OK;
  }
  LFE_TRY(ensure_f64(c, c->clw.rsum, c->clw.rsum_cap, 2));
  const double d = (double)v;
  LFE_TRY(h2d_small(c, c->clw.rsum, &d, sizeof(double)));
  LFE_TRY(allreduce_sum_f64(c, c->clw.rsum, 1));
  double h = 0.0;
  LFE_TRY(d2h_sync(c, &h, c->clw.rsum, sizeof(double)));
  *out = (int64_t)h;
  return LFE_OK;
}

static int subset_meat_fix(lfe_ctx* c, int j, int win, bool bucketed, double* meat, int64_t* G_out,
                           bool stats_pass = false, bool owner_local = false) {
  const int k = c->score_k;
  const int64_t n = c->n;
  const int32_t G = c->cl_levels[j];
  auto& W = c->clw;
  const int32_t* keep = c->L.P >= 0 ? c->L.code[c->L.P] : nullptr;
  const int nch = (int)std::max<int64_t>(1, (n + kClFixChunk - 1) / kClFixChunk);
  const size_t m = (size_t)G * std::max(k, 1);
  LFE_TRY(ensure_f64(c, W.fixst, W.fixst_cap, (size_t)kColStatHead + (size_t)std::max(k, 1) * nch));
  LFE_TRY(ensure_f64(c, W.fixq, W.fixq_cap, (size_t)kFqRows * kFqCols));
  LFE_TRY(ensure_cluster_ws(c, m, (size_t)G + 4));   // clS: coarse limbs; clP: counts, then [nonzero, max]
  LFE_TRY(ensure_f64(c, W.srec, W.srec_cap, m));      // fine limbs -> S
  int32_t* cnt = c->clP;
  int32_t* cm = c->clP + G;
  double* S = W.srec;
  LFE_HIP(hipMemsetAsync(W.fixst, 0, sizeof(double) * kColStatHead, c->stream));
  LFE_HIP(hipMemsetAsync(cnt, 0, sizeof(int32_t) * ((size_t)G + 4), c->stream));
  LFE_HIP(hipMemsetAsync(c->clS, 0, sizeof(double) * m, c->stream));
  LFE_HIP(hipMemsetAsync(S, 0, sizeof(double) * m, c->stream));
  {
    ProfScope _ps(c, K_CLUSTER_FIX);
    // kept rows per cluster: the primary FE's kept counts (bucketed: the column repeats it), an LDS
    // histogram (a small table), else global adds in the statistics pass
    int32_t* cnt_in_stats = nullptr;
    if (bucketed) {
      LFE_HIP(hipMemcpyAsync(cnt, c->fe[c->L.P].cnt, sizeof(int32_t) * G, hipMemcpyDeviceToDevice, c->stream));
    } else if ((size_t)G * 4 <= kClFixLds) {
      if (n > 0)
        hipLaunchKernelGGL(k_clfix_hist, dim3(std::max(1, std::min<int>(2 * c->n_cu, (int)((n + 8191) / 8192)))),
                           dim3(1024), sizeof(int32_t) * G, c->stream, W.lay[j], keep, n, G, cnt);
    } else {
      cnt_in_stats = cnt;
    }
    // quanta: from the residual pass's meat (one process: Σ_i s_ic^2 ≈ its diagonal, deterministic;
    // max |s| taken as 64 rms, every value checked against the coarse sums' bound in the adds) or
    // from a statistics pass over the score rows
    // (score_meat_ok: the meat is exactly sum s s' - one process, no weights, no records)
    const bool from_meat = !stats_pass && !cnt_in_stats && c->world == 1 && c->score_meat_ok &&
                           c->score_meat.size() == (size_t)k * k && k > 0 && k <= 64;
    if (from_meat) {
      // max |s_c| assumed 16 rms (the typical range of the fine limb; a larger value takes a coarse
      // limb, one past the coarse sums' bound raises the overflow flag)
      ClMeatStats ms{};
      ms.k = k;
      const double nk = (double)std::max<int64_t>(c->n_kept, 1);
      for (int e = 0; e < k; ++e) {
        const double d = std::max(c->score_meat[(size_t)e * k + e], 0.0);
        ms.M[e] = std::isfinite(d) ? 16.0 * std::sqrt(d / nk) : d;
        ms.d[e] = d;
      }
      hipLaunchKernelGGL(k_clfix_meat_stats, dim3(1), dim3(64), 0, c->stream, ms, W.fixst);
    } else if (n > 0) {
      hipLaunchKernelGGL(k_clfix_stats, dim3(nch), dim3(256), 0, c->stream, W.lay[j], keep, n, c->scores, std::max(k, 1),
                         nch, cnt_in_stats, W.fixst);
    }
    LFE_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_clfix_count, dim3(grid_for(G, 256, 1024)), dim3(256), 0, c->stream, cnt, G, cm);
    LFE_HIP(hipGetLastError());
    if (k > 0 && n > 0) {
      LFE_TRY(launch_fix_quanta(c, W.fixst, from_meat ? 1 : nch,
                                std::max<int64_t>(from_meat ? c->n_kept : c->n_kept_local, 1), cm + 1, 1, W.fixq, k));
      if (from_meat) hipLaunchKernelGGL(k_fq_all_big, dim3(1), dim3(64), 0, c->stream, W.fixq, k);
      ClFixAdd a{};
      a.code = W.lay[j];
      a.keep = keep;
      a.U = c->scores;
      a.fq = W.fixq;
      a.items = reinterpret_cast<const int4*>(c->items_d);
      a.S = reinterpret_cast<unsigned long long*>(S);
      a.hi = c->clS;
      a.n_items = c->L.n_items;
      a.k = k;
      a.s = c->L.s;
      a.win = win;
      a.G = G;
      a.bucketed = bucketed ? 1 : 0;
      a.cmax = cm + 1;
      a.oflag = from_meat ? cm + 2 : nullptr;
      const size_t lds = sizeof(unsigned long long) * (size_t)win * k;
      const void* fn = from_meat ? reinterpret_cast<const void*>(&k_clfix_add<true>)
                                 : reinterpret_cast<const void*>(&k_clfix_add<false>);
      LFE_HIP(set_max_lds(fn, (int)std::max<size_t>(lds, 8)));
      const int grid = std::max(1, std::min(c->L.n_items, 2 * c->n_cu));
      if (from_meat) hipLaunchKernelGGL(k_clfix_add<true>, dim3(grid), dim3(kClFixThreads), lds, c->stream, a);
      else hipLaunchKernelGGL(k_clfix_add<false>, dim3(grid), dim3(kClFixThreads), lds, c->stream, a);
      LFE_HIP(hipGetLastError());
      LFE_TRY(launch_fix_convert(c, S, c->clS, (int64_t)m, k, W.fixq));
    }
  }
  if (owner_local) {  // each cluster on one rank: the counts of present clusters summed
    LFE_TRY(allreduce_sum_i32(c, cm, 1));
    LFE_TRY(allreduce_max_i32(c, cm + 2, 1));
  } else if (c->world > 1) {  // every rank's sums in the key-indexed table (global codes): all-reduced
    LFE_TRY(allreduce_sum_f64(c, S, (size_t)G * k));
    LFE_TRY(allreduce_sum_i32(c, cnt, (size_t)G));
    LFE_HIP(hipMemsetAsync(cm, 0, sizeof(int32_t) * 2, c->stream));
    hipLaunchKernelGGL(k_clfix_count, dim3(grid_for(G, 256, 1024)), dim3(256), 0, c->stream, cnt, G, cm);
    LFE_HIP(hipGetLastError());
  }
  int32_t hc[3] = {0, 0, 0};
  LFE_TRY(d2h_sync(c, hc, cm, sizeof(hc)));
  if (hc[2] != 0)  // a value past the assumed range: the quanta from the statistics pass instead
    return subset_meat_fix(c, j, win, bucketed, meat, G_out, true, owner_local);
  *G_out = hc[0];
  if (k == 0) return LFE_OK;
  // S is replicated after the all-reduce: reduce its Gram locally; owner-local: each rank's S'S of
  // its own clusters, summed over ranks by the Gram's reduction
  const int world = c->world;
  if (!owner_local) c->world = 1;
  const int rc = launch_table_gram(c, S, G, k, meat);
  c->world = world;
  return rc;
}

// meat and cluster count of the one-column subset whose column repeats FE f, by the FE's segment
// layout (the general sweeps' sorted build orders the kept rows by the code and keeps the row
// permutation): two-limb sums of the score rows per segment (seg_score_sums), quanta from a
// statistics pass over the score rows - no keys, no radix sort, no segment heads (config 4's 1e5-
// and 1e4-level columns; one process)
static int subset_meat_seg(lfe_ctx* c, int f, double* meat, int64_t* G_out) {
  const int k = c->score_k;
  const int64_t n = c->n;
  const int32_t G = c->fe[f].G;
  auto& W = c->clw;
  const int32_t* keep = c->L.P >= 0 ? c->L.code[c->L.P] : nullptr;
  const int nch = (int)std::max<int64_t>(1, (n + kClFixChunk - 1) / kClFixChunk);
  const size_t m = (size_t)G * k;
  LFE_TRY(ensure_f64(c, W.fixq, W.fixq_cap, (size_t)kFqRows * kFqCols));
  LFE_TRY(ensure_cluster_ws(c, m, 4));            // clS: coarse limbs; clP: [nonzero, max]
  LFE_TRY(ensure_f64(c, W.srec, W.srec_cap, m));  // fine limbs -> S
  int32_t* cm = c->clP;
  double* S = W.srec;
  // the score rows' statistics: once per launch_cluster_subsets call (its subsets share the rows)
  const bool stats = !W.segst_ok;
  if (stats) {
    LFE_TRY(ensure_f64(c, W.segst, W.segst_cap, (size_t)kColStatHead + (size_t)k * nch));
    LFE_HIP(hipMemsetAsync(W.segst, 0, sizeof(double) * kColStatHead, c->stream));
    W.segst_ok = true;
  }
  LFE_HIP(hipMemsetAsync(cm, 0, sizeof(int32_t) * 4, c->stream));
  LFE_HIP(hipMemsetAsync(c->clS, 0, sizeof(double) * m, c->stream));
  LFE_HIP(hipMemsetAsync(S, 0, sizeof(double) * m, c->stream));
  {
    ProfScope _ps(c, K_CLUSTER_FIX);  // one scope: statistics (first subset), sums, conversion
    hipLaunchKernelGGL(k_clfix_count, dim3(grid_for(G, 256, 1024)), dim3(256), 0, c->stream, c->fe[f].cnt, G, cm);
    if (stats && n > 0)
      hipLaunchKernelGGL(k_clfix_stats, dim3(nch), dim3(256), 0, c->stream, keep, keep, n, c->scores, k, nch, nullptr,
                         W.segst);
    LFE_HIP(hipGetLastError());
    LFE_TRY(launch_fix_quanta(c, W.segst, nch, std::max<int64_t>(c->n_kept_local, 1), cm + 1, 1, W.fixq, k));
    LFE_TRY(seg_score_sums(c, f, c->scores, k, W.fixq, S, c->clS, -1));
    LFE_TRY(launch_fix_convert(c, S, c->clS, (int64_t)m, k, W.fixq));
  }
  int32_t hc[2] = {0, 0};
  LFE_TRY(d2h_sync(c, hc, cm, sizeof(hc)));
  *G_out = hc[0];
  return launch_table_gram(c, S, G, k, meat);
}

// ---------------------------------------------------------------------------
// One-way cluster on the primary FE, summed in the residual pass (lfe_gram.hip k_resid_rows<.., true>)
// ---------------------------------------------------------------------------
// Quanta before the pass, from its Gram tile and beta (both on the device): rms of the score column
// x~_j r taken as rms(x~_j) rms(r), with sum r^2 = v' T v (v = [-b0, 1, -b]) in fixed order; the
// fine limb's range is 16 rms, every column may carry coarse limbs, and one past the exact-sum bound
// raises the flag (the subset is then redone from score rows).  Deterministic: a fixed function of
// the tile.
__global__ void k_clfused_quanta(const double* __restrict__ tile, const double* __restrict__ beta, int p, int64_t n,
                                 int32_t* __restrict__ cmax, double* __restrict__ fq) {
  __shared__ double rss;
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i <= p; ++i) {
      const double vi = i == 0 ? -beta[0] : i == 1 ? 1.0 : -beta[i - 1];
      double u = 0.0;
      for (int j = 0; j <= p; ++j) {
        const double vj = j == 0 ? -beta[0] : j == 1 ? 1.0 : -beta[j - 1];
        u += tile[i * 16 + j] * vj;
      }
      t += vi * u;
    }
    rss = t > 0.0 ? t : 0.0;
    // a near-perfect fit: v'Tv has cancelled, so rms(r) says nothing about the scores' scale -
    // raise the bound flag (cmax[1]) and the subset is summed from score rows with the
    // statistics-pass quanta instead
    const double yy = tile[1 * 16 + 1];
    if (!(rss > 0x1p-40 * yy)) cmax[1] = 1;
  }
  __syncthreads();
  const double nn = n > 0 ? (double)n : 1.0;
  const double N = (double)max(*cmax, 1);
  for (int e = threadIdx.x; e < p - 1; e += blockDim.x) {
    const double g = tile[(e + 2) * 16 + (e + 2)];
    const double rms = sqrt((g > 0.0 ? g : 0.0) / nn) * sqrt(rss / nn);
    fix_quanta_col(16.0 * rms, rms, N, fq, e);
    fq[FQ_BIG * kFqCols + e] = 1.0;
  }
}

// the cluster column whose one-way sums the residual pass can form (it repeats the primary FE),
// or -1
int cluster_fused_col(const lfe_ctx* c) {
  const bool env_on = [] {  // "LFE_CL_FUSED=0": score rows and the separate sums (A/B)
    const char* e = knob("LFE_CL_FUSED");
    const char* s = knob("LFE_CL_STATS");
    return !(e && e[0] == '0') && !(s && s[0] == '1');
  }();
  const int k = c->p - 1;
  if (!(env_on && clfix_on() && !(c->test_hooks & (LFE_TEST_CLUSTER_SORTED | LFE_TEST_CLUSTER_STATS)) &&
        (c->world == 1 || c->owner_on) && c->L.P >= 0 && c->L.permuted && !c->w && !c->records && k >= 1 && k <= 63))
    return -1;
  for (int j = 0; j < (int)c->cl_fe.size() && j < (int)c->cl.size(); ++j)
    if (c->cl_fe[j] == c->L.P) return j;
  return -1;
}

int cluster_fused_prepare(lfe_ctx* c) {
  const int k = c->p - 1, G = c->fe[c->L.P].G;
  LFE_TRY(ensure_f64(c, c->clf_S, c->clf_S_cap, (size_t)G * k));      // fine limbs
  LFE_TRY(ensure_f64(c, c->clf_hi, c->clf_hi_cap, (size_t)G * k));    // coarse limbs
  LFE_TRY(ensure_i32(c, c->clf_cnt, c->clf_cnt_cap, (size_t)G + 4));  // counts, then [G, max, flag]
  LFE_TRY(ensure_f64(c, c->clf_fq, c->clf_fq_cap, (size_t)kFqRows * kFqCols));
  int32_t* cm = c->clf_cnt + G;
  LFE_HIP(hipMemcpyAsync(c->clf_cnt, c->fe[c->L.P].cnt, sizeof(int32_t) * G, hipMemcpyDeviceToDevice, c->stream));
  LFE_HIP(hipMemsetAsync(cm, 0, sizeof(int32_t) * 4, c->stream));
  hipLaunchKernelGGL(k_clfix_count, dim3(grid_for(G, 256, 1024)), dim3(256), 0, c->stream, c->clf_cnt, G, cm);
  LFE_HIP(hipGetLastError());
  // owner-sharded ranks: the largest cluster over all ranks, so every rank takes the same quanta
  LFE_TRY(allreduce_max_i32(c, cm + 1, 1));
  return LFE_OK;
}

int cluster_fused_reset(lfe_ctx* c, const double* tile, const double* beta) {
  const int k = c->p - 1, G = c->fe[c->L.P].G;
  LFE_HIP(hipMemsetAsync(c->clf_S, 0, sizeof(double) * (size_t)G * k, c->stream));
  LFE_HIP(hipMemsetAsync(c->clf_hi, 0, sizeof(double) * (size_t)G * k, c->stream));
  LFE_HIP(hipMemsetAsync(c->clf_cnt + G + 2, 0, sizeof(int32_t), c->stream));
  hipLaunchKernelGGL(k_clfused_quanta, dim3(1), dim3(64), 0, c->stream, tile, beta, c->p,
                     std::max<int64_t>(c->n_kept, 1), c->clf_cnt + G + 1, c->clf_fq);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

// the fused pass's sums -> meat (S'S) and cluster count; 1: its bound flag is up (redo from score rows)
static int cluster_fused_finish(lfe_ctx* c, double* meat, int64_t* G_out, int* redo) {
  const int k = c->score_k, G = c->fe[c->L.P].G;
  *redo = 0;
  if (c->clfused_done) {  // asked again after the same pass
    std::copy(c->clfused_meat.begin(), c->clfused_meat.end(), meat);
    *G_out = c->clfused_G;
    return LFE_OK;
  }
  int32_t hc[3] = {0, 0, 0};
  // owner-sharded ranks: clusters present and the bound flag over all ranks (the redo is everyone's)
  LFE_TRY(allreduce_sum_i32(c, c->clf_cnt + G, 1));
  LFE_TRY(allreduce_max_i32(c, c->clf_cnt + G + 2, 1));
  LFE_TRY(d2h_sync(c, hc, c->clf_cnt + G, sizeof(hc)));
  *redo = hc[2] != 0;
  if (*redo) return LFE_OK;
  {
    ProfScope _ps(c, K_CLUSTER_FIX);
    LFE_TRY(launch_fix_convert(c, c->clf_S, c->clf_hi, (int64_t)G * k, k, c->clf_fq));
  }
  *G_out = hc[0];
  LFE_TRY(launch_table_gram(c, c->clf_S, G, k, meat));
  c->clfused_meat.assign(meat, meat + (size_t)k * k);
  c->clfused_G = hc[0];
  c->clfused_done = true;
  return LFE_OK;
}

int launch_codes_differ(lfe_ctx* c, const int32_t* a, const int32_t* b, int64_t n, int32_t* flag) {
  if (n > 0) hipLaunchKernelGGL(k_cl_same, dim3(grid_for(n, 256, 2048)), dim3(256), 0, c->stream, a, b, n, flag);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

// meat and cluster count of one subset (mask over the loaded cluster columns)
static int subset_meat(lfe_ctx* c, int mask, double* meat, int64_t* G_out) {
  if (c->clfused) {  // the residual pass summed the cluster column that repeats the primary FE
    int redo = 0;
    if (c->clfused_j >= 0 && mask == 1 << c->clfused_j) {
      LFE_TRY(cluster_fused_finish(c, meat, G_out, &redo));
      if (!redo) return LFE_OK;
    }
    // a subset the pass did not sum (from its score rows, if it wrote them), or a value past the
    // fused quanta's bound: the pass again, writing score rows
    if (redo || !c->clfused_scores) {
      double st[4];
      LFE_TRY(launch_resid(c, c->clfused_beta.data(), st, nullptr, 1, 0));
    }
  }
  const int k = c->score_k;
  const int64_t n = c->n;
  auto& W = c->clw;
  if (clfix_on() && !(c->test_hooks & LFE_TEST_CLUSTER_SORTED) && __builtin_popcount((unsigned)mask) == 1 && k >= 1 &&
      k <= 63 && c->L.n_items > 0) {
    // one column: the sort-free sums when its table window fits in LDS - the whole table (few
    // clusters), or the bucket slice when the column is the primary FE; all-reduced whole across
    // ranks up to 64 MB.  Otherwise the sorted path below (global atomics per score value were
    // measured slower than the sort: 4.7 vs 2.5 ms on config 4's 1e5-level column, round 5)
    const int j = __builtin_ctz((unsigned)mask);
    const int64_t G = c->cl_levels[j];
    const bool own = owner_col(c, mask) == j;
    if (c->world == 1 || own || G * k * 8 <= (64ll << 20)) {
      int win = 0;
      bool bucketed = false;
      if ((size_t)G * k * 8 <= kClFixLds) {
        win = (int)G;
      } else if ((c->world == 1 || own) && c->L.permuted && c->L.P >= 0 && j < (int)c->cl_fe.size() &&
                 c->cl_fe[j] == c->L.P && ((size_t)8 << c->L.s) * k <= kClFixLds) {
        bucketed = true;  // the column repeats the primary FE (lfe_load_clusters compared them)
        win = 1 << c->L.s;
      }
      const bool stats_env = [] {  // "1": quanta from the statistics pass (A/B, tests)
        const char* e = knob("LFE_CL_STATS");
        return e && e[0] == '1';
      }();
      if (win > 0)
        return subset_meat_fix(c, j, win, bucketed, meat, G_out,
                               stats_env || (c->test_hooks & LFE_TEST_CLUSTER_STATS) != 0, own);
    }
    // a column that repeats an FE of the general sweeps: that FE's segment layout
    const int f = j < (int)c->cl_fe.size() ? c->cl_fe[j] : -1;
    if (c->world == 1 && f >= 0 && f < c->F && c->seg_ready && c->fe[f].perm_ok && c->fe[f].G == G)
      return subset_meat_seg(c, f, meat, G_out);
  }
  KeyArgs ka{};
  uint64_t span = 1;
  for (int j = 0; j < (int)c->cl.size(); ++j) {
    if (!(mask >> j & 1)) continue;
    if (ka.m == kMaxCl) return fail(LFE_EINVAL, "too many cluster columns in one subset");
    const uint64_t g = (uint64_t)c->cl_levels[j];
    if (span > ((1ull << 62) / g)) return fail(LFE_EINVAL, "cluster intersection span exceeds 2^62");
    ka.code[ka.m] = W.lay[j];
    ka.mult[ka.m] = span;  // key = c_0 + G_0 (c_1 + G_1 (...)): any injective mixed radix groups the same rows
    ++ka.m;
    span *= g;
  }
  ka.keep = c->L.P >= 0 ? c->L.code[c->L.P] : nullptr;
  ka.n = n;
  ka.drop = span;
  ka.keys = W.keys[0];
  ka.rows = W.rows[0];
  ka.pj = -1;
  int sort_bits = bit_length(span);
  // one process, a column that repeats the primary FE: the layout's bucket order already sorts the
  // key's top part (HDFE_CLUSTER2, MEGA_CLUSTER2: 4 -> 3 radix passes).  Dropped rows take the low
  // part past every kept row's, so they end the sorted order as one run.
  const bool own = owner_col(c, mask) >= 0;  // every cluster of the subset on one rank
  if ((c->world == 1 || own) && c->L.permuted && c->L.P >= 0 && ka.m >= 2 && !(c->test_hooks & LFE_TEST_CLUSTER_SORTED)) {
    int jp = -1, kj = 0;
    for (int j = 0; j < (int)c->cl.size(); ++j) {
      if (!(mask >> j & 1)) continue;
      if (jp < 0 && j < (int)c->cl_fe.size() && c->cl_fe[j] == c->L.P && c->cl_levels[j] == c->fe[c->L.P].G) jp = kj;
      ++kj;
    }
    if (jp >= 0) {
      uint64_t other = 1;  // product of the other columns' levels
      kj = 0;
      for (int j = 0; j < (int)c->cl.size(); ++j) {
        if (!(mask >> j & 1)) continue;
        if (kj != jp) other *= (uint64_t)c->cl_levels[j];
        ++kj;
      }
      const int s = c->L.s;
      const uint64_t lmax = (other << s);  // low parts < lmax; dropped rows: exactly lmax
      // whole 8-bit digits: the sort's last digit must not reach into the bucket part (else a kept
      // row's low bucket bits would order it after the dropped rows)
      const int lbits = (bit_length(lmax) + 7) / 8 * 8;
      const uint64_t nb = (uint64_t)c->L.nb;
      if ((lbits + 7) / 8 < (sort_bits + 7) / 8 && lbits + bit_length(nb) <= 62) {
        // mixed radix of the other columns as before (their multipliers skip the primary's), the
        // primary's low bits above them
        uint64_t mul = 1;
        kj = 0;
        for (int j = 0; j < (int)c->cl.size(); ++j) {
          if (!(mask >> j & 1)) continue;
          if (kj != jp) {
            ka.mult[kj] = mul;
            mul *= (uint64_t)c->cl_levels[j];
          }
          ++kj;
        }
        ka.mult[jp] = other;
        ka.pj = jp;
        ka.ps = s;
        ka.pshift = lbits;
        ka.drop = lmax;
        sort_bits = lbits;
      }
    }
  }
  const uint64_t drop = ka.drop;
  if (n > 0) hipLaunchKernelGGL(k_cl_keys, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, ka);
  LFE_HIP(hipGetLastError());

  int buf = 0;
  if (n > 0) LFE_TRY(radix_sort(c, n, sort_bits, &buf));
  int32_t G = 0, nv = 0;
  LFE_TRY(group_segments(c, n, drop, W.keys[buf], &G, &nv));
  // one process, unweighted, mostly singletons (mean cluster size below 2): D + the multi-row
  // clusters' corrections, without gathering every row
  if (c->world == 1 && k > 0 && c->score_meat_ok && (int)c->score_meat.size() == k * k && G > 0 &&
      2 * (int64_t)G > (int64_t)nv && knob("LFE_CL_NO_SINGLETON") == nullptr) {
    *G_out = G;
    return singleton_meat(c, W.rows[buf], G, k, meat);
  }
  if (k > 0) LFE_TRY(group_sums(c, n, drop, W.keys[buf], W.rows[buf], c->scores, k, G, nv));
  if (own) {  // owner-local: this rank's clusters are whole; the meat and the count summed over ranks
    LFE_TRY(sum_over_ranks(c, G, G_out));
    if (k == 0) return LFE_OK;
    return launch_table_gram(c, c->clS, G, k, meat);
  }

  // multi-rank, few clusters: a key-indexed table, all-reduced (smaller than the exchange)
  const char* own_env = knob("LFE_CL_OWNER_MIN_SPAN");  // tests: force the owner-partitioned form
  const uint64_t owner_min = own_env ? (uint64_t)atoll(own_env) : ((64ull << 20) / (8ull * std::max(k, 1)));
  if (c->world > 1 && span < owner_min && span < (1ull << 31)) {
    const int32_t C = (int32_t)span;
    LFE_TRY(ensure_cluster_ws(c, (size_t)std::max(G, 1) * std::max(k, 1), (size_t)C + 4));
    LFE_TRY(ensure_f64(c, W.srec, W.srec_cap, (size_t)C * std::max(k, 1)));
    double* S = W.srec;  // the key-indexed table (the exchange's send buffer is idle here)
    int32_t* present = c->clP;
    int32_t* cntG = present + C;
    LFE_HIP(hipMemsetAsync(S, 0, sizeof(double) * (size_t)C * std::max(k, 1), c->stream));
    LFE_HIP(hipMemsetAsync(present, 0, sizeof(int32_t) * ((size_t)C + 4), c->stream));
    if (G > 0) {
      ProfScope _ps(c, K_CLUSTER_SCATTER);
      hipLaunchKernelGGL(k_cl_dense_put, dim3(grid_for((int64_t)G * std::max(k, 1))), dim3(kBlock), 0, c->stream,
                         W.keys[buf], W.seg_off, G, c->clS, k, S, present);
    }
    LFE_HIP(hipGetLastError());
    LFE_TRY(allreduce_sum_f64(c, S, (size_t)C * k));
    LFE_TRY(allreduce_sum_i32(c, present, C));
    hipLaunchKernelGGL(k_count_nonzero, dim3(grid_for(C, 256, 1024)), dim3(256), 0, c->stream, present, C, cntG);
    LFE_HIP(hipGetLastError());
    int32_t hG = 0;
    LFE_TRY(d2h_sync(c, &hG, cntG, sizeof(int32_t)));
    *G_out = hG;
    if (k > 0) {
      const int world = c->world;  // S is replicated after the all-reduce: reduce its Gram locally
      c->world = 1;
      const int rc = launch_table_gram(c, S, C, k, meat);
      c->world = world;
      if (rc) return rc;
    }
    return LFE_OK;
  }
  if (c->world > 1) return owner_meat(c, W.keys[buf], W.seg_off, c->clS, G, k, span, meat, G_out);
  *G_out = G;
  if (k == 0) return LFE_OK;
  return launch_table_gram(c, c->clS, G, k, meat);
}

int launch_cluster_subsets(lfe_ctx* c, int n_subsets, const int32_t* masks, double* meats, int64_t* G_out) {
  const int k = c->score_k;
  const int64_t n = c->n;
  const int m = (int)c->cl.size();
  for (int s = 0; s < n_subsets; ++s)
    if (masks[s] <= 0 || masks[s] >= (1 << m)) return fail(LFE_EINVAL, "subset mask must select loaded cluster columns");
  auto& W = c->clw;
  const size_t ld = (size_t)c->ld;
  LFE_TRY(ensure_sort_ws(c, ld));
  LFE_TRY(ensure_i32(c, W.seg_off, W.seg_off_cap, ld + 1));
  LFE_TRY(ensure_i32(c, W.ufirst, W.ufirst_cap, (size_t)seg_units_needed(c->ld)));
  if (!W.lay_valid) {
    LFE_TRY(ensure_layout_orig(c));
    W.lay.resize(m, nullptr);
    W.lay_cap.resize(m, 0);
    for (int j = 0; j < m; ++j) {
      LFE_TRY(ensure_i32(c, W.lay[j], W.lay_cap[j], ld));
      if (n > 0)
        hipLaunchKernelGGL(k_cl_layout, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, c->cl[j],
                           c->L.orig, n, W.lay[j]);
      LFE_HIP(hipGetLastError());
    }
    W.lay_valid = true;
  }
  W.segst_ok = false;  // (subset_meat_seg: the score rows' statistics, formed by the first subset)
  for (int s = 0; s < n_subsets; ++s)
    LFE_TRY(subset_meat(c, masks[s], meats + (size_t)s * k * k, G_out + s));
  return LFE_OK;
}

void free_cluster_ws(lfe_ctx* c) {
  auto& W = c->clw;
  dfree_any(W.fixst);
  dfree_any(W.rsum);
  W.rsum_cap = 0;
  dfree_any(W.fixq);
  dfree_any(W.segst);
  W.fixst_cap = W.fixq_cap = W.segst_cap = 0;
  W.segst_ok = false;
  for (int b = 0; b < 2; ++b) {
    dfree_any(W.keys[b]);
    dfree_any(W.rows[b]);
    W.keys_cap[b] = W.rows_cap[b] = 0;
  }
  dfree_any(W.counts);
  dfree_any(W.flag);
  dfree_any(W.seg_off);
  dfree_any(W.ufirst);
  W.counts_cap = W.flag_cap = W.seg_off_cap = W.ufirst_cap = 0;
  for (auto& p : W.lay) dfree_any(p);
  W.lay.clear();
  W.lay_cap.clear();
  W.lay_valid = false;
}

}  // namespace lfe

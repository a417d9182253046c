// leanfe HIP engine — alternating projections for two fixed effects, the
// headline case (polars_impl.py:490-526, strategy 'alt_proj', unweighted).
//
// alpha-form sweep, order [Q, P] (ascending cardinality, polars_impl.py:476-480):
//     T_P[h]   = sum_{i in h} alpha_Q[q_i]            (K1)
//     alpha_P  = (S_P - T_P) / n_P                     projection of P
//     T_Q'[q]  = sum_{i in q} alpha_P[h_i]            (K2)
//     alpha_Q' = (S_Q - T_Q') / n_Q                    next sweep's Q projection
// The stop test after a sweep (max_g |mean_g(y~)|, y only, polars_impl.py:511-521)
// is exactly |alpha_Q' - alpha_Q| on the y column (0 for the just-projected P),
// so it costs nothing extra.
//
// Both cross terms are segmented sums over a codes-only row layout, so neither
// pass needs a per-row atomic (per-row LDS f64 atomics bound the earlier
// version at ~2.7 lane-ops/clk/CU):
//   segment layout: kept rows of each bucket sorted by the primary code h;
//                   per row the secondary code q (int32).  K1: per segment,
//                   gather alpha_Q[q] rows from an LDS copy of alpha_Q.
//   run layout:     kept rows of each bucket sorted by q; per row h - lo
//                   (uint16).  K2: per (bucket, q) run, gather alpha_P rows
//                   from the bucket's LDS slice; one global atomic add per run
//                   and column (nb * G_Q runs, ~1/128 of the rows here).
// Both passes use the MFMA lane layout of the Gram kernels (lane = row quad x
// column): a 16-row group is one aligned int4 / ushort4 load per lane and four
// conflict-free LDS row gathers; rows outside the current segment/run index a
// zero row of the LDS table, so nothing is predicated.  Codes are loaded a
// batch of groups ahead.  Multi-GPU: T_P (when P's projection needs the
// all-reduce) and T_Q are reduced over ranks between the passes.
#include "lfe_internal.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>

namespace lfe {

// ===========================================================================
// 1. bucket-local counting sort (segment and run layouts)
// ===========================================================================
// Key of a kept row: KEYQ ? its secondary code : its primary code - lo (the
// offset in its bucket); value stored: the other one.  Deterministic: per-wave
// 16-bit cursors, rows ranked within a wave from ballots (as in the partition
// scatter of lfe_prep.hip), never by the return order of LDS atomics.

// both layouts' per-item histograms in one pass over the codes: itemcnt1[item][h - lo]
// (K1 = 2^s keys) and itemcnt2[item][q] (K2 = G_Q keys)
__global__ __launch_bounds__(256) void k_ls_hist2(const int4* __restrict__ items, const int32_t* __restrict__ codeP,
                                                  const int32_t* __restrict__ codeQ, int s, int K1, int K2,
                                                  int32_t* __restrict__ cnt1, int32_t* __restrict__ cnt2) {
  extern __shared__ int32_t h[];
  int32_t* h1 = h;
  int32_t* h2 = h + K1;
  const int4 it = items[blockIdx.x];
  const int lo = it.x << s;
  for (int j = threadIdx.x; j < K1 + K2; j += blockDim.x) h[j] = 0;
  __syncthreads();
  // 16-byte code loads over the 4-aligned middle of the item, scalar at its two ends
  const int32_t a0 = min(it.z, (it.y + 3) & ~3), a1 = max(a0, it.z & ~3);
  auto one = [&](int32_t g, int32_t q) {
    if (g >= 0) {
      atomicAdd(&h1[g - lo], 1);
      atomicAdd(&h2[q], 1);
    }
  };
  for (int32_t i = it.y + threadIdx.x; i < a0; i += blockDim.x) one(codeP[i], codeQ[i]);
  for (int32_t i = a0 + 4 * threadIdx.x; i < a1; i += 4 * blockDim.x) {
    const int4 g = *reinterpret_cast<const int4*>(codeP + i);
    const int4 q = *reinterpret_cast<const int4*>(codeQ + i);
    one(g.x, q.x);
    one(g.y, q.y);
    one(g.z, q.z);
    one(g.w, q.w);
  }
  for (int32_t i = a1 + threadIdx.x; i < it.z; i += blockDim.x) one(codeP[i], codeQ[i]);
  __syncthreads();
  for (int j = threadIdx.x; j < K1; j += blockDim.x) cnt1[(int64_t)blockIdx.x * K1 + j] = h1[j];
  for (int j = threadIdx.x; j < K2; j += blockDim.x) cnt2[(int64_t)blockIdx.x * K2 + j] = h2[j];
}

// per (bucket, key): exclusive scan over the bucket's items -> item bases; total -> off[b K + key]
__device__ __forceinline__ void ls_base_one(const int32_t* __restrict__ bitems, int nb, int K,
                                            int32_t* __restrict__ itemcnt, int32_t* __restrict__ off, int64_t e) {
  if (e == (int64_t)nb * K) {  // the scan's trailing element (the total after the exclusive scan)
    off[e] = 0;
    return;
  }
  const int b = (int)(e / K), j = (int)(e % K);
  int32_t run = 0;
  // eight items' counts loaded before any is rewritten (the chain is latency-bound otherwise)
  for (int i = bitems[b], i1 = bitems[b + 1]; i < i1; i += 8) {
    int32_t t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = i + u < i1 ? itemcnt[(int64_t)(i + u) * K + j] : 0;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (i + u < i1) {
        itemcnt[(int64_t)(i + u) * K + j] = run;
        run += t[u];
      }
  }
  off[e] = run;
}

__global__ void k_ls_base(const int32_t* __restrict__ bitems, int nb, int K, int32_t* __restrict__ itemcnt,
                          int32_t* __restrict__ off) {
  const int64_t total = (int64_t)nb * K;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e <= total; e += (int64_t)gridDim.x * blockDim.x)
    ls_base_one(bitems, nb, K, itemcnt, off, e);
}

// both layouts' item bases and key totals in one launch (the fused sort)
__global__ void k_ls_base2(const int32_t* __restrict__ bitems, int nb, int K1, int32_t* __restrict__ cnt1,
                           int32_t* __restrict__ off1, int K2, int32_t* __restrict__ cnt2, int32_t* __restrict__ off2) {
  const int64_t t1 = (int64_t)nb * K1 + 1, t2 = (int64_t)nb * K2 + 1;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < t1 + t2; e += (int64_t)gridDim.x * blockDim.x) {
    if (e < t1) ls_base_one(bitems, nb, K1, cnt1, off1, e);
    else ls_base_one(bitems, nb, K2, cnt2, off2, e - t1);
  }
}

constexpr int kLsThreads = 512;
constexpr int kLsWaves = kLsThreads / 64;
// rows per thread of the local sorts (16 rows, one 8192-row item per pass and one workgroup per
// CU: 0.575 vs 0.51 ms for the layout phase)
constexpr int kLsPer = 8;
static int ls_per() { return kLsPer; }

static __host__ __device__ inline int even(int K) { return (K + 1) & ~1; }  // 16-bit counter rows in words


// LDS of the single-layout sort: per-wave 16-bit counters [kLsWaves][K], run / tot / delta [K],
// the stage [kLsRows]
static size_t ls_scatter_lds(int K, int per = 16) {
  return sizeof(int32_t) * (3 * (size_t)K + (size_t)kLsThreads * per) + sizeof(uint16_t) * kLsWaves * (size_t)even(K);
}

// Deterministic ranking of a sub-chunk's rows by key (both local sorts).  Every wave has its
// own 16-bit counter per key (two per 32-bit word), so a row's slot is its wave's first slot
// for the key (ls_offsets_n) + the counter value its returning LDS add got.  The adds of one wave
// are issued in slot order without waits in between (lanes without a key add 0 to the wave's
// spare word), a wave's LDS operations complete in issue order, and the lanes of one
// instruction that hit the same counter are served in the LDS's fixed lane order; no other
// wave touches the counters, so the layout - and with it the summation order of every
// segmented sum over it - does not depend on how the waves are scheduled.  (Matching the
// lanes of a key with one ballot per key bit, as the partition scatter does for its 8-bit
// bucket ids, costs ~15 VALU ops per bit and row: 1.06 vs 0.33 ms for this kernel.)
template <int PER>
__device__ __forceinline__ void wave_rank(const int32_t (&key)[PER], uint32_t* cw, uint32_t* spare,
                                          int32_t (&rank)[PER]) {
  uint32_t old[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const bool act = key[k] >= 0;
    const int sh = (key[k] & 1) << 4;
    old[k] = atomicAdd(act ? &cw[key[k] >> 1] : spare, act ? (1u << sh) : 0u);
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) rank[k] = (int32_t)((old[k] >> ((key[k] & 1) << 4)) & 0xffffu);
}

// per key j < K (cw: [kLsWaves][Kp] 16-bit counters): cw[w][j] <- the first slot of wave w's rows with key j in the sub-chunk,
// delta[j] <- run[j] - (the key's first slot); the keys' offsets are an exclusive scan of the
// totals (one thread per `per` keys, then the waves).  NS key sets (the fused sort's two
// layouts) share the barriers, and a key's eight wave counters are read before any is rewritten
// (one LDS round trip per pass, not a dependent chain of eight).
struct LsKeys {
  uint16_t* cw;
  int Kp;
  int32_t* tot;
  const int32_t* run;
  int32_t* delta;
  int K;
};
template <int NS>
__device__ void ls_offsets_n(const LsKeys (&ks)[NS], int32_t (*wsum)[kLsWaves], int tid, int lane, int wave) {
#pragma unroll
  for (int S = 0; S < NS; ++S) {
    const LsKeys& k = ks[S];
    for (int j = tid; j < k.K; j += kLsThreads) {
      uint16_t h[kLsWaves];
#pragma unroll
      for (int w2 = 0; w2 < kLsWaves; ++w2) h[w2] = k.cw[w2 * k.Kp + j];
      int32_t t = 0;
#pragma unroll
      for (int w2 = 0; w2 < kLsWaves; ++w2) {
        k.cw[w2 * k.Kp + j] = (uint16_t)t;
        t += h[w2];
      }
      k.tot[j] = t;
    }
  }
  __syncthreads();
  int32_t x[NS], sum[NS];
#pragma unroll
  for (int S = 0; S < NS; ++S) {
    const LsKeys& k = ks[S];
    const int per = (k.K + kLsThreads - 1) / kLsThreads;
    const int b0 = tid * per;
    sum[S] = 0;
    for (int q = 0; q < per; ++q)
      if (b0 + q < k.K) sum[S] += k.tot[b0 + q];
    x[S] = sum[S];
  }
  for (int o = 1; o < 64; o <<= 1) {
#pragma unroll
    for (int S = 0; S < NS; ++S) {
      const int32_t y = __shfl_up(x[S], o, 64);
      if (lane >= o) x[S] += y;
    }
  }
#pragma unroll
  for (int S = 0; S < NS; ++S)
    if (lane == 63) wsum[S][wave] = x[S];
  __syncthreads();
#pragma unroll
  for (int S = 0; S < NS; ++S) {
    const LsKeys& k = ks[S];
    const int per = (k.K + kLsThreads - 1) / kLsThreads;
    const int b0 = tid * per;
    int32_t wofs = 0;
    for (int w2 = 0; w2 < wave; ++w2) wofs += wsum[S][w2];
    int32_t acc = x[S] - sum[S] + wofs;
    for (int q = 0; q < per; ++q)
      if (b0 + q < k.K) {
        const int32_t t = k.tot[b0 + q];
        k.tot[b0 + q] = acc;
        acc += t;
      }
  }
  __syncthreads();
#pragma unroll
  for (int S = 0; S < NS; ++S) {
    const LsKeys& k = ks[S];
    for (int j = tid; j < k.K; j += kLsThreads) {
      const int32_t boff = k.tot[j];
      k.delta[j] = k.run[j] - boff;
      uint16_t h[kLsWaves];
#pragma unroll
      for (int w2 = 0; w2 < kLsWaves; ++w2) h[w2] = k.cw[w2 * k.Kp + j];
#pragma unroll
      for (int w2 = 0; w2 < kLsWaves; ++w2) k.cw[w2 * k.Kp + j] = (uint16_t)(h[w2] + boff);
    }
  }
  __syncthreads();
}

// kept rows of the wave's sub-chunk slice -> wkept[wave] (lane 0)
template <int PER>
__device__ __forceinline__ void wave_kept(const int32_t (&key)[PER], int lane, int wave, int32_t* wkept) {
  int cnt = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) cnt += __popcll(__ballot(key[k] >= 0));
  if (lane == 0) wkept[wave] = cnt;
}

// one layout (the fallback when both do not fit in LDS together): KEYQ ? the run layout (key q,
// value h - lo) : the segment layout (key h - lo, value q)
template <bool KEYQ, typename VT, int kLsPer>
__global__ __launch_bounds__(kLsThreads) void k_ls_scatter(const int4* __restrict__ items,
                                                           const int32_t* __restrict__ codeP,
                                                           const int32_t* __restrict__ codeQ, int s, int K,
                                                           const int32_t* __restrict__ off,
                                                           const int32_t* __restrict__ itembase,
                                                           const int32_t* __restrict__ xitems,
                                                           VT* __restrict__ out) {
  constexpr int kLsRows = kLsThreads * kLsPer;
  extern __shared__ int32_t sm[];
  int32_t* run = sm;             // [K] next free slot of each key
  int32_t* tot = run + K;        // [K]
  int32_t* delta = tot + K;      // [K]
  int32_t* stage = delta + K;    // [kLsRows] slot keys, then slot values
  const int Kp = even(K);
  uint16_t* cw = reinterpret_cast<uint16_t*>(stage + kLsRows);  // [kLsWaves][Kp]
  __shared__ int32_t wsum[kLsWaves], wkept[kLsWaves];
  __shared__ uint32_t spare[kLsWaves];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int item = xitems[blockIdx.x];  // XCD-grouped order (build_items)
  if (item < 0) return;
  const int4 it = items[item];
  const int lo = it.x << s;
  for (int j = tid; j < K; j += kLsThreads)
    run[j] = off[(int64_t)it.x * K + j] + itembase[(int64_t)item * K + j];
  // sub-chunks start at multiples of 4 rows and slots k .. k + 3 of a lane are 4 consecutive
  // rows, so the codes come in 16-byte loads (rows before it.y are masked)
  static_assert(kLsPer % 4 == 0, "rows per thread in fours");
  for (int32_t r0 = it.y & ~3; r0 < it.z; r0 += kLsRows) {
    const int32_t r1 = min(it.z, r0 + kLsRows);
    const int32_t wbase = r0 + wave * kLsPer * 64;
    __syncthreads();
    for (int j = tid; j < kLsWaves * Kp / 2; j += kLsThreads) reinterpret_cast<uint32_t*>(cw)[j] = 0u;
    __syncthreads();
    int32_t key[kLsPer], val[kLsPer];
#pragma unroll
    for (int k = 0; k < kLsPer; k += 4) {
      const int32_t i0 = wbase + (k >> 2) * 256 + 4 * lane;
      int4 g4 = int4{-1, -1, -1, -1}, q4 = int4{0, 0, 0, 0};
      if (i0 < r1) {
        g4 = *reinterpret_cast<const int4*>(codeP + i0);
        q4 = *reinterpret_cast<const int4*>(codeQ + i0);
      }
      const int32_t gv[4] = {g4.x, g4.y, g4.z, g4.w}, qv[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int32_t i = i0 + t;
        key[k + t] = -1;
        val[k + t] = 0;
        if (i >= it.y && i < r1 && gv[t] >= 0) {
          key[k + t] = KEYQ ? qv[t] : gv[t] - lo;
          val[k + t] = KEYQ ? gv[t] - lo : qv[t];
        }
      }
    }
    int32_t pos[kLsPer];
    wave_rank(key, reinterpret_cast<uint32_t*>(cw + wave * Kp), &spare[wave], pos);
    wave_kept(key, lane, wave, wkept);
    __syncthreads();
    {
      const LsKeys ks[1] = {{cw, Kp, tot, run, delta, K}};
      ls_offsets_n<1>(ks, reinterpret_cast<int32_t(*)[kLsWaves]>(wsum), tid, lane, wave);
    }
    int32_t nk = 0;  // kept rows of this sub-chunk
    for (int w2 = 0; w2 < kLsWaves; ++w2) nk += wkept[w2];
#pragma unroll
    for (int k = 0; k < kLsPer; ++k)
      if (key[k] >= 0) {
        pos[k] += cw[wave * Kp + key[k]];
        stage[pos[k]] = key[k];
      }
    __syncthreads();
    // each thread keeps the destinations of the slots it writes out (j = tid + k * threads)
    int32_t dd[kLsPer];
#pragma unroll
    for (int k = 0; k < kLsPer; ++k) {
      const int j = tid + k * kLsThreads;
      dd[k] = j < nk ? delta[stage[j]] + j : -1;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kLsPer; ++k)
      if (key[k] >= 0) stage[pos[k]] = val[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kLsPer; ++k)
      if (dd[k] >= 0) out[dd[k]] = (VT)stage[tid + k * kLsThreads];
    __syncthreads();
    // next sub-chunk: each key continues after this one's rows (its end = the next key's start)
    for (int j = tid; j < K; j += kLsThreads) run[j] = delta[j] + (j + 1 < K ? tot[j + 1] : nk);
  }
}

// Both layouts in one pass over the codes: the segment layout (key h - lo, value q -> seg_q)
// and the run layout (key q, value h - lo -> run_h) of the same sub-chunk, ranked with the
// same deterministic wave ranking as k_ls_scatter, so the two code columns are read once.
struct Ls2Args {
  const int4* items;
  const int32_t* codeP;
  const int32_t* codeQ;
  int s, K1, K2;
  const int32_t* off1;   // [nb K1 + 1]
  const int32_t* off2;   // [nb K2 + 1]
  const int32_t* base1;  // [n_items][K1] item bases
  const int32_t* base2;  // [n_items][K2]
  const int32_t* xitems;
  int32_t* seg_q;
  uint16_t* run_h;
};

static size_t ls2_lds(int K1, int K2, int per) {
  return sizeof(int32_t) * (3 * ((size_t)K1 + K2) + 2 * (size_t)kLsThreads * per) +
         sizeof(uint16_t) * kLsWaves * ((size_t)even(K1) + even(K2));
}

template <int kLsPer>
// (4 waves per SIMD, <= 128 VGPRs: two workgroups per CU, as the LDS allows)
__global__ __launch_bounds__(kLsThreads, 4) void k_ls_scatter2(Ls2Args a) {
  constexpr int kLsRows = kLsThreads * kLsPer;
  extern __shared__ int32_t sm[];
  const int K1 = a.K1, K2 = a.K2;
  int32_t* run1 = sm;           // [K1] next free slot of each key
  int32_t* run2 = run1 + K1;    // [K2]
  int32_t* tot1 = run2 + K2;    // [K1] the keys' local offsets
  int32_t* tot2 = tot1 + K1;    // [K2]
  int32_t* del1 = tot2 + K2;    // [K1]
  int32_t* del2 = del1 + K1;    // [K2]
  int32_t* st1 = del2 + K2;     // [kLsRows]
  int32_t* st2 = st1 + kLsRows; // [kLsRows]
  const int K1p = even(K1), K2p = even(K2);
  uint16_t* cw1 = reinterpret_cast<uint16_t*>(st2 + kLsRows);  // [kLsWaves][K1p]
  uint16_t* cw2 = cw1 + kLsWaves * K1p;                         // [kLsWaves][K2p]
  __shared__ int32_t wsum[2][kLsWaves], wkept[kLsWaves];
  __shared__ uint32_t spare[kLsWaves];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int item = a.xitems[blockIdx.x];  // XCD-grouped order (build_items)
  if (item < 0) return;
  const int4 it = a.items[item];
  const int lo = it.x << a.s;
  for (int j = tid; j < K1; j += kLsThreads)
    run1[j] = a.off1[(int64_t)it.x * K1 + j] + a.base1[(int64_t)item * K1 + j];
  for (int j = tid; j < K2; j += kLsThreads)
    run2[j] = a.off2[(int64_t)it.x * K2 + j] + a.base2[(int64_t)item * K2 + j];
  static_assert(kLsPer % 4 == 0, "rows per thread in fours");
  for (int32_t r0 = it.y & ~3; r0 < it.z; r0 += kLsRows) {
    const int32_t r1 = min(it.z, r0 + kLsRows);
    const int32_t wbase = r0 + wave * kLsPer * 64;
    __syncthreads();
    for (int j = tid; j < kLsWaves * (K1p + K2p) / 2; j += kLsThreads) reinterpret_cast<uint32_t*>(cw1)[j] = 0u;
    __syncthreads();
    int32_t hk[kLsPer], qk[kLsPer];  // h - lo (key of layout 1) and q (key of layout 2); -1: not kept
#pragma unroll
    for (int k = 0; k < kLsPer; k += 4) {
      const int32_t i0 = wbase + (k >> 2) * 256 + 4 * lane;
      int4 g4 = int4{-1, -1, -1, -1}, q4 = int4{0, 0, 0, 0};
      if (i0 < r1) {
        g4 = *reinterpret_cast<const int4*>(a.codeP + i0);
        q4 = *reinterpret_cast<const int4*>(a.codeQ + i0);
      }
      const int32_t gv[4] = {g4.x, g4.y, g4.z, g4.w}, qv[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int32_t i = i0 + t;
        const bool kept = i >= it.y && i < r1 && gv[t] >= 0;
        hk[k + t] = kept ? gv[t] - lo : -1;
        qk[k + t] = kept ? qv[t] : -1;
      }
    }
    int32_t p1[kLsPer], p2[kLsPer];
    wave_rank(hk, reinterpret_cast<uint32_t*>(cw1 + wave * K1p), &spare[wave], p1);
    wave_rank(qk, reinterpret_cast<uint32_t*>(cw2 + wave * K2p), &spare[wave], p2);
    wave_kept(hk, lane, wave, wkept);
    __syncthreads();
    {
      const LsKeys ks[2] = {{cw1, K1p, tot1, run1, del1, K1}, {cw2, K2p, tot2, run2, del2, K2}};
      ls_offsets_n<2>(ks, wsum, tid, lane, wave);
    }
    int32_t nk = 0;  // kept rows of this sub-chunk
    for (int w2 = 0; w2 < kLsWaves; ++w2) nk += wkept[w2];
#pragma unroll
    for (int k = 0; k < kLsPer; ++k)
      if (hk[k] >= 0) {
        p1[k] += cw1[wave * K1p + hk[k]];
        p2[k] += cw2[wave * K2p + qk[k]];
        st1[p1[k]] = hk[k];
        st2[p2[k]] = qk[k];
      }
    __syncthreads();
    int32_t d1[kLsPer], d2[kLsPer];
#pragma unroll
    for (int k = 0; k < kLsPer; ++k) {
      const int j = tid + k * kLsThreads;
      d1[k] = j < nk ? del1[st1[j]] + j : -1;
      d2[k] = j < nk ? del2[st2[j]] + j : -1;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kLsPer; ++k)
      if (hk[k] >= 0) {
        st1[p1[k]] = qk[k];
        st2[p2[k]] = hk[k];
      }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kLsPer; ++k) {
      if (d1[k] >= 0) a.seg_q[d1[k]] = st1[tid + k * kLsThreads];
      if (d2[k] >= 0) a.run_h[d2[k]] = (uint16_t)st2[tid + k * kLsThreads];
    }
    __syncthreads();
    for (int j = tid; j < K1; j += kLsThreads) run1[j] = del1[j] + (j + 1 < K1 ? tot1[j + 1] : nk);
    for (int j = tid; j < K2; j += kLsThreads) run2[j] = del2[j] + (j + 1 < K2 ? tot2[j + 1] : nk);
  }
}

// first segment (primary group) of each work unit of ~U kept rows
// first segment of work unit k (H past the last unit): the first h with seg_off[h] >= k U, then
// the first segment from there on that holds rows, so no unit starts with a run of empty segments
// (an owner shard's buckets hold every other rank's levels too)
__device__ __forceinline__ int unit_first(const int32_t* __restrict__ seg_off, int32_t H, int64_t U, int k,
                                          int n_units) {
  if (k >= n_units) return H;
  const int64_t target = (int64_t)k * U;
  int lo = 0, hi = H;  // first h with seg_off[h] >= target
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (seg_off[mid] < target) lo = mid + 1;
    else hi = mid;
  }
  const int32_t t = lo < H ? seg_off[lo] : 0;
  hi = H;
  while (lo < hi) {  // first h with seg_off[h + 1] > t
    const int mid = (lo + hi) >> 1;
    if (seg_off[mid + 1] <= t) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// K1's unit descriptors {first segment h, end segment h1, first row seg_off[h], end row
// seg_off[h1]}: one 16-byte load starts a unit (no dependent segment-offset loads)
__global__ void k_unit_bounds(const int32_t* __restrict__ seg_off, int32_t H, int64_t U, int n_units,
                              int4* __restrict__ desc) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n_units; k += gridDim.x * blockDim.x) {
    const int h = unit_first(seg_off, H, U, k, n_units), h1 = unit_first(seg_off, H, U, k + 1, n_units);
    desc[k] = int4{h, h1, seg_off[h], seg_off[h1]};
  }
}

// bucket-local counting sort of the kept rows given the per-item histograms
// itemcnt [n_items][K] (k_ls_hist2); off = [nb K + 1] exclusive offsets.  The rows of a
// key are placed in the deterministic wave-ranking order (ls_offsets_n / wave_rank), so the
// summation order of K1 / K2 - and with it every bit of the sweeps - repeats run to run.
template <bool KEYQ, typename VT>
static int local_sort(lfe_ctx* c, int Q, int K, int32_t* itemcnt, int32_t*& off, size_t& off_cap, VT* out) {
  auto& L = c->L;
  const int P = L.P;
  const size_t m = (size_t)L.nb * K;
  LFE_TRY(ensure_i32(c, off, off_cap, m + 1));
  const int4* items = reinterpret_cast<const int4*>(c->items_d);
  {
    ProfScope _ps(c, K_LAYOUT_BASE);
    hipLaunchKernelGGL(k_ls_base, dim3(grid_for((int64_t)m + 1)), dim3(kBlock), 0, c->stream, c->bitems_d, L.nb, K,
                       itemcnt, off);
  }
  LFE_HIP(hipGetLastError());
  if (!out) return LFE_OK;  // per-key totals and item bases only (the fused sort scans both)
  LFE_TRY(exclusive_scan(c, off, (int64_t)m + 1));
  const int per = ls_per();
  const size_t lds = ls_scatter_lds(K, per);
  const void* fn = reinterpret_cast<const void*>(&k_ls_scatter<KEYQ, VT, kLsPer>);
  if (lds > 64 * 1024) LFE_HIP(set_max_lds(fn, (int)lds));
  {
    ProfScope _ps(c, K_LAYOUT_SCATTER);
    hipLaunchKernelGGL((k_ls_scatter<KEYQ, VT, kLsPer>), dim3(c->n_xgrid), dim3(kLsThreads), lds, c->stream,
                       items, L.code[P], L.code[Q], L.s, K, off, itemcnt, c->xitems_d, out);
  }
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

// per-item histograms of both keys in one pass (seg_aux = [n_items][B] ++ [n_items][G_Q]) over
// the rows whose primary code is >= 0 (before the singleton marks: every row)
int layout_hists(lfe_ctx* c, int Q) {
  auto& L = c->L;
  const int B = 1 << L.s;
  const int32_t G_Q = c->fe[Q].G;
  const size_t n1 = (size_t)L.n_items * B;
  LFE_TRY(ensure_i32(c, c->seg_aux, c->seg_aux_cap, n1 + (size_t)L.n_items * G_Q));
  ProfScope _ps(c, K_LAYOUT_HIST);
  hipLaunchKernelGGL(k_ls_hist2, dim3(L.n_items), dim3(256), sizeof(int32_t) * ((size_t)B + G_Q), c->stream,
                     reinterpret_cast<const int4*>(c->items_d), L.code[L.P], L.code[Q], L.s, B, (int)G_Q, c->seg_aux,
                     c->seg_aux + n1);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

static int build_layouts(lfe_ctx* c, int Q) {
  auto& L = c->L;
  const int B = 1 << L.s;
  const int32_t G_Q = c->fe[Q].G;
  const size_t n1 = (size_t)L.n_items * B;
  // the pre-filter histograms of prepare_layout are the kept rows' when nothing was dropped
  // (used once: the local sorts below turn them into item bases)
  if (!c->hists_kept) LFE_TRY(layout_hists(c, Q));
  c->hists_kept = false;
  LFE_TRY(ensure_i32(c, c->seg_q, c->seg_q_cap, (size_t)c->ld));
  LFE_TRY(ensure_u16(c, c->run_h, c->run_h_cap, (size_t)c->ld));
  const int per = ls_per();
  const size_t lds2 = ls2_lds(B, G_Q, per);
  if (lds2 <= 150 * 1024) {
    // both layouts' item bases and key totals, then one scan of both
    const size_t m1 = (size_t)L.nb * B, m2 = (size_t)L.nb * G_Q;
    LFE_TRY(ensure_i32(c, c->seg_off, c->seg_off_cap, m1 + 1));
    LFE_TRY(ensure_i32(c, c->run_off, c->run_off_cap, m2 + 1));
    {
      ProfScope _ps(c, K_LAYOUT_BASE);
      hipLaunchKernelGGL(k_ls_base2, dim3(grid_for((int64_t)(m1 + m2 + 2))), dim3(kBlock), 0, c->stream, c->bitems_d,
                         L.nb, B, c->seg_aux, c->seg_off, (int)G_Q, c->seg_aux + n1, c->run_off);
    }
    LFE_HIP(hipGetLastError());
    LFE_TRY(exclusive_scan2(c, c->seg_off, (int64_t)m1 + 1, c->run_off, (int64_t)m2 + 1));
    Ls2Args a{};
    a.items = reinterpret_cast<const int4*>(c->items_d);
    a.codeP = L.code[L.P];
    a.codeQ = L.code[Q];
    a.s = L.s;
    a.K1 = B;
    a.K2 = G_Q;
    a.off1 = c->seg_off;
    a.off2 = c->run_off;
    a.base1 = c->seg_aux;
    a.base2 = c->seg_aux + n1;
    a.xitems = c->xitems_d;
    a.seg_q = c->seg_q;
    a.run_h = c->run_h;
    const void* fn = reinterpret_cast<const void*>(&k_ls_scatter2<kLsPer>);
    if (lds2 > 64 * 1024) LFE_HIP(set_max_lds(fn, (int)lds2));
    {
      ProfScope _ps(c, K_LAYOUT_SCATTER);
      void* args[] = {&a};
      LFE_HIP(hipLaunchKernel(fn, dim3(c->n_xgrid), dim3(kLsThreads), args, lds2, c->stream));
    }
    LFE_HIP(hipGetLastError());
  } else {
    LFE_TRY((local_sort<false, int32_t>(c, Q, B, c->seg_aux, c->seg_off, c->seg_off_cap, c->seg_q)));
    LFE_TRY((local_sort<true, uint16_t>(c, Q, G_Q, c->seg_aux + n1, c->run_off, c->run_off_cap, c->run_h)));
  }
  // K1 work units: one per wave, rows / waves each (whole segments, multiples of 16 rows).  A
  // unit start costs a chain of dependent loads (unit bounds, segment ends, codes); same-box A/B,
  // ms per solve for K1: 50M rows 0.505 -> 0.474 (2048-row units before), 6.25M (8-rank owner
  // shard) 0.107 -> 0.090 (512), 1M (config 1) 0.121 -> 0.080 (512).  LFE_K1_UNIT: a fixed size.
  const int64_t waves = (int64_t)c->n_cu * 16;  // K1: one 1024-thread workgroup per CU
  int64_t U = std::max<int64_t>(256, ((c->n_kept_local + waves - 1) / waves + 15) / 16 * 16);
  if (const char* e = knob("LFE_K1_UNIT")) U = std::max<int64_t>(16, atoll(e) / 16 * 16);
  const int32_t H = L.nb * B;
  c->n_units = (int)std::max<int64_t>(1, (c->n_kept_local + U - 1) / U);
  LFE_TRY(ensure_i32(c, c->seg_units, c->seg_units_cap, (size_t)4 * c->n_units));
  {
    ProfScope _ps(c, K_MISC);
    hipLaunchKernelGGL(k_unit_bounds, dim3(grid_for(c->n_units)), dim3(kBlock), 0, c->stream, c->seg_off, H, U,
                       c->n_units, reinterpret_cast<int4*>(c->seg_units));
  }
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

// ===========================================================================
// 2. the two cross-term passes
// ===========================================================================

constexpr int kTpThreads = 1024;  // K1: one workgroup per CU (alpha_Q in LDS)
// K2 workgroup size: 16 waves while the columns fit two 16-lane slots (<= 128 VGPRs)
template <int NT>
constexpr int tq_threads() { return NT <= 2 ? 1024 : 512; }
constexpr int kTqSplitDefault = 2;
constexpr int kIterLds = 150 * 1024;

// reduce over the 4 row quads of the lane layout (lanes 16 and 32 apart)
__device__ __forceinline__ double quad_sum(double v) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

// DPP row_newbcast:D (gfx90a+): every lane of a 16-lane row receives lane D of
// that row (checked on the device by tools/dpp_check.hip)
template <int D>
__device__ __forceinline__ int rowbc(int v) {
  return __builtin_amdgcn_update_dpp(0, v, 0x150 + D, 0xF, 0xF, false);
}
template <int D>
__device__ __forceinline__ int4 rowbc4(const int4& v) {
  return int4{rowbc<D>(v.x), rowbc<D>(v.y), rowbc<D>(v.z), rowbc<D>(v.w)};
}
// compile-time loop D = B, B + 4, ..., < E
template <int B, int E, typename Fn>
__device__ __forceinline__ void static_for4(Fn&& fn) {
  if constexpr (B < E) {
    fn(std::integral_constant<int, B>{});
    static_for4<B + 4, E>(fn);
  }
}
template <int B, int E, typename Fn>
__device__ __forceinline__ void static_for8(Fn&& fn) {
  if constexpr (B < E) {
    fn(std::integral_constant<int, B>{});
    static_for8<B + 8, E>(fn);
  }
}

// Codes of 16 consecutive 16-row groups [gb, gb + 16) are one load per lane:
// lane (kq, c) holds quad kq of group gb + c; group gb + d's codes reach the
// lanes of row kq by row_newbcast:d.  Two such batches are in flight (ping-pong).
constexpr int kBatch = 16;

struct TpArgs {
  const int32_t* seg_off;  // [H + 1] segment offsets (h = bucket * B + offset)
  const int32_t* seg_q;    // secondary code of each kept row, segment order
  const int4* units;       // [n_units] work unit descriptors (k_unit_bounds)
  int n_units;
  int G_Q, G_P, p;
  const double* alphaQ;  // [G_Q][p]
  const double* S_P;     // [G_P][p]
  const int32_t* cntP;   // [G_P] kept counts (all ranks)
  double* out;           // fused: alpha_P [G_P][p]; else T_P [G_P][p]
  int fused;
  double* zeroT;         // T_Q [zero_n], zeroed for the K2 pass that follows (saves a fill launch)
  int64_t zero_n;
  double* zero_check;    // the stop test's max, zeroed for the check after K2 (or null)
  unsigned long long* dbg;  // LFE_SWEEP_TIMING (diagnostic): [block][2] wall-clock start, end
};

// K1: T_P[h] = sum_{i in h} alpha_Q[q_i]; fused: alpha_P[h] = (S_P[h] - T_P[h]) / n_h
// (the body of k_tp as workgroup blk of nblk, aq = [G_Q + 1][p] LDS)
template <int NT>
__device__ __forceinline__ void tp_body(const TpArgs& a, double* __restrict__ aq, int blk, int nblk) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kq = lane >> 4, c = lane & 15;
  const int p = a.p, G_Q = a.G_Q;
  // the wave's first unit descriptor is loaded before the staging, so its latency overlaps it
  const int u_first = blk * (kTpThreads / 64) + wave;
  const int4 d_first = u_first < a.n_units ? a.units[u_first] : int4{0, 0, 0, 0};
  stage_lds<kTpThreads>(aq, a.alphaQ, G_Q * p, tid);
  for (int j = tid; j < p; j += kTpThreads) aq[G_Q * p + j] = 0.0;
  for (int64_t j = (int64_t)blk * kTpThreads + tid; j < a.zero_n; j += (int64_t)nblk * kTpThreads)
    a.zeroT[j] = 0.0;
  if (a.zero_check && blk == 0 && tid == 0) *a.zero_check = 0.0;
  __syncthreads();
  uint32_t cl8[NT];  // byte offset of the lane's column (dead lanes read column 0)
#pragma unroll
  for (int I = 0; I < NT; ++I) cl8[I] = 8 * (16 * I + c < p ? 16 * I + c : 0);
  const uint32_t p8 = 8 * p;
  const int nwaves = nblk * (kTpThreads / 64);
  for (int u = u_first; u < a.n_units; u += nwaves) {
    const int4 ud = u == u_first ? d_first : a.units[u];
    int h = ud.x;
    const int h1 = ud.y;
    if (h >= h1) continue;
    int r0 = ud.z;
    const int rend = ud.w;  // the unit's rows end here
    const int g0 = r0 >> 4, g1 = (rend + 15) >> 4;
    double acc[NT];
#pragma unroll
    for (int I = 0; I < NT; ++I) acc[I] = 0.0;
    // the fused projection's operands of segment h (count, S_P row), loaded when the segment
    // starts so that their latency hides under its rows (short segments: one stall each before)
    int32_t pn = 0;
    double ps[NT];
    auto prefetch = [&]() {
      if (!a.fused || h >= a.G_P) return;
      pn = a.cntP[h];
#pragma unroll
      for (int I = 0; I < NT; ++I) ps[I] = a.S_P[(int64_t)h * p + (16 * I + c < p ? 16 * I + c : 0)];
    };
    prefetch();
    auto finalize = [&]() {  // segment h complete
#pragma unroll
      for (int I = 0; I < NT; ++I) {
        const double t = quad_sum(acc[I]);
        const int col = 16 * I + c;
        if (kq == 0 && col < p && h < a.G_P) {
          const int64_t e = (int64_t)h * p + col;
          if (a.fused) a.out[e] = pn > 0 ? (ps[I] - t) / (double)pn : 0.0;
          else a.out[e] = t;
        }
        acc[I] = 0.0;
      }
    };
    bool done = false;
    // the ends of segments hb .. hb + 63 in the lanes of one register (no global load per
    // segment).  Segments without rows are passed over unwritten: their outputs are 0 from the
    // zeroed table (T_P: the memset before K1; alpha_P: prepare_layout)
    int hb = h;
    int win = hb + lane < h1 ? a.seg_off[hb + lane + 1] : 0x7fffffff;
    int r1 = __builtin_amdgcn_readlane(win, 0);  // seg_off[h + 1]
    auto next_seg = [&]() -> bool {  // segment h is complete
      ++h;
      r0 = r1;
      if (r0 >= rend) return false;  // the rest of the unit's segments are empty
      while (true) {  // a segment with rows lies ahead in the unit
        const int d = h - hb;
        if (d >= 64) {
          hb = h;
          win = hb + lane < h1 ? a.seg_off[hb + lane + 1] : 0x7fffffff;
          continue;
        }
        const uint64_t m = __ballot(win > r0) & (~0ull << d);
        if (m) {
          const int k = (int)__builtin_ctzll(m);
          h = hb + k;
          r1 = __builtin_amdgcn_readlane(win, k);
          prefetch();
          return true;
        }
        h = hb + 64;
      }
    };
    // one 16-row group: lane rows g*16 + 4 kq + s
    auto group = [&](int g, const int4& q4) {
      const int gs = g * 16, rb = gs + 4 * kq;
      const int qv[4] = {q4.x, q4.y, q4.z, q4.w};
      if (gs >= r0 && gs + 16 <= r1) {  // inside segment h (wave-uniform): no masks
#pragma unroll
        for (int s = 0; s < 4; ++s) {
#pragma unroll
          for (int I = 0; I < NT; ++I) acc[I] += lds_row(aq, qv[s], p8, cl8[I]);
        }
        if (gs + 16 < r1) return;
        finalize();
        if (!next_seg()) done = true;
        return;
      }
      while (true) {  // the group holds a segment boundary
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int row = rb + s;
          const uint32_t ro = row >= r0 && row < r1 ? qv[s] : G_Q;
#pragma unroll
          for (int I = 0; I < NT; ++I) acc[I] += lds_row(aq, ro, p8, cl8[I]);
        }
        if (r1 > gs + 16) return;  // segment h continues in the next group
        finalize();
        if (!next_seg()) {
          done = true;
          return;
        }
      }
    };
    auto load = [&](int gb) -> int4 {
      const int g = gb + c;
      return g < g1 ? *reinterpret_cast<const int4*>(a.seg_q + g * 16 + 4 * kq) : int4{0, 0, 0, 0};
    };
    auto four = [&](const int4& v, int gb, auto dc) {
        constexpr int d = decltype(dc)::value;
        if (gb + d >= g1 || done) return;
        const int4 q[4] = {rowbc4<d>(v), rowbc4<d + 1>(v), rowbc4<d + 2>(v), rowbc4<d + 3>(v)};
        const int gs = (gb + d) * 16;
        if (gs >= r0 && gs + 64 < r1) {  // 4 groups inside segment h, which continues after them
          double t[4][NT];
#pragma unroll
          for (int dd = 0; dd < 4; ++dd) {
            const int qv[4] = {q[dd].x, q[dd].y, q[dd].z, q[dd].w};
#pragma unroll
            for (int s = 0; s < 4; ++s) {
#pragma unroll
              for (int I = 0; I < NT; ++I) {
                const double v = lds_row(aq, qv[s], p8, cl8[I]);
                t[s][I] = dd == 0 ? v : t[s][I] + v;
              }
            }
          }
#pragma unroll
          for (int I = 0; I < NT; ++I) acc[I] += (t[0][I] + t[1][I]) + (t[2][I] + t[3][I]);
          return;
        }
#pragma unroll
        for (int dd = 0; dd < 4; ++dd) {
          if (gb + d + dd >= g1 || done) return;
          group(gb + d + dd, q[dd]);
        }
    };
    // 8 groups inside the segment: all 32 row gathers issued before their sums (more LDS reads in
    // flight per wave; the pass is latency-bound at 4 waves per SIMD); else two 4-group steps
    auto batch = [&](const int4& v, int gb) {
      static_for8<0, kBatch>([&](auto dc) {
        constexpr int d = decltype(dc)::value;
        if (gb + d >= g1 || done) return;
        const int gs = (gb + d) * 16;
        if (gs >= r0 && gs + 128 < r1) {
          const int4 q[8] = {rowbc4<d>(v),     rowbc4<d + 1>(v), rowbc4<d + 2>(v), rowbc4<d + 3>(v),
                             rowbc4<d + 4>(v), rowbc4<d + 5>(v), rowbc4<d + 6>(v), rowbc4<d + 7>(v)};
          double t[4][NT];
#pragma unroll
          for (int dd = 0; dd < 8; ++dd) {
            const int qv[4] = {q[dd].x, q[dd].y, q[dd].z, q[dd].w};
#pragma unroll
            for (int s = 0; s < 4; ++s) {
#pragma unroll
              for (int I = 0; I < NT; ++I) {
                const double x = lds_row(aq, qv[s], p8, cl8[I]);
                t[s][I] = dd == 0 ? x : t[s][I] + x;
              }
            }
          }
#pragma unroll
          for (int I = 0; I < NT; ++I) acc[I] += (t[0][I] + t[1][I]) + (t[2][I] + t[3][I]);
          return;
        }
        four(v, gb, std::integral_constant<int, d>{});
        four(v, gb, std::integral_constant<int, d + 4>{});
      });
    };
    // batches on absolute 16-group boundaries (the groups before the unit's first add zero rows),
    // so a segment's summation tree depends on its rows only, not on where units begin
    const int ga = g0 & ~(kBatch - 1);
    int4 va = load(ga), vb;
    for (int gb = ga; gb < g1 && !done;) {
      vb = load(gb + kBatch);
      batch(va, gb);
      gb += kBatch;
      if (gb >= g1 || done) break;
      va = load(gb + kBatch);
      batch(vb, gb);
      gb += kBatch;
    }
  }
}

template <int NT>
__global__ __launch_bounds__(kTpThreads) void k_tp(TpArgs a) {
  extern __shared__ __attribute__((aligned(16))) double aq[];  // [G_Q + 1][p], row G_Q = 0
  if (a.dbg && threadIdx.x == 0) a.dbg[2 * blockIdx.x] = wall_clock64();
  tp_body<NT>(a, aq, blockIdx.x, gridDim.x);
  if (a.dbg) {
    __syncthreads();
    if (threadIdx.x == 0) a.dbg[2 * blockIdx.x + 1] = wall_clock64();
  }
}

struct TqArgs {
  const int32_t* run_off;  // [nb * G_Q + 1] run offsets
  const uint16_t* run_h;   // primary code - lo of each kept row, run order
  const int32_t* blist;    // [nbe] the buckets that hold rows, in order (null: all nb buckets)
  int nbe, s, G_Q, G_P, p;
  const double* alphaP;  // [G_P][p]
  double* runs;          // [nbe * G_Q][p]: the sum of every (listed bucket, q) run (empty runs: 0)
  int split;             // workgroups per bucket (each takes 1 / split of the bucket's runs)
  unsigned long long* dbg;  // LFE_SWEEP_TIMING (diagnostic): [block][2] wall-clock start, end
};

// K2: runs[i][q] = sum over the (bucket blist[i], q) run of alpha_P[h_i].  Every run is summed by
// one wave in row order and every slot is written, so T_Q[q] = sum_i runs[i][q] (k_tq_reduce, in
// bucket order) is bit-reproducible: no cross-workgroup atomics.  Buckets without rows contribute
// nothing and are not visited.
// (the body of k_tq as workgroup blk of nblk, sl = [B + 1][p] LDS)
template <int NT>
__device__ __forceinline__ void tq_body(const TqArgs& a, double* __restrict__ sl, int blk, int nblk) {
  constexpr int kTqThreads = tq_threads<NT>();
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr int NW = kTqThreads / 64;
  const int kq = lane >> 4, c = lane & 15;
  const int p = a.p, G_Q = a.G_Q, B = 1 << a.s;
  uint32_t cl8[NT];  // byte offset of the lane's column (dead lanes read column 0)
#pragma unroll
  for (int I = 0; I < NT; ++I) cl8[I] = 8 * (16 * I + c < p ? 16 * I + c : 0);
  const uint32_t p8 = 8 * p;
  const int kTqSplit = a.split;
  for (int bs = blk; bs < a.nbe * kTqSplit; bs += nblk) {
    const int bi = bs / kTqSplit, part = bs % kTqSplit;
    const int b = a.blist ? a.blist[bi] : bi;  // no list: every bucket holds rows
    const int lo = b << a.s;
    // wave: runs q in [q, q1) of bucket b; their offsets (and the ends of runs q .. q + 63 in the
    // lanes of one register) are loaded before the staging, so their latency overlaps it
    const int slot = part * NW + wave;
    int q = slot * G_Q / (NW * kTqSplit);
    const int q1 = (slot + 1) * G_Q / (NW * kTqSplit);
    const int32_t* off = a.run_off + (int64_t)b * G_Q;
    int r0 = 0, r1 = 0, rq1 = 0, win = 0;
    if (q < q1) {
      r0 = off[q];
      r1 = off[q + 1];
      rq1 = off[q1];
      win = q + lane < q1 ? off[q + lane + 1] : 0;
    }
    __syncthreads();
    {  // the bucket's rows of alpha_P are contiguous (16-byte aligned: lo p 8 = b 2^s p 8); rows
       // past G_P and the zero row B are cleared
      const int nv = max(0, min(B, a.G_P - lo)) * p;
      stage_lds<kTqThreads>(sl, a.alphaP + (int64_t)lo * p, nv, tid);
      for (int j = nv + tid; j < (B + 1) * p; j += kTqThreads) sl[j] = 0.0;
    }
    __syncthreads();
    if (q >= q1) continue;
    double* const runs = a.runs + (int64_t)bi * G_Q * p;
    const int g0 = r0 >> 4, g1 = (rq1 + 15) >> 4;
    if (g0 >= g1) {  // no rows in these runs
      for (int j = lane; j < (q1 - q) * p; j += 64) runs[(int64_t)q * p + j] = 0.0;
      continue;
    }
    int qb = q;  // win holds the ends of runs qb .. qb + 63: no global load per run
    auto run_end = [&](int qq) -> int {
      if (qq - qb >= 64) {
        qb = qq;
        win = qb + lane < q1 ? off[qb + lane + 1] : 0;
      }
      return __builtin_amdgcn_readlane(win, qq - qb);
    };
    double acc[NT];
#pragma unroll
    for (int I = 0; I < NT; ++I) acc[I] = 0.0;
    typedef unsigned short us4 __attribute__((ext_vector_type(4)));
    auto finalize = [&]() {  // run q complete (an empty run stores 0)
#pragma unroll
      for (int I = 0; I < NT; ++I) {
        const double t = quad_sum(acc[I]);
        const int col = 16 * I + c;
        if (kq == 0 && col < p) runs[(int64_t)q * p + col] = t;
        acc[I] = 0.0;
      }
    };
    bool done = false;
    auto group = [&](int g, const us4& h4) {
      const int gs = g * 16, rb = gs + 4 * kq;
      if (gs >= r0 && gs + 16 <= r1) {  // inside run q (wave-uniform): no masks
#pragma unroll
        for (int s = 0; s < 4; ++s) {
#pragma unroll
          for (int I = 0; I < NT; ++I) acc[I] += lds_row(sl, h4[s], p8, cl8[I]);
        }
        if (gs + 16 < r1) return;
        finalize();
        if (++q >= q1) {
          done = true;
          return;
        }
        r0 = r1;
        r1 = run_end(q);
        return;
      }
      while (true) {  // the group holds a run boundary
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int row = rb + s;
          const uint32_t ro = row >= r0 && row < r1 ? (uint32_t)h4[s] : (uint32_t)B;
#pragma unroll
          for (int I = 0; I < NT; ++I) acc[I] += lds_row(sl, ro, p8, cl8[I]);
        }
        if (r1 > gs + 16) return;  // run continues in the next group
        finalize();
        if (++q >= q1) {
          done = true;
          return;
        }
        r0 = r1;
        r1 = run_end(q);
      }
    };
    // ushort4 of codes = 2 dwords per lane; broadcast dword-wise
    auto load = [&](int gb) -> int2 {
      const int g = gb + c;
      return g < g1 ? *reinterpret_cast<const int2*>(a.run_h + g * 16 + 4 * kq) : int2{0, 0};
    };
    auto unpack = [](int lo32, int hi32) {
      return us4{(unsigned short)(lo32 & 0xFFFF), (unsigned short)((unsigned)lo32 >> 16),
                 (unsigned short)(hi32 & 0xFFFF), (unsigned short)((unsigned)hi32 >> 16)};
    };
    auto batch = [&](const int2& v, int gb) {
      static_for4<0, kBatch>([&](auto dc) {
        constexpr int d = decltype(dc)::value;
        if (gb + d >= g1 || done) return;
        const us4 hh[4] = {unpack(rowbc<d>(v.x), rowbc<d>(v.y)), unpack(rowbc<d + 1>(v.x), rowbc<d + 1>(v.y)),
                           unpack(rowbc<d + 2>(v.x), rowbc<d + 2>(v.y)), unpack(rowbc<d + 3>(v.x), rowbc<d + 3>(v.y))};
        const int gs = (gb + d) * 16;
        if (gs >= r0 && gs + 64 < r1) {  // 4 groups inside run q, which continues after them
          double t[4][NT];
#pragma unroll
          for (int dd = 0; dd < 4; ++dd)
#pragma unroll
            for (int s = 0; s < 4; ++s) {
#pragma unroll
              for (int I = 0; I < NT; ++I) {
                const double v = lds_row(sl, hh[dd][s], p8, cl8[I]);
                t[s][I] = dd == 0 ? v : t[s][I] + v;
              }
            }
#pragma unroll
          for (int I = 0; I < NT; ++I) acc[I] += (t[0][I] + t[1][I]) + (t[2][I] + t[3][I]);
          return;
        }
#pragma unroll
        for (int dd = 0; dd < 4; ++dd) {
          if (gb + d + dd >= g1 || done) return;
          group(gb + d + dd, hh[dd]);
        }
      });
    };
    int2 va = load(g0), vb;
    for (int gb = g0; gb < g1 && !done;) {
      vb = load(gb + kBatch);
      batch(va, gb);
      gb += kBatch;
      if (gb >= g1 || done) break;
      va = load(gb + kBatch);
      batch(vb, gb);
      gb += kBatch;
    }
  }
}

template <int NT>
__global__ __launch_bounds__(tq_threads<NT>()) void k_tq(TqArgs a) {
  extern __shared__ __attribute__((aligned(16))) double sl[];  // [B + 1][p], row B = 0
  if (a.dbg && threadIdx.x == 0) a.dbg[2 * blockIdx.x] = wall_clock64();
  tq_body<NT>(a, sl, blockIdx.x, gridDim.x);
  if (a.dbg) {
    __syncthreads();
    if (threadIdx.x == 0) a.dbg[2 * blockIdx.x + 1] = wall_clock64();
  }
}

// T_Q[q][col] = sum over buckets b (in order) of runs[b][q][col]
// 16 consecutive entries per block (128-byte loads), 16 bucket slices (slice s: buckets s, s + 16,
// ...), each thread four loads in flight; the slices are added in order: a fixed summation order
constexpr int kTqRedE = 16, kTqRedS = 16;
// slice sl's sum of entry e over its buckets sl, sl + 16, ... (in order, four loads in flight)
__device__ __forceinline__ double tq_red_slice(const double* __restrict__ runs, int nb, int64_t m, int64_t e, int sl) {
  double t = 0.0;
  if (e < m) {
    int b = sl;
    for (; b + 3 * kTqRedS < nb; b += 4 * kTqRedS) {
      const double v0 = runs[(int64_t)b * m + e], v1 = runs[(int64_t)(b + kTqRedS) * m + e];
      const double v2 = runs[(int64_t)(b + 2 * kTqRedS) * m + e], v3 = runs[(int64_t)(b + 3 * kTqRedS) * m + e];
      t = (((t + v0) + v1) + v2) + v3;
    }
    for (; b < nb; b += kTqRedS) t += runs[(int64_t)b * m + e];
  }
  return t;
}
// the slices of entry ei added in order
__device__ __forceinline__ double tq_red_total(const double (*part)[kTqRedE], int ei) {
  double r = part[0][ei];
  for (int k = 1; k < kTqRedS; ++k) r += part[k][ei];
  return r;
}
// T_Q[e] = r, the next projection alpha_new[e] = (S_Q[e] - r) / n; returns the stop test's term
// |alpha_new - alpha_cur| on column 0 of a present group (else 0)
__device__ __forceinline__ double tq_red_fin(double r, int64_t e, double* __restrict__ T, const double* __restrict__ S,
                                             const int32_t* __restrict__ cnt, int p, const double* __restrict__ cur,
                                             double* __restrict__ out, bool check) {
  T[e] = r;
  const int32_t n = cnt[e / p];
  const double v = n > 0 ? (S[e] - r) / (double)n : 0.0;
  out[e] = v;
  return (check && n > 0 && e % p == 0) ? fabs(v - cur[e]) : 0.0;
}
// max over the wave (NaN propagates) into *check by lane 0
__device__ __forceinline__ void tq_red_check(double mx, int lane, unsigned long long* check) {
  for (int off = 32; off > 0; off >>= 1) {
    const double o = __shfl_down(mx, off, 64);
    mx = (isnan(o) || isnan(mx)) ? __builtin_nan("") : fmax(mx, o);
  }
  if (lane == 0) atomicMax(check, (unsigned long long)__double_as_longlong(fabs(mx)));
}

// T_Q[q][col] = sum over buckets b (in order) of runs[b][q][col]
// 16 consecutive entries per block (128-byte loads), 16 bucket slices (slice s: buckets s, s + 16,
// ...), each thread four loads in flight; the slices are added in order: a fixed summation order
__global__ __launch_bounds__(256) void k_tq_reduce(const double* __restrict__ runs, int nb, int64_t m,
                                                   double* __restrict__ T) {
  __shared__ double part[kTqRedS][kTqRedE];
  const int ei = threadIdx.x % kTqRedE, sl = threadIdx.x / kTqRedE;
  const int64_t e = (int64_t)blockIdx.x * kTqRedE + ei;
  part[sl][ei] = tq_red_slice(runs, nb, m, e, sl);
  __syncthreads();
  if (sl == 0 && e < m) T[e] = tq_red_total(part, ei);
}

// one rank: k_tq_reduce and the next Q projection (k_fin_check) in one launch.  T_Q[e] is summed
// as k_tq_reduce sums it, then alpha_new[e] = (S_Q[e] - T_Q[e]) / n and, on column 0, the stop
// test |alpha_new - alpha_cur| (NaN propagates); wave 0 holds the block's 16 writers.
__global__ __launch_bounds__(256) void k_tq_reduce_fin(const double* __restrict__ runs, int nb, int64_t m,
                                                       double* __restrict__ T, const double* __restrict__ S,
                                                       const int32_t* __restrict__ cnt, int p,
                                                       const double* __restrict__ cur, double* __restrict__ out,
                                                       unsigned long long* __restrict__ check,
                                                       const double* __restrict__ flag_in, double* __restrict__ flag_out,
                                                       unsigned int* __restrict__ done,
                                                       unsigned long long* __restrict__ msg, unsigned long long seq) {
  __shared__ double part[kTqRedS][kTqRedE];
  // the digits' guard flag beside the stop test, for the same read-back (no separate copy)
  if (flag_in && blockIdx.x == 0 && threadIdx.x == 0) *flag_out = *flag_in;
  const int ei = threadIdx.x % kTqRedE, sl = threadIdx.x / kTqRedE;
  const int64_t e = (int64_t)blockIdx.x * kTqRedE + ei;
  part[sl][ei] = tq_red_slice(runs, nb, m, e, sl);
  __syncthreads();
  double mx = 0.0;
  if (sl == 0 && e < m) mx = tq_red_fin(tq_red_total(part, ei), e, T, S, cnt, p, cur, out, check != nullptr);
  if (check && threadIdx.x < 64) tq_red_check(mx, threadIdx.x, check);
  // the stop test (and the guard's flag) straight into mapped host memory by the last workgroup:
  // no copy kernel and no event between the sweep and the host's decision
  if (msg && last_block_done(done) && threadIdx.x == 0) {
    double v[2];
    v[0] = __longlong_as_double((long long)__hip_atomic_load(check, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    v[1] = flag_in ? __hip_atomic_load(flag_out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
    host_msg_publish(msg, seq, v, 2);
  }
}

// alpha_new = (S - T) / cnt; check = max_g |alpha_new[g][0] - alpha_cur[g][0]| over groups present
// (= |mean_g(y~)| after the sweep); NaN propagates (a NaN panel never converges).
__global__ void k_fin_check(const double* __restrict__ S, const double* __restrict__ T,
                            const int32_t* __restrict__ cnt, int32_t G, int p, const double* __restrict__ cur,
                            double* __restrict__ out, unsigned long long* __restrict__ check,
                            const double* __restrict__ flag_in = nullptr, double* __restrict__ flag_out = nullptr) {
  if (flag_in && blockIdx.x == 0 && threadIdx.x == 0) *flag_out = *flag_in;
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

static int fin_check(lfe_ctx* c, int f, const double* T, const double* cur, double* out, bool check,
                     const double* flag_in = nullptr) {
  auto& fe = c->fe[f];
  ProfScope _ps(c, K_FINALIZE);
  hipLaunchKernelGGL(k_fin_check, dim3(grid_for((int64_t)fe.G * c->p)), dim3(kBlock), 0, c->stream, fe.S, T, fe.cnt,
                     fe.G, c->p, cur, out, check ? reinterpret_cast<unsigned long long*>(c->dred) : nullptr,
                     check ? flag_in : nullptr, c->dred + 1);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

// two FEs whose row layouts do not fit LDS (wide fits: alpha_Q or the primary slice too large)
// but whose dense count tables serve both cross terms (lfe_dense.hip, 16-column groups)
static bool fast_dense_only_ok(const lfe_ctx* c) {
  if (c->F != 2 || c->L.w || c->L.P < 0 || !c->L.permuted || (1ll << c->L.s) > 65536) return false;
  return dense_ok(c);
}

bool fast_path_ok(const lfe_ctx* c, const std::vector<int>& order) {
  return order.back() == c->L.P && (fast_layout_ok(c) || fast_dense_only_ok(c));
}

bool fast_layout_ok(const lfe_ctx* c) {
  if (c->F != 2 || c->L.w || c->L.P < 0 || !c->L.permuted) return false;
  const int Q = 1 - c->L.P, p = c->p;
  const int64_t G_Q = c->fe[Q].G, B = 1ll << c->L.s;
  return (G_Q + 1) * p * 8 <= kIterLds                 // K1: alpha_Q in LDS
         && (B + 1) * p * 8 <= 96 * 1024               // K2: primary slice in LDS
         && ls_scatter_lds((int)G_Q, ls_per()) <= 150 * 1024  // run layout sort
         && (B + G_Q) * 4 <= 64 * 1024                 // both histograms in LDS
         && B <= 65536;                                // uint16 offsets
}

template <int NT>
static void launch_tp(lfe_ctx* c, const TpArgs& a, size_t lds) {
  hipLaunchKernelGGL(k_tp<NT>, dim3(c->n_cu), dim3(kTpThreads), lds, c->stream, a);
}
template <int NT>
static void launch_tq(lfe_ctx* c, const TqArgs& a, size_t lds) {
  hipLaunchKernelGGL(k_tq<NT>, dim3(std::max(a.nbe, 1) * a.split), dim3(tq_threads<NT>()), lds, c->stream, a);
}

int demean_fast(lfe_ctx* c, double tol, int max_iter, int check_from, int* iterations_out, double* last_out) {
  const int P = c->L.P, Q = 1 - P, p = c->p;
  auto& fp = c->fe[P];
  auto& fq = c->fe[Q];
  const int NT = (p + 15) / 16;
  // dense count tables where the primary x secondary table holds >= ~0.15 rows per cell (both
  // cross terms on the matrix cores, lfe_dense.hip); else the segment / run layouts
  // the tables prepare_layout built on every row hold the kept rows when nothing was dropped
  // (owner-sharded ranks: dense_ok alone, a decision every rank takes alike; dn_pre_valid is local)
  const bool dense = !c->dense_off && ((c->dn_pre_valid && c->world == 1) || dense_ok(c));
  c->dense_cells = 0;
  if (dense) {
    c->hists_kept = false;
    if (c->dn_pre_valid) c->dense_cells = dense_table_cells(c);
    else LFE_TRY(dense_build(c));
  } else {
    LFE_TRY(build_layouts(c, Q));
  }
  LFE_TRY(ensure_f64(c, c->alpha_spare, c->alpha_spare_cap, (size_t)fq.G * p));
  LFE_TRY(ensure_dred(c, 2));
  // the i8 digits' dynamic-range guard: its flag rides with the stop test's read-back (and, with
  // several ranks, with every sweep's T_Q all-reduce, so all ranks see the same flag)
  const bool guard = dense && c->dn8;
  // the sums' epilogue already formed the first projection alpha_Q = S_Q / n_Q and zeroed the
  // guard's flag (one rank; consumed once: a redo without the dense passes projects again)
  const bool first_done = c->q_first != nullptr && c->q_first == fq.alpha;
  c->q_first = nullptr;
  if (guard && !first_done) LFE_TRY(range_flag_reset(c));
  const size_t lds_tp = sizeof(double) * ((size_t)fq.G + 1) * p;
  const size_t lds_tq = sizeof(double) * (((size_t)1 << c->L.s) + 1) * p;
  const void* ftp = NT == 1 ? reinterpret_cast<const void*>(&k_tp<1>)
                    : NT == 2 ? reinterpret_cast<const void*>(&k_tp<2>)
                    : NT == 3 ? reinterpret_cast<const void*>(&k_tp<3>)
                              : reinterpret_cast<const void*>(&k_tp<4>);
  const void* ftq = NT == 1 ? reinterpret_cast<const void*>(&k_tq<1>)
                    : NT == 2 ? reinterpret_cast<const void*>(&k_tq<2>)
                    : NT == 3 ? reinterpret_cast<const void*>(&k_tq<3>)
                              : reinterpret_cast<const void*>(&k_tq<4>);
  if (!dense) {  // the row passes' LDS tables (a wide fit runs the dense passes only)
    LFE_HIP(set_max_lds(ftp, (int)std::max<size_t>(lds_tp, 1)));
    LFE_HIP(set_max_lds(ftq, (int)std::max<size_t>(lds_tq, 1)));
  }
  TpArgs tp{};
  tp.seg_off = c->seg_off;
  tp.seg_q = c->seg_q;
  tp.units = reinterpret_cast<const int4*>(c->seg_units);
  tp.n_units = c->n_units;
  tp.G_Q = fq.G;
  tp.G_P = fp.G;
  tp.p = p;
  tp.S_P = fp.S;
  tp.cntP = fp.cnt;
  tp.fused = c->world == 1 || c->owner_on;  // owner-sharded: T_P is complete on each rank
  tp.out = tp.fused ? fp.alpha : fp.T;
  TqArgs tq{};
  tq.run_off = c->run_off;
  tq.run_h = c->run_h;
  tq.blist = c->nbe == c->L.nb ? nullptr : c->blist_d;
  tq.nbe = c->nbe;
  tq.s = c->L.s;
  tq.G_Q = fq.G;
  tq.G_P = fp.G;
  tq.p = p;
  tq.alphaP = fp.alpha;
  const int nbe = std::max(c->nbe, 1);
  LFE_TRY(ensure_f64(c, c->tq_runs, c->tq_runs_cap, (size_t)nbe * fq.G * p));
  tq.runs = c->tq_runs;
  // about four workgroups per CU in all (two resident at a time), so no CU is left with a lone
  // tail: 196 buckets -> 5 per bucket (tq 0.61 -> 0.49 ms per step at 50M rows, measured)
  tq.split = std::max(kTqSplitDefault / 2, (int)std::lround(4.0 * c->n_cu / nbe));
  {  // every workgroup stages its bucket's 45 KB alpha_P slice: >= 8K rows per workgroup at p = 11
     // (LFE_K2_MINROWS sweep, ms per solve for K2: 6.25M rows over 25 buckets 0.113 at 16K, 0.105
     // at 8K, 0.117 at 4K; 48K 0.142; config 2 (p = 6) 0.362 / 0.314 / 0.314 at 16K / 8K / 4K, config
     // 1 (p = 4) 0.108 / 0.075 at 8K / 4K; 50M rows unchanged); a narrower slice (p < 11) pays for
     // proportionally fewer rows
    const int64_t per_bucket = c->n_kept_local / nbe;
    int64_t min_rows = std::max<int64_t>(2048, (int64_t)8192 * p / 11);
    if (const char* e = knob("LFE_K2_MINROWS")) min_rows = std::max<int64_t>(256, atoll(e));  // A/B only
    tq.split = (int)std::max<int64_t>(1, std::min<int64_t>(tq.split, per_bucket / min_rows));
    // ... but no fewer workgroups than CUs while each keeps >= 8K rows (6.25M rows over 196
    // buckets: 196 -> 392 workgroups)
    const int64_t fill = (c->n_cu + nbe - 1) / nbe;
    if (tq.split < fill && per_bucket / fill >= 8192) tq.split = (int)fill;
    // whole rounds of resident workgroups: the split with the least rounds per share of a bucket
    // (a workgroup's time goes as 1 / split), e.g. config 1's 40 buckets at one resident workgroup
    // per CU: 6 per bucket (240, one round) instead of 8 (320: two rounds; K2 16.4 -> 12.9 us,
    // per-workgroup wall clock from LFE_SWEEP_TIMING; config 1 0.46 -> 0.42 ms per solve)
    if (!dense) {
      const int res = std::max(1, resident_blocks(c, ftq, NT <= 2 ? 1024 : 512, std::max<size_t>(lds_tq, 1)));
      double best = 1e30;
      int bs = tq.split;
      for (int sp = tq.split; sp >= 1; --sp) {
        const double cost = (double)(((int64_t)nbe * sp + res - 1) / res) / sp;
        if (cost < best - 1e-12) {
          best = cost;
          bs = sp;
        }
      }
      tq.split = bs;
    }
  }
  // LFE_SWEEP_TIMING (diagnostic): per-workgroup wall clock of the last K1 / K2 launch to stderr
  const bool timing = !dense && knob("LFE_SWEEP_TIMING") != nullptr;
  const int tp_grid = c->n_cu, tq_grid_wg = std::max(tq.nbe, 1) * tq.split;
  if (timing) {
    LFE_HIP(hipMalloc(&tp.dbg, sizeof(unsigned long long) * 2 * tp_grid));
    LFE_HIP(hipMalloc(&tq.dbg, sizeof(unsigned long long) * 2 * tq_grid_wg));
  }
  // sweep 1's Q projection: alpha_P = 0 -> alpha_Q = S_Q / n_Q (alpha_P is first written by K1,
  // which covers every primary group)
  if (!first_done) LFE_TRY(fin_check(c, Q, nullptr, nullptr, fq.alpha, false));
  int iterations = 0;
  double last = -1.0;
  int flag_read = 0;  // the sweep whose check read the guard's flag
  for (int it = 1; it <= max_iter; ++it) {
    tp.alphaQ = fq.alpha;
    tp.zeroT = nullptr;  // K2 writes every run slot; k_tq_reduce writes T_Q
    tp.zero_n = 0;
    tp.zero_check = it >= check_from ? c->dred : nullptr;
    // T_P partials: segments with no local rows are not written by K1
    if (!tp.fused) LFE_HIP(hipMemsetAsync(fp.T, 0, sizeof(double) * (size_t)fp.G * p, c->stream));
    if (dense) {
      ProfScope _ps(c, K_TP);
      LFE_TRY(dense_tp(c, fq.alpha, tp.zero_check));
    } else {
      ProfScope _ps(c, K_TP);
      switch (NT) {
        case 1: launch_tp<1>(c, tp, lds_tp); break;
        case 2: launch_tp<2>(c, tp, lds_tp); break;
        case 3: launch_tp<3>(c, tp, lds_tp); break;
        default: launch_tp<4>(c, tp, lds_tp); break;
      }
    }
    LFE_HIP(hipGetLastError());
    if (!tp.fused) {
      LFE_TRY(allreduce_sum_f64(c, fp.T, (size_t)fp.G * p));
      LFE_TRY(fin_check(c, P, fp.T, nullptr, fp.alpha, false));
    }
    if (dense) {  // the check's max was zeroed by K1
      ProfScope _ps(c, K_TQ);
      LFE_TRY(dense_tq(c, c->tq_runs));
    } else {
      ProfScope _ps(c, K_TQ);
      switch (NT) {
        case 1: launch_tq<1>(c, tq, lds_tq); break;
        case 2: launch_tq<2>(c, tq, lds_tq); break;
        case 3: launch_tq<3>(c, tq, lds_tq); break;
        default: launch_tq<4>(c, tq, lds_tq); break;
      }
    }
    LFE_HIP(hipGetLastError());
    iterations = it;
    const bool check = it >= check_from;
    const int64_t m = (int64_t)fq.G * p;
    const unsigned tq_grid = (unsigned)((m + kTqRedE - 1) / kTqRedE);
    unsigned long long seq = 0;  // the stop test published to mapped host memory (one rank)
    if (c->world == 1) {  // T_Q and the next Q projection in one launch
      if (check && host_msg_on(c)) seq = next_msg_seq(c);
      {
        ProfScope _ps(c, K_TQ_REDUCE);
        hipLaunchKernelGGL(k_tq_reduce_fin, dim3(tq_grid), dim3(kTqRedE * kTqRedS), 0, c->stream, c->tq_runs,
                           c->nbe, m, fq.T, fq.S, fq.cnt, p, fq.alpha, c->alpha_spare,
                           check ? reinterpret_cast<unsigned long long*>(c->dred) : nullptr,
                           check && guard ? c->rflag : nullptr, c->dred + 1, c->gsync + GS_TQ_REDUCE,
                           seq ? c->dmsg : nullptr, seq);
      }
      LFE_HIP(hipGetLastError());
      if (!check && it == max_iter) break;
    } else {
      {
        ProfScope _ps(c, K_TQ_REDUCE);
        hipLaunchKernelGGL(k_tq_reduce, dim3(tq_grid), dim3(kTqRedE * kTqRedS), 0, c->stream, c->tq_runs, c->nbe,
                           m, fq.T);
      }
      LFE_HIP(hipGetLastError());
      if (guard)
        LFE_TRY(allreduce_sum_f64_many(c, {{fq.T, (size_t)fq.G * p}, {c->rflag, 1}}));
      else
        LFE_TRY(allreduce_sum_f64(c, fq.T, (size_t)fq.G * p));
      if (!check && it == max_iter) break;
      LFE_TRY(fin_check(c, Q, fq.T, fq.alpha, c->alpha_spare, check, guard ? c->rflag : nullptr));
    }
    if (check) {
      // the check's read-back first, then - when this check is likely the last (the first one,
      // or the previous was within 100x of tol: the check falls ~100x per sweep) - the Gram of
      // the tables and its Cholesky, so the GPU works through the host's decision and the
      // return to the caller; lfe_gram_resid then starts at the residual pass
      // (the guard's flag was copied beside the check by the reduce / projection kernel)
      if (!seq) LFE_TRY(d2h_async(c, c->dred, sizeof(double) * (guard ? 2 : 1)));
      int spec = 0;
      c->tq_final = true;
      // at every check, gated on the device by the check itself: an unconverged sweep pays two empty
      // launches (the old host-side guess - the first check, or the previous within 100x of tol -
      // ran the whole tables Gram at two of config 1's three checks for nothing: ~15 us each)
      LFE_TRY(gram_spec_enqueue(c, &spec, reinterpret_cast<const unsigned long long*>(c->dred), tol));
      c->tq_final = false;
      double rb[2] = {0.0, 0.0};
      if (seq) LFE_TRY(host_msg_wait(c, seq, rb, 2));
      else LFE_TRY(d2h_wait(c, rb, sizeof(double) * (guard ? 2 : 1)));
      last = rb[0];
      flag_read = it;
      if (rb[1] != 0.0) {  // a tile's digits lost precision: lfe_demean redoes the solve without them
        c->dense_coarse = true;
        break;
      }
      if (last < tol) {  // converged after sweep `it`: keep alpha_Q of this sweep
        c->gram_spec = spec != 0;
        break;
      }
    }
    if (it == max_iter) break;
    std::swap(fq.alpha, c->alpha_spare);
  }
  if (guard && !c->dense_coarse && flag_read != iterations) {  // the loop ended without a check
    double f = 0.0;
    LFE_TRY(d2h_sync(c, &f, c->rflag, sizeof(double)));
    c->dense_coarse = f != 0.0;
  }
  if (timing) {
    auto report = [&](const char* name, unsigned long long* d, int n) -> int {
      std::vector<unsigned long long> h((size_t)2 * n);
      LFE_HIP(hipMemcpy(h.data(), d, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
      (void)hipFree(d);
      unsigned long long t0 = ~0ull, t1 = 0;
      std::vector<double> dur(n), st(n);
      for (int b = 0; b < n; ++b) t0 = std::min(t0, h[2 * b]);
      for (int b = 0; b < n; ++b) {
        st[b] = (h[2 * b] - t0) / 100.0;
        dur[b] = (h[2 * b + 1] - h[2 * b]) / 100.0;
        t1 = std::max(t1, h[2 * b + 1]);
      }
      std::vector<double> sd = dur, ss = st;
      std::sort(sd.begin(), sd.end());
      std::sort(ss.begin(), ss.end());
      fprintf(stderr, "%s: %d workgroups, span %.2f us; start offset median %.2f max %.2f; duration min %.2f median %.2f p90 %.2f max %.2f us\n",
              name, n, (t1 - t0) / 100.0, ss[n / 2], ss[n - 1], sd[0], sd[n / 2], sd[(n * 9) / 10], sd[n - 1]);
      return LFE_OK;
    };
    LFE_TRY(report("K1 k_tp", tp.dbg, tp_grid));
    LFE_TRY(report("K2 k_tq", tq.dbg, tq_grid_wg));
  }
  *iterations_out = iterations;
  *last_out = last;
  c->tq_final = true;  // fq.T was formed from the final alpha_P (the Gram-from-tables cross term)
  return LFE_OK;
}

}  // namespace lfe

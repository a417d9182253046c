// leanfe HIP engine — the two cross terms of the two-FE sweep (polars_impl.py:490-526) as dense
// products on the matrix cores, for panels where the primary-by-secondary count table is dense.
//
// Per bucket b of the primary FE P (2^s groups h, rows sorted by bucket in the layout) let
// N_b[h][q] = the number of kept rows with codes (h, q).  Then
//     T_P[h]     = sum_q N_b[h][q] alpha_Q[q]        (K1: N_b alpha_Q)
//     T_Q,b[q]   = sum_h N_b[h][q] alpha_P[h]        (K2: N_b' alpha_P slice)
// which is what the segment / run passes of lfe_iter.hip gather row by row.  At 50M rows over
// 196 buckets x 512 x 1000 cells (0.5 rows per cell) the table holds 2 bytes per cell where the
// layouts hold 6 per row, and both products run on v_mfma_f64_16x16x4f64 with the counts (small
// integers, exact in f64) as one operand: no LDS row gathers, no per-row work in the sweeps.
//
// Storage (uint16 counts; the caller guarantees every count <= 65535 from the largest primary
// level's kept count): 16 x 16 blocks of 512 bytes.
//   NA [bi][hb][qb] blocks, element (hh, qq) at 16 hh + qq  (K1: lane (kq, c) loads 4 counts
//       of group h = 16 hb + c, levels q = 16 qb + 4 kq .. + 3: the A operand of four MFMAs)
//   NB [bi][qb][hb] blocks, element (qq, hh) at 16 qq + hh  (K2: the same with h and q swapped)
// bi indexes the buckets that hold rows (blist), so an owner shard's table covers its own levels.
//
// Every T entry is a fixed sequence of MFMAs and fixed-order adds: the bits repeat run to run.
// T_Q,b goes to the same per-bucket slots (tq_runs) as K2 of lfe_iter.hip, so the bucket
// reduction, the Q projection, the stop test and the multi-rank all-reduce are shared.
//
// Exact integer form ("dn8", the default where it fits).  The f64 MFMA is 64 cycles per 16x16x4
// product; v_mfma_i32_16x16x64_i8 is 16 cycles per 16x16x64, 16x the MACs per cycle, and sums
// exactly in int32.  The counts are small integers (i8 when <= 127) and the other FE's effects
// are cut into exact integer digits: per tile of 512 k rows and per column, with 2^e > max |alpha|,
//     round(alpha 2^(54 - e)) = sum_{d < 8} digit_d 128^d,   digit_d in [-64, 63]
// so T = sum_d (N digit_d) 128^d 2^(e - 54) with every N digit_d product summed exactly on the
// matrix cores and one f64 conversion per tile - the effects rounded to 2^-54 of the tile's largest,
// below the f64 rounding of a sum of them.  The i8 tables hold 1 byte per cell (half the u16 tables'
// traffic per pass) in MFMA fragment order; a 16 x 64 block with a cell over 127 is flagged and
// zero in the i8 table, and its u16 counts (NA / NB storage) are summed in f64 by the pass.
#include "lfe_internal.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace lfe {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef unsigned short us4 __attribute__((ext_vector_type(4)));

constexpr int kDnHC = 64;      // primary groups per build workgroup (LDS: kDnHC x GQ16 u16 counters)
constexpr int kDnWaves = 16;   // waves per workgroup of the product passes
constexpr int kDnThreads = 64 * kDnWaves;

struct DnBuildArgs {
  const int4* items;      // work items (bucket, r0, r1): a bucket's rows are its items' union
  const int32_t* bitems;  // [nb + 1] first item of each bucket
  const int32_t* blist;   // [nbe] buckets that hold rows
  const int32_t* codeP;   // layout order; -1: a dropped row
  const int32_t* codeQ;
  int nbe, s, B, GQ16, nch;
  int GQW;                // LDS counter row width (GQ16, or GQ64 for the i8 tables)
  uint16_t* NA;           // u16 tables (dn8: the counts of flagged blocks only, 16 x 64 natural order)
  uint16_t* NB;
  // dn8: i8 fragment tables and per-block flags
  int dn8, GQ64, fa_stride, fb_stride;
  int8_t* NA8;            // [bi][hb][q kb] 1 KB: lane (g, i) bytes jj = count (16 hb + i, 64 kb + 16 g + jj)
  int8_t* NB8;            // [bi][qb][h kb] 1 KB: lane (g, i) bytes jj = count (64 kb + 16 g + jj, 16 qb + i)
  uint8_t* FA;            // [bi][hb][fa_stride]: block has a count > 127
  uint8_t* FB;            // [bi][qb][fb_stride]
  // pre-filter mode (the table built before the singleton marks, every row counted): the
  // pre-filter counts of both FEs from the table's row / column sums, replacing the layout
  // histograms; flag: a primary level with more than 65535 rows (a 16-bit cell could have wrapped)
  int32_t* cntP;
  int32_t* cntQ;
  int32_t* flag;
  int G_P, G_Q;
  // one rank: the singleton test of k_any_singleton folded in - a primary count of 1 where it is
  // written; the secondary counts (summed by atomics over the workgroups) by launch_any_eq1 after
  int32_t* any;
};

// pre-filter mode: row sums of the chunk's counters = the primary counts of its groups (each group is
// one workgroup's), column sums added into the secondary counts (integer atomics: any order)
template <typename CT>
__device__ void dn_counts(const DnBuildArgs& a, const CT* cnt, int hlo, int HW) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int r = wave; r < HW; r += nw) {
    int s = 0;
    for (int q = lane; q < a.GQW; q += 64) s += (int)cnt[r * a.GQW + q];
    for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
    if (lane == 0 && hlo + r < a.G_P) {
      a.cntP[hlo + r] = s;
      if (s > 65535) atomicOr(a.flag, 1);
      if (s == 1 && a.any) atomicAdd(a.any, 1);
    }
  }
  for (int q = threadIdx.x; q < a.G_Q; q += blockDim.x) {
    int s = 0;
    for (int r = 0; r < HW; ++r) s += (int)cnt[r * a.GQW + q];
    if (s) atomicAdd(&a.cntQ[q], s);
  }
}

// Counts of the bucket's kept rows with h in [hlo, hlo + HW) into LDS counters of CT (8 or 16
// bits, packed in 32-bit words: cnt[h - hlo][q]); returns whether some 8-bit counter overflowed.
template <typename CT>
__device__ bool dn_count(const DnBuildArgs& a, uint32_t* cw, int hlo, int HW, int r0, int r1) {
  constexpr int PER = 4 / sizeof(CT), SH = 8 * sizeof(CT);
  const int W = a.GQW / PER;  // words per group row
  __shared__ int ovf;
  for (int j = threadIdx.x; j < HW * W; j += blockDim.x) cw[j] = 0u;
  if (threadIdx.x == 0) ovf = 0;
  __syncthreads();
  bool over = false;
  auto one = [&](int h, int q) {
    const uint32_t d = (uint32_t)(h - hlo);
    if (h < 0 || d >= (uint32_t)HW) return;
    const int sh = (q % PER) * SH;
    const uint32_t old = atomicAdd(&cw[d * W + q / PER], 1u << sh);
    if (sizeof(CT) == 1 && ((old >> sh) & 0xffu) == 0xffu) over = true;  // carried into the next byte
  };
  // 16-byte code loads over the 4-aligned middle, four of each in flight per thread (the rows of
  // a bucket are read by its workgroups: from L2 or the Infinity Cache after the first; eight in
  // flight measured the same, 0.276 vs 0.269 ms per build at 50M rows)
  const int a0 = min(r1, (r0 + 3) & ~3), a1 = max(a0, r1 & ~3);
  for (int row = r0 + (int)threadIdx.x; row < a0; row += blockDim.x) one(a.codeP[row], a.codeQ[row]);
  for (int row = a1 + (int)threadIdx.x; row < r1; row += blockDim.x) one(a.codeP[row], a.codeQ[row]);
  const int4* cP = reinterpret_cast<const int4*>(a.codeP);
  const int4* cQ = reinterpret_cast<const int4*>(a.codeQ);
  constexpr int V = 4;
  for (int v0 = a0 / 4 + (int)threadIdx.x; v0 < a1 / 4; v0 += V * blockDim.x) {
    int4 hv[V], qv[V];
#pragma unroll
    for (int u = 0; u < V; ++u) {
      const int v = v0 + u * blockDim.x;
      hv[u] = v < a1 / 4 ? cP[v] : int4{-1, -1, -1, -1};
      qv[u] = v < a1 / 4 ? cQ[v] : int4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < V; ++u) {
      one(hv[u].x, qv[u].x);
      one(hv[u].y, qv[u].y);
      one(hv[u].z, qv[u].z);
      one(hv[u].w, qv[u].w);
    }
  }
  if (over) ovf = 1;
  __syncthreads();
  return ovf != 0;
}

// NA and NB blocks of the primary group blocks [hb0, hb0 + HW / 16) from the LDS counters
template <typename CT>
__device__ void dn_write(const DnBuildArgs& a, const CT* cnt, int bi, int hb0, int HW) {
  const int nqb = a.GQ16 >> 4, nhb = a.B >> 4, hbl_n = HW / 16;
  const int nel4 = hbl_n * nqb * 64;  // 4 counts (8 bytes) per store
  us4* na = reinterpret_cast<us4*>(a.NA + (int64_t)bi * nhb * nqb * 256);
  for (int e = threadIdx.x; e < nel4; e += blockDim.x) {  // NA blocks (hb, qb): rows h, 4 q's per store
    const int blk = e >> 6, el = (e & 63) * 4, hbl = blk / nqb, qb = blk - hbl * nqb;
    const CT* src = cnt + (hbl * 16 + (el >> 4)) * a.GQW + qb * 16 + (el & 15);
    na[((int64_t)(hb0 + hbl) * nqb + qb) * 64 + (e & 63)] = us4{src[0], src[1], src[2], src[3]};
  }
  us4* nbp = reinterpret_cast<us4*>(a.NB + (int64_t)bi * nqb * nhb * 256);
  for (int e = threadIdx.x; e < nel4; e += blockDim.x) {  // NB blocks (qb, hb): rows q, 4 h's per store
    const int blk = e >> 6, el = (e & 63) * 4, qb = blk / hbl_n, hbl = blk - qb * hbl_n;
    const CT* src = cnt + (hbl * 16 + (el & 15)) * a.GQW + qb * 16 + (el >> 4);
    nbp[((int64_t)qb * nhb + hb0 + hbl) * 64 + (e & 63)] = us4{src[0], src[a.GQW], src[2 * a.GQW], src[3 * a.GQW]};
  }
}

// dn8: the i8 fragment blocks of the primary rows [hb0 16, hb0 16 + HW) (HW = 64 or 128: whole
// 64-row h k-blocks) from the LDS counters.  Every fragment is written as its counts' low bytes in
// one pass (an NA8 fragment is 16 contiguous counters, an NB8 fragment 16 counters a row apart);
// a block holding a count over 127 is flagged, then (rare) zeroed in the i8 table and stored as u16
// (16 x 64, natural order) in NA / NB.
template <typename CT>
__device__ void dn_write8(const DnBuildArgs& a, const CT* cnt, int bi, int hb0, int HW) {
  __shared__ int ov[1024];
  typedef int v4 __attribute__((ext_vector_type(4)));
  const int nkq = a.GQ64 >> 6, nhb = a.B >> 4, nqb = a.GQ64 >> 4, nhk = a.B >> 6;
  const int hbl_n = HW >> 4, hkl_n = HW >> 6, hk0 = hb0 >> 2;
  const int na_b = hbl_n * nkq, nb_b = nqb * hkl_n;
  for (int j = threadIdx.x; j < na_b + nb_b; j += blockDim.x) ov[j] = 0;
  __syncthreads();
  for (int e = threadIdx.x; e < na_b * 64; e += blockDim.x) {
    const int blk = e >> 6, l = e & 63, hbl = blk / nkq, kb = blk - hbl * nkq;
    const CT* src = cnt + (hbl * 16 + (l & 15)) * a.GQW + kb * 64 + 16 * (l >> 4);
    v4 w;
    bool big;
    if (sizeof(CT) == 1) {  // 16 byte counters: one 16-byte LDS read, a byte over 127 has its top bit
      w = *reinterpret_cast<const v4*>(src);
      big = ((w.x | w.y | w.z | w.w) & 0x80808080) != 0;
    } else {
      const v4 u0 = reinterpret_cast<const v4*>(src)[0], u1 = reinterpret_cast<const v4*>(src)[1];
      const int hi = (u0.x | u0.y | u0.z | u0.w | u1.x | u1.y | u1.z | u1.w) & (int)0xff80ff80;
      big = hi != 0;
      // two u16 counters per word -> their low bytes, four per word
      auto pk = [](int x, int y) {
        const uint32_t ux = (uint32_t)x, uy = (uint32_t)y;
        return (int)((ux & 0xffu) | ((ux >> 8) & 0xff00u) | ((uy & 0xffu) << 16) | ((uy << 8) & 0xff000000u));
      };
      w = v4{pk(u0.x, u0.y), pk(u0.z, u0.w), pk(u1.x, u1.y), pk(u1.z, u1.w)};
    }
    if (big) ov[blk] = 1;
    *reinterpret_cast<v4*>(a.NA8 + (((int64_t)bi * nhb + hb0 + hbl) * nkq + kb) * 1024 + l * 16) = w;
  }
  for (int e = threadIdx.x; e < nb_b * 64; e += blockDim.x) {
    const int blk = e >> 6, l = e & 63, qb = blk / hkl_n, hkl = blk - qb * hkl_n;
    const CT* src = cnt + (hkl * 64 + 16 * (l >> 4)) * a.GQW + qb * 16 + (l & 15);
    v4 w = v4{0, 0, 0, 0};
    int m = 0;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {
      const int v = (int)src[jj * a.GQW];
      m |= v;
      w[jj >> 2] |= (v & 0xff) << (8 * (jj & 3));
    }
    if (m & ~127) ov[na_b + blk] = 1;
    *reinterpret_cast<v4*>(a.NB8 + (((int64_t)bi * nqb + qb) * nhk + hk0 + hkl) * 1024 + l * 16) = w;
  }
  __syncthreads();
  for (int j = threadIdx.x; j < na_b; j += blockDim.x) {
    const int hbl = j / nkq, kb = j - hbl * nkq;
    a.FA[((int64_t)bi * nhb + hb0 + hbl) * a.fa_stride + kb] = (uint8_t)ov[j];
  }
  for (int j = threadIdx.x; j < nb_b; j += blockDim.x) {
    const int qb = j / hkl_n, hkl = j - qb * hkl_n;
    a.FB[((int64_t)bi * nqb + qb) * a.fb_stride + hk0 + hkl] = (uint8_t)ov[na_b + j];
  }
  // the flagged blocks (rare: a (h, q) pair with more than 127 kept rows): i8 block zeroed, counts as u16
  for (int blk = 0; blk < na_b + nb_b; ++blk) {
    if (!ov[blk]) continue;  // uniform (LDS)
    if (blk < na_b) {
      const int hbl = blk / nkq, kb = blk - hbl * nkq;
      const int64_t bo = (((int64_t)bi * nhb + hb0 + hbl) * nkq + kb) * 1024;
      for (int t = threadIdx.x; t < 1024; t += blockDim.x) {
        a.NA[bo + t] = (uint16_t)cnt[(hbl * 16 + (t >> 6)) * a.GQW + kb * 64 + (t & 63)];
        a.NA8[bo + t] = 0;
      }
    } else {
      const int qb = (blk - na_b) / hkl_n, hkl = (blk - na_b) - qb * hkl_n;
      const int64_t bo = (((int64_t)bi * nqb + qb) * nhk + hk0 + hkl) * 1024;
      for (int t = threadIdx.x; t < 1024; t += blockDim.x) {
        a.NB[bo + t] = (uint16_t)cnt[(hkl * 64 + (t & 63)) * a.GQW + qb * 16 + (t >> 6)];
        a.NB8[bo + t] = 0;
      }
    }
  }
}


// 4-bit counters (eight per word, row-major [HW][GQW]) of the chunk's rows with h in [hlo, hlo + HW);
// returns whether a counter reached 16 (it carried into its neighbour: the chunk is counted again)
__device__ bool dn_count4(const DnBuildArgs& a, uint32_t* cw, int hlo, int HW, int r0, int r1) {
  const int W = a.GQW / 8;
  __shared__ int ovf4;
  for (int j = threadIdx.x; j < HW * W; j += blockDim.x) cw[j] = 0u;
  if (threadIdx.x == 0) ovf4 = 0;
  __syncthreads();
  bool over = false;
  auto one = [&](int h, int q) {
    const uint32_t d = (uint32_t)(h - hlo);
    if (h < 0 || d >= (uint32_t)HW) return;
    const int sh = (q & 7) * 4;
    const uint32_t old = atomicAdd(&cw[d * W + (q >> 3)], 1u << sh);
    if (((old >> sh) & 0xfu) == 0xfu) over = true;
  };
  const int a0 = min(r1, (r0 + 3) & ~3), a1 = max(a0, r1 & ~3);
  for (int row = r0 + (int)threadIdx.x; row < a0; row += blockDim.x) one(a.codeP[row], a.codeQ[row]);
  for (int row = a1 + (int)threadIdx.x; row < r1; row += blockDim.x) one(a.codeP[row], a.codeQ[row]);
  const int4* cP = reinterpret_cast<const int4*>(a.codeP);
  const int4* cQ = reinterpret_cast<const int4*>(a.codeQ);
  constexpr int V = 4;
  for (int v0 = a0 / 4 + (int)threadIdx.x; v0 < a1 / 4; v0 += V * blockDim.x) {
    int4 hv[V], qv[V];
#pragma unroll
    for (int u = 0; u < V; ++u) {
      const int v = v0 + u * blockDim.x;
      hv[u] = v < a1 / 4 ? cP[v] : int4{-1, -1, -1, -1};
      qv[u] = v < a1 / 4 ? cQ[v] : int4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < V; ++u) {
      one(hv[u].x, qv[u].x);
      one(hv[u].y, qv[u].y);
      one(hv[u].z, qv[u].z);
      one(hv[u].w, qv[u].w);
    }
  }
  if (over) ovf4 = 1;
  __syncthreads();
  return ovf4 != 0;
}

// four nibbles (the low 16 bits) -> four bytes, in order
__device__ __forceinline__ int nib_spread(uint32_t w) {
  uint32_t t = w & 0xffffu;
  t = (t | (t << 8)) & 0x00ff00ffu;
  t = (t | (t << 4)) & 0x0f0f0f0fu;
  return (int)t;
}

// pre-filter mode on 4-bit counters: as dn_counts
__device__ void dn_counts4(const DnBuildArgs& a, const uint32_t* cw, int hlo, int HW) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6, W = a.GQW / 8;
  for (int r = wave; r < HW; r += nw) {
    int s = 0;
    for (int j = lane; j < W; j += 64) {
      const uint32_t w = cw[r * W + j];
      const uint32_t b = (w & 0x0f0f0f0fu) + ((w >> 4) & 0x0f0f0f0fu);  // four byte sums <= 30
      s += (int)((b * 0x01010101u) >> 24);
    }
    for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
    if (lane == 0 && hlo + r < a.G_P) {
      a.cntP[hlo + r] = s;
      if (s > 65535) atomicOr(a.flag, 1);
      if (s == 1 && a.any) atomicAdd(a.any, 1);
    }
  }
  for (int q = threadIdx.x; q < a.G_Q; q += blockDim.x) {
    int s = 0;
    const int sh = (q & 7) * 4;
    for (int r = 0; r < HW; ++r) s += (int)((cw[r * W + (q >> 3)] >> sh) & 0xfu);
    if (s) atomicAdd(&a.cntQ[q], s);
  }
}

// dn8 fragments of the primary rows [hb0 16, hb0 16 + HW) from 4-bit counters: no count exceeds 15,
// so no block is flagged
__device__ void dn_write4(const DnBuildArgs& a, const uint32_t* cw, int bi, int hb0, int HW) {
  typedef int v4 __attribute__((ext_vector_type(4)));
  const int W = a.GQW / 8;
  const int nkq = a.GQ64 >> 6, nhb = a.B >> 4, nqb = a.GQ64 >> 4, nhk = a.B >> 6;
  const int hbl_n = HW >> 4, hkl_n = HW >> 6, hk0 = hb0 >> 2;
  const int na_b = hbl_n * nkq, nb_b = nqb * hkl_n;
  for (int e = threadIdx.x; e < na_b * 64; e += blockDim.x) {
    const int blk = e >> 6, l = e & 63, hbl = blk / nkq, kb = blk - hbl * nkq;
    const uint32_t* src = cw + (hbl * 16 + (l & 15)) * W + ((kb * 64 + 16 * (l >> 4)) >> 3);
    const uint32_t w0 = src[0], w1 = src[1];
    const v4 w = v4{nib_spread(w0), nib_spread(w0 >> 16), nib_spread(w1), nib_spread(w1 >> 16)};
    *reinterpret_cast<v4*>(a.NA8 + (((int64_t)bi * nhb + hb0 + hbl) * nkq + kb) * 1024 + l * 16) = w;
  }
  for (int e = threadIdx.x; e < nb_b * 64; e += blockDim.x) {
    const int blk = e >> 6, l = e & 63, qb = blk / hkl_n, hkl = blk - qb * hkl_n;
    const int row = hkl * 64 + 16 * (l >> 4), q = qb * 16 + (l & 15), sh = (q & 7) * 4;
    const uint32_t* src = cw + row * W + (q >> 3);
    v4 w = v4{0, 0, 0, 0};
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) w[jj >> 2] |= (int)((src[jj * W] >> sh) & 0xfu) << (8 * (jj & 3));
    *reinterpret_cast<v4*>(a.NB8 + (((int64_t)bi * nqb + qb) * nhk + hk0 + hkl) * 1024 + l * 16) = w;
  }
  for (int j = threadIdx.x; j < na_b; j += blockDim.x) {
    const int hbl = j / nkq, kb = j - hbl * nkq;
    a.FA[((int64_t)bi * nhb + hb0 + hbl) * a.fa_stride + kb] = 0;
  }
  for (int j = threadIdx.x; j < nb_b; j += blockDim.x) {
    const int qb = j / hkl_n, hkl = j - qb * hkl_n;
    a.FB[((int64_t)bi * nqb + qb) * a.fb_stride + hk0 + hkl] = 0;
  }
}

// one 128-group chunk on 8-bit counters, recounted in two halves on 16-bit counters if a pair
// passes 255 rows
__device__ void dn_chunk8(const DnBuildArgs& a, uint32_t* cw, int bi, int hlo, int hb0, int r0, int r1) {
  constexpr int HC = 2 * kDnHC;
  if (!dn_count<uint8_t>(a, cw, hlo, HC, r0, r1)) {
    if (a.cntP) dn_counts<uint8_t>(a, reinterpret_cast<const uint8_t*>(cw), hlo, HC);
    if (a.dn8) dn_write8<uint8_t>(a, reinterpret_cast<const uint8_t*>(cw), bi, hb0, HC);
    else dn_write<uint8_t>(a, reinterpret_cast<const uint8_t*>(cw), bi, hb0, HC);
    return;
  }
  for (int half = 0; half < 2; ++half) {
    __syncthreads();
    dn_count<uint16_t>(a, cw, hlo + half * kDnHC, kDnHC, r0, r1);
    if (a.cntP) dn_counts<uint16_t>(a, reinterpret_cast<const uint16_t*>(cw), hlo + half * kDnHC, kDnHC);
    if (a.dn8) dn_write8<uint16_t>(a, reinterpret_cast<const uint16_t*>(cw), bi, hb0 + half * (kDnHC / 16), kDnHC);
    else dn_write<uint16_t>(a, reinterpret_cast<const uint16_t*>(cw), bi, hb0 + half * (kDnHC / 16), kDnHC);
  }
}

// Workgroup (bucket bi, chunk of HC primary groups): counts the chunk's rows in LDS and writes its
// NA and NB blocks.  HC = 128 groups on 8-bit counters (the bucket's codes are read by B / 128
// workgroups); a chunk where some (h, q) pair holds more than 255 rows is counted again in two
// halves on 16-bit counters (counts <= 65535 by the caller's check).  dn8 tables of sparse panels
// (~0.5 rows per cell): HC = 256 groups on 4-bit counters (the codes read B / 256 times), a chunk
// with a 16-row cell counted again as two 128-group chunks.  The workgroups of a bucket share an
// XCD (block i -> XCD i % 8), so its codes are read from one L2.
__device__ void dn_build_body(const DnBuildArgs& a, uint32_t* cw);

__global__ __launch_bounds__(1024) void k_dn_build(DnBuildArgs a) {
  extern __shared__ uint32_t cw[];  // [HC][GQ16] 8-bit or [HC / 2][GQ16] 16-bit counters
  dn_build_body(a, cw);
}

__device__ void dn_build_body(const DnBuildArgs& a, uint32_t* cw) {
  const int i = blockIdx.x, x = i & 7, r = i >> 3;
  const int chunk = r % a.nch, bi = (r / a.nch) * 8 + x;
  if (bi >= a.nbe) return;
  const int b = a.blist[bi];
  const int it0 = a.bitems[b], it1 = a.bitems[b + 1];
  const int r0 = it1 > it0 ? a.items[it0].y : 0, r1 = it1 > it0 ? a.items[it1 - 1].z : 0;
  const int HC = a.B / a.nch, hlo = (b << a.s) + chunk * HC, hb0 = chunk * (HC / 16);
  if (HC == 4 * kDnHC) {  // 4-bit counters (dn8 only)
    if (!dn_count4(a, cw, hlo, HC, r0, r1)) {
      if (a.cntP) dn_counts4(a, cw, hlo, HC);
      dn_write4(a, cw, bi, hb0, HC);
      return;
    }
    for (int half = 0; half < 2; ++half) {
      __syncthreads();
      dn_chunk8(a, cw, bi, hlo + half * 2 * kDnHC, hb0 + half * (2 * kDnHC / 16), r0, r1);
    }
    return;
  }
  if (HC == 2 * kDnHC) {
    dn_chunk8(a, cw, bi, hlo, hb0, r0, r1);
    return;
  }
  dn_count<uint16_t>(a, cw, hlo, HC, r0, r1);
  if (a.cntP) dn_counts<uint16_t>(a, reinterpret_cast<const uint16_t*>(cw), hlo, HC);
  if (a.dn8) dn_write8<uint16_t>(a, reinterpret_cast<const uint16_t*>(cw), bi, hb0, HC);
  else dn_write<uint16_t>(a, reinterpret_cast<const uint16_t*>(cw), bi, hb0, HC);
}

struct DnPassArgs {
  const uint16_t* Nm;     // NA (K1) or NB (K2)
  const int32_t* blist;
  int nbe, s, B, GQ16, G_Q, G_P, p;
  int KP;                 // waves sharing one output block (k-range parts, summed in part order)
  const double* alpha;    // K1: alpha_Q [G_Q][p]; K2: alpha_P [G_P][p]
  // K1: alpha_P = (S_P - T_P) / n_P
  const double* S_P;
  const int32_t* cntP;
  double* alphaP;
  double* zero_check;     // K1: the stop test's max, zeroed for the check after K2 (or null)
  // K2: per-bucket slots [nbe][G_Q][p]
  double* runs;
};

// R output blocks of 16 rows (K1: primary groups of one bucket; K2: secondary levels) x 16 columns
// per wave (or per KP waves, each over 1 / KP of the k range).  The B operand (the other FE's
// effects) comes from LDS - K1 the whole alpha_Q, K2 the bucket's alpha_P slice - and one B value
// feeds the wave's R blocks.  R = 1: two blocks per wave (half the B reads per MFMA) measured
// slower, K1 + K2 0.71 vs 0.65 ms per solve at 50M rows on one box: the passes are not bound by
// the B operand's LDS reads.
constexpr int kDnR = 1;
template <bool K2>
__global__ __launch_bounds__(kDnThreads) void k_dn_pass(DnPassArgs a) {
  constexpr int R = kDnR;
  extern __shared__ __attribute__((aligned(16))) double tb[];  // K1: [GQ16][p]; K2: [B][p]
  __shared__ d4 red[kDnWaves][64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kq = lane >> 4, c = lane & 15;
  const int p = a.p, nqb = a.GQ16 >> 4, nhb = a.B >> 4;
  const int upw = kDnWaves / a.KP * R;             // output blocks per workgroup
  const int nrb = K2 ? nqb : nhb;                  // output blocks per bucket
  const int nkb = K2 ? nhb : nqb;                  // k blocks per output block
  // workgroups never straddle buckets (K2 stages the bucket's slice)
  const int wgpb = (nrb + upw - 1) / upw;
  const int bi = blockIdx.x / wgpb;
  const int rb0 = (blockIdx.x - bi * wgpb) * upw + (wave / a.KP) * R;  // the wave's first block
  const int part = wave % a.KP;
  const int b = a.blist[bi];
  const int lo = b << a.s;
  if (K2) {  // the bucket's alpha_P rows (rows past G_P: 0)
    const int nv = max(0, min(a.B, a.G_P - lo)) * p;
    for (int j = tid; j < a.B * p; j += kDnThreads) tb[j] = j < nv ? a.alpha[(int64_t)lo * p + j] : 0.0;
  } else {
    const int nv = a.G_Q * p;
    for (int j = tid; j < a.GQ16 * p; j += kDnThreads) tb[j] = j < nv ? a.alpha[j] : 0.0;
    if (a.zero_check && blockIdx.x == 0 && tid == 0) *a.zero_check = 0.0;
  }
  __syncthreads();
  const int cc = c < p ? c : 0;
#ifndef LFE_DN_CH
#define LFE_DN_CH 4
#endif
  constexpr int CH = LFE_DN_CH;  // accumulator chains per block (steps t, and k-block parity at 8)
  d4 acc[R][CH];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int t = 0; t < CH; ++t) acc[r][t] = d4{0.0, 0.0, 0.0, 0.0};
  if (rb0 < nrb) {
    const int k0 = part * nkb / a.KP, k1 = (part + 1) * nkb / a.KP;
    // lane (kq, c): counts of row 16 rb + c at k = 16 kb + 4 kq + t; the matching B row is k.  A
    // block past the bucket's last (odd nrb) reads block rb0's counts and is not stored.
    const uint16_t* nm[R];
#pragma unroll
    for (int r = 0; r < R; ++r)
      nm[r] = a.Nm + (((int64_t)bi * nrb + min(rb0 + r, nrb - 1)) * nkb) * 256 + c * 16 + 4 * kq;
    // two register sets of U k blocks' counts: the next set is in flight while the MFMAs consume
    // the current one.  Loads are unconditional (a block index past the range is clamped: valid
    // memory, its MFMAs skipped), so the compiler keeps them out of branches, and a set's B values
    // are all read from LDS before its MFMAs; four accumulator chains per block.
    constexpr int U = 4;
    auto load = [&](us4 (&nv)[U][R], int kb) {
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < R; ++r)
          nv[u][r] = *reinterpret_cast<const us4*>(nm[r] + (int64_t)min(kb + u, k1 - 1) * 256);
    };
    auto use = [&](const us4 (&nv)[U][R], int kb) {
      double bv[U][4];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int kr = min(kb + u, k1 - 1) * 16 + 4 * kq;
#pragma unroll
        for (int t = 0; t < 4; ++t) bv[u][t] = tb[(kr + t) * p + cc];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (kb + u >= k1) break;  // wave-uniform
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const double b = c < p ? bv[u][t] : 0.0;
#pragma unroll
          for (int r = 0; r < R; ++r)
            acc[r][(t + 4 * u) % CH] =
                __builtin_amdgcn_mfma_f64_16x16x4f64((double)nv[u][r][t], b, acc[r][(t + 4 * u) % CH], 0, 0, 0);
        }
      }
    };
    us4 na[U][R], nb[U][R];
    load(na, k0);
    for (int kb = k0; kb < k1; kb += 2 * U) {
      load(nb, kb + U);
      use(na, kb);
      if (kb + U >= k1) break;
      load(na, kb + 2 * U);
      use(nb, kb + U);
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    d4 d = (acc[r][0] + acc[r][1]) + (acc[r][2] + acc[r][3]);
#pragma unroll
    for (int t = 4; t < CH; ++t) d += acc[r][t];
    if (a.KP > 1) {  // the KP parts of an output block, added in part order (every wave syncs)
      __syncthreads();
      if (part != 0) red[wave][lane] = d;
      __syncthreads();
      if (part != 0) continue;
      for (int k = 1; k < a.KP; ++k) d += red[wave + k][lane];
    }
    const int rb = rb0 + r;
    if (rb >= nrb || c >= p) continue;
    // lane (kq, c), register rr: row 16 rb + kq + 4 rr of the output block, column c
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = rb * 16 + kq + 4 * rr;
      if (K2) {
        if (row < a.G_Q) a.runs[((int64_t)bi * a.G_Q + row) * p + c] = d[rr];
      } else {
        const int h = lo + row;
        if (row < a.B && h < a.G_P) {
          const int32_t n = a.cntP[h];
          const int64_t e = (int64_t)h * p + c;
          a.alphaP[e] = n > 0 ? (a.S_P[e] - d[rr]) / (double)n : 0.0;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// dn8: the passes on v_mfma_i32_16x16x64_i8
// ---------------------------------------------------------------------------
// Operand maps (tools/mfma_i8_probe.hip, exact integer data): lane l = (g = l >> 4, i = l & 15)
// holds A[row i][k = 16 g + jj] and B[k = 16 g + jj][col i] in bytes jj = 0..15; D (4 x i32):
// row 4 g + x, col i.  A = the count fragments of the tables, B = the digit fragments of the other
// FE's effects, [kb][digit][1 KB] per 512-row tile, lane l's 16 bytes at l * 16.
typedef int v4i __attribute__((ext_vector_type(4)));
constexpr int kDn8Tile = 512;           // k rows per digit tile (8 k blocks of 64)
constexpr int kDn8TileBytes = 8 * 8 * 1024;

// balanced base-128 digits of A = round(v * s1 * s2) (|A| <= 2^54; s1, s2 powers of two, so both
// products are exact): A = hi 2^28 + lo with |hi| <= 2^26, |lo| <= 2^27 split in f64 (exact:
// integers), then four digits in [-64, 63] from each int32 half (lo's remainder, in [-1, 1], carried
// into hi)
__device__ __forceinline__ void dn8_split(double v, double s1, double s2, int (&dg)[8]) {
  const double A = rint(v * s1 * s2);
  const double hf = rint(A * 0x1p-28);
  int lo = (int)__builtin_fma(hf, -0x1p28, A);
  int hi = (int)hf;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    int r = lo & 127;
    r -= (r & 64) << 1;
    dg[d] = r;
    lo = (lo - r) >> 7;
  }
  hi += lo;
#pragma unroll
  for (int d = 4; d < 8; ++d) {
    int r = hi & 127;
    r -= (r & 64) << 1;
    dg[d] = r;
    hi = (hi - r) >> 7;
  }
}

// One tile of rows [0, rows) (rows <= 512) of a row-major [.][p] table (p <= 16) into digit
// fragments fr [8 kb][8 d][1024] and per-column scales sc[16] = 2^(e - 54) (NaN for a column with a
// non-finite value, so that it propagates), by a block of NT threads.  Thread t holds column t & 15
// of RPT consecutive rows in registers: one round of loads, no dependent load chain.
// mid() runs right after the tile's loads are issued (the caller's own loads - the streaming
// passes' A ring - then queue behind them instead of in front: vmcnt retires loads in order)
struct Dn8NoMid {
  __device__ void operator()() const {}
};
// Dynamic-range guard.  Digits keep every effect to 2^-54 of its tile's largest, so
// an effect below 2^-kDn8RangeBits of the largest keeps fewer than 54 - kDn8RangeBits bits (f64
// keeps 53 of each).  When more than a quarter of a tile column's nonzero effects lie that far
// below its largest (one level with a 1e8 effect, a 5e9 outlier's group), the tile sets *rflag and
// the solve is redone without the dense cross terms (lfe_demean): the result is then the row
// passes', whose rounding is the f64 sums' own.
constexpr int kDn8RangeBits = 16;

template <int NT, class Mid = Dn8NoMid>
__device__ void dn8_tile_digits(const double* __restrict__ src, int rows, int p, int ld, int8_t* __restrict__ fr,
                                double* __restrict__ sc, double* __restrict__ red, Mid mid = Mid(),
                                unsigned long long* tdbg = nullptr, double* rflag = nullptr) {
  constexpr int RPT = kDn8Tile * 16 / NT;  // rows per thread (32 or 16)
  const int tid = threadIdx.x, col = tid & 15, r0 = (tid >> 4) * RPT;
  double v[RPT];
#pragma unroll
  for (int u = 0; u < RPT; ++u) v[u] = (col < p && r0 + u < rows) ? src[(int64_t)(r0 + u) * ld + col] : 0.0;
  mid();
  if (tdbg && tid == 0) {  // diagnostic phase stamps (LFE_DN8_TIMING): this thread's loads landed
    __builtin_amdgcn_s_waitcnt(0);
    tdbg[0] = wall_clock64();
  }
  double m = 0.0;
  bool bad = false;
#pragma unroll
  for (int u = 0; u < RPT; ++u) {
    bad |= !isfinite(v[u]);
    m = fmax(m, fabs(v[u]));
  }
  // column max over the wave's four row groups (lanes c, c + 16, c + 32, c + 48), then over the
  // waves: 16 LDS values per column instead of a 64-long serial loop (NaN marks a bad column)
  double mv = bad ? __builtin_nan("") : m;
#pragma unroll
  for (int off = 16; off < 64; off <<= 1) {
    const double o = __shfl_xor(mv, off, 64);
    mv = (isnan(o) || isnan(mv)) ? __builtin_nan("") : fmax(mv, o);
  }
  constexpr int NW = NT / 64;
  if ((tid & 63) < 16) red[(tid >> 6) * 16 + col] = mv;
  __syncthreads();
  if (tdbg && tid == 0) tdbg[1] = wall_clock64();
  if (tid < 16) {
    double mm = 0.0;
    bool nb = false;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const double t = red[w * 16 + tid];
      nb |= isnan(t);
      mm = fmax(mm, t);
    }
    // max |alpha| < 2^e.  The digit scale 2^(54 - e) goes in two factors, each finite down to the
    // smallest subnormals (one factor overflows for e < -969); e >= -1020 keeps the
    // inverse scale 2^(e - 54) >= 2^-1074 exact, and every subnormal effect an exact integer
    const int e = mm > 0.0 ? max(ilogb(mm) + 1, -1020) : 0;
    sc[tid] = nb ? __builtin_nan("") : ldexp(1.0, e - 54);
    red[NT + tid] = (double)e;
  }
  __syncthreads();
  if (tdbg && tid == 0) tdbg[2] = wall_clock64();
  const int ec = (int)red[NT + col], h1 = (54 - ec) >> 1;
  const double s1 = ldexp(1.0, h1), s2 = ldexp(1.0, 54 - ec - h1);
  // rows 4 q .. 4 q + 3 of the thread's -> one 32-bit word per digit at lane (16 g + col), bytes 4 jq
#pragma unroll
  for (int q4 = 0; q4 < RPT / 4; ++q4) {
    const int rq = (r0 >> 2) + q4, kb = rq >> 4, g = (rq >> 2) & 3, jq = rq & 3;
    int word[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const double x = v[4 * q4 + u];
      int dg[8];
      dn8_split(isfinite(x) ? x : 0.0, s1, s2, dg);
#pragma unroll
      for (int d = 0; d < 8; ++d) word[d] |= (dg[d] & 255) << (8 * u);
    }
    const int off = (16 * g + col) * 16 + 4 * jq;
#pragma unroll
    for (int d = 0; d < 8; ++d) *reinterpret_cast<int*>(fr + (kb * 8 + d) * 1024 + off) = word[d];
  }
  if (rflag) {  // the guard: per column, effects far below the largest vs nonzero effects
    const double thr = ldexp(1.0, ec - kDn8RangeBits);
    int pk = 0;  // small | nonzero << 16 (each <= 512 per column)
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      const double x = fabs(v[u]);
      // (a subnormal effect keeps fewer bits in f64 too: not counted as small)
      pk += (x != 0.0) ? ((x < thr && x >= 0x1p-1022 ? 1 : 0) | (1 << 16)) : 0;
    }
    pk += __shfl_xor(pk, 16, 64);
    pk += __shfl_xor(pk, 32, 64);
    // red's first NW x 16 slots (the column maxima) were read before the second barrier
    if ((tid & 63) < 16) red[(tid >> 6) * 16 + col] = (double)pk;
    __syncthreads();
    if (tid < 16 && !isnan(sc[tid])) {
      int small = 0, nz = 0;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        const int t = (int)red[w * 16 + tid];
        small += t & 0xffff;
        nz += t >> 16;
      }
      if (4 * small > nz) *rflag = 1.0;
    }
  }
}

// alpha_Q -> digit tiles dq [tile][kb][d][1 KB] and scales eq [tile][16] (one block per tile)
__global__ __launch_bounds__(256) void k_dn8_digits(const double* __restrict__ alpha, int G, int p, int ld,
                                                    int8_t* __restrict__ dq, double* __restrict__ eq,
                                                    double* __restrict__ rflag) {
  extern __shared__ __attribute__((aligned(16))) int8_t fr[];
  __shared__ double red[256 + 16];
  __shared__ double sc[16];
  const int t = blockIdx.x, r0 = t * kDn8Tile;
  dn8_tile_digits<256>(alpha + (int64_t)r0 * ld, min(kDn8Tile, G - r0), p, ld, fr, sc, red, Dn8NoMid(), nullptr,
                       rflag);
  __syncthreads();
  const int4* s4 = reinterpret_cast<const int4*>(fr);
  int4* d4p = reinterpret_cast<int4*>(dq + (int64_t)t * kDn8TileBytes);
  for (int j = threadIdx.x; j < kDn8TileBytes / 16; j += blockDim.x) d4p[j] = s4[j];
  if (threadIdx.x < 16) eq[t * 16 + threadIdx.x] = sc[threadIdx.x];
}

struct Dn8Args {
  const int8_t* Nm;       // NA8 (K1) or NB8 (K2)
  const uint8_t* flags;   // FA / FB: block holds a count over 127 (its u16 counts in X)
  int fstride;
  const uint16_t* X;      // the flagged blocks' u16 counts (16 x 64, natural order)
  const int32_t* blist;
  int nbe, s, B, G_Q, G_P, p;
  int lda, ldo;           // row strides: K1 alpha_Q / S_P and alpha_P, K2 alpha_P / the slots (the
                          // fit's p; `p` is then the pass's column group, <= 16)
  int nkb;                // 64-row k blocks per output block (K1: GQ64 / 64, K2: B / 64)
  int nrb;                // output blocks per bucket (K1: B / 16, K2: GQ64 / 16)
  int rbw;                // output blocks per workgroup
  const int8_t* dq;       // K1: alpha_Q digit tiles
  const double* eq;       // K1: their scales
  const double* alpha;    // K1: alpha_Q (flagged blocks); K2: alpha_P (digitized per bucket tile)
  const double* S_P;      // K1: alpha_P = (S_P - T_P) / n_P
  const int32_t* cntP;
  double* alphaP;
  double* zero_check;
  double* runs;           // K2: per-bucket slots [nbe][G_Q][p]
  double* rflag;          // the digits' dynamic-range guard (dn8_tile_digits: 1.0 when set), null: off
  unsigned long long* dbg;  // diagnostic (LFE_DN8_TIMING): per workgroup wall clock at start / prologue end / end
};

// K1 (K2 = false): T_P of R output blocks (16 primary groups each) per wave; K2: T_Q,b of R blocks
// of 16 secondary levels.  Per tile: its digit fragments staged in LDS (K1: copied from k_dn8_digits'
// output; K2: the bucket's alpha_P rows digitized here), the A fragments of the next k block in
// flight while 8 digit MFMAs per block run, then the int32 sums of the tile to f64 and the flagged
// blocks' f64 sums, in that fixed order.
template <bool K2, int R>
__global__ __launch_bounds__(512) void k_dn8_pass(Dn8Args a) {
  extern __shared__ __attribute__((aligned(16))) int8_t fr[];  // [8 kb][8 d][1024]
  __shared__ double red[512 + 16];
  __shared__ double sc[16];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c = lane & 15;
  const int p = a.p;
  const int wgpb = (a.nrb + a.rbw - 1) / a.rbw;
  const int bi = blockIdx.x / wgpb;
  const int rb0 = (blockIdx.x - bi * wgpb) * a.rbw + wave * R;
  const int b = a.blist[bi];
  const int lo = b << a.s;
  if (!K2 && a.zero_check && blockIdx.x == 0 && tid == 0) *a.zero_check = 0.0;
  double acc[R][4];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int x = 0; x < 4; ++x) acc[r][x] = 0.0;
  const int8_t* nm[R];
#pragma unroll
  for (int r = 0; r < R; ++r)
    nm[r] = a.Nm + ((int64_t)bi * a.nrb + min(rb0 + r, a.nrb - 1)) * a.nkb * 1024 + lane * 16;
  const int ntile = (a.nkb + 7) / 8;
  for (int t = 0; t < ntile; ++t) {
    const int kb0 = t * 8, nk = min(8, a.nkb - kb0);
    __syncthreads();
    if (K2) {
      const int r0 = lo + t * kDn8Tile;
      dn8_tile_digits<512>(a.alpha + (int64_t)r0 * a.lda, max(0, min(kDn8Tile, min(a.B - t * kDn8Tile, a.G_P - r0))),
                           p, a.lda, fr, sc, red, Dn8NoMid(), nullptr, a.rflag);
    } else {
      // the tile's fragments, every load of a thread issued before its stores (4 KB per thread
      // round: no chain of L2 round trips)
      const int4* s4 = reinterpret_cast<const int4*>(a.dq + (int64_t)t * kDn8TileBytes);
      int4* d4p = reinterpret_cast<int4*>(fr);
      constexpr int kStage = 16;  // int4 per thread per round (256 threads: one 64 KB tile)
      for (int j0 = 0; j0 < nk * 512; j0 += kStage * (int)blockDim.x) {
        int4 tmp[kStage];
#pragma unroll
        for (int u = 0; u < kStage; ++u) {
          const int j = j0 + u * (int)blockDim.x + tid;
          tmp[u] = j < nk * 512 ? s4[j] : int4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < kStage; ++u) {
          const int j = j0 + u * (int)blockDim.x + tid;
          if (j < nk * 512) d4p[j] = tmp[u];
        }
      }
      if (tid < 16) sc[tid] = a.eq[t * 16 + tid];
    }
    // the tile's A fragments, all in flight together (the table streams from HBM), and its blocks'
    // flags: one 8-byte word per output block (fstride and kb0 are multiples of 8)
    v4i A[R][8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int r = 0; r < R; ++r)
        A[r][k] = *reinterpret_cast<const v4i*>(nm[r] + (int64_t)(kb0 + min(k, nk - 1)) * 1024);
    uint64_t fw[R];
#pragma unroll
    for (int r = 0; r < R; ++r)
      fw[r] = *reinterpret_cast<const uint64_t*>(a.flags + ((int64_t)bi * a.nrb + min(rb0 + r, a.nrb - 1)) * a.fstride + kb0);
    __syncthreads();
    v4i D[R][8];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int d = 0; d < 8; ++d) D[r][d] = v4i{0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k >= nk) break;  // uniform
#pragma unroll
      for (int d = 0; d < 8; ++d) {
        const v4i bv = *reinterpret_cast<const v4i*>(fr + (k * 8 + d) * 1024 + lane * 16);
#pragma unroll
        for (int r = 0; r < R; ++r) D[r][d] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[r][k], bv, D[r][d], 0, 0, 0);
      }
    }
    // the tile's exact digit sums -> f64 (digit order), then its flagged blocks
    const double s0 = sc[c];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      double tsum[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int d = 7; d >= 0; --d) {
        const double sd = ldexp(s0, 7 * d);
#pragma unroll
        for (int x = 0; x < 4; ++x) tsum[x] += (double)D[r][d][x] * sd;
      }
#pragma unroll
      for (int x = 0; x < 4; ++x) acc[r][x] += tsum[x];
      const int rb = rb0 + r;
      if (rb >= a.nrb || fw[r] == 0) continue;  // wave-uniform; a flagged block is rare
      for (int k = 0; k < nk; ++k) {
        if (!((fw[r] >> (8 * k)) & 0xff)) continue;
        const uint16_t* X = a.X + (((int64_t)bi * a.nrb + rb) * a.nkb + kb0 + k) * 1024;
        const int kr0 = (kb0 + k) * 64;  // first k row of the block
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          double sx = 0.0;
          for (int jj = 0; jj < 64; ++jj) {
            const int kr = kr0 + jj;
            double al = 0.0;
            if (c < p) {
              if (K2) al = (kr < a.B && lo + kr < a.G_P) ? a.alpha[(int64_t)(lo + kr) * a.lda + c] : 0.0;
              else al = kr < a.G_Q ? a.alpha[(int64_t)kr * a.lda + c] : 0.0;
            }
            sx += (double)X[(4 * g + x) * 64 + jj] * al;
          }
          acc[r][x] += sx;
        }
      }
    }
  }
  // lane (g, c), register x: row 16 rb + 4 g + x of the output block, column c
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int rb = rb0 + r;
    if (rb >= a.nrb || c >= p) continue;
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const int row = rb * 16 + 4 * g + x;
      if (K2) {
        if (row < a.G_Q) a.runs[((int64_t)bi * a.G_Q + row) * a.ldo + c] = acc[r][x];
      } else {
        const int h = lo + row;
        if (row < a.B && h < a.G_P) {
          const int32_t n = a.cntP[h];
          const int64_t e = (int64_t)h * a.ldo + c;
          a.alphaP[e] = n > 0 ? (a.S_P[e] - acc[r][x]) / (double)n : 0.0;
        }
      }
    }
  }
}

// Streaming forms of the two passes (the default where the k range fits LDS: K1 <= 16 k blocks of
// alpha_Q digits, K2 <= 8).  A pass moves ~100 MB of i8 table against ~2 MFMA-microseconds of
// work: its time is the table's streaming.  Every wave walks the flattened (output block, k block)
// steps of its output blocks with a ring of kDn8Ring A fragments in flight (a load issued 8 steps
// before its MFMAs, across block boundaries), the 8 digit fragments of a step read from LDS into
// separate registers before its 8 MFMAs; per 8 k blocks (one digit tile) the int32 sums go to f64.
// The digit tiles are formed in the workgroup's prologue (K1: all of alpha_Q, persistent
// workgroups, one per CU; K2: the bucket's alpha_P rows, two workgroups per CU).
constexpr int kDn8MaxKb = 16;
constexpr int kDn8Ring = 8;

// the A-fragment ring of one wave: its first kDn8Ring loads are issued before the workgroup's
// digit prologue, so the table's HBM latency overlaps the digitization
struct Dn8Ring {
  v4i A[kDn8Ring];
  int64_t rl;  // load cursor: step -> (row rl, k block kl)
  int kl;
};

__device__ __forceinline__ void dn8_ring_fill(const Dn8Args& a, Dn8Ring& R, int64_t base, int first, int stride,
                                              int end, int lane) {
  R.rl = base + first;
  R.kl = 0;
  if (first >= end) return;
  const int nkb = a.nkb;
  const int steps = (end - first + stride - 1) / stride * nkb;
  const int8_t* tab = a.Nm + lane * 16;
#pragma unroll
  for (int u = 0; u < kDn8Ring; ++u) {
    if (u < steps) R.A[u] = *reinterpret_cast<const v4i*>(tab + (R.rl * nkb + R.kl) * 1024);
    if (++R.kl == nkb) {
      R.kl = 0;
      R.rl += stride;
    }
  }
}

// the steps of one wave: output blocks first, first + stride, ... < end (table rows base + i)
template <bool K2>
__device__ __forceinline__ void dn8_wave_stream(const Dn8Args& a, const int8_t* __restrict__ fr,
                                                const double* __restrict__ sc, int64_t base, int first, int stride,
                                                int end, int lane, Dn8Ring& R) {
  const int g = lane >> 4, c = lane & 15, p = a.p, nkb = a.nkb;
  if (first >= end) return;
  const int nblk = (end - first + stride - 1) / stride;
  const int steps = nblk * nkb;
  const int8_t* tab = a.Nm + lane * 16;
  auto adv_l = [&]() {
    if (++R.kl == nkb) {
      R.kl = 0;
      R.rl += stride;
    }
  };
  // consume cursor
  int64_t rc = base + first;
  int kc = 0;
  v4i D[8];
#pragma unroll
  for (int d = 0; d < 8; ++d) D[d] = v4i{0, 0, 0, 0};
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  uint64_t fw0 = 0, fw1 = 0;
  // K1: the block's projection operands (n_P and S_P of its rows), loaded at its first step and
  // used at its last, so the epilogue does not wait on dependent global loads
  double sp[4] = {0.0, 0.0, 0.0, 0.0};
  int32_t np4[4] = {0, 0, 0, 0};
  int hrow = 0;
  for (int j0 = 0; j0 < steps; j0 += kDn8Ring) {
#pragma unroll
    for (int u = 0; u < kDn8Ring; ++u) {
      if (j0 + u >= steps) break;  // uniform
      if (kc == 0) {  // the block's flag words (read at its first step, used at its tile ends)
        const uint8_t* fl = a.flags + rc * a.fstride;
        fw0 = *reinterpret_cast<const uint64_t*>(fl);
        fw1 = nkb > 8 ? *reinterpret_cast<const uint64_t*>(fl + 8) : 0ull;
        if (!K2) {
          const int bi = (int)(rc / a.nrb), rb = (int)(rc - (int64_t)bi * a.nrb);
          hrow = (a.blist[bi] << a.s) + rb * 16 + 4 * g;  // rows hrow + q, q < 4
          const int lo = a.blist[bi] << a.s;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int h = hrow + q, row = h - lo;
            const bool ok = c < p && row < a.B && h < a.G_P;
            np4[q] = ok ? a.cntP[h] : 0;
            sp[q] = ok ? a.S_P[(int64_t)h * a.ldo + c] : 0.0;
          }
        }
      }
      const v4i av = R.A[u];
      if (j0 + u + kDn8Ring < steps) R.A[u] = *reinterpret_cast<const v4i*>(tab + (R.rl * nkb + R.kl) * 1024);
      adv_l();
#pragma unroll
      for (int h = 0; h < 2; ++h) {  // the digit fragments in two halves of four (register pressure)
        v4i bv[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) bv[d] = *reinterpret_cast<const v4i*>(fr + (kc * 8 + 4 * h + d) * 1024 + lane * 16);
#pragma unroll
        for (int d = 0; d < 4; ++d) D[4 * h + d] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv[d], D[4 * h + d], 0, 0, 0);
      }
      if ((kc & 7) == 7 || kc == nkb - 1) {  // a digit tile ends: its exact sums to f64, then its flagged blocks
        const int t = kc >> 3;
        const double s0 = sc[t * 16 + c];
        double ts[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int d = 7; d >= 0; --d) {
          const double sd = ldexp(s0, 7 * d);
#pragma unroll
          for (int q = 0; q < 4; ++q) ts[q] += (double)D[d][q] * sd;
          D[d] = v4i{0, 0, 0, 0};
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] += ts[q];
        const uint64_t fw = t ? fw1 : fw0;
        if (fw != 0) {  // rare: blocks with a count over 127, summed in f64 from their u16 counts
          const int bi = (int)(rc / a.nrb), rb = (int)(rc - (int64_t)bi * a.nrb);
          const int lo = a.blist[bi] << a.s;
          for (int k = 0; k < 8 && t * 8 + k < nkb; ++k) {
            if (!((fw >> (8 * k)) & 0xff)) continue;
            const int kb = t * 8 + k;
            const uint16_t* X = a.X + (((int64_t)bi * a.nrb + rb) * nkb + kb) * 1024;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              double sx = 0.0;
              for (int jj = 0; jj < 64; ++jj) {
                const int kr = kb * 64 + jj;
                double al = 0.0;
                if (c < p) {
                  if (K2) al = (kr < a.B && lo + kr < a.G_P) ? a.alpha[(int64_t)(lo + kr) * a.lda + c] : 0.0;
                  else al = kr < a.G_Q ? a.alpha[(int64_t)kr * a.lda + c] : 0.0;
                }
                sx += (double)X[(4 * g + q) * 64 + jj] * al;
              }
              acc[q] += sx;
            }
          }
        }
      }
      if (kc == nkb - 1) {  // the block's outputs: lane (g, c) holds rows 16 rb + 4 g + q of column c
        const int bi = (int)(rc / a.nrb), rb = (int)(rc - (int64_t)bi * a.nrb);
        if (c < p) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int row = rb * 16 + 4 * g + q;
            if (K2) {
              if (row < a.G_Q) a.runs[((int64_t)bi * a.G_Q + row) * a.ldo + c] = acc[q];
            } else {
              const int h = hrow + q;
              if (row < a.B && h < a.G_P)
                a.alphaP[(int64_t)h * a.ldo + c] = np4[q] > 0 ? (sp[q] - acc[q]) / (double)np4[q] : 0.0;
            }
          }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = 0.0;
      }
      if (++kc == nkb) {
        kc = 0;
        rc += stride;
      }
    }
  }
}

// K1, persistent: the digit tiles of alpha_Q formed in LDS by every workgroup, then workgroup i takes
// output blocks [i T / grid, (i + 1) T / grid) of the T = nbe x B/16 primary blocks, wave w every 16th
__global__ __launch_bounds__(1024) void k_dn8_k1s(Dn8Args a) {
  extern __shared__ __attribute__((aligned(16))) int8_t fr[];  // [ntile][8 kb][8 d][1 KB]
  __shared__ double red[1024 + 16];
  __shared__ double sc[32];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), W = blockDim.x >> 6;
  if (a.zero_check && blockIdx.x == 0 && tid == 0) *a.zero_check = 0.0;
  const int64_t total = (int64_t)a.nbe * a.nrb;
  const int i0 = (int)(total * blockIdx.x / gridDim.x), i1 = (int)(total * (blockIdx.x + 1) / gridDim.x);
  if (a.dbg && tid == 0) a.dbg[blockIdx.x * 3] = wall_clock64();
  Dn8Ring R;
  const int ntile = (a.nkb + 7) / 8;
  for (int t = 0; t < ntile; ++t) {
    if (t) __syncthreads();
    // every workgroup forms the same digits (measured faster than one k_dn8_digits pass whose
    // 64 KB tiles every workgroup copies: 0.448 vs 0.474 ms per config-1 solve, round 5)
    dn8_tile_digits<1024>(a.alpha + (int64_t)t * kDn8Tile * a.lda, min(kDn8Tile, a.G_Q - t * kDn8Tile), a.p, a.lda,
                          fr + (size_t)t * kDn8TileBytes, sc + 16 * t, red,
                          [&]() {
                            if (t == 0) dn8_ring_fill(a, R, 0, i0 + wave, W, i1, lane);
                          },
                          nullptr, blockIdx.x == 0 ? a.rflag : nullptr);
  }
  if (ntile == 0) dn8_ring_fill(a, R, 0, i0 + wave, W, i1, lane);
  __syncthreads();
  if (a.dbg && tid == 0) a.dbg[blockIdx.x * 3 + 1] = wall_clock64();
  dn8_wave_stream<false>(a, fr, sc, 0, i0 + wave, W, i1, lane, R);
  if (a.dbg) {
    __syncthreads();
    if (tid == 0) a.dbg[blockIdx.x * 3 + 2] = wall_clock64();
  }
}

// K2: workgroup (bucket bi, part j of np): the bucket's alpha_P rows digitized in LDS, then output
// blocks [j nrb / np, (j + 1) nrb / np) of the bucket's secondary blocks, wave w every 8th
__device__ __forceinline__ void dn8_k2s_body(const Dn8Args& a, int np, int blk) {
  extern __shared__ __attribute__((aligned(16))) int8_t fr[];  // [8 kb][8 d][1 KB]
  __shared__ double red[512 + 16];
  __shared__ double sc[16];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), W = blockDim.x >> 6;
  const int bi = blk / np, part = blk - bi * np;
  const int i0 = a.nrb * part / np, i1 = a.nrb * (part + 1) / np;
  if (a.dbg && tid == 0) a.dbg[blockIdx.x * 3] = wall_clock64();
  Dn8Ring R;
  const int lo = a.blist[bi] << a.s;
  dn8_tile_digits<512>(a.alpha + (int64_t)lo * a.lda, max(0, min(a.B, a.G_P - lo)), a.p, a.lda, fr, sc, red,
                       [&]() { dn8_ring_fill(a, R, (int64_t)bi * a.nrb, i0 + wave, W, i1, lane); },
                       a.dbg ? a.dbg + 3 * 65536 + (size_t)blockIdx.x * 4 : nullptr, a.rflag);
  __syncthreads();
  if (a.dbg && tid == 0) a.dbg[blockIdx.x * 3 + 1] = wall_clock64();
  dn8_wave_stream<true>(a, fr, sc, (int64_t)bi * a.nrb, i0 + wave, W, i1, lane, R);
  if (a.dbg) {
    __syncthreads();
    if (tid == 0) a.dbg[blockIdx.x * 3 + 2] = wall_clock64();
  }
}

__global__ __launch_bounds__(512, 4) void k_dn8_k2s(Dn8Args a, int np) { dn8_k2s_body(a, np, blockIdx.x); }

// several K2-form passes in one launch (the pair-table sweeps: every partner FE and column group of
// one projection), workgroups [start[j], start[j + 1]) running pass j: one launch's latency and
// digit prologues in parallel instead of one launch after another
constexpr int kDn8Batch = 8;
struct Dn8Batch {
  Dn8Args a[kDn8Batch];
  int np[kDn8Batch];
  int start[kDn8Batch + 1];
  int n;
};
__global__ __launch_bounds__(512, 4) void k_dn8_k2s_batch(Dn8Batch b) {
  int j = 0;
  while (j + 1 < b.n && (int)blockIdx.x >= b.start[j + 1]) ++j;
  dn8_k2s_body(b.a[j], b.np[j], (int)blockIdx.x - b.start[j]);
}

// K1's fewest output blocks per workgroup (LFE_DN8_K1_MIN: A/B)
static int64_t dn8_k1_min_blocks() {
  const int64_t v = [] {
    const char* e = knob("LFE_DN8_K1_MIN");
    const long long x = e ? atoll(e) : 4;
    return (int64_t)(x >= 1 ? x : 4);
  }();
  return v;
}

// LFE_DN8_TIMING=1 (diagnostic): per-workgroup phase times of the last K1 / K2 launch to stderr
static bool dn8_timing() {
  const bool on = [] {
    const char* e = knob("LFE_DN8_TIMING");
    return e && e[0] == '1';
  }();
  return on;
}
static unsigned long long* g_dn8_dbg = nullptr;
static int dn8_timing_report(lfe_ctx* c, const char* name, int grid) {
  std::vector<unsigned long long> h((size_t)grid * 3);
  LFE_HIP(hipStreamSynchronize(c->stream));
  LFE_HIP(hipMemcpy(h.data(), g_dn8_dbg, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
  unsigned long long t0 = ~0ull, t1 = 0;
  double pro = 0, str = 0, pro_max = 0, str_max = 0;
  for (int b = 0; b < grid; ++b) {
    t0 = std::min(t0, h[3 * b]);
    t1 = std::max(t1, h[3 * b + 2]);
    const double p = (double)(h[3 * b + 1] - h[3 * b]) / 100.0, q = (double)(h[3 * b + 2] - h[3 * b + 1]) / 100.0;
    pro += p;
    str += q;
    pro_max = std::max(pro_max, p);
    str_max = std::max(str_max, q);
  }
  fprintf(stderr, "[dn8 %s] grid %d span %.1f us, prologue avg %.1f max %.1f us, stream avg %.1f max %.1f us\n", name,
          grid, (double)(t1 - t0) / 100.0, pro / grid, pro_max, str / grid, str_max);
  std::vector<unsigned long long> hd((size_t)grid * 4);
  LFE_HIP(hipMemcpy(hd.data(), g_dn8_dbg + 3 * 65536, sizeof(unsigned long long) * hd.size(), hipMemcpyDeviceToHost));
  double l = 0, r = 0, q = 0, sp = 0;
  int cnt = 0;
  for (int b = 0; b < grid; ++b) {
    if (hd[4 * b] == 0 || hd[4 * b] < h[3 * b]) continue;
    l += (double)(hd[4 * b] - h[3 * b]) / 100.0;
    r += (double)(hd[4 * b + 1] - hd[4 * b]) / 100.0;
    q += (double)(hd[4 * b + 2] - hd[4 * b + 1]) / 100.0;
    sp += (double)(h[3 * b + 1] - hd[4 * b + 2]) / 100.0;
    ++cnt;
  }
  if (cnt)
    fprintf(stderr, "[dn8 %s] first tile: loads %.1f, max + barrier %.1f, scale + barrier %.1f, split + rest %.1f us\n",
            name, l / cnt, r / cnt, q / cnt, sp / cnt);
  LFE_HIP(hipMemset(g_dn8_dbg + 3 * 65536, 0, sizeof(unsigned long long) * hd.size()));
  return LFE_OK;
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------

static int64_t dn_cells(const lfe_ctx* c) {
  const int Q = 1 - c->L.P;
  const int64_t GQ16 = ((int64_t)c->fe[Q].G + 15) / 16 * 16;
  return (int64_t)std::max(c->nbe, 1) * ((int64_t)1 << c->L.s) * GQ16;
}

static int dn_gq64(const lfe_ctx* c) { return (c->fe[1 - c->L.P].G + 63) / 64 * 64; }

// cells of the tables dense_build writes (i8 tables: GQ64 columns)
int64_t dense_table_cells(const lfe_ctx* c) {
  return c->dn8 ? (int64_t)std::max(c->nbe, 1) * ((int64_t)1 << c->L.s) * dn_gq64(c) : dn_cells(c);
}

// the exact i8 passes: the counters of a 64-group chunk of GQ64 columns fit the build's LDS, the
// bucket is whole 64-row k blocks (LFE_DN8=0: the f64 passes, for A/B)
static bool dn8_tiled() {  // A/B: the tiled forms of the i8 passes
  const char* e = knob("LFE_DN8_TILED");
  return e && e[0] == '1';
}

static bool dn8_ok(const lfe_ctx* c) {
  const char* e = knob("LFE_DN8");
  if (e && e[0] == '0') return false;
  const int64_t B = 1ll << c->L.s;
  if (!(B % 64 == 0 && (size_t)kDnHC * dn_gq64(c) * 2 <= 150 * 1024)) return false;
  // more than 16 columns: the streaming passes, one per 16-column group (K1's digit tiles in LDS)
  return c->p <= 16 || (dn_gq64(c) / 64 <= kDn8MaxKb && !dn8_tiled());
}

static bool dn8_ok(const lfe_ctx* c);

// before the singleton marks (prepare_layout, two-FE item path): build the i8 tables on every row and
// take the pre-filter counts from them (dense_build(c, true)) where the dense passes would run on a
// panel without drops (the cmax bound is checked on the device) - LFE_DN_PRE=0 turns it off
bool dense_pre_ok(const lfe_ctx* c) {
  if (c->dense_off) return false;
  const char* e = knob("LFE_DENSE");
  if (e && e[0] == '0') return false;
  const char* pe = knob("LFE_DN_PRE");
  if (pe && pe[0] == '0') return false;
  const int P = c->L.P, Q = 1 - P;
  (void)P;
  if (!(c->world == 1 || c->owner_on) || c->nbe < 1 || !dn8_ok(c)) return false;
  const int64_t B = 1ll << c->L.s;
  (void)Q;
  if (B % kDnHC != 0) return false;
  return (e && e[0] == '1') || (double)c->n >= 0.3 * (double)dn_cells(c);
}

bool dense_ok(const lfe_ctx* c) {
  if (c->dense_off) return false;  // the digits' range guard fired (lfe_demean)
  const char* e = knob("LFE_DENSE");  // "0": never (A/B); "1": whenever it fits
  if (e && e[0] == '0') return false;
  const int P = c->L.P, Q = 1 - P, p = c->p;
  if (!(c->world == 1 || c->owner_on) || c->nbe < 1) return false;
  const int64_t B = 1ll << c->L.s, GQ16 = ((int64_t)c->fe[Q].G + 15) / 16 * 16;
  if (B % kDnHC != 0) return false;
  // the f64 passes hold the B operand tables in LDS (p <= 16); the i8 passes their digit tiles
  if (!dn8_ok(c) && (p > 16 || GQ16 * p * 8 > 100 * 1024 || B * p * 8 > 64 * 1024)) return false;
  if (kDnHC * GQ16 * 2 > 150 * 1024) return false;                        // the build's counters
  if (c->fe[P].cmax > 65535 || c->cmax_over_ranks > 0) return false;      // uint16 counts
  // the products cost ~ the cells (~1.1 ns per cell and pass), the row passes ~ the rows (~3.2 ns
  // per row and pass): dense from 0.3 rows per cell (50M rows over 1e5 x 1e3: 0.5; config 2's 10M:
  // 0.1, where the dense passes measured 1.5x the row passes).  Owner-sharded ranks decide from the
  // whole panel's rows and cells, so every rank takes the same sweeps (a rank on the row
  // layouts beside ranks on the tables rounds its cross terms differently)
  if (e && e[0] == '1') return true;
  if (c->owner_on && c->world > 1) {
    const int64_t nb_all = ((int64_t)c->fe[P].G + B - 1) / B;
    return (double)c->n_kept >= 0.3 * (double)(nb_all * B * GQ16);
  }
  return (double)c->n_kept_local >= 0.3 * (double)dn_cells(c);
}

int dense_build(lfe_ctx* c, bool pre) {
  auto& L = c->L;
  const int Q = 1 - L.P;
  const int B = 1 << L.s, GQ16 = (c->fe[Q].G + 15) / 16 * 16;
  c->dn8 = dn8_ok(c);
  const int GQ64 = dn_gq64(c), GQW = c->dn8 ? GQ64 : GQ16;
  const size_t cells = c->dn8 ? (size_t)std::max(c->nbe, 1) * B * GQ64 : (size_t)dn_cells(c);
  c->dense_cells = (int64_t)cells;
  LFE_TRY(ensure_u16(c, c->dn_na, c->dn_na_cap, cells));
  LFE_TRY(ensure_u16(c, c->dn_nb, c->dn_nb_cap, cells));
  DnBuildArgs a{};
  a.GQW = GQW;
  a.G_P = c->fe[L.P].G;
  a.G_Q = c->fe[Q].G;
  if (pre) {
    a.cntP = c->fe[L.P].cnt_pre;
    a.cntQ = c->fe[Q].cnt_pre;
    a.flag = c->iscratch + kIsDnPre;
    if (c->world == 1) {  // (several ranks: the counts are summed afterwards, k_any_singleton tests them)
      a.any = c->iscratch + kIsAny;
      c->any_ready = true;
    }
  }
  if (c->dn8) {
    const int nbe = std::max(c->nbe, 1);
    a.dn8 = 1;
    a.GQ64 = GQ64;
    a.fa_stride = (GQ64 / 64 + 7) / 8 * 8;
    a.fb_stride = (B / 64 + 7) / 8 * 8;
    LFE_TRY(ensure_i8(c, c->dn8_a, c->dn8_a_cap, cells));
    LFE_TRY(ensure_i8(c, c->dn8_b, c->dn8_b_cap, cells));
    LFE_TRY(ensure_u8(c, c->dn8_fa, c->dn8_fa_cap, (size_t)nbe * (B / 16) * a.fa_stride));
    LFE_TRY(ensure_u8(c, c->dn8_fb, c->dn8_fb_cap, (size_t)nbe * (GQ64 / 16) * a.fb_stride));
    a.NA8 = c->dn8_a;
    a.NB8 = c->dn8_b;
    a.FA = c->dn8_fa;
    a.FB = c->dn8_fb;
  }
  a.items = reinterpret_cast<const int4*>(c->items_d);
  a.bitems = c->bitems_d;
  a.blist = c->blist_d;
  a.codeP = L.code[L.P];
  a.codeQ = L.code[Q];
  a.nbe = c->nbe;
  a.s = L.s;
  a.B = B;
  a.GQ16 = GQ16;
  // 128-group chunks on 8-bit counters (each bucket's codes read B / 128 times) when they fit LDS
  // and still give every CU a workgroup; else 64-group chunks on 16-bit counters (twice the
  // workgroups).  Same box, ms per build: 50M rows 0.269 (8-bit) vs 0.368 (16-bit); the 8-rank
  // owner shard's 25 buckets 0.068 vs 0.055
  const bool c8_fits = (size_t)2 * kDnHC * GQW <= 150 * 1024 && B % (2 * kDnHC) == 0;
  bool c8 = c8_fits && (int64_t)c->nbe * (B / (2 * kDnHC)) >= c->n_cu;
  if (const char* e = knob("LFE_DN_C8")) c8 = c8_fits && e[0] == '1';  // tests: force either form
  // 256-group chunks on 4-bit counters (the i8 tables; half the code reads of the 8-bit form) where
  // cells average under 2 rows (a 16-row cell is then rare) and the chunks still fill the CUs
  const bool c4_fits = c8_fits && c->dn8 && B % (4 * kDnHC) == 0;
  bool c4 = c4_fits && (int64_t)c->nbe * (B / (4 * kDnHC)) >= c->n_cu &&
            (double)c->n < 2.0 * (double)std::max(c->nbe, 1) * B * GQ64;
  if (const char* e = knob("LFE_DN_C4")) c4 = c4_fits && e[0] == '1';  // A/B, tests
  a.nch = B / (c4 ? 4 * kDnHC : c8 ? 2 * kDnHC : kDnHC);
  a.NA = c->dn_na;
  a.NB = c->dn_nb;
  const size_t lds = sizeof(uint16_t) * kDnHC * GQW;  // both forms
  LFE_HIP(set_max_lds(reinterpret_cast<const void*>(&k_dn_build), (int)lds));
  const int grid = (c->nbe + 7) / 8 * 8 * a.nch;
  ProfScope _ps(c, K_LAYOUT_SCATTER);
  hipLaunchKernelGGL(k_dn_build, dim3(grid), dim3(1024), lds, c->stream, a);
  LFE_HIP(hipGetLastError());
  // the secondary FE's singleton levels once its counts are final (its own small kernel: a test in
  // the build's last workgroup cost every workgroup a fence and a counter add, +13 us at 50M rows)
  if (a.any) LFE_TRY(launch_any_eq1(c, a.cntQ, a.G_Q, a.any));
  return LFE_OK;
}

// k-range parts per output block: at least one round of the resident waves (wpc per CU; an owner
// shard has few buckets).  More parts per block cost more than the shorter tail saves (headline,
// same box: K1 + K2 0.66 ms per solve at one round, 0.85 ms at four)
static int dn_parts(const lfe_ctx* c, int blocks, int wpc) {
  int kp = 1;
  int64_t rounds = 1;
  if (const char* e = knob("LFE_DN_ROUNDS")) rounds = std::max(1ll, atoll(e));  // A/B only
  while (kp < kDnWaves && (int64_t)blocks * kp < rounds * c->n_cu * wpc) kp *= 2;
  return kp;
}

static DnPassArgs dn_args(const lfe_ctx* c) {
  const int P = c->L.P, Q = 1 - P;
  DnPassArgs a{};
  a.blist = c->blist_d;
  a.nbe = c->nbe;
  a.s = c->L.s;
  a.B = 1 << c->L.s;
  a.GQ16 = (c->fe[Q].G + 15) / 16 * 16;
  a.G_Q = c->fe[Q].G;
  a.G_P = c->fe[P].G;
  a.p = c->p;
  return a;
}

static Dn8Args dn8_args(const lfe_ctx* c) {
  const int P = c->L.P, Q = 1 - P;
  Dn8Args a{};
  a.blist = c->blist_d;
  a.nbe = c->nbe;
  a.s = c->L.s;
  a.B = 1 << c->L.s;
  a.G_Q = c->fe[Q].G;
  a.G_P = c->fe[P].G;
  a.p = c->p;
  a.lda = a.ldo = c->p;
  a.rflag = c->rflag;
  return a;
}

int range_flag_reset(lfe_ctx* c) {
  LFE_TRY(ensure_f64(c, c->rflag, c->rflag_cap, 2));
  LFE_HIP(hipMemsetAsync(c->rflag, 0, sizeof(double) * 2, c->stream));
  return LFE_OK;
}

// K2 streaming workgroups per bucket (tile): two are resident per CU (64 KB of LDS each), so the
// parts fill one round of those 2 n_cu slots (a second, partial round costs a whole workgroup time:
// 196 buckets x 3 parts = 588 > 512), at least 8 output blocks each
static int k2_parts(const lfe_ctx* c, int nbe, int nrb) {
  int np = (int)std::max<int64_t>(1, (2 * (int64_t)c->n_cu) / std::max(nbe, 1));
  if (const char* e = knob("LFE_K2_NP")) np = std::max(1, atoi(e));  // A/B only
  return std::min(np, std::max(1, nrb / 8));
}

template <bool K2>
static int dn8_launch(lfe_ctx* c, const Dn8Args& a, int waves, int grid) {
  const size_t lds = kDn8TileBytes;
  const void* f1 = reinterpret_cast<const void*>(&k_dn8_pass<K2, 1>);
  const void* f2 = reinterpret_cast<const void*>(&k_dn8_pass<K2, 2>);
  const bool two = a.rbw == 2 * waves;
  LFE_HIP(set_max_lds(two ? f2 : f1, (int)lds));
  if (two) hipLaunchKernelGGL((k_dn8_pass<K2, 2>), dim3(grid), dim3(64 * waves), lds, c->stream, a);
  else hipLaunchKernelGGL((k_dn8_pass<K2, 1>), dim3(grid), dim3(64 * waves), lds, c->stream, a);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

// output blocks per wave: two while that leaves >= 2 workgroups per CU, else one
static int dn8_rbw(const lfe_ctx* c, int nrb, int waves) {
  const int64_t wg2 = (int64_t)std::max(c->nbe, 1) * ((nrb + 2 * waves - 1) / (2 * waves));
  return wg2 >= 2 * (int64_t)c->n_cu ? 2 * waves : waves;
}

int dense_tp(lfe_ctx* c, const double* alphaQ, double* zero_check) {
  const int P = c->L.P;
  if (c->dn8) {
    Dn8Args a = dn8_args(c);
    const int GQ64 = dn_gq64(c), nkb = GQ64 / 64, ntile = (nkb + 7) / 8;
    a.Nm = c->dn8_a;
    a.flags = c->dn8_fa;
    a.fstride = (nkb + 7) / 8 * 8;
    a.X = c->dn_na;
    a.nkb = nkb;
    a.nrb = a.B / 16;
    a.dq = c->dn8_dq;
    a.eq = c->dn8_eq;
    a.alpha = alphaQ;
    a.S_P = c->fe[P].S;
    a.cntP = c->fe[P].cnt;
    a.alphaP = c->fe[P].alpha;
    a.zero_check = zero_check;
    if (nkb <= kDn8MaxKb && !dn8_tiled()) {  // persistent streaming form (LFE_DN8_TILED=1: A/B)
      const size_t lds = (size_t)ntile * kDn8TileBytes;
      LFE_HIP(set_max_lds(reinterpret_cast<const void*>(&k_dn8_k1s), (int)lds));
      const int64_t total = (int64_t)std::max(c->nbe, 1) * a.nrb;
      // every CU a workgroup down to 4 output blocks each: an owner shard's few buckets (the 8-rank
      // shard: 800 blocks) ran on 50 workgroups at 16 blocks each, its stream phase 11.5 us after a
      // 12.7 us digit prologue that more workgroups do not lengthen (LFE_DN8_TIMING)
      const int64_t per_wg = dn8_k1_min_blocks();
      const int grid = (int)std::min<int64_t>(c->n_cu, (total + per_wg - 1) / per_wg);
      if (dn8_timing()) {
        if (!g_dn8_dbg) {
          LFE_HIP(hipMalloc(reinterpret_cast<void**>(&g_dn8_dbg), sizeof(unsigned long long) * 7 * 65536));
          LFE_HIP(hipMemset(g_dn8_dbg, 0, sizeof(unsigned long long) * 7 * 65536));
        }
        a.dbg = g_dn8_dbg;
      }
      // wide fits: one pass per 16-column group (each projects its own columns of alpha_P)
      const int p = c->p;
      for (int c0 = 0; c0 < p; c0 += 16) {
        Dn8Args g = a;
        g.p = std::min(16, p - c0);
        g.alpha = alphaQ + c0;
        g.S_P = a.S_P + c0;
        g.alphaP = a.alphaP + c0;
        if (c0) g.zero_check = nullptr;
        hipLaunchKernelGGL(k_dn8_k1s, dim3(grid), dim3(1024), lds, c->stream, g);
        LFE_HIP(hipGetLastError());
      }
      if (a.dbg) return dn8_timing_report(c, "K1", grid);
      return LFE_OK;
    }
    // tiled form: alpha_Q's digit tiles formed once per pass by k_dn8_digits
    LFE_TRY(ensure_i8(c, c->dn8_dq, c->dn8_dq_cap, (size_t)ntile * kDn8TileBytes));
    LFE_TRY(ensure_f64(c, c->dn8_eq, c->dn8_eq_cap, (size_t)ntile * 16));
    LFE_HIP(set_max_lds(reinterpret_cast<const void*>(&k_dn8_digits), kDn8TileBytes));
    hipLaunchKernelGGL(k_dn8_digits, dim3(ntile), dim3(256), kDn8TileBytes, c->stream, alphaQ, a.G_Q, a.p, a.p,
                       c->dn8_dq, c->dn8_eq, a.rflag);
    LFE_HIP(hipGetLastError());
    constexpr int waves = 4;
    a.rbw = dn8_rbw(c, a.nrb, waves);
    return dn8_launch<false>(c, a, waves, std::max(c->nbe, 1) * ((a.nrb + a.rbw - 1) / a.rbw));
  }
  DnPassArgs a = dn_args(c);
  a.Nm = c->dn_na;
  a.alpha = alphaQ;
  a.S_P = c->fe[P].S;
  a.cntP = c->fe[P].cnt;
  a.alphaP = c->fe[P].alpha;
  a.zero_check = zero_check;
  const int nrb = a.B / 16;
  a.KP = dn_parts(c, c->nbe * ((nrb + kDnR - 1) / kDnR), 16);  // alpha_Q in LDS: one workgroup per CU
  const int upw = kDnWaves / a.KP * kDnR, wgpb = (nrb + upw - 1) / upw;
  const size_t lds = sizeof(double) * a.GQ16 * a.p;
  LFE_HIP(set_max_lds(reinterpret_cast<const void*>(&k_dn_pass<false>), (int)lds));
  hipLaunchKernelGGL(k_dn_pass<false>, dim3(c->nbe * wgpb), dim3(kDnThreads), lds, c->stream, a);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

int dense_tq(lfe_ctx* c, double* runs) {
  if (c->dn8) {
    Dn8Args a = dn8_args(c);
    const int GQ64 = dn_gq64(c);
    a.Nm = c->dn8_b;
    a.flags = c->dn8_fb;
    a.nkb = a.B / 64;
    a.fstride = (a.nkb + 7) / 8 * 8;
    a.X = c->dn_nb;
    a.nrb = GQ64 / 16;
    a.alpha = c->fe[c->L.P].alpha;
    a.runs = runs;
    if (a.nkb <= 8 && !dn8_tiled()) {  // streaming form: two workgroups per bucket and CU
      LFE_HIP(set_max_lds(reinterpret_cast<const void*>(&k_dn8_k2s), kDn8TileBytes));
      const int nbe = std::max(c->nbe, 1);
      const int np = k2_parts(c, nbe, a.nrb);
      if (dn8_timing()) {
        if (!g_dn8_dbg) {
          LFE_HIP(hipMalloc(reinterpret_cast<void**>(&g_dn8_dbg), sizeof(unsigned long long) * 7 * 65536));
          LFE_HIP(hipMemset(g_dn8_dbg, 0, sizeof(unsigned long long) * 7 * 65536));
        }
        a.dbg = g_dn8_dbg;
      }
      const int p = c->p;
      for (int c0 = 0; c0 < p; c0 += 16) {  // wide fits: one pass per 16-column group
        Dn8Args g = a;
        g.p = std::min(16, p - c0);
        g.alpha = a.alpha + c0;
        g.runs = runs + c0;
        hipLaunchKernelGGL(k_dn8_k2s, dim3(nbe * np), dim3(512), kDn8TileBytes, c->stream, g, np);
        LFE_HIP(hipGetLastError());
      }
      if (a.dbg) return dn8_timing_report(c, "K2", nbe * np);
      return LFE_OK;
    }
    constexpr int waves = 8;  // every workgroup digitizes its bucket's alpha_P rows: 16 blocks each
    a.rbw = dn8_rbw(c, a.nrb, waves);
    return dn8_launch<true>(c, a, waves, std::max(c->nbe, 1) * ((a.nrb + a.rbw - 1) / a.rbw));
  }
  DnPassArgs a = dn_args(c);
  a.Nm = c->dn_nb;
  a.alpha = c->fe[c->L.P].alpha;
  a.runs = runs;
  const int nrb = a.GQ16 / 16;
  a.KP = dn_parts(c, c->nbe * ((nrb + kDnR - 1) / kDnR), 32);  // a 45 KB slice: two workgroups per CU
  const int upw = kDnWaves / a.KP * kDnR, wgpb = (nrb + upw - 1) / upw;
  const size_t lds = sizeof(double) * a.B * a.p;
  LFE_HIP(set_max_lds(reinterpret_cast<const void*>(&k_dn_pass<true>), (int)lds));
  hipLaunchKernelGGL(k_dn_pass<true>, dim3(c->nbe * wgpb), dim3(kDnThreads), lds, c->stream, a);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

// one pair-table pass of the general dense sweeps (lfe_dense3.hip): the K2 streaming kernel with
// "buckets" = the 512-level tiles of the k-side FE and "secondary levels" = the output FE's levels
static Dn8Args pair_args(const PairPass& pp) {
  Dn8Args a{};
  a.Nm = pp.tab;
  a.flags = pp.flg;
  a.fstride = 8;
  a.X = pp.X;
  a.blist = pp.tiles;
  a.nbe = pp.ntile_k;
  a.s = 9;
  a.B = kDn8Tile;
  a.G_Q = pp.G_rows;
  a.G_P = pp.G_k;
  a.p = pp.pc;
  a.lda = pp.lda;
  a.ldo = pp.ldo;
  a.nkb = 8;
  a.nrb = pp.nrb;
  a.alpha = pp.alpha;
  a.runs = pp.runs;
  return a;
}

int dn8_pair_pass(lfe_ctx* c, const PairPass& pp) { return dn8_pair_passes(c, &pp, 1); }

int dn8_pair_passes(lfe_ctx* c, const PairPass* pp, int n) {
  static bool attr = false;
  if (!attr) {
    LFE_HIP(set_max_lds(reinterpret_cast<const void*>(&k_dn8_k2s_batch), kDn8TileBytes));
    attr = true;
  }
  for (int j0 = 0; j0 < n; j0 += kDn8Batch) {
    Dn8Batch b{};
    int grid = 0;
    for (int j = j0; j < n && b.n < kDn8Batch; ++j) {
      if (pp[j].ntile_k < 1 || pp[j].nrb < 1) continue;
      const int q = b.n++;
      b.a[q] = pair_args(pp[j]);
      b.a[q].rflag = c->rflag;
      // the batch shares the chip: its passes' workgroups together fill one round of the resident ones
      b.np[q] = 1;
      b.start[q] = grid;
      grid += pp[j].ntile_k;
    }
    if (b.n == 0) continue;
    // parts per tile: as many as keep the whole batch within one round (two per CU), >= 8 blocks each
    const int per = std::max(1, (int)((2 * (int64_t)c->n_cu) / std::max(grid, 1)));
    grid = 0;
    for (int q = 0; q < b.n; ++q) {
      b.np[q] = std::min(per, std::max(1, b.a[q].nrb / 8));
      b.start[q] = grid;
      grid += b.a[q].nbe * b.np[q];
    }
    b.start[b.n] = grid;
    hipLaunchKernelGGL(k_dn8_k2s_batch, dim3(grid), dim3(512), kDn8TileBytes, c->stream, b);
    LFE_HIP(hipGetLastError());
  }
  return LFE_OK;
}

}  // namespace lfe

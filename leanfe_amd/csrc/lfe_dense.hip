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
#include "lfe_internal.h"

#include <algorithm>
#include <cstdlib>

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
  uint16_t* NA;
  uint16_t* NB;
};

// Counts of the bucket's kept rows with h in [hlo, hlo + HW) into LDS counters of CT (8 or 16
// bits, packed in 32-bit words: cnt[h - hlo][q]); returns whether some 8-bit counter overflowed.
template <typename CT>
__device__ bool dn_count(const DnBuildArgs& a, uint32_t* cw, int hlo, int HW, int r0, int r1) {
  constexpr int PER = 4 / sizeof(CT), SH = 8 * sizeof(CT);
  const int W = a.GQ16 / PER;  // words per group row
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
    const CT* src = cnt + (hbl * 16 + (el >> 4)) * a.GQ16 + qb * 16 + (el & 15);
    na[((int64_t)(hb0 + hbl) * nqb + qb) * 64 + (e & 63)] = us4{src[0], src[1], src[2], src[3]};
  }
  us4* nbp = reinterpret_cast<us4*>(a.NB + (int64_t)bi * nqb * nhb * 256);
  for (int e = threadIdx.x; e < nel4; e += blockDim.x) {  // NB blocks (qb, hb): rows q, 4 h's per store
    const int blk = e >> 6, el = (e & 63) * 4, qb = blk / hbl_n, hbl = blk - qb * hbl_n;
    const CT* src = cnt + (hbl * 16 + (el & 15)) * a.GQ16 + qb * 16 + (el >> 4);
    nbp[((int64_t)qb * nhb + hb0 + hbl) * 64 + (e & 63)] = us4{src[0], src[a.GQ16], src[2 * a.GQ16], src[3 * a.GQ16]};
  }
}

// Workgroup (bucket bi, chunk of HC primary groups): counts the chunk's rows in LDS and writes its
// NA and NB blocks.  HC = 128 groups on 8-bit counters (the bucket's codes are read by B / 128
// workgroups); a chunk where some (h, q) pair holds more than 255 rows is counted again in two
// halves on 16-bit counters (counts <= 65535 by the caller's check).  The workgroups of a bucket
// share an XCD (block i -> XCD i % 8), so its codes are read from one L2.
__global__ __launch_bounds__(1024) void k_dn_build(DnBuildArgs a) {
  extern __shared__ uint32_t cw[];  // [HC][GQ16] 8-bit or [HC / 2][GQ16] 16-bit counters
  const int i = blockIdx.x, x = i & 7, r = i >> 3;
  const int chunk = r % a.nch, bi = (r / a.nch) * 8 + x;
  if (bi >= a.nbe) return;
  const int b = a.blist[bi];
  const int it0 = a.bitems[b], it1 = a.bitems[b + 1];
  const int r0 = it1 > it0 ? a.items[it0].y : 0, r1 = it1 > it0 ? a.items[it1 - 1].z : 0;
  const int HC = a.B / a.nch, hlo = (b << a.s) + chunk * HC, hb0 = chunk * (HC / 16);
  if (HC == 2 * kDnHC) {
    if (!dn_count<uint8_t>(a, cw, hlo, HC, r0, r1)) {
      dn_write<uint8_t>(a, reinterpret_cast<const uint8_t*>(cw), bi, hb0, HC);
      return;
    }
    for (int half = 0; half < 2; ++half) {
      __syncthreads();
      dn_count<uint16_t>(a, cw, hlo + half * kDnHC, kDnHC, r0, r1);
      dn_write<uint16_t>(a, reinterpret_cast<const uint16_t*>(cw), bi, hb0 + half * (kDnHC / 16), kDnHC);
    }
    return;
  }
  dn_count<uint16_t>(a, cw, hlo, HC, r0, r1);
  dn_write<uint16_t>(a, reinterpret_cast<const uint16_t*>(cw), bi, hb0, HC);
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
// host side
// ---------------------------------------------------------------------------

static int64_t dn_cells(const lfe_ctx* c) {
  const int Q = 1 - c->L.P;
  const int64_t GQ16 = ((int64_t)c->fe[Q].G + 15) / 16 * 16;
  return (int64_t)std::max(c->nbe, 1) * ((int64_t)1 << c->L.s) * GQ16;
}

bool dense_ok(const lfe_ctx* c) {
  const char* e = getenv("LFE_DENSE");  // "0": never (A/B); "1": whenever it fits
  if (e && e[0] == '0') return false;
  const int P = c->L.P, Q = 1 - P, p = c->p;
  if (!(c->world == 1 || c->owner_on) || p > 16 || c->nbe < 1) return false;
  const int64_t B = 1ll << c->L.s, GQ16 = ((int64_t)c->fe[Q].G + 15) / 16 * 16;
  if (B % kDnHC != 0) return false;
  if (GQ16 * p * 8 > 100 * 1024 || B * p * 8 > 64 * 1024) return false;  // the B operand tables in LDS
  if (kDnHC * GQ16 * 2 > 150 * 1024) return false;                        // the build's counters
  if (c->fe[P].cmax > 65535) return false;                                 // uint16 counts
  // the products cost ~ the cells (~1.1 ns per cell and pass), the row passes ~ the rows (~3.2 ns
  // per row and pass): dense from 0.3 rows per cell (50M rows over 1e5 x 1e3: 0.5; config 2's 10M:
  // 0.1, where the dense passes measured 1.5x the row passes)
  if (!(e && e[0] == '1') && (double)c->n_kept_local < 0.3 * (double)dn_cells(c)) return false;
  return true;
}

int dense_build(lfe_ctx* c) {
  auto& L = c->L;
  const int Q = 1 - L.P;
  const int B = 1 << L.s, GQ16 = (c->fe[Q].G + 15) / 16 * 16;
  const size_t cells = (size_t)dn_cells(c);
  c->dense_cells = (int64_t)cells;
  LFE_TRY(ensure_u16(c, c->dn_na, c->dn_na_cap, cells));
  LFE_TRY(ensure_u16(c, c->dn_nb, c->dn_nb_cap, cells));
  DnBuildArgs a{};
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
  const bool c8_fits = (size_t)2 * kDnHC * GQ16 <= 150 * 1024 && B % (2 * kDnHC) == 0;
  bool c8 = c8_fits && (int64_t)c->nbe * (B / (2 * kDnHC)) >= c->n_cu;
  if (const char* e = getenv("LFE_DN_C8")) c8 = c8_fits && e[0] == '1';  // tests: force either form
  a.nch = B / (c8 ? 2 * kDnHC : kDnHC);
  a.NA = c->dn_na;
  a.NB = c->dn_nb;
  const size_t lds = sizeof(uint16_t) * kDnHC * GQ16;  // both forms
  LFE_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_dn_build), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds));
  const int grid = (c->nbe + 7) / 8 * 8 * a.nch;
  ProfScope _ps(c, K_LAYOUT_SCATTER);
  hipLaunchKernelGGL(k_dn_build, dim3(grid), dim3(1024), lds, c->stream, a);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

// k-range parts per output block: at least one round of the resident waves (wpc per CU; an owner
// shard has few buckets).  More parts per block cost more than the shorter tail saves (headline,
// same box: K1 + K2 0.66 ms per solve at one round, 0.85 ms at four)
static int dn_parts(const lfe_ctx* c, int blocks, int wpc) {
  int kp = 1;
  int64_t rounds = 1;
  if (const char* e = getenv("LFE_DN_ROUNDS")) rounds = std::max(1ll, atoll(e));  // A/B only
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

int dense_tp(lfe_ctx* c, const double* alphaQ, double* zero_check) {
  const int P = c->L.P;
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
  LFE_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_dn_pass<false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(k_dn_pass<false>, dim3(c->nbe * wgpb), dim3(kDnThreads), lds, c->stream, a);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

int dense_tq(lfe_ctx* c, double* runs) {
  DnPassArgs a = dn_args(c);
  a.Nm = c->dn_nb;
  a.alpha = c->fe[c->L.P].alpha;
  a.runs = runs;
  const int nrb = a.GQ16 / 16;
  a.KP = dn_parts(c, c->nbe * ((nrb + kDnR - 1) / kDnR), 32);  // a 45 KB slice: two workgroups per CU
  const int upw = kDnWaves / a.KP * kDnR, wgpb = (nrb + upw - 1) / upw;
  const size_t lds = sizeof(double) * a.B * a.p;
  LFE_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_dn_pass<true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(k_dn_pass<true>, dim3(c->nbe * wgpb), dim3(kDnThreads), lds, c->stream, a);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

}  // namespace lfe

// leanfe HIP engine — Gram, residual/HC1 meat and cluster scores on MFMA.
//
//   Gram   X'X, X'y with X = [1, x~]          (polars_impl.py:165-209)
//   resid  r = y~ - X beta_full, sum w r^2, sum r^2, HC1 meat sum (w) r^2 x~ x~'
//                                              (polars_impl.py:229, 281-282; std_errors.py:196-264)
//   scores S_c = sum_{i in c} x~_i r_i (w_i) and meat S'S: the one-hot SpMM
//          W_C'(X.e)                           (std_errors.py:317-336, compress.py:929-942)
//
// "MFMA-native" lane layout.  v_mfma_f64_16x16x4_f64 takes lane l's operand
// as A[i = l&15][k = l>>4] = B[k][j = l&15]; for a Gram G = Z'Z over 4 rows
// that is Z[row_k][col], so lane (k = l>>4, c = l&15) owns column c (plus
// 16*I for wider designs) of rows 16g + 4k + s, s = 0..3 of a 16-row group g.
// A lane therefore loads its 4 consecutive rows of a column as one 32-byte
// vector (a 16-row group of a column is one full 128-byte line), gathers the
// group effects of its column for 4 rows (16 lanes = 16 consecutive doubles
// of an alpha row), and feeds step s of the MFMA straight from registers: no
// LDS tile, no barrier per tile, waves run independently.  Only the primary
// FE's alpha slice for the item's bucket is staged in LDS (once per item).
#include "lfe_internal.h"

#include <algorithm>
#include <cstdlib>

namespace lfe {

typedef double d4 __attribute__((ext_vector_type(4)));

enum { GRAM_DESIGN = 0, GRAM_RESID = 1, GRAM_TABLE = 2 };

constexpr int kGramThreads = 256;  // 4 independent waves

struct GramArgs {
  LayoutArgs la;
  const double* X;
  int64_t ld;
  const double* w;
  const double* beta;   // GRAM_RESID: beta_full [p] = {intercept, b_1..b_{p-1}}
  double* scores;       // GRAM_RESID: optional row-major [ld][p-1+icpt] output u r (w)
  int icpt;             // GRAM_RESID: the intercept takes y's slot in the meat / scores (u = [1, x~])
  int yoco;             // GRAM_RESID on YOCO records: sufficient-statistic residuals (compress.py:754-811)
  const double* rsy;    // yoco: [ld] _sum_y, layout order
  const double* rsyy;   // yoco: [ld] _sum_y_sq, layout order
  const double* table;  // GRAM_TABLE: row-major [rows][tcols]
  const int32_t* tidx;  // GRAM_TABLE: optional row index (row q of the Gram = table row tidx[q])
  int64_t rows;         // GRAM_TABLE
  int tcols;
  int B;                // 1 << s
  int G_P;
  int stage;            // 1: the primary FE's alpha slice is staged in LDS per item
  int nq;               // number of non-primary FEs
  int qf[kMaxFE];       // their FE indices
  int G_Q;              // levels of qf[0] (its alpha table staged in LDS when it fits)
  // k_resid_rows<.., CL = true>: the one-way cluster sums on the primary FE formed in the residual
  // pass itself - every score value's fine limb into the bucket's LDS window of the [G_P][k]
  // table, coarse limbs into clHi, a coarse limb past the exact-sum bound raises *clFlag
  unsigned long long* clS;
  double* clHi;
  const double* clFq;
  const int32_t* clCmax;
  int32_t* clFlag;
};

template <int NT>
struct GramShape {
  static constexpr int NP = NT * (NT + 1) / 2;
  static constexpr int LEN = NP * 256;
};

__device__ __forceinline__ d4 ld4(const double* p) { return *reinterpret_cast<const d4*>(p); }
__device__ __forceinline__ void st4(double* p, d4 v) { *reinterpret_cast<d4*>(p) = v; }

// one 64-bit DPP lane move (two 32-bit halves)
template <int CTRL>
__device__ __forceinline__ double dppd(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
// sum over the 16 lanes of a DPP row (quad xor 1, xor 2, half mirror, mirror); all lanes get it
__device__ __forceinline__ double row16_sum(double v) {
  v += dppd<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dppd<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dppd<0x141>(v);  // row_half_mirror
  v += dppd<0x140>(v);  // row_mirror
  return v;
}

// z[s][I] -> acc (4 MFMA steps per pair)
template <int NT>
__device__ __forceinline__ void mfma_rows(const double (&z)[4][NT], d4* acc) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    int q = 0;
#pragma unroll
    for (int I = 0; I < NT; ++I)
#pragma unroll
      for (int J = I; J < NT; ++J, ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(z[s][I], z[s][J], acc[q], 0, 0, 0);
  }
}

// LDS reduction of the 4 waves' accumulators -> partial[blockIdx.x]
template <int NT, int TH>
__device__ __forceinline__ void block_reduce_store(const d4* acc, double* red, double* out, int tid) {
  using Sh = GramShape<NT>;
  const int lane = tid & 63, wave = tid >> 6;
  for (int wv = 0; wv < TH / 64; ++wv) {
    __syncthreads();
    if (wave == wv) {
#pragma unroll
      for (int q = 0; q < Sh::NP; ++q)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int e = q * 256 + ((lane >> 4) + 4 * rr) * 16 + (lane & 15);
          red[e] = (wv == 0) ? acc[q][rr] : red[e] + acc[q][rr];
        }
    }
  }
  __syncthreads();
  for (int e = tid; e < Sh::LEN; e += TH) out[e] = red[e];
}

// Gram of a small row-major table (cluster score sums): Z = table[rows][tcols]
template <int NT>
__global__ __launch_bounds__(kGramThreads) void k_gram_table(GramArgs a, double* __restrict__ partial, int64_t pstride) {
  using Sh = GramShape<NT>;
  __shared__ double red[Sh::LEN];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kq = lane >> 4, c = lane & 15;
  d4 acc[Sh::NP];
#pragma unroll
  for (int q = 0; q < Sh::NP; ++q) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
  const int64_t ngroups = (a.rows + 15) / 16;
  for (int64_t gi = (int64_t)blockIdx.x * 4 + wave; gi < ngroups; gi += (int64_t)gridDim.x * 4) {
    double z[4][NT];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int64_t r = gi * 16 + kq * 4 + s;
#pragma unroll
      for (int I = 0; I < NT; ++I) {
        const int col = 16 * I + c;
        const int64_t tr = a.tidx && r < a.rows ? (int64_t)a.tidx[r] : r;
        z[s][I] = (r < a.rows && col < a.tcols) ? a.table[tr * a.tcols + col] : 0.0;
      }
    }
    mfma_rows<NT>(z, acc);
  }
  block_reduce_store<NT, kGramThreads>(acc, red, partial + (int64_t)blockIdx.x * pstride, tid);
}

// Design Gram / residual pass over the bucket layout.
// MODE: design / resid; NT: 16-column slots per lane; FQ: max non-primary FEs;
// GU: 16-row groups per wave iteration; WT: weighted fit; QL: the (single)
// non-primary FE's alpha table is staged in LDS (an L2 gather of 88-byte rows
// costs half the bandwidth of the pass, tools/ubench_gram.hip); TH: threads.
// Every load address is valid for every lane: lanes without a data column read
// column 0 and rows outside the item get primary code -1, so nothing is
// predicated and each row's validity is the single test h >= 0.
// (NT = 2, GU = 1, 256 threads: three workgroups per CU, i.e. three waves per SIMD - the register
// budget 168 the unweighted residual variant needs four registers of spill-free slack for)
template <int MODE, int NT, int FQ, int GU, bool WT, bool QL, int TH>
__global__ __launch_bounds__(TH, (NT == 2 && GU == 1 && TH == 256 && FQ == 1) ? 3 : 1) void k_gram(
    GramArgs a, double* __restrict__ partial, int64_t pstride) {
  using Sh = GramShape<NT>;
  constexpr int NW = TH / 64;
  constexpr bool PF = NT == 1 && !QL && FQ == 2;  // (the generic FQ 7 variant measured slower with it)
  __shared__ double red[Sh::LEN];
  __shared__ double stat_red[NW][4];
  extern __shared__ __attribute__((aligned(16))) double dyn_lds[];
  // dynamic LDS: [B][p] alpha_P slice of the item's bucket, then (QL) [G_Q][p] alpha_Q
  double* slice = dyn_lds;
  double* aqL = dyn_lds + (QL ? a.B * a.la.p : 0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kq = lane >> 4, c = lane & 15;
  const int p = a.la.p, P = a.la.P;

  d4 acc[Sh::NP];
#pragma unroll
  for (int q = 0; q < Sh::NP; ++q) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
  double st[4] = {0.0, 0.0, 0.0, 0.0};  // sum w r^2, sum r^2, sum y~, sum y~^2

  // columns held by this lane: design column col = 16I + c -> data column xc
  int xl[NT];          // data column loaded (0 for lanes without one)
  bool dat[NT];        // lane holds a data column
  double fill[NT];     // DESIGN: value of a non-data column (1 for the intercept)
  double coef[NT];     // RESID: row term y~ - sum_j beta_j x~_j
  bool one[NT];        // RESID with icpt: this slot is the intercept (value 1 in the meat / scores)
  const double* xb[NT];
#pragma unroll
  for (int I = 0; I < NT; ++I) {
    const int col = 16 * I + c;
    int xc = (MODE == GRAM_DESIGN) ? col - 1 : col;  // DESIGN: col 0 = intercept, col 1 = y
    if (xc >= p) xc = -2;
    dat[I] = xc >= 0;
    xl[I] = xc >= 0 ? xc : 0;
    fill[I] = xc == -1 ? 1.0 : 0.0;
    coef[I] = (MODE == GRAM_RESID) ? (xc == 0 ? 1.0 : (xc >= 1 ? -a.beta[xc] : 0.0)) : 0.0;
    one[I] = MODE == GRAM_RESID && a.icpt && xc == 0;
    if (MODE == GRAM_RESID) dat[I] = xc >= 1 || one[I];  // meat columns
    xb[I] = a.X + (int64_t)xl[I] * a.ld;
  }
  const double beta0 = (MODE == GRAM_RESID) ? a.beta[0] : 0.0;
  const int nq = a.nq < FQ ? a.nq : FQ;
  if (QL) {
    const double* src = a.la.alpha[a.qf[0]];
    for (int j = tid; j < a.G_Q * p; j += TH) aqL[j] = src[j];
    __syncthreads();
  }

  // a contiguous range of items per block (all blocks co-resident): the
  // primary slice is staged again only when the bucket changes
  const BlockRows br = block_rows(a.la.items, a.la.n_items, lane);
  int staged = -1;
  for (int item = br.first; item < a.la.n_items; ++item) {
    int4 it = a.la.items[item];
    if (it.y >= br.hi) break;
    it.y = max(it.y, br.lo);
    it.z = min(it.z, br.hi);
    const int lo = it.x << a.la.s;
    if (a.stage && it.x != staged) {
      __syncthreads();
      for (int j = tid; j < a.B * p; j += TH) {
        const int g = lo + j / p;
        slice[j] = g < a.G_P ? a.la.alpha[P][(int64_t)g * p + (j % p)] : 0.0;
      }
      __syncthreads();
      staged = it.x;
    }
    const int g0 = it.y >> 4, g1 = (it.z + 15) >> 4;
    constexpr int step = NW * GU;
    // software pipeline: the codes of a batch are loaded one iteration ahead,
    // so X loads, every group's alpha gathers and the next codes are in flight together
    int hq[GU][4], cq[GU][FQ][4];
    auto load_codes = [&](int gb) {
#pragma unroll
      for (int u = 0; u < GU; ++u) {
        const int gi = gb + u;
        const int r = gi * 16 + kq * 4;
        int4 h = int4{-1, -1, -1, -1};
        if (gi < g1) h = P >= 0 ? *reinterpret_cast<const int4*>(a.la.code[P] + r) : int4{0, 0, 0, 0};
        hq[u][0] = h.x; hq[u][1] = h.y; hq[u][2] = h.z; hq[u][3] = h.w;
#pragma unroll
        for (int q = 0; q < FQ; ++q) {
          int4 v = int4{0, 0, 0, 0};
          if (q < nq && gi < g1) v = *reinterpret_cast<const int4*>(a.la.code[a.qf[q]] + r);
          cq[u][q][0] = v.x; cq[u][q][1] = v.y; cq[u][q][2] = v.z; cq[u][q][3] = v.w;
        }
        // a group straddling the item edge (wave-uniform test): rows outside the
        // item are marked dropped and their other codes zeroed (rows past n hold
        // uninitialised codes, and the gathers below are not predicated)
        if (gi < g1 && (gi * 16 < it.y || gi * 16 + 16 > it.z)) {
#pragma unroll
          for (int s = 0; s < 4; ++s)
            if (r + s < it.y || r + s >= it.z) {
              hq[u][s] = -1;
#pragma unroll
              for (int q = 0; q < FQ; ++q) cq[u][q][s] = 0;
            }
        }
      }
    };
    // PF: the X columns of a batch are loaded one iteration ahead too (the wave then waits on the
    // L2 gathers only, not on an HBM round trip per batch)
    d4 xn[GU][NT];
    auto load_x = [&](int gb) {
#pragma unroll
      for (int u = 0; u < GU; ++u) {
        const int gi = gb + u;
        const int r = gi * 16 + kq * 4;
#pragma unroll
        for (int I = 0; I < NT; ++I) xn[u][I] = gi < g1 ? ld4(xb[I] + r) : d4{0.0, 0.0, 0.0, 0.0};
      }
    };
    load_codes(g0 + wave * GU);
    if (PF) load_x(g0 + wave * GU);
    for (int gb = g0 + wave * GU; gb < g1; gb += step) {
      d4 xv[GU][NT], wv[GU], yr[GU], s1[GU], s2[GU];
      bool valid[GU][4];
#pragma unroll
      for (int u = 0; u < GU; ++u) {
        const int gi = gb + u;
        const int r = gi * 16 + kq * 4;
#pragma unroll
        for (int I = 0; I < NT; ++I) xv[u][I] = PF ? xn[u][I] : gi < g1 ? ld4(xb[I] + r) : d4{0.0, 0.0, 0.0, 0.0};
        if (WT) wv[u] = gi < g1 ? ld4(a.w + r) : d4{0.0, 0.0, 0.0, 0.0};
        if (MODE == GRAM_RESID && WT && a.yoco) {  // record mean of y (raw column 0), _sum_y, _sum_y_sq
          yr[u] = gi < g1 ? ld4(a.X + r) : d4{0.0, 0.0, 0.0, 0.0};
          s1[u] = gi < g1 ? ld4(a.rsy + r) : d4{0.0, 0.0, 0.0, 0.0};
          s2[u] = gi < g1 ? ld4(a.rsyy + r) : d4{0.0, 0.0, 0.0, 0.0};
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) valid[u][s] = hq[u][s] >= 0;
      }
      // group effects: non-primary FEs gathered from global (L2-resident tables)
      double ga[GU][4][NT];
#pragma unroll
      for (int u = 0; u < GU; ++u)
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int I = 0; I < NT; ++I) ga[u][s][I] = 0.0;
#pragma unroll
      for (int q = 0; q < FQ; ++q) {
        if (q >= nq) continue;
        const double* aq = a.la.alpha[a.qf[q]];
#pragma unroll
        for (int u = 0; u < GU; ++u)
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const uint32_t ro = (uint32_t)cq[u][q][s] * (uint32_t)p;
#pragma unroll
            for (int I = 0; I < NT; ++I) {
              const double v = QL ? aqL[ro + (uint32_t)xl[I]] : aq[ro + (uint32_t)xl[I]];
              ga[u][s][I] = (q == 0) ? v : ga[u][s][I] + v;
            }
          }
      }
      int hv[GU][4];
#pragma unroll
      for (int u = 0; u < GU; ++u)
#pragma unroll
        for (int s = 0; s < 4; ++s) hv[u][s] = hq[u][s];
      load_codes(gb + step);  // next batch
      if (PF) load_x(gb + step);
      if (P >= 0) {
        // separate LDS / global paths: a generic pointer over both address
        // spaces trips a gfx950 codegen error (flat address-space check)
        if (a.stage) {
#pragma unroll
          for (int u = 0; u < GU; ++u)
#pragma unroll
            for (int s = 0; s < 4; ++s) {
              const uint32_t ro = (uint32_t)(valid[u][s] ? hv[u][s] - lo : 0) * (uint32_t)p;
#pragma unroll
              for (int I = 0; I < NT; ++I) ga[u][s][I] += slice[ro + (uint32_t)xl[I]];
            }
        } else {
          const double* ap = a.la.alpha[P];
#pragma unroll
          for (int u = 0; u < GU; ++u)
#pragma unroll
            for (int s = 0; s < 4; ++s) {
              const uint32_t ro = (uint32_t)(valid[u][s] ? hv[u][s] : 0) * (uint32_t)p;
#pragma unroll
              for (int I = 0; I < NT; ++I) ga[u][s][I] += ap[ro + (uint32_t)xl[I]];
            }
        }
      }
#pragma unroll
      for (int u = 0; u < GU; ++u) {
        double xt[4][NT];
#pragma unroll
        for (int I = 0; I < NT; ++I)
#pragma unroll
          for (int s = 0; s < 4; ++s) xt[s][I] = xv[u][I][s] - ga[u][s][I];
        double z[4][NT];
        if (MODE == GRAM_DESIGN) {
          // Z = sqrt(w) [1, y~, x~]   (X_w = X * sqrt(w), polars_impl.py:202-203)
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const double sw = WT ? sqrt(wv[u][s]) : 1.0;
#pragma unroll
            for (int I = 0; I < NT; ++I) {
              double v = dat[I] ? xt[s][I] : fill[I];
              if (WT) v *= sw;
              z[s][I] = valid[u][s] ? v : 0.0;
            }
          }
        } else {
          // r = y~ - beta0 - sum_j beta_j x~_j (unweighted residual, polars_impl.py:229)
          double sc[4];
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            double t = coef[0] * xt[s][0];
#pragma unroll
            for (int I = 1; I < NT; ++I) t += coef[I] * xt[s][I];
            const double res = row16_sum(t) - beta0;
            double m;
            if (WT && a.yoco) {
              // record g: LSDV fitted value = mean_y - r; rss_g = sum_y_sq - 2 fit sum_y + n fit^2
              // (compress.py:803-808); residual sum e_g = sum_y - n fit (:1118-1124).  The HC1
              // meat is sum_g rss_g x~ x~' (:907-919): rss_g >= 0 up to rounding, clamped for the sqrt
              const double fit = yr[u][s] - res;
              const double rss = s2[u][s] - 2.0 * fit * s1[u][s] + wv[u][s] * fit * fit;
              if (c == 0 && valid[u][s]) {
                st[0] += rss;
                st[1] += wv[u][s] * res * res;
                st[2] += xt[s][0];
                st[3] += xt[s][0] * xt[s][0];
              }
              sc[s] = s1[u][s] - wv[u][s] * fit;
              m = sqrt(fmax(rss, 0.0));
            } else {
              if (c == 0 && valid[u][s]) {  // lane c = 0 holds y~ (column 0)
                const double rr = res * res;
                st[0] += WT ? wv[u][s] * rr : rr;
                st[1] += rr;
                st[2] += xt[s][0];
                st[3] += xt[s][0] * xt[s][0];
              }
              sc[s] = WT ? res * wv[u][s] : res;
              m = WT ? res * sqrt(wv[u][s]) : res;
            }
#pragma unroll
            for (int I = 0; I < NT; ++I) z[s][I] = (valid[u][s] && dat[I]) ? (one[I] ? 1.0 : xt[s][I]) * m : 0.0;
          }
          if (a.scores) {
            const int gi = gb + u;
            const int r = gi * 16 + kq * 4;
            const bool full = gi * 16 >= it.y && gi * 16 + 16 <= it.z;
#pragma unroll
            for (int I = 0; I < NT; ++I) {
              if (!dat[I]) continue;
              // row-major [row][k]: the 16 column lanes of a row quad write one contiguous row
              const int64_t ks = a.la.p - 1 + a.icpt;
              double* dst = a.scores + (int64_t)r * ks + (xl[I] - 1 + a.icpt);
              d4 v;
#pragma unroll
              for (int s = 0; s < 4; ++s) v[s] = valid[u][s] ? (one[I] ? 1.0 : xt[s][I]) * sc[s] : 0.0;
              if (full) {
#pragma unroll
                for (int s = 0; s < 4; ++s) dst[s * ks] = v[s];
              } else if (gi < g1) {
#pragma unroll
                for (int s = 0; s < 4; ++s)
                  if (valid[u][s]) dst[s * ks] = v[s];
              }
            }
          }
        }
        mfma_rows<NT>(z, acc);
      }
    }
  }

  double* out = partial + (int64_t)blockIdx.x * pstride;
  block_reduce_store<NT, TH>(acc, red, out, tid);
  if (MODE == GRAM_RESID) {
#pragma unroll
    for (int s = 0; s < 4; ++s) st[s] = wave_reduce63(st[s], 0.0, [](double x, double y) { return x + y; });
    if (lane == 63)
      for (int s = 0; s < 4; ++s) stat_red[wave][s] = st[s];
    __syncthreads();
    if (tid < 4) {
      double t = 0.0;
      for (int w = 0; w < NW; ++w) t += stat_red[w][tid];
      out[Sh::LEN + tid] = t;
    }
  }
}

// Residual pass, row per lane (two FEs, unweighted, p <= PM <= 16).  The lane
// layout above needs a 16-lane DPP reduction for every row's residual (~6 VALU
// per row); here each lane owns whole rows: it loads the row's p columns
// (coalesced across the wave), gathers the two alpha rows from LDS (tables padded
// to PM doubles per row so a row is PM/2 16-byte reads), forms the residual with
// a lane-local dot product and accumulates the HC1 meat (upper triangle, VALU
// f64 FMAs) and the residual statistics.  Output: the same [16][16] tile + 4
// statistics per block as k_gram<RESID>.
constexpr int kResThreads = 512;

// CL: the one-way cluster sums on the primary FE (GramArgs.cl*): alpha_Q comes from global memory
// (L2) and the LDS holds the slice and the bucket's [B][k] window of fine limbs instead; the
// window goes out by int64 global adds when the bucket changes and at the end (no score rows).
template <int PM, int UR, bool CL>
__global__ __launch_bounds__(kResThreads) void k_resid_rows(GramArgs a, double* __restrict__ partial, int64_t pstride) {
  constexpr int KM = PM - 1;              // regressor columns held
  constexpr int NM = KM * (KM + 1) / 2;   // meat upper triangle
  constexpr int NW = kResThreads / 64;
  typedef double d2 __attribute__((ext_vector_type(2)));
  typedef unsigned long long u64;
  extern __shared__ __attribute__((aligned(16))) double lds[];
  double* slice = lds;                    // [B][PM] alpha_P slice of the current bucket
  double* aqL = lds + a.B * PM;           // [G_Q][PM] alpha_Q (!CL)
  u64* win = reinterpret_cast<u64*>(lds + a.B * PM);  // [B][p - 1] cluster fine limbs (CL)
  __shared__ double red[NW][NM + 4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int p = a.la.p, P = a.la.P;
  const int Q = a.qf[0];
  const double* aQg = a.la.alpha[Q];
  const int kc = p - 1;  // CL: score columns
  // the pad columns [p, PM) of both tables once, then the rows (the slice rows are restaged per
  // bucket below; their pads stay 0)
  for (int j = tid; j < (CL ? a.B : a.B + a.G_Q) * PM; j += kResThreads)
    if (j % PM >= p) lds[j] = 0.0;
  if (CL) {
    for (int j = tid; j < a.B * kc; j += kResThreads) win[j] = 0ull;
  } else {
    stage_lds<kResThreads>(aqL, aQg, a.G_Q * p, tid, p, PM);
  }
  const double hlim = CL ? 0x1p51 / (double)max(*a.clCmax, 1) - 1.0 : 0.0;
  bool over = false;
  auto flush = [&](int lo) {  // (between barriers) the window's nonzero limbs out, the window zeroed
    for (int j = tid; j < a.B * kc; j += kResThreads) {
      const u64 v = win[j];
      if (v != 0ull && lo + j / kc < a.G_P) atomicAdd(&a.clS[(int64_t)lo * kc + j], v);
      win[j] = 0ull;
    }
  };
  double beta[PM];
#pragma unroll
  for (int cc = 0; cc < PM; ++cc) beta[cc] = cc < p ? a.beta[cc] : 0.0;
  double m[NM];
#pragma unroll
  for (int e = 0; e < NM; ++e) m[e] = 0.0;
  double st[4] = {0.0, 0.0, 0.0, 0.0};  // sum r^2 (w = 1), sum r^2, sum y~, sum y~^2
  const int32_t* codeP = a.la.code[P];
  const int32_t* codeQ = a.la.code[Q];
  const BlockRows br = block_rows(a.la.items, a.la.n_items, lane);
  int staged = -1;
  for (int item = br.first; item < a.la.n_items; ++item) {
    int4 it = a.la.items[item];
    if (it.y >= br.hi) break;
    it.y = max(it.y, br.lo);
    it.z = min(it.z, br.hi);
    const int lo = it.x << a.la.s;
    if (it.x != staged) {
      __syncthreads();
      if (CL && staged >= 0) flush(staged << a.la.s);
      {  // rows past G_P: data columns cleared (their codes never occur)
        const int nr = max(0, min(a.B, a.G_P - lo));
        stage_lds<kResThreads>(slice, a.la.alpha[P] + (int64_t)lo * p, nr * p, tid, p, PM);
        for (int j = nr * PM + tid; j < a.B * PM; j += kResThreads) slice[j] = 0.0;
      }
      __syncthreads();
      staged = it.x;
    }
    // a lane takes UR = 2 consecutive rows (from an even base; rows before it.y are masked), so
    // columns come in 16-byte loads and the two code arrays in 8-byte loads
    static_assert(UR == 2, "row pairs");
    for (int rb = (it.y & ~1) + wave * 64 * UR; rb < it.z; rb += NW * 64 * UR) {
      int hq[UR], qq[UR];
      double x[UR][PM];
      typedef double d2 __attribute__((ext_vector_type(2)));
      const int r0 = rb + 2 * lane;
      const bool in0 = r0 < it.z;  // r0 + 1 <= ld - 1: r0 is even and ld a multiple of 64
      {
        const int2 h2 = in0 ? *reinterpret_cast<const int2*>(codeP + r0) : int2{-1, -1};
        const int2 q2 = in0 ? *reinterpret_cast<const int2*>(codeQ + r0) : int2{0, 0};
        const bool lo_in = in0 && r0 >= it.y, hi_in = in0 && r0 + 1 < it.z;
        hq[0] = lo_in ? h2.x : -1;
        hq[1] = hi_in ? h2.y : -1;
        qq[0] = lo_in ? q2.x : 0;
        qq[1] = hi_in ? q2.y : 0;
#pragma unroll
        for (int cc = 0; cc < PM; ++cc) {
          const d2 v = (in0 && cc < p) ? *reinterpret_cast<const d2*>(a.X + (int64_t)cc * a.ld + r0) : d2{0.0, 0.0};
          x[0][cc] = v.x;
          x[1][cc] = v.y;
        }
      }
#pragma unroll
      for (int u = 0; u < UR; ++u) {
        const bool valid = hq[u] >= 0;
        const d2* sp = reinterpret_cast<const d2*>(slice + (valid ? hq[u] - lo : 0) * PM);
        double xt[PM];
        if (CL) {  // alpha_Q rows from global memory (an L2-resident table, unpadded rows)
          const double* qg = aQg + (int64_t)qq[u] * p;
#pragma unroll
          for (int c2 = 0; c2 < PM / 2; ++c2) {
            const d2 s2 = sp[c2];
            xt[2 * c2] = x[u][2 * c2] - s2.x - (2 * c2 < p ? qg[2 * c2] : 0.0);
            xt[2 * c2 + 1] = x[u][2 * c2 + 1] - s2.y - (2 * c2 + 1 < p ? qg[2 * c2 + 1] : 0.0);
          }
        } else {
          const d2* qp = reinterpret_cast<const d2*>(aqL + qq[u] * PM);
#pragma unroll
          for (int c2 = 0; c2 < PM / 2; ++c2) {
            const d2 s2 = sp[c2], q2 = qp[c2];
            xt[2 * c2] = x[u][2 * c2] - s2.x - q2.x;
            xt[2 * c2 + 1] = x[u][2 * c2 + 1] - s2.y - q2.y;
          }
        }
        // r = y~ - beta0 - sum_j beta_j x~_j (polars_impl.py:229)
        double res = xt[0] - beta[0];
#pragma unroll
        for (int cc = 1; cc < PM; ++cc) res -= beta[cc] * xt[cc];
        if (!valid) continue;
        const double rr = res * res;
        st[0] += rr;
        st[1] += rr;
        st[2] += xt[0];
        st[3] += xt[0] * xt[0];
        double wv[KM];
#pragma unroll
        for (int j = 0; j < KM; ++j) wv[j] = xt[j + 1] * res;
        int e = 0;
#pragma unroll
        for (int i = 0; i < KM; ++i)
#pragma unroll
          for (int j = i; j < KM; ++j, ++e) m[e] += wv[i] * wv[j];
        if (a.scores) {
          const int r = rb + 2 * lane + u;
#pragma unroll
          for (int j = 0; j < KM; ++j)
            if (j + 1 < p) a.scores[(int64_t)r * (p - 1) + j] = wv[j];
        }
        if (CL) {  // the score row into the cluster's window entries (lfe_cluster.hip's two limbs)
          const int hl = (hq[u] - lo) * kc;
#pragma unroll
          for (int j = 0; j < KM; ++j) {
            if (j + 1 >= p) break;
            double hh;
            const u64 xi = fix_split(wv[j], fix_col(a.clFq, j), hh);
            if (xi) atomicAdd(&win[hl + j], xi);
            if (hh != 0.0) atomicAdd(&a.clHi[(int64_t)hq[u] * kc + j], hh);
            over |= !(fabs(hh) <= hlim);
          }
        }
      }
    }
  }
  if (CL) {
    __syncthreads();
    if (staged >= 0) flush(staged << a.la.s);
    if (__any(over) && lane == 0) *a.clFlag = 1;
  }
  // block reduction: wave sums over DPP lane moves (VALU, fixed order; xor shuffles of the
  // NM + 4 sums cost ds_bpermute latency at the kernel's tail), then the NW wave rows in LDS
  const auto addop = [](double x, double y) { return x + y; };
#pragma unroll
  for (int e = 0; e < NM; ++e) {
    const double v = wave_reduce63(m[e], 0.0, addop);
    if (lane == 63) red[wave][e] = v;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const double v = wave_reduce63(st[e], 0.0, addop);
    if (lane == 63) red[wave][NM + e] = v;
  }
  __syncthreads();
  double* out = partial + (int64_t)blockIdx.x * pstride;
  for (int t = tid; t < 256 + 4; t += kResThreads) {
    double v = 0.0;
    if (t < 256) {
      const int i = t / 16 - 1, j = t % 16 - 1;  // tile (1 + i, 1 + j) = meat (i, j)
      if (i >= 0 && j >= 0 && i < KM && j < KM) {
        const int lo2 = i < j ? i : j, hi2 = i < j ? j : i;
        const int e = lo2 * KM - lo2 * (lo2 - 1) / 2 + (hi2 - lo2);
        for (int w = 0; w < NW; ++w) v += red[w][e];
      }
    } else {
      for (int w = 0; w < NW; ++w) v += red[w][NM + (t - 256)];
    }
    out[t] = v;
  }
}

// Design Gram, row per lane (same conditions as k_resid_rows).  Accumulates, for
// the data columns d = [y~, x~_1..x~_k] (PM >= p slots), the row count, the column
// sums (intercept row of [1, d]'[1, d]) and the upper triangle of d'd, on VALU f64
// FMAs; output in the [16][16] tile order of k_gram<DESIGN> (column 0 = intercept).
template <int PM, int UR>
__global__ __launch_bounds__(kResThreads) void k_design_rows(GramArgs a, double* __restrict__ partial,
                                                             int64_t pstride) {
  constexpr int PS = (PM + 1) & ~1;      // LDS row stride (even: 16-byte pair reads)
  constexpr int NG = PM * (PM + 1) / 2;  // upper triangle of d'd
  constexpr int NA = NG + PM + 1;        // + column sums + count
  constexpr int NW = kResThreads / 64;
  typedef double d2 __attribute__((ext_vector_type(2)));
  extern __shared__ __attribute__((aligned(16))) double lds[];
  double* slice = lds;           // [B][PS]
  double* aqL = lds + a.B * PS;  // [G_Q][PS]
  __shared__ double red[NW][NA];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int p = a.la.p, P = a.la.P;
  const int Q = a.qf[0];
  const double* aQg = a.la.alpha[Q];
  for (int j = tid; j < a.G_Q * PS; j += kResThreads) {
    const int g = j / PS, cc = j % PS;
    aqL[j] = cc < p ? aQg[(int64_t)g * p + cc] : 0.0;
  }
  double acc[NA];
#pragma unroll
  for (int e = 0; e < NA; ++e) acc[e] = 0.0;
  const int32_t* codeP = a.la.code[P];
  const int32_t* codeQ = a.la.code[Q];
  const BlockRows br = block_rows(a.la.items, a.la.n_items, lane);
  int staged = -1;
  for (int item = br.first; item < a.la.n_items; ++item) {
    int4 it = a.la.items[item];
    if (it.y >= br.hi) break;
    it.y = max(it.y, br.lo);
    it.z = min(it.z, br.hi);
    const int lo = it.x << a.la.s;
    if (it.x != staged) {
      __syncthreads();
      for (int j = tid; j < a.B * PS; j += kResThreads) {
        const int g = lo + j / PS, cc = j % PS;
        slice[j] = (g < a.G_P && cc < p) ? a.la.alpha[P][(int64_t)g * p + cc] : 0.0;
      }
      __syncthreads();
      staged = it.x;
    }
    for (int rb = it.y + wave * 64 * UR; rb < it.z; rb += NW * 64 * UR) {
      int hq[UR], qq[UR];
      double x[UR][PS];
#pragma unroll
      for (int u = 0; u < UR; ++u) {
        const int r = rb + u * 64 + lane;
        const bool in = r < it.z;
        hq[u] = in ? codeP[r] : -1;
        qq[u] = in ? codeQ[r] : 0;
#pragma unroll
        for (int cc = 0; cc < PS; ++cc) x[u][cc] = (in && cc < p) ? a.X[(int64_t)cc * a.ld + r] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < UR; ++u) {
        if (hq[u] < 0) continue;
        const d2* sp = reinterpret_cast<const d2*>(slice + (hq[u] - lo) * PS);
        const d2* qp = reinterpret_cast<const d2*>(aqL + qq[u] * PS);
        double d[PS];
#pragma unroll
        for (int c2 = 0; c2 < PS / 2; ++c2) {
          const d2 s2 = sp[c2], q2 = qp[c2];
          d[2 * c2] = x[u][2 * c2] - s2.x - q2.x;
          d[2 * c2 + 1] = x[u][2 * c2 + 1] - s2.y - q2.y;
        }
        int e = 0;
#pragma unroll
        for (int i = 0; i < PM; ++i)
#pragma unroll
          for (int j = i; j < PM; ++j, ++e) acc[e] += d[i] * d[j];
#pragma unroll
        for (int i = 0; i < PM; ++i) acc[NG + i] += d[i];
        acc[NG + PM] += 1.0;
      }
    }
  }
  const auto addop = [](double x, double y) { return x + y; };
#pragma unroll
  for (int e = 0; e < NA; ++e) {
    const double v = wave_reduce63(acc[e], 0.0, addop);
    if (lane == 63) red[wave][e] = v;
  }
  __syncthreads();
  double* out = partial + (int64_t)blockIdx.x * pstride;
  for (int t = tid; t < 256; t += kResThreads) {
    const int i = t / 16, j = t % 16;  // design column 0 = intercept, 1 + c = data column c
    int e = -1;
    if (i == 0 && j == 0) e = NG + PM;
    else if (i == 0 && j - 1 < PM) e = NG + (j - 1);
    else if (j == 0 && i - 1 < PM) e = NG + (i - 1);
    else if (i >= 1 && j >= 1 && i - 1 < PM && j - 1 < PM) {
      const int lo2 = (i < j ? i : j) - 1, hi2 = (i < j ? j : i) - 1;
      e = lo2 * PM - lo2 * (lo2 - 1) / 2 + (hi2 - lo2);
    }
    double v = 0.0;
    if (e >= 0)
      for (int w = 0; w < NW; ++w) v += red[w][e];
    out[t] = v;
  }
}

// fixed-order tree sum of per-block partials: one workgroup per output entry
__global__ __launch_bounds__(256) void k_reduce_partials(const double* __restrict__ partial, int nblocks,
                                                         int64_t pstride, double* __restrict__ out) {
  __shared__ double red[256];
  const int e = blockIdx.x;
  double s = 0.0;
  for (int b = threadIdx.x; b < nblocks; b += 256) s += partial[(int64_t)b * pstride + e];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[e] = red[0];
}

// k_reduce_partials whose last workgroup then publishes src[0, count) (the whole result block the
// host reads: spec tile, beta, guard and this residual tile) into mapped host memory (one rank)
__global__ __launch_bounds__(256) void k_reduce_partials_msg(const double* __restrict__ partial, int nblocks,
                                                             int64_t pstride, double* __restrict__ out,
                                                             unsigned int* __restrict__ done, const double* src,
                                                             int count, unsigned long long* __restrict__ msg,
                                                             unsigned long long seq) {
  __shared__ double red[256];
  const int e = blockIdx.x;
  double s = 0.0;
  for (int b = threadIdx.x; b < nblocks; b += 256) s += partial[(int64_t)b * pstride + e];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[e] = red[0];
  if (!last_block_done(done)) return;
  for (int i = threadIdx.x; i < count; i += 256) {
    const unsigned long long b =
        (unsigned long long)__double_as_longlong(__hip_atomic_load(&src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    host_msg_word(msg, 2 * i, seq, (unsigned int)b);
    host_msg_word(msg, 2 * i + 1, seq, (unsigned int)(b >> 32));
  }
}

__global__ void k_validate(const int32_t* __restrict__ code, int64_t n, int32_t lo, int32_t hi,
                           int32_t* __restrict__ flag) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t g = code[i];
    if (g < lo || g >= hi) atomicOr(flag, 1);
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
  return launch_validate_range(code, n, 0, G, flag, s);
}

int launch_validate_range(const int32_t* code, int64_t n, int32_t lo, int32_t hi, int32_t* flag, hipStream_t s) {
  if (n == 0) return LFE_OK;
  hipLaunchKernelGGL(k_validate, dim3(grid_for(n)), dim3(kBlock), 0, s, code, n, lo, hi, flag);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

// row groups per wave iteration for the 2-FE kernels: GU 2 beats 1 and 4 at NT = 1 (occupancy
// 4 vs 2 waves/SIMD, measured)
constexpr int kGramGU = 2;

constexpr int kGramThreadsQL = 1024;  // alpha_Q in LDS: one 110 KB workgroup per CU, 16 waves

template <int MODE, int NT>
static const void* gram_kernel(bool general, bool weighted, bool ql, bool nq2 = false) {
  if (MODE == GRAM_TABLE) return reinterpret_cast<const void*>(&k_gram_table<NT>);
  constexpr int M = MODE == GRAM_TABLE ? GRAM_DESIGN : MODE;
  if (general) {
    // three FEs at p <= 16: two 16-row groups per wave iteration with X loaded a batch ahead
    // (config 4: residual 3.76 -> 3.47 ms, design 2.39 -> 2.29 ms; round 5).  LFE_GRAM_GEN=0: the
    // generic variant (A/B)
    const int gen = [] {
      const char* e = knob("LFE_GRAM_GEN");
      return e ? atoi(e) : 2;
    }();
    if (gen == 2 && nq2 && NT == 1)
      return weighted ? reinterpret_cast<const void*>(&k_gram<M, NT, 2, 2, true, false, kGramThreads>)
                      : reinterpret_cast<const void*>(&k_gram<M, NT, 2, 2, false, false, kGramThreads>);
    return weighted ? reinterpret_cast<const void*>(&k_gram<M, NT, kMaxFE - 1, 1, true, false, kGramThreads>)
                    : reinterpret_cast<const void*>(&k_gram<M, NT, kMaxFE - 1, 1, false, false, kGramThreads>);
  }
  if (ql && NT == 1) {
    // 16 waves per CU need <= 128 VGPRs: GU 2
    return weighted ? reinterpret_cast<const void*>(&k_gram<M, 1, 1, 2, true, true, kGramThreadsQL>)
                    : reinterpret_cast<const void*>(&k_gram<M, 1, 1, 2, false, true, kGramThreadsQL>);
  }
#define GRAM_FN(GU) (weighted ? reinterpret_cast<const void*>(&k_gram<M, NT, 1, GU, true, false, kGramThreads>) \
                              : reinterpret_cast<const void*>(&k_gram<M, NT, 1, GU, false, false, kGramThreads>))
  // wide fits: one 16-row group per wave iteration (GU 2 holds 232 registers at NT = 2: two waves
  // per SIMD) unless LFE_GRAM_GU=2 (A/B)
  const int gu_wide = [] {
    const char* e = knob("LFE_GRAM_GU");
    return e ? atoi(e) : 1;
  }();
  if (NT >= 2 && gu_wide == 1) return GRAM_FN(1);
  return GRAM_FN(kGramGU);
#undef GRAM_FN
}

template <int MODE, int NT>
static int run_gram(lfe_ctx* c, GramArgs a, double* host_out, int extra) {
  using Sh = GramShape<NT>;
  int nblocks;
  size_t dyn = 0;
  int threads = kGramThreads;
  a.nq = 0;
  for (int f = 0; f < a.la.F; ++f)
    if (f != a.la.P) a.qf[a.nq++] = f;
  a.G_Q = a.nq > 0 ? c->fe[a.qf[0]].G : 0;
  const void* fn = nullptr;
  if (MODE == GRAM_TABLE) {
    fn = gram_kernel<MODE, NT>(false, false, false);
    const int64_t ngroups = (a.rows + 15) / 16;
    nblocks = (int)std::min<int64_t>(std::max<int64_t>((ngroups + 3) / 4, 1), 2048);
  } else {
    const size_t sbytes = sizeof(double) * (size_t)a.B * a.la.p;
    a.stage = (a.la.P >= 0 && sbytes <= 96 * 1024) ? 1 : 0;
    dyn = a.stage ? sbytes : 0;
    // one non-primary FE whose alpha table fits next to the slice: stage it in LDS
    const size_t qbytes = sizeof(double) * (size_t)a.G_Q * a.la.p;
    const bool ql = NT == 1 && a.nq == 1 && a.stage && dyn + qbytes <= 150 * 1024;
    if (ql) {
      dyn += qbytes;
      threads = kGramThreadsQL;
    }
    fn = gram_kernel<MODE, NT>(a.nq > 1, a.w != nullptr, ql, a.nq == 2);
    if (dyn > 64 * 1024)  // dynamic LDS above 64 KB must be opted in
      LFE_HIP(set_max_lds(fn, (int)dyn));
    nblocks = row_blocks(c, resident_blocks(c, fn, threads, dyn));
  }
  const int64_t pstride = Sh::LEN + 4;
  LFE_TRY(ensure_scratch(c, (size_t)nblocks * pstride));
  LFE_TRY(ensure_dred(c, (size_t)pstride));
  {
    ProfScope _ps(c, MODE == GRAM_DESIGN ? K_GRAM_DESIGN : (MODE == GRAM_RESID ? K_GRAM_RESID : K_GRAM_TABLE));
    double* part = c->scratch;
    void* args[] = {&a, &part, const_cast<int64_t*>(&pstride)};
    LFE_HIP(hipLaunchKernel(fn, dim3(nblocks), dim3(threads), args, dyn, c->stream));
  }
  LFE_HIP(hipGetLastError());
  const int len = Sh::LEN + extra;
  {
    ProfScope _ps(c, K_REDUCE);
    hipLaunchKernelGGL(k_reduce_partials, dim3(len), dim3(256), 0, c->stream, c->scratch, nblocks, pstride, c->dred);
  }
  LFE_HIP(hipGetLastError());
  LFE_TRY(allreduce_sum_f64(c, c->dred, len));
  LFE_TRY(d2h_sync(c, host_out, c->dred, sizeof(double) * len));
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

// gram of `tile_cols` staged columns; the dense output keeps columns [off, off + ncols)
template <int MODE>
static int gram_dispatch(lfe_ctx* c, GramArgs a, int tile_cols, int off, int ncols, double* dense_out,
                         double* extra_out, int extra) {
  const int NT = (std::max(tile_cols, 1) + 15) / 16;
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
  if (dense_out) {
    std::vector<double> full((size_t)tile_cols * tile_cols);
    unpack_tiles(h.data(), NT, tile_cols, full.data());
    for (int i = 0; i < ncols; ++i)
      for (int j = 0; j < ncols; ++j) dense_out[i * ncols + j] = full[(size_t)(i + off) * tile_cols + (j + off)];
  }
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

static bool resid_rows_ok(const lfe_ctx* c, const GramArgs& a) {
  // p <= 12: the meat's upper triangle stays in registers (p = 16 would spill)
  const int PM = c->p <= 4 ? 4 : c->p <= 8 ? 8 : 12;
  // both alpha tables as dynamic LDS beside the row kernels' static LDS (k_design_rows /
  // k_resid_rows: at most 960, 2880, 4992 bytes for PM 4, 8, 12) within the CU's 160 KB
  const size_t stat = PM == 4 ? 1024 : PM == 8 ? 3072 : 5120;
  return c->F == 2 && c->p <= 12 && c->p >= 2 && !a.w && a.la.P >= 0 && c->L.permuted &&
         ((size_t)a.B + c->fe[1 - a.la.P].G) * PM * 8 + stat <= 160 * 1024;
}

// row-per-lane design Gram (k_design_rows): the reduced [16][16] tile (column 0 =
// intercept, 1 + c = data column c; all ranks) is left in out_dev
static int design_rows_enqueue(lfe_ctx* c, GramArgs a, double* out_dev) {
  a.nq = 1;
  a.qf[0] = 1 - a.la.P;
  a.G_Q = c->fe[a.qf[0]].G;
  const int p = c->p;
  const int PM = p <= 4 ? 4 : p <= 8 ? 8 : 11;
  const size_t dyn = sizeof(double) * ((size_t)a.B + a.G_Q) * ((PM + 1) & ~1);
  const void* fn = PM == 4   ? reinterpret_cast<const void*>(&k_design_rows<4, 2>)
                   : PM == 8 ? reinterpret_cast<const void*>(&k_design_rows<8, 2>)
                             : reinterpret_cast<const void*>(&k_design_rows<11, 1>);
  if (dyn > 64 * 1024) LFE_HIP(set_max_lds(fn, (int)dyn));
  const int nblocks = row_blocks(c, resident_blocks(c, fn, kResThreads, dyn));
  const int64_t pstride = 256 + 4;
  LFE_TRY(ensure_scratch(c, (size_t)nblocks * pstride));
  {
    ProfScope _ps(c, K_GRAM_DESIGN);
    double* part = c->scratch;
    void* args[] = {&a, &part, const_cast<int64_t*>(&pstride)};
    LFE_HIP(hipLaunchKernel(fn, dim3(nblocks), dim3(kResThreads), args, dyn, c->stream));
  }
  LFE_HIP(hipGetLastError());
  {
    ProfScope _ps(c, K_REDUCE);
    hipLaunchKernelGGL(k_reduce_partials, dim3(256), dim3(256), 0, c->stream, c->scratch, nblocks, pstride, out_dev);
  }
  LFE_HIP(hipGetLastError());
  return allreduce_sum_f64(c, out_dev, 256);
}

// ---------------------------------------------------------------------------
// Gram from group tables (two FEs after demean_fast, unweighted, one process).
// With d~ = d - a_h - b_q (a = alpha_P, b = alpha_Q) and every data column shifted
// by its first layout row c (a shift the FEs absorb: d - c - a - (b - c) = d~):
//   sum d~ d~' = R + sum_h [n a a' - S a' - a S'] + sum_q [n b' b'' - V b'' - b' V']
//   sum d~     = C - sum_h n a - sum_q n b'
// with R, C the raw Gram / column sums of d - c over kept rows (k_sums2_raw / k_sums4<RAW>),
// S the group sums, b' = b - c, V = S_Q - n c - T_Q and T_Q = sum_{i in q} a_{h_i}
// (the last sweep's cross term, formed from the final a).  Per group the bracket is
// n a_i a_j - V_i a_j - a_i V_j: symmetric, so only the upper triangle is summed.
// The group tables replace the design pass over X (8p + 4F bytes per row).
// Cancellation guard: the assembled diagonal must keep > 1/kTabKappa of R's.
// ---------------------------------------------------------------------------
constexpr double kTabKappa = 1e4;

struct TabArgs {
  const double* alpha[2];  // [G][p]: P, Q
  const double* S[2];
  const double* TQ;        // [G_Q][p]
  const int32_t* cnt[2];
  int G[2];
  int p;
  const double* shift;     // [16] the raw tile's shift c
  int q_on;                // 0: skip the secondary groups (owner-sharded ranks other than 0)
  // speculative Gram (gram_spec_enqueue): run only when the stop test just computed on the device
  // (u64 bits of the check's max) is below tol - an unconverged sweep pays an empty launch
  const unsigned long long* gate;
  double gate_tol;
};

__device__ __forceinline__ bool gate_closed(const unsigned long long* gate, double tol) {
  return gate && !(__longlong_as_double((long long)*gate) < tol);
}

// the final step of the tables Gram (k_tables_final_chol): partials -> tile, guard flag, Cholesky
struct TabFinal {
  const double* raw;
  double* tile;
  double* flag;
  double* beta;
  double* beta_copy;
  double* ok;
};

template <int PM>
__global__ __launch_bounds__(256) void k_tables_gram(TabArgs t, double* __restrict__ partial) {
  constexpr int NG = PM * (PM + 1) / 2;
  constexpr int NA = NG + PM;
  __shared__ double red[4][NA];
  if (gate_closed(t.gate, t.gate_tol)) return;
  const int p = t.p;
  double sh[PM];
#pragma unroll
  for (int j = 0; j < PM; ++j) sh[j] = j < p ? t.shift[j] : 0.0;
  double acc[NA];
#pragma unroll
  for (int e = 0; e < NA; ++e) acc[e] = 0.0;
  const int total = t.G[0] + (t.q_on ? t.G[1] : 0);
  for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < total; g += gridDim.x * blockDim.x) {
    const int f = g < t.G[0] ? 0 : 1;
    const int gg = f ? g - t.G[0] : g;
    const double n = (double)t.cnt[f][gg];
    if (n == 0.0) continue;
    const double* al = t.alpha[f] + (int64_t)gg * p;
    const double* Sg = t.S[f] + (int64_t)gg * p;
    const double* Tg = t.TQ + (int64_t)gg * p;
    double av[PM], V[PM];
#pragma unroll
    for (int j = 0; j < PM; ++j) {
      if (j < p) {
        av[j] = f ? al[j] - sh[j] : al[j];
        V[j] = Sg[j] - n * sh[j] - (f ? Tg[j] : 0.0);
      } else {
        av[j] = V[j] = 0.0;
      }
    }
    int e = 0;
#pragma unroll
    for (int i = 0; i < PM; ++i)
#pragma unroll
      for (int j = i; j < PM; ++j, ++e) acc[e] += (n * av[i] - V[i]) * av[j] - av[i] * V[j];
#pragma unroll
    for (int i = 0; i < PM; ++i) acc[NG + i] += n * av[i];
  }
  // wave sums over DPP lane moves (VALU; a shuffle reduction of the NA sums kept this kernel
  // on ds_bpermute latency), then the four waves in order
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const auto addop = [](double x, double y) { return x + y; };
#pragma unroll
  for (int e = 0; e < NA; ++e) {
    const double v = wave_reduce63(acc[e], 0.0, addop);
    if (lane == 63) red[wave][e] = v;
  }
  __syncthreads();
  // entry-major [NA][blocks]: the final kernel's lanes then read consecutive blocks of one entry
  for (int e = threadIdx.x; e < NA; e += blockDim.x)
    partial[(int64_t)e * gridDim.x + blockIdx.x] = ((red[0][e] + red[1][e]) + red[2][e]) + red[3][e];
}

// out[e] = sum over the row e of an entry-major [rows][nblk] partial table, blocks in order
__global__ __launch_bounds__(256) void k_sum_rows(const double* __restrict__ partial, int nblk,
                                                  double* __restrict__ out) {
  __shared__ double red[256];
  const int e = blockIdx.x;
  double s = 0.0;
  for (int b = threadIdx.x; b < nblk; b += 256) s += partial[(int64_t)e * nblk + b];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[e] = red[0];
}

static bool tables_gram_ok(const lfe_ctx* c) {
  return c->raw_ready && c->tq_final && c->F == 2 && c->p <= 12 && c->L.P >= 0 && !c->L.w;
}

template <int PM>
__global__ __launch_bounds__(1024) void k_tables_final_chol(const double* __restrict__ partial, int nblk,
                                                            const double* __restrict__ raw, int p,
                                                            double* __restrict__ tile, double* __restrict__ flag,
                                                            double* __restrict__ beta, double* __restrict__ beta_copy,
                                                            double* __restrict__ ok, const unsigned long long* gate,
                                                            double gate_tol);

__global__ void k_chol_solve(const double* __restrict__ tile, int p, double* __restrict__ beta,
                             double* __restrict__ beta_copy, double* __restrict__ ok);

// design tile into out_dev[0, 256) and the guard flag into *flag_dev, from the group tables; with
// beta, also the Cholesky solve of the tile (beta, beta_copy, ok as k_chol_solve)
static int tables_gram_enqueue(lfe_ctx* c, double* out_dev, double* flag_dev, double* beta = nullptr,
                               double* beta_copy = nullptr, double* ok = nullptr,
                               const unsigned long long* gate = nullptr, double gate_tol = 0.0) {
  const int P = c->L.P, Q = 1 - P, p = c->p;
  TabArgs t{};
  t.alpha[0] = c->fe[P].alpha;
  t.alpha[1] = c->fe[Q].alpha;
  t.S[0] = c->fe[P].S;
  t.S[1] = c->fe[Q].S;
  t.TQ = c->fe[Q].T;
  t.cnt[0] = c->fe[P].cnt;
  t.cnt[1] = c->fe[Q].cnt;
  t.G[0] = c->fe[P].G;
  t.G[1] = c->fe[Q].G;
  t.p = p;
  t.shift = c->raw_shift;
  // owner-sharded rows: each rank's primary groups are its own (partial sums over ranks), the
  // secondary tables are global (counted on rank 0 only); the sums are all-reduced before the
  // final tile.  Otherwise every rank holds the same global tables.
  t.q_on = (!c->owner_on || c->rank == 0) ? 1 : 0;
  t.gate = gate;
  t.gate_tol = gate_tol;
  const int PM = p <= 4 ? 4 : p <= 8 ? 8 : 12;
  const int NA = PM * (PM + 1) / 2 + PM;
  const int nblk = grid_for((int64_t)t.G[0] + t.G[1], 256, 256);  // the final sums the partials by waves
  LFE_TRY(ensure_scratch(c, (size_t)nblk * NA + NA));
  ProfScope _ps(c, K_GRAM_TABLES);
  double* part = c->scratch;
  double* msum = c->scratch + (size_t)nblk * NA;
  const bool split = [] {  // diagnostic: the Cholesky as its own launch (rocprof A/B)
    const char* e = knob("LFE_CHOL_SPLIT");
    return e && e[0] == '1';
  }();
  auto final_from = [&](auto kfinal) -> int {
    // one block sums the block partials in a fixed order, forms the tile and (beta) solves it.
    // Owner-sharded rows: one workgroup per entry sums the partials first, then the sums over
    // ranks, then the tile
    const double* src = part;
    int ns = nblk;
    if (c->owner_on) {
      hipLaunchKernelGGL(k_sum_rows, dim3(NA), dim3(256), 0, c->stream, part, nblk, msum);
      LFE_HIP(hipGetLastError());
      LFE_TRY(allreduce_sum_f64(c, msum, (size_t)NA));
      src = msum;
      ns = 1;
    }
    hipLaunchKernelGGL(kfinal, dim3(1), dim3(1024), 0, c->stream, src, ns, c->raw_tile, p, out_dev, flag_dev,
                       split ? nullptr : beta, beta_copy, ok, gate, gate_tol);
    if (split && beta)
      hipLaunchKernelGGL(k_chol_solve, dim3(1), dim3(64), 0, c->stream, out_dev, p, beta, beta_copy, ok);
    return LFE_OK;
  };
  // (a fused form - the last block of k_tables_gram summing the partials and solving on 256 threads -
  // measured 43 us against 14 + 14 us for the two launches at the 8-rank shard: kept apart)
  switch (PM) {
    case 4:
      hipLaunchKernelGGL(k_tables_gram<4>, dim3(nblk), dim3(256), 0, c->stream, t, part);
      LFE_TRY(final_from(k_tables_final_chol<4>));
      break;
    case 8:
      hipLaunchKernelGGL(k_tables_gram<8>, dim3(nblk), dim3(256), 0, c->stream, t, part);
      LFE_TRY(final_from(k_tables_final_chol<8>));
      break;
    default:
      hipLaunchKernelGGL(k_tables_gram<12>, dim3(nblk), dim3(256), 0, c->stream, t, part);
      LFE_TRY(final_from(k_tables_final_chol<12>));
      break;
  }
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

void reduce_tiles(lfe_ctx* c, const double* part, int nblocks, double* out) {
  hipLaunchKernelGGL(k_reduce_partials, dim3(256), dim3(256), 0, c->stream, part, nblocks, (int64_t)256, out);
}

// beta_full of X = [1, x] from the reduced design tile (column 0 intercept, 1 y, 2.. x):
// Cholesky of X'X and two triangular solves, one thread (m <= 12).  ok = 0 when X'X is
// not positive definite (the host then solves as polars_impl.py:217-220 does).
// beta_full from the Gram tile by Cholesky (p <= 12).  Fixed loop bounds with
// guards unroll completely, so L stays in registers (a runtime-bounded version
// indexed a scratch array and took ~70 us).
// the block's threads: right-looking Cholesky in LDS (a column step is a sqrt, a scaled column
// and a trailing update spread over the threads), then the two triangular solves on thread 0.
// tile: global or LDS.  Every thread of the block must call it (it holds barriers).
constexpr int kCholM = 12;
// beta_full from the Cholesky factor of the design tile (intercept + the k regressors: tile rows
// 0, 2, 3, ..), by ONE wave in registers: lane i holds row i of L (columns by register), the
// column elements other lanes need arrive by shuffles, and the forward / back substitutions run
// in the order of the serial loops of polars_impl.py:212-226's LAPACK-free restatement (so the
// bits are those of the one-thread form this replaced: ~1.5 us instead of ~15 us of LDS round trips)
// lane k's value to every lane (k wave-uniform: two v_readlane, no LDS round trip as ds_bpermute)
__device__ __forceinline__ double bcast_lane(double v, int k) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), k);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), k);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ void chol_solve_wave(const double* tile, int p, double* __restrict__ beta,
                                                double* __restrict__ beta_copy, double* __restrict__ ok,
                                                double (*Ls)[kCholM + 1]) {
  // every loop runs its constant bound with the active range as a predicate, so all of them
  // unroll and r / col / xs stay in registers (a loop left rolled indexes them in scratch memory)
  constexpr int M = kCholM;
  const int lane = threadIdx.x & 63;
  const int m = p;  // intercept + k regressors
  auto idx = [](int i) { return i == 0 ? 0 : i + 1; };
  double r[M];
#pragma unroll
  for (int k = 0; k < M; ++k) r[k] = (lane < m && k < m) ? tile[idx(lane) * 16 + idx(k)] : 0.0;
  const double bv = lane < m ? tile[idx(lane) * 16 + 1] : 0.0;
  bool bad = false;
#pragma unroll
  for (int j = 0; j < M; ++j) {
    const bool live = j < m;  // uniform
    const double d = bcast_lane(r[j], j);
    bad |= live && !(d > 0.0);
    const double ljj = sqrt(d > 0.0 ? d : 1.0);
    if (live) {
      if (lane == j) r[j] = ljj;
      else if (lane > j && lane < m) r[j] /= ljj;
    }
#pragma unroll
    for (int k = j + 1; k < M; ++k) {
      const double lkj = bcast_lane(r[j], k);
      if (live && k < m && lane >= k && lane < m) r[k] -= r[j] * lkj;  // L[i][k] -= L[i][j] L[k][j], j < k <= i
    }
  }
  if (bad) {
    if (lane == 0) *ok = 0.0;
    return;
  }
  // forward: y_i = (b_i - sum_{k < i} L[i][k] y_k) / L[i][i], the k in ascending order
  double acc = bv;
#pragma unroll
  for (int k = 0; k < M; ++k) {
    const double yk = bcast_lane(acc / (r[k] != 0.0 ? r[k] : 1.0), k);  // lane k: r[k] = L[k][k]
    if (k < m) {
      if (lane == k) acc = yk;
      else if (lane > k) acc -= r[k] * yk;
    }
  }
  // back: x_i = (y_i - sum_{k > i} L[k][i] x_k) / L[i][i], k ascending: lane i's column of L via LDS
  if (lane < m)
#pragma unroll
    for (int k = 0; k < M; ++k) Ls[lane][k] = r[k];
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  double col[M], xs[M];
#pragma unroll
  for (int k = 0; k < M; ++k) {
    col[k] = (lane < m && k < m) ? Ls[k][lane] : 0.0;
    xs[k] = 0.0;
  }
  double diag = 1.0;
#pragma unroll
  for (int k = 0; k < M; ++k)
    if (k == lane) diag = r[k];
#pragma unroll
  for (int i = M - 1; i >= 0; --i) {
    double v = acc;  // lane i: y_i
#pragma unroll
    for (int k = i + 1; k < M; ++k) v -= col[k] * xs[k];  // xs[k] = 0 for k >= m
    const double xi = bcast_lane(v / diag, i);
    if (i < m) xs[i] = xi;
  }
  if (lane < m) {
    double x = 0.0;
#pragma unroll
    for (int k = 0; k < M; ++k)
      if (k == lane) x = xs[k];
    beta[lane] = beta_copy[lane] = x;
  }
  if (lane == 0) *ok = 1.0;
}

__global__ void k_chol_solve(const double* __restrict__ tile, int p, double* __restrict__ beta,
                             double* __restrict__ beta_copy, double* __restrict__ ok) {
  __shared__ double L[kCholM][kCholM + 1];
  if (threadIdx.x < 64) chol_solve_wave(tile, p, beta, beta_copy, ok, L);
}

// The design tile from the raw tile + the table partials (the waves sum the block partials of one
// entry each, lanes over blocks in a fixed order); *flag = 1 when the cancellation guard holds;
// with beta, the Cholesky solve of the tile too, in the same launch.  NTH threads (>= 256): the
// one-block finisher (1024) or the last block of k_tables_gram (256)
template <int PM, int NTH>
__device__ void tables_final_body(const double* __restrict__ partial, int nblk, int p, const TabFinal& f) {
  constexpr int NG = PM * (PM + 1) / 2;
  constexpr int NA = NG + PM;
  constexpr int NW = NTH / 64;
  __shared__ double m[NA];
  __shared__ double tl[256];
  __shared__ int bad;
  __shared__ double L[kCholM][kCholM + 1];
  const double* raw = f.raw;
  if (threadIdx.x == 0) bad = 0;
  {
    // wave w sums entries w, w + NW, ..; lane l the blocks l, l + 64, .. (<= 256 blocks) in that
    // order: every load issued before the first add
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const auto addop = [](double x, double y) { return x + y; };
    constexpr int EU = (NA + NW - 1) / NW;
    double v[EU][4];
#pragma unroll
    for (int u = 0; u < EU; ++u)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int e = wave + NW * u, q = lane + 64 * rr;
        v[u][rr] = (e < NA && q < nblk) ? partial[(int64_t)e * nblk + q] : 0.0;
      }
#pragma unroll
    for (int u = 0; u < EU; ++u) {
      const int e = wave + NW * u;
      double s = 0.0;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        if (lane + 64 * rr < nblk) s += v[u][rr];
      s = wave_reduce63(s, 0.0, addop);
      if (lane == 63 && e < NA) m[e] = s;
    }
  }
  __syncthreads();
  if (threadIdx.x < 256) {
    const int t = threadIdx.x;
    const int i = t / 16 - 1, j = t % 16 - 1;  // design indices -> data columns
    double v = 0.0;
    if (i < p && j < p) {
      if (i < 0 && j < 0) {
        v = raw[15 * 16 + 15];
      } else if (i < 0 || j < 0) {
        const int d = i < 0 ? j : i;
        v = raw[15 * 16 + d] - m[NG + d];
      } else {
        const int lo = i < j ? i : j, hi = i < j ? j : i;
        v = raw[i * 16 + j] + m[lo * PM - lo * (lo - 1) / 2 + (hi - lo)];
        if (i == j && !(v > 0.0 && raw[i * 16 + i] <= kTabKappa * v)) atomicAdd(&bad, 1);
      }
    }
    f.tile[t] = v;
    tl[t] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) *f.flag = bad ? 0.0 : 1.0;
  if (f.beta && threadIdx.x < 64) chol_solve_wave(tl, p, f.beta, f.beta_copy, f.ok, L);
}

template <int PM>
__global__ __launch_bounds__(1024) void k_tables_final_chol(const double* __restrict__ partial, int nblk,
                                                            const double* __restrict__ raw, int p,
                                                            double* __restrict__ tile, double* __restrict__ flag,
                                                            double* __restrict__ beta, double* __restrict__ beta_copy,
                                                            double* __restrict__ ok, const unsigned long long* gate,
                                                            double gate_tol) {
  if (gate_closed(gate, gate_tol)) return;
  const TabFinal f{raw, tile, flag, beta, beta_copy, ok};
  tables_final_body<PM, 1024>(partial, nblk, p, f);
}

// ---------------------------------------------------------------------------
// Gram from group tables, three or more FEs (after the pair-table sweeps of lfe_dense3.hip,
// unweighted, one process).  With d' = d - c (every data column shifted by the first layout row),
// a'_f = alpha_f except a'_s = alpha_s - c for one FE s (the FEs absorb the shift), S'_f = S_f - n c
// and T'_f[g] = sum over g's rows of sum_{h != f} a'_h (the final cross term, T_f - n c for f != s):
//   sum d~ d~' = R + sum_f sum_g [n a' a'' - V a'' - a' V'],   V = S' - T' / 2
//   sum d~     = C - sum_f sum_g n a'
// (the cross products sum_{f != h} a'_f a'_h' over the rows are sum_f sum_g a' T'', symmetric in
// total, so each FE carries half of its T').  R, C: the raw Gram of [1, d'] over the kept rows, one
// MFMA pass over X with no effect gathers (k_raw_gram); the table terms are one pass over the
// groups of every FE (k_tab3_gram).  Cancellation guard as the two-FE form (kTabKappa).
// ---------------------------------------------------------------------------
template <int NT>
__global__ __launch_bounds__(kGramThreads) void k_raw_gram(GramArgs a, double* __restrict__ partial, int64_t pstride) {
  using Sh = GramShape<NT>;
  __shared__ double red[Sh::LEN];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kq = lane >> 4, c = lane & 15;
  const int p = a.la.p, P = a.la.P;
  d4 acc[Sh::NP];
#pragma unroll
  for (int q = 0; q < Sh::NP; ++q) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
  const double* xb[NT];
  double sh[NT], fill[NT];
  bool dat[NT];
#pragma unroll
  for (int I = 0; I < NT; ++I) {
    int xc = 16 * I + c - 1;  // design column 0 = intercept, 1 + d = data column d
    if (xc >= p) xc = -2;
    dat[I] = xc >= 0;
    fill[I] = xc == -1 ? 1.0 : 0.0;
    xb[I] = a.X + (int64_t)(xc >= 0 ? xc : 0) * a.ld;
    sh[I] = dat[I] && a.la.n_items > 0 ? xb[I][0] : 0.0;
  }
  constexpr int GU = 2;
  const BlockRows br = block_rows(a.la.items, a.la.n_items, lane);
  for (int item = br.first; item < a.la.n_items; ++item) {
    int4 it = a.la.items[item];
    if (it.y >= br.hi) break;
    it.y = max(it.y, br.lo);
    it.z = min(it.z, br.hi);
    const int g0 = it.y >> 4, g1 = (it.z + 15) >> 4;
    for (int gb = g0 + wave * GU; gb < g1; gb += (kGramThreads / 64) * GU) {
      int4 h[GU];
      d4 xv[GU][NT];
#pragma unroll
      for (int u = 0; u < GU; ++u) {  // every load of the GU groups first
        const int gi = gb + u, r = gi * 16 + kq * 4;
        h[u] = gi < g1 ? *reinterpret_cast<const int4*>(a.la.code[P] + r) : int4{-1, -1, -1, -1};
#pragma unroll
        for (int I = 0; I < NT; ++I) xv[u][I] = gi < g1 ? ld4(xb[I] + r) : d4{0.0, 0.0, 0.0, 0.0};
      }
#pragma unroll
      for (int u = 0; u < GU; ++u) {
        const int r = (gb + u) * 16 + kq * 4;
        const int hv[4] = {h[u].x, h[u].y, h[u].z, h[u].w};
        double z[4][NT];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const bool valid = hv[s] >= 0 && r + s >= it.y && r + s < it.z;
#pragma unroll
          for (int I = 0; I < NT; ++I) z[s][I] = valid ? (dat[I] ? xv[u][I][s] - sh[I] : fill[I]) : 0.0;
        }
        mfma_rows<NT>(z, acc);
      }
    }
  }
  block_reduce_store<NT, kGramThreads>(acc, red, partial + (int64_t)blockIdx.x * pstride, tid);
}

constexpr int kT3Chunk = 64;  // groups staged per round
constexpr int kT3MaxP = 32;   // (NG + p <= 560 entries: three per thread)
constexpr int kT3E = 3;

struct Tab3Args {
  const double* alpha[kMaxFE];
  const double* S[kMaxFE];
  const double* T[kMaxFE];
  const int32_t* cnt[kMaxFE];
  int64_t gstart[kMaxFE + 1];  // FE f's groups are [gstart[f], gstart[f + 1]) of the concatenation
  int F, p, sfe;               // sfe: the FE whose effects absorb the shift
  double tw[kMaxFE];           // share of its cross term each FE carries (1/2 each; two FEs: 0 and 1)
  const double* X;             // the shift c_d = X[d][0] (the raw pass's)
  int64_t ld;
};

// block partials [NG upper-triangle entries of sum_g (n a' a'' - V a'' - a' V')][p entries of sum_g n a']
__global__ __launch_bounds__(256) void k_tab3_gram(Tab3Args t, double* __restrict__ partial, int pstride) {
  __shared__ double av[kT3Chunk][kT3MaxP + 1];
  __shared__ double vv[kT3Chunk][kT3MaxP + 1];
  __shared__ double nn[kT3Chunk];
  const int p = t.p, tid = threadIdx.x, NG = p * (p + 1) / 2;
  const int64_t total = t.gstart[t.F];
  int ei[kT3E], ej[kT3E];
#pragma unroll
  for (int k = 0; k < kT3E; ++k) {  // entry -> (i, j), j >= i; or the column sums (i = -1)
    int e = tid + 256 * k, i = -2, j = 0;
    if (e < NG) {
      i = 0;
      while (e >= p - i) {
        e -= p - i;
        ++i;
      }
      j = i + e;
    } else if (e < NG + p) {
      i = -1;
      j = e - NG;
    }
    ei[k] = i;
    ej[k] = j;
  }
  double acc[kT3E] = {0.0, 0.0, 0.0};
  for (int64_t g0 = (int64_t)blockIdx.x * kT3Chunk; g0 < total; g0 += (int64_t)gridDim.x * kT3Chunk) {
    __syncthreads();
    for (int idx = tid; idx < kT3Chunk * p; idx += 256) {
      const int gl = idx / p, d = idx - gl * p;
      const int64_t g = g0 + gl;
      double a = 0.0, v = 0.0, n = 0.0;
      if (g < total) {
        int f = 0;
        while (g >= t.gstart[f + 1]) ++f;
        const int64_t gg = g - t.gstart[f], e = gg * p + d;
        n = (double)t.cnt[f][gg];
        if (n > 0.0) {
          const double c = t.X[(int64_t)d * t.ld];
          a = f == t.sfe ? t.alpha[f][e] - c : t.alpha[f][e];
          const double w = t.tw[f];
          const double Tp = w == 0.0 ? 0.0 : (f == t.sfe ? t.T[f][e] : t.T[f][e] - n * c);
          v = t.S[f][e] - n * c - w * Tp;
        }
      }
      av[gl][d] = a;
      vv[gl][d] = v;
      if (d == 0) nn[gl] = n;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kT3E; ++k) {
      const int i = ei[k], j = ej[k];
      if (i == -2) continue;
      double s = 0.0;
      if (i >= 0) {
        for (int gl = 0; gl < kT3Chunk; ++gl) s += (nn[gl] * av[gl][i] - vv[gl][i]) * av[gl][j] - av[gl][i] * vv[gl][j];
      } else {
        for (int gl = 0; gl < kT3Chunk; ++gl) s += nn[gl] * av[gl][j];
      }
      acc[k] += s;
    }
  }
#pragma unroll
  for (int k = 0; k < kT3E; ++k)
    if (ei[k] != -2) partial[(int64_t)blockIdx.x * pstride + tid + 256 * k] = acc[k];
}

// the design tiles (I <= J tiles of 16 x 16, design column 0 = intercept, 1 + d = data column d)
// from the raw tiles and the table sums m; *flag = 1 when the cancellation guard holds
__global__ __launch_bounds__(256) void k_tab3_assemble(const double* __restrict__ raw, const double* __restrict__ m,
                                                       int p, int NT, double* __restrict__ tile,
                                                       double* __restrict__ flag) {
  __shared__ int bad;
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  const int NG = p * (p + 1) / 2, len = NT * (NT + 1) / 2 * 256, D = p + 1;
  for (int t = threadIdx.x; t < len; t += blockDim.x) {
    int q = t >> 8, I = 0;
    while (q >= NT - I) {
      q -= NT - I;
      ++I;
    }
    const int J = I + q, a = 16 * I + ((t & 255) >> 4), b = 16 * J + (t & 15);
    double v = raw[t];
    if (a < D && b < D) {
      if (a == 0 && b == 0) {
      } else if (a == 0 || b == 0) {
        v -= m[NG + (a > b ? a : b) - 1];
      } else {
        const int lo = (a < b ? a : b) - 1, hi = (a < b ? b : a) - 1;
        v += m[lo * p - lo * (lo - 1) / 2 + (hi - lo)];
        if (a == b && !(v > 0.0 && raw[t] <= kTabKappa * v)) atomicAdd(&bad, 1);
      }
    }
    tile[t] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) *flag = bad ? 0.0 : 1.0;
}

// the group-sum pass's raw tile (k_sums2_raw: lane c < p = data column c shifted by its first
// layout row, lane 15 = the intercept) as tables3_gram's reduced raw tile (design column 0 = the
// intercept, 1 + d = data column d; D = p + 1 <= 16: one tile)
__global__ __launch_bounds__(256) void k_raw_perm(const double* __restrict__ rt, double* __restrict__ raw) {
  const int a = threadIdx.x >> 4, b = threadIdx.x & 15;
  const int ma = a == 0 ? 15 : a - 1, mb = b == 0 ? 15 : b - 1;
  raw[threadIdx.x] = rt[ma * 16 + mb];
}

static bool tables3_ok(const lfe_ctx* c) {
  const char* e = knob("LFE_TAB3");  // "0": the design pass (A/B)
  if (e && e[0] == '0') return false;
  if (!(c->world == 1 && !c->L.w && !c->records && !c->sw.on && c->p <= kT3MaxP && c->L.P >= 0 && c->L.n_items > 0))
    return false;
  // three or more FEs after the pair-table sweeps, or two FEs too wide for the raw Gram of the
  // group-sum pass (p > 12) whose sweeps left T_Q from the final alpha_P
  return c->d3.on || (c->F == 2 && c->tq_final && c->p > 12);
}

// the design Gram of [1, y~, x~] from the raw pass and the group tables into host_out (dense D x D);
// returns 1 when the guard trips (the caller runs the design pass)
template <int NT>
static int tables3_gram(lfe_ctx* c, double* host_out) {
  using Sh = GramShape<NT>;
  const int p = c->p, D = p + 1, NG = p * (p + 1) / 2;
  if (c->d3.on) LFE_TRY(dense3_final_T(c));
  GramArgs a = base_args(c);
  const void* fn = reinterpret_cast<const void*>(&k_raw_gram<NT>);
  const int nblocks = row_blocks(c, resident_blocks(c, fn, kGramThreads, 0));
  const int64_t pstride = Sh::LEN;
  int64_t total = 0;
  Tab3Args t{};
  for (int f = 0; f < c->F; ++f) {
    t.alpha[f] = c->fe[f].alpha;
    t.S[f] = c->fe[f].S;
    t.T[f] = c->fe[f].T;
    t.cnt[f] = c->fe[f].cnt;
    t.gstart[f] = total;
    total += c->fe[f].G;
  }
  t.gstart[c->F] = total;
  t.F = c->F;
  t.p = p;
  if (c->d3.on) {  // every FE carries half of its cross term (all final)
    t.sfe = c->L.P;
    for (int f = 0; f < c->F; ++f) t.tw[f] = 0.5;
  } else {  // two FEs: the whole cross term on Q's side (T_Q final), the shift on Q's effects
    const int Q = 1 - c->L.P;
    t.sfe = Q;
    t.tw[c->L.P] = 0.0;
    t.tw[Q] = 1.0;
  }
  t.X = c->L.X;
  t.ld = c->ld;
  const int nblk3 = (int)std::max<int64_t>(1, std::min<int64_t>(256, (total + kT3Chunk - 1) / kT3Chunk));
  const int ps3 = 256 * kT3E;
  LFE_TRY(ensure_scratch(c, (size_t)nblocks * pstride + (size_t)nblk3 * ps3));
  LFE_TRY(ensure_dred(c, (size_t)2 * Sh::LEN + NG + p + 8));
  double* part = c->scratch;
  double* part3 = c->scratch + (size_t)nblocks * pstride;
  double* raw = c->dred;                // [LEN] reduced raw tiles
  double* m = c->dred + Sh::LEN;        // [NG + p] table sums
  double* tile = m + NG + p;            // [LEN] design tiles, then the flag
  // two FEs with p <= 15: the group-sum pass left the raw tile (same shift), so no pass over X
  const bool reuse = NT == 1 && !c->d3.on && c->F == 2 && c->raw_ready && p <= 15;
  if (!reuse) {
    ProfScope _ps(c, K_GRAM_DESIGN);
    void* args[] = {&a, &part, const_cast<int64_t*>(&pstride)};
    LFE_HIP(hipLaunchKernel(fn, dim3(nblocks), dim3(kGramThreads), args, 0, c->stream));
  }
  LFE_HIP(hipGetLastError());
  {
    ProfScope _ps(c, K_GRAM_TABLES);
    if (reuse) hipLaunchKernelGGL(k_raw_perm, dim3(1), dim3(256), 0, c->stream, c->raw_tile, raw);
    else hipLaunchKernelGGL(k_reduce_partials, dim3(Sh::LEN), dim3(256), 0, c->stream, part, nblocks, pstride, raw);
    hipLaunchKernelGGL(k_tab3_gram, dim3(nblk3), dim3(256), 0, c->stream, t, part3, ps3);
    hipLaunchKernelGGL(k_reduce_partials, dim3(NG + p), dim3(256), 0, c->stream, part3, nblk3, (int64_t)ps3, m);
    hipLaunchKernelGGL(k_tab3_assemble, dim3(1), dim3(256), 0, c->stream, raw, m, p, NT, tile, tile + Sh::LEN);
  }
  LFE_HIP(hipGetLastError());
  std::vector<double> h((size_t)Sh::LEN + 1);
  LFE_TRY(d2h_sync(c, h.data(), tile, sizeof(double) * (Sh::LEN + 1)));
  if (h[Sh::LEN] != 1.0) return 1;
  std::vector<double> full((size_t)D * D);
  unpack_tiles(h.data(), NT, D, full.data());
  for (int e = 0; e < D * D; ++e) host_out[e] = full[e];
  return LFE_OK;
}

int launch_gram(lfe_ctx* c, double* host_gram) {
  if (tables3_ok(c)) {  // three or more FEs after the pair-table sweeps: no effect gathers
    const int NT = (c->p + 1 + 15) / 16;
    const int rc = NT == 1 ? tables3_gram<1>(c, host_gram) : tables3_gram<2>(c, host_gram);
    if (rc != 1) return rc;  // else the guard tripped: the design pass
  }

  GramArgs a = base_args(c);
  const bool spec = c->gram_spec;  // the tables tile is already on the stream (lfe_demean)
  c->gram_spec = false;
  if (resid_rows_ok(c, a) && c->p <= 11) {
    LFE_TRY(ensure_dred(c, 260));
    std::vector<double> h(533);
    bool done = false;
    if (spec) {
      LFE_TRY(d2h_sync(c, h.data(), c->dspec, sizeof(double) * 533));
      done = h[532] == 1.0;
    } else if (tables_gram_ok(c)) {  // the Gram from the group tables, unless its guard trips
      LFE_TRY(tables_gram_enqueue(c, c->dred, c->dred + 256));
      LFE_TRY(d2h_sync(c, h.data(), c->dred, sizeof(double) * 257));
      done = h[256] == 1.0;
    }
    if (!done && c->sw.on) return 2;  // streamed X: the caller streams the design-Gram pass
    if (!done) {
      LFE_TRY(design_rows_enqueue(c, a, c->dred));
      LFE_TRY(d2h_sync(c, h.data(), c->dred, sizeof(double) * 256));
    }
    const int D = c->p + 1;
    for (int i = 0; i < D; ++i)
      for (int j = 0; j < D; ++j) host_gram[i * D + j] = h[(size_t)i * 16 + j];
    return LFE_OK;
  }
  if (c->sw.on) return 2;
  return gram_dispatch<GRAM_DESIGN>(c, a, c->p + 1, 0, c->p + 1, host_gram, nullptr, 0);
}

// row-per-lane residual pass (k_resid_rows): two FEs, unweighted, p <= 12, both
// alpha tables (padded to PM doubles per row) in LDS; leaves the reduced [16][16]
// tile + 4 statistics (260 doubles, all ranks) in out_dev
static int resid_rows_enqueue(lfe_ctx* c, GramArgs a, double* out_dev, bool cl = false,
                              const double* msg_src = nullptr, int msg_count = 0, unsigned long long msg_seq = 0) {
  const int p = c->p;
  const int PM = p <= 4 ? 4 : p <= 8 ? 8 : 12;
  const size_t dyn = cl ? sizeof(double) * (size_t)a.B * (PM + (p - 1))
                        : sizeof(double) * ((size_t)a.B + a.G_Q) * PM;
  const void* fn = cl ? (PM == 4   ? reinterpret_cast<const void*>(&k_resid_rows<4, 2, true>)
                         : PM == 8 ? reinterpret_cast<const void*>(&k_resid_rows<8, 2, true>)
                                   : reinterpret_cast<const void*>(&k_resid_rows<12, 2, true>))
                      : (PM == 4   ? reinterpret_cast<const void*>(&k_resid_rows<4, 2, false>)
                         : PM == 8 ? reinterpret_cast<const void*>(&k_resid_rows<8, 2, false>)
                                   : reinterpret_cast<const void*>(&k_resid_rows<12, 2, false>));
  if (dyn > 64 * 1024) LFE_HIP(set_max_lds(fn, (int)dyn));
  const int nblocks = row_blocks(c, resident_blocks(c, fn, kResThreads, dyn));
  const int64_t pstride = 256 + 4;
  LFE_TRY(ensure_scratch(c, (size_t)nblocks * pstride));
  {
    ProfScope _ps(c, K_GRAM_RESID);
    double* part = c->scratch;
    void* args[] = {&a, &part, const_cast<int64_t*>(&pstride)};
    LFE_HIP(hipLaunchKernel(fn, dim3(nblocks), dim3(kResThreads), args, dyn, c->stream));
  }
  LFE_HIP(hipGetLastError());
  {
    ProfScope _ps(c, K_REDUCE);
    if (msg_src)  // one rank: the result block straight to mapped host memory
      hipLaunchKernelGGL(k_reduce_partials_msg, dim3(pstride), dim3(256), 0, c->stream, c->scratch, nblocks, pstride,
                         out_dev, c->gsync + GS_RESID, msg_src, msg_count, c->dmsg, msg_seq);
    else
      hipLaunchKernelGGL(k_reduce_partials, dim3(pstride), dim3(256), 0, c->stream, c->scratch, nblocks, pstride,
                         out_dev);
  }
  LFE_HIP(hipGetLastError());
  return allreduce_sum_f64(c, out_dev, (size_t)pstride);
}

static void unpack_resid(const double* h, int k, double* meat, double* stats) {
  for (int i = 0; i < k; ++i)
    for (int j = 0; j < k; ++j) meat[i * k + j] = h[(size_t)(1 + i) * 16 + (1 + j)];
  for (int e = 0; e < 4; ++e) stats[e] = h[256 + e];
}

static int resid_rows(lfe_ctx* c, GramArgs a, double* meat, double* stats) {
  LFE_TRY(ensure_dred(c, 260));
  LFE_TRY(resid_rows_enqueue(c, a, c->dred));
  std::vector<double> h(260);
  LFE_TRY(d2h_sync(c, h.data(), c->dred, sizeof(double) * 260));
  unpack_resid(h.data(), c->p - 1, meat, stats);
  return LFE_OK;
}

// ---------------------------------------------------------------------------
// out-of-core X: residual / design-Gram pass over one streamed chunk
// ---------------------------------------------------------------------------
// Row per lane in input order; x~ = x - sum_f alpha_f[g_f] with the alpha rows gathered from the
// global tables (L2 / MALL resident; the pass is bound by the host link, not by these gathers).
// MODE 0: r = y~ - beta0 - sum_j beta_j x~_j (unweighted residual, polars_impl.py:229), the
// statistics (sum w r^2, sum r^2, sum y~, sum y~^2) and the meat sum w r^2 u u' over u = x~ (IC 0)
// or u = [1, x~, z~] (IC 1, the IV residual of std_errors.py:448-602) - tile (1 + i, 1 + j) =
// meat (i, j), stats at 256..259 - and, with `scores`, the chunk's score rows u r w ([rows][ks]);
// MODE 1: the Gram of sqrt(w) [1, y~, x~] (as k_design_rows: column 0 = intercept, 1 + c = data
// column c, polars_impl.py:201-209).
struct StreamRowArgs {
  const double* X;
  int64_t ld, rows;
  int p, F;
  const int32_t* code[kMaxFE];
  const int32_t* cnt_pre[kMaxFE];
  const double* alpha[kMaxFE];
  const double* w;     // the chunk's weights (null: unweighted)
  const double* beta;  // MODE 0: [p] beta_full (IC 1: the coefficients of u)
  double* scores;      // MODE 0: [rows][ks] score rows, or null
  int ks;
};

template <int PM, int MODE, int IC>
__global__ __launch_bounds__(256) void k_stream_rows(StreamRowArgs a, double* __restrict__ partial) {
  constexpr int KM = PM - 1 + IC;  // meat width (u)
  constexpr int NM = MODE == 0 ? KM * (KM + 1) / 2 : (PM + 1) * (PM + 2) / 2;  // meat / Gram of [1, d]
  constexpr int NS = MODE == 0 ? 4 : 0;
  __shared__ double red[4][NM + NS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int p = a.p, F = a.F;
  const int km = p - 1 + IC;  // live meat columns
  double beta[PM];
#pragma unroll
  for (int cc = 0; cc < PM; ++cc) beta[cc] = (MODE == 0 && cc < p) ? a.beta[cc] : 0.0;
  double m[NM];
#pragma unroll
  for (int e = 0; e < NM; ++e) m[e] = 0.0;
  double st[4] = {0.0, 0.0, 0.0, 0.0};
  for (int64_t row = (int64_t)blockIdx.x * 256 + tid; row < a.rows; row += (int64_t)gridDim.x * 256) {
    bool keep = true;
    int32_t g[kMaxFE];
#pragma unroll
    for (int f = 0; f < kMaxFE; ++f) {
      g[f] = 0;
      if (f < F) {
        g[f] = a.code[f][row];
        keep = keep && a.cnt_pre[f][g[f]] > 1;
      }
    }
    if (!keep) {  // dropped singleton (its score row stays zero)
      if (MODE == 0 && a.scores)
        for (int j = 0; j < km; ++j) a.scores[row * a.ks + j] = 0.0;
      continue;
    }
    double xt[PM];
#pragma unroll
    for (int cc = 0; cc < PM; ++cc) xt[cc] = cc < p ? a.X[(int64_t)cc * a.ld + row] : 0.0;
#pragma unroll
    for (int f = 0; f < kMaxFE; ++f) {
      if (f >= F) continue;
      const double* af = a.alpha[f] + (int64_t)g[f] * p;
#pragma unroll
      for (int cc = 0; cc < PM; ++cc)
        if (cc < p) xt[cc] -= af[cc];
    }
    const double wi = a.w ? a.w[row] : 1.0;
    if (MODE == 0) {
      double res = xt[0] - beta[0];  // polars_impl.py:229
#pragma unroll
      for (int cc = 1; cc < PM; ++cc) res -= beta[cc] * xt[cc];
      const double rr = res * res;
      st[0] += a.w ? wi * rr : rr;
      st[1] += rr;
      st[2] += xt[0];
      st[3] += xt[0] * xt[0];
      const double mr = a.w ? res * sqrt(wi) : res;
      double u[KM];
#pragma unroll
      for (int j = 0; j < KM; ++j) u[j] = IC ? (j == 0 ? 1.0 : xt[j]) : xt[j + 1];
      if (a.scores) {
        const double sc = a.w ? res * wi : res;
#pragma unroll
        for (int j = 0; j < KM; ++j)
          if (j < km) a.scores[row * a.ks + j] = u[j] * sc;
      }
      double wv[KM];
#pragma unroll
      for (int j = 0; j < KM; ++j) wv[j] = u[j] * mr;
      int e = 0;
#pragma unroll
      for (int i = 0; i < KM; ++i)
#pragma unroll
        for (int j = i; j < KM; ++j, ++e) m[e] += wv[i] * wv[j];
    } else {
      const double sw = a.w ? sqrt(wi) : 1.0;  // X_w = X sqrt(w), polars_impl.py:202-203
      double d[PM + 1];
      d[0] = sw;
#pragma unroll
      for (int cc = 0; cc < PM; ++cc) d[cc + 1] = xt[cc] * sw;
      int e = 0;
#pragma unroll
      for (int i = 0; i <= PM; ++i)
#pragma unroll
        for (int j = i; j <= PM; ++j, ++e) m[e] += d[i] * d[j];
    }
  }
  const auto addop = [](double x, double y) { return x + y; };
#pragma unroll
  for (int e = 0; e < NM; ++e) {
    const double v = wave_reduce63(m[e], 0.0, addop);
    if (lane == 63) red[wave][e] = v;
  }
#pragma unroll
  for (int e = 0; e < NS; ++e) {
    const double v = wave_reduce63(st[e], 0.0, addop);
    if (lane == 63) red[wave][NM + e] = v;
  }
  __syncthreads();
  double* out = partial + (int64_t)blockIdx.x * 260;
  for (int t = tid; t < 260; t += 256) {
    double v = 0.0;
    if (t < 256) {
      int i = t / 16, j = t % 16, e = -1;
      if (MODE == 0) {
        --i;
        --j;  // tile (1 + i, 1 + j) = meat (i, j)
        if (i >= 0 && j >= 0 && i < KM && j < KM) {
          const int lo2 = i < j ? i : j, hi2 = i < j ? j : i;
          e = lo2 * KM - lo2 * (lo2 - 1) / 2 + (hi2 - lo2);
        }
      } else if (i <= PM && j <= PM) {  // design index 0 = intercept, 1 + c = column c
        const int lo2 = i < j ? i : j, hi2 = i < j ? j : i;
        e = lo2 * (PM + 1) - lo2 * (lo2 - 1) / 2 + (hi2 - lo2);
      }
      if (e >= 0) v = ((red[0][e] + red[1][e]) + red[2][e]) + red[3][e];
    } else if (MODE == 0) {
      const int e = NM + (t - 256);
      v = ((red[0][e] + red[1][e]) + red[2][e]) + red[3][e];
    }
    out[t] = v;
  }
}

// Wide fits (p > 11: the row-per-lane kernel above would hold a (p + 1)^2 / 2 accumulator per lane).
// The MFMA lane layout of k_gram over the chunk's rows in input order: lane (kq, c) owns design
// column 16 I + c (I < NT) of rows 16 g + 4 kq + s, gathers its columns of every FE's alpha rows
// from the global tables, and the Gram / meat accumulates on v_mfma_f64_16x16x4f64 in NT (NT + 1) / 2
// output blocks.  MODE 1: column 0 = sqrt(w), 1 + c = sqrt(w) x~_c (the Gram of X_w = [1, y~, x~] sqrt(w),
// polars_impl.py:201-209).  MODE 0: the residual r = y~ - beta0 - sum_j beta_j x~_j (polars_impl.py:229)
// is one 16-lane DPP sum per row; the meat columns are u r sqrt(w) with u = x~ (IC 0: column c = x~_c,
// tile (1 + i, 1 + j) = meat (i, j)) or u = [1, x~, z~] (IC 1: the intercept in y's column 0; the
// tile conversion shifts it by one so both forms unpack alike), the statistics after the blocks.
template <int NT, int MODE, int IC>
__global__ __launch_bounds__(256) void k_stream_wide(StreamRowArgs a, double* __restrict__ partial, int64_t pstride) {
  using Sh = GramShape<NT>;
  __shared__ double red[Sh::LEN];
  __shared__ double stat_red[4][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kq = lane >> 4, c = lane & 15;
  const int p = a.p, F = a.F;
  d4 acc[Sh::NP];
#pragma unroll
  for (int q = 0; q < Sh::NP; ++q) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
  double st[4] = {0.0, 0.0, 0.0, 0.0};
  int xl[NT];
  bool dat[NT], one[NT];
  double fill[NT], coef[NT];
#pragma unroll
  for (int I = 0; I < NT; ++I) {
    const int col = 16 * I + c;
    int xc = MODE == 1 ? col - 1 : col;  // MODE 1: column 0 = intercept
    if (xc >= p) xc = -2;
    xl[I] = xc >= 0 ? xc : 0;
    fill[I] = xc == -1 ? 1.0 : 0.0;
    coef[I] = MODE == 0 ? (xc == 0 ? 1.0 : (xc >= 1 ? -a.beta[xc] : 0.0)) : 0.0;
    one[I] = MODE == 0 && IC && xc == 0;
    dat[I] = MODE == 0 ? (xc >= 1 || one[I]) : xc >= 0;
  }
  const double beta0 = MODE == 0 ? a.beta[0] : 0.0;
  const int64_t ngroups = (a.rows + 15) >> 4;
  for (int64_t g = (int64_t)blockIdx.x * 4 + wave; g < ngroups; g += (int64_t)gridDim.x * 4) {
    const int64_t r = g * 16 + kq * 4;
    double xt[4][NT], wv[4];
    bool valid[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int64_t row = r + s;
      bool keep = row < a.rows;
      int32_t gc[kMaxFE];
#pragma unroll
      for (int f = 0; f < kMaxFE; ++f) {
        gc[f] = 0;
        if (f < F) {
          gc[f] = keep ? a.code[f][row] : 0;
          keep = keep && a.cnt_pre[f][gc[f]] > 1;
        }
      }
      valid[s] = keep;
      wv[s] = (a.w && keep) ? a.w[row] : 1.0;
#pragma unroll
      for (int I = 0; I < NT; ++I) xt[s][I] = row < a.rows ? a.X[(int64_t)xl[I] * a.ld + row] : 0.0;
#pragma unroll
      for (int f = 0; f < kMaxFE; ++f) {
        if (f >= F) continue;
        const double* af = a.alpha[f] + (int64_t)gc[f] * p;
#pragma unroll
        for (int I = 0; I < NT; ++I) xt[s][I] -= af[xl[I]];
      }
    }
    double z[4][NT];
    if (MODE == 1) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const double sw = a.w ? sqrt(wv[s]) : 1.0;
#pragma unroll
        for (int I = 0; I < NT; ++I) z[s][I] = valid[s] ? (dat[I] ? xt[s][I] : fill[I]) * sw : 0.0;
      }
    } else {
      double sc[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        double t = coef[0] * xt[s][0];
#pragma unroll
        for (int I = 1; I < NT; ++I) t += coef[I] * xt[s][I];
        const double res = row16_sum(t) - beta0;
        if (c == 0 && valid[s]) {  // lane c = 0 holds y~ (column 0)
          const double rr = res * res;
          st[0] += a.w ? wv[s] * rr : rr;
          st[1] += rr;
          st[2] += xt[s][0];
          st[3] += xt[s][0] * xt[s][0];
        }
        sc[s] = a.w ? res * wv[s] : res;
        const double m = a.w ? res * sqrt(wv[s]) : res;
#pragma unroll
        for (int I = 0; I < NT; ++I) z[s][I] = (valid[s] && dat[I]) ? (one[I] ? 1.0 : xt[s][I]) * m : 0.0;
      }
      if (a.scores) {  // row-major [rows][ks]; a dropped row's score row is zero
#pragma unroll
        for (int I = 0; I < NT; ++I) {
          if (!dat[I]) continue;
          const int j = xl[I] - 1 + IC;
#pragma unroll
          for (int s = 0; s < 4; ++s)
            if (r + s < a.rows) a.scores[(r + s) * a.ks + j] = valid[s] ? (one[I] ? 1.0 : xt[s][I]) * sc[s] : 0.0;
        }
      }
    }
    mfma_rows<NT>(z, acc);
  }
  double* out = partial + (int64_t)blockIdx.x * pstride;
  block_reduce_store<NT, 256>(acc, red, out, tid);
  if (MODE == 0) {
#pragma unroll
    for (int e = 0; e < 4; ++e) st[e] = wave_reduce63(st[e], 0.0, [](double x, double y) { return x + y; });
    if (lane == 63)
      for (int e = 0; e < 4; ++e) stat_red[wave][e] = st[e];
    __syncthreads();
    if (tid < 4) out[Sh::LEN + tid] = ((stat_red[0][tid] + stat_red[1][tid]) + stat_red[2][tid]) + stat_red[3][tid];
  } else if (tid < 4) {
    out[Sh::LEN + tid] = 0.0;
  }
}

// tile[(16 I + i + off) * ts + 16 J + j + off] += block (I, J)[i][j] (both triangles), statistics after
// ts * ts: the chunk's reduced MFMA blocks added to the streamed tile in chunk order
__global__ void k_wide_tile_add(double* __restrict__ tile, const double* __restrict__ blk, int NT, int ts, int off) {
  const int np = NT * (NT + 1) / 2;
  for (int e = threadIdx.x; e < np * 256; e += blockDim.x) {
    const int q = e >> 8, i = (e >> 4) & 15, j = e & 15;
    int I = 0, rem = q;
    while (rem >= NT - I) {
      rem -= NT - I;
      ++I;
    }
    const int J = I + rem;
    const int gi = 16 * I + i + off, gj = 16 * J + j + off;
    if (gi >= ts || gj >= ts) continue;
    tile[(size_t)gi * ts + gj] += blk[e];
    if (I != J) tile[(size_t)gj * ts + gi] += blk[e];
  }
  if (threadIdx.x < 4) tile[(size_t)ts * ts + threadIdx.x] += blk[np * 256 + threadIdx.x];
}

// the wide (p > 11) form of stream_rows_chunk: k_stream_wide, its blocks reduced in block order and
// added to the streamed tile (stride c->sw.ts = 16 NT)
static int stream_wide_chunk(lfe_ctx* c, int mode, int icpt, const StreamRowArgs& a) {
  auto& w = c->sw;
  const int NT = w.ts / 16;
  const int np = NT * (NT + 1) / 2;
  const int64_t len = (int64_t)np * 256 + 4;
  const int64_t groups = (a.rows + 15) / 16;
  const int nblocks = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)c->n_cu * 4, (groups + 3) / 4));
  LFE_TRY(ensure_scratch(c, (size_t)nblocks * len));
  LFE_TRY(ensure_f64(c, w.red, w.red_cap, (size_t)len));
  {
    ProfScope _ps(c, mode == 0 ? K_GRAM_RESID : K_GRAM_DESIGN);
#define SW(NT_, M_, I_) \
  hipLaunchKernelGGL((k_stream_wide<NT_, M_, I_>), dim3(nblocks), dim3(256), 0, c->stream, a, c->scratch, len)
#define SWM(M_, I_)                      \
  switch (NT) {                          \
    case 1: SW(1, M_, I_); break;        \
    case 2: SW(2, M_, I_); break;        \
    case 3: SW(3, M_, I_); break;        \
    default: SW(4, M_, I_); break;       \
  }
    if (mode == 1) {
      SWM(1, 0)
    } else if (icpt) {
      SWM(0, 1)
    } else {
      SWM(0, 0)
    }
#undef SWM
#undef SW
    LFE_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL(k_reduce_partials, dim3(len), dim3(256), 0, c->stream, c->scratch, nblocks, len, w.red);
  LFE_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_wide_tile_add, dim3(1), dim3(256), 0, c->stream, w.tile, w.red, NT, w.ts,
                     mode == 0 && icpt ? 1 : 0);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

// One streamed chunk of the residual (mode 0; icpt 1: the IV residual over u = [1, x~, z~]) or
// design-Gram (mode 1) pass: the chunk's tile is added to c->sw.tile in chunk order; `scores`
// ([rows][ks], or null) receives the chunk's score rows for the cluster sums.
int stream_rows_chunk(lfe_ctx* c, int mode, int icpt, const double* X, int64_t ld, int64_t row0, int64_t rows,
                      double* scores) {
  const int p = c->p;
  StreamRowArgs a{};
  a.X = X;
  a.ld = ld;
  a.rows = rows;
  a.p = p;
  a.F = c->F;
  for (int f = 0; f < c->F; ++f) {
    a.code[f] = c->fe[f].code + row0;
    a.cnt_pre[f] = c->fe[f].cnt_pre;
    a.alpha[f] = c->fe[f].alpha;
  }
  a.w = c->w ? c->w + row0 : nullptr;
  a.beta = c->dbeta;
  a.scores = mode == 0 ? scores : nullptr;
  a.ks = p - 1 + icpt;
  if (p > 11) return stream_wide_chunk(c, mode, icpt, a);
  const int nblocks = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)c->n_cu * 4, (rows + 255) / 256));
  LFE_TRY(ensure_scratch(c, (size_t)nblocks * 260));
  {
    ProfScope _ps(c, mode == 0 ? K_GRAM_RESID : K_GRAM_DESIGN);
    const int PM = p <= 4 ? 4 : p <= 8 ? 8 : 12;
#define SR(PM_, M_, I_) \
  hipLaunchKernelGGL((k_stream_rows<PM_, M_, I_>), dim3(nblocks), dim3(256), 0, c->stream, a, c->scratch)
    if (mode == 0 && !icpt) {
      if (PM == 4) SR(4, 0, 0); else if (PM == 8) SR(8, 0, 0); else SR(12, 0, 0);
    } else if (mode == 0) {
      if (PM == 4) SR(4, 0, 1); else if (PM == 8) SR(8, 0, 1); else SR(12, 0, 1);
    } else {
      if (PM == 4) SR(4, 1, 0); else if (PM == 8) SR(8, 1, 0); else SR(12, 1, 0);
    }
#undef SR
    LFE_HIP(hipGetLastError());
  }
  LFE_TRY(ensure_dred(c, 544));
  hipLaunchKernelGGL(k_reduce_partials, dim3(260), dim3(256), 0, c->stream, c->scratch, nblocks, (int64_t)260,
                     c->dred + 272);
  LFE_HIP(hipGetLastError());
  stream_tile_add(c, c->dred + 272, 260);
  return LFE_OK;
}

// Gram, device solve and residual pass with one host round trip (row-kernel case:
// two FEs, unweighted, p <= 11).  Returns 1 (nothing done) when unavailable.
int gram_spec_enqueue(lfe_ctx* c, int* queued, const unsigned long long* gate, double tol) {
  *queued = 0;
  c->gram_spec = false;
  GramArgs a = base_args(c);
  if (!(resid_rows_ok(c, a) && c->p <= 11 && tables_gram_ok(c))) return LFE_OK;
  LFE_TRY(ensure_f64(c, c->dspec, c->dspec_elems, 544));
  LFE_TRY(tables_gram_enqueue(c, c->dspec, c->dspec + 532, c->dspec + 520, c->dspec + 520, c->dspec + 516, gate,
                              tol));
  *queued = 1;
  return LFE_OK;
}

int launch_gram_resid(lfe_ctx* c, double* host_gram, double* beta_full, double* stats, double* hc1, int keep_scores) {
  GramArgs a = base_args(c);
  const bool spec = c->gram_spec;  // the tables tile and beta are already on the stream (lfe_demean)
  c->gram_spec = false;
  if (!(resid_rows_ok(c, a) && c->p <= 11)) return 1;
  const int p = c->p, k = p - 1;
  // a one-way cluster on the primary FE: its sums in this pass (no score rows written)
  // (one cluster column: with more, the other subsets need the score rows, and the pass that both
  // writes them and sums was slower than the separate sums - HDFE_CLUSTER2 4.00-4.04 vs 3.98 ms)
  const int clj = keep_scores && c->cl.size() == 1 ? cluster_fused_col(c) : -1;
  const bool cl = clj >= 0 && (size_t)a.B * (12 + k) * 8 + 5120 <= 160 * 1024;
  const bool cl_scores = false;
  c->clfused = false;
  if (cl) LFE_TRY(cluster_fused_prepare(c));
  // dred: [0, 256) design tile | [256, 516) residual tile + stats | 516 ok | [520, 532) beta | 532 tables guard
  LFE_TRY(ensure_dred(c, 544));
  std::vector<double> h(533);
  for (int pass = tables_gram_ok(c) ? 0 : 1; pass < 2; ++pass) {
    // the speculative chain left tile, ok, beta and guard in dspec: the residual pass reads its
    // beta there and adds its tile beside them, so one read-back returns everything
    double* buf = pass == 0 && spec ? c->dspec : c->dred;
    if (buf == c->dred) {
      if (pass == 0) {
        LFE_TRY(tables_gram_enqueue(c, c->dred, c->dred + 532, c->dbeta, c->dred + 520, c->dred + 516));
      } else {
        LFE_TRY(design_rows_enqueue(c, a, c->dred));
        hipLaunchKernelGGL(k_chol_solve, dim3(1), dim3(64), 0, c->stream, c->dred, p, c->dbeta, c->dred + 520,
                           c->dred + 516);
      }
    }
    LFE_HIP(hipGetLastError());
    GramArgs ar = a;
    ar.nq = 1;
    ar.qf[0] = 1 - a.la.P;
    ar.G_Q = c->fe[ar.qf[0]].G;
    ar.beta = buf == c->dred ? c->dbeta : c->dspec + 520;
    ar.scores = keep_scores && (!cl || cl_scores) ? c->scores : nullptr;
    if (cl) {  // quanta from this pass's Gram tile and beta (on the device), the sums zeroed
      LFE_TRY(cluster_fused_reset(c, buf, ar.beta));
      const int G = c->fe[c->L.P].G;
      ar.clS = reinterpret_cast<unsigned long long*>(c->clf_S);
      ar.clHi = c->clf_hi;
      ar.clFq = c->clf_fq;
      ar.clCmax = c->clf_cnt + G + 1;
      ar.clFlag = c->clf_cnt + G + 2;
    }
    const unsigned long long seq = host_msg_on(c) ? next_msg_seq(c) : 0;
    LFE_TRY(resid_rows_enqueue(c, ar, buf + 256, cl, seq ? buf : nullptr, 533, seq));
    if (seq) LFE_TRY(host_msg_wait(c, seq, h.data(), 533));
    else LFE_TRY(d2h_sync(c, h.data(), buf, sizeof(double) * 533));
    if (pass == 1 || h[532] == 1.0) break;  // guard failed: the explicit design pass
  }
  if (h[516] != 1.0) return 1;  // not positive definite: the caller takes the two-call path
  const int D = p + 1;
  for (int i = 0; i < D; ++i)
    for (int j = 0; j < D; ++j) host_gram[i * D + j] = h[(size_t)i * 16 + j];
  for (int i = 0; i < p; ++i) beta_full[i] = h[520 + i];
  std::vector<double> meat((size_t)std::max(k, 1) * std::max(k, 1));
  unpack_resid(h.data() + 256, k, meat.data(), stats);
  if (hc1)
    for (int e = 0; e < k * k; ++e) hc1[e] = meat[e];
  c->scores_valid = keep_scores != 0;
  c->score_k = k;
  c->score_meat = meat;  // the row kernel's meat is sum s s' (unweighted two-FE case)
  c->score_meat_ok = keep_scores && c->world == 1;
  c->clfused = cl;
  c->clfused_done = false;
  c->clfused_j = clj;
  c->clfused_scores = cl_scores;
  if (cl) c->clfused_beta.assign(beta_full, beta_full + p);
  return LFE_OK;
}

int launch_resid(lfe_ctx* c, const double* beta_full, double* stats, double* hc1, int keep_scores, int icpt) {
  c->clfused = false;  // this pass writes the score rows
  GramArgs a = base_args(c);
  LFE_TRY(h2d_small(c, c->dbeta, beta_full, sizeof(double) * c->p));
  a.beta = c->dbeta;
  a.scores = keep_scores ? c->scores : nullptr;
  a.icpt = icpt ? 1 : 0;
  if (c->records) {
    LFE_TRY(records_layout(c));
    a.yoco = 1;
    a.rsy = c->rec_lay;
    a.rsyy = c->rec_lay + c->ld;
  }
  const int k = c->p - 1 + a.icpt;  // meat / score width
  c->score_k = k;
  std::vector<double> meat((size_t)std::max(k, 1) * std::max(k, 1));
  if (!icpt && !a.yoco && resid_rows_ok(c, a)) {
    a.nq = 1;
    a.qf[0] = 1 - a.la.P;
    a.G_Q = c->fe[a.qf[0]].G;
    LFE_TRY(resid_rows(c, a, meat.data(), stats));
    if (hc1)
      for (int e = 0; e < k * k; ++e) hc1[e] = meat[e];
    c->scores_valid = keep_scores != 0;
    c->score_meat = meat;
    c->score_meat_ok = keep_scores && c->world == 1;
    return LFE_OK;
  }
  // staged columns 0..p-1 (col 0 = y, zeroed in the meat, or the intercept with icpt);
  // meat = columns 1..p-1, or 0..p-1 with icpt
  const int rc = gram_dispatch<GRAM_RESID>(c, a, c->p, 1 - a.icpt, k, meat.data(), stats, 4);
  if (rc) return rc;
  if (hc1)
    for (int e = 0; e < k * k; ++e) hc1[e] = meat[e];
  c->scores_valid = keep_scores != 0;
  // the meat is sum s s' over the score rows s = u r only without weights (weighted: w r^2 u u'
  // against scores u r w) and outside records mode
  c->score_meat = meat;
  c->score_meat_ok = keep_scores && c->world == 1 && !a.w && !a.yoco;
  return LFE_OK;
}

// meat = table' table of a row-major [rows][k] score table (summed over ranks
// unless the caller sets world = 1 for a replicated table)
int launch_table_gram(lfe_ctx* c, const double* table, int64_t rows, int k, double* meat, const int32_t* idx) {
  GramArgs a{};
  a.table = table;
  a.tidx = idx;
  a.rows = rows;
  a.tcols = k;
  return gram_dispatch<GRAM_TABLE>(c, a, k, 0, k, meat, nullptr, 0);
}

int launch_copy_demeaned(lfe_ctx* c, double* dev_out) {
  LFE_TRY(ensure_layout_orig(c));
  if (c->n)
    hipLaunchKernelGGL(k_copy_demeaned, dim3(grid_for(c->n)), dim3(kBlock), 0, c->stream, layout_args(c), c->L.X,
                       c->ld, c->n, c->L.orig, dev_out);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

}  // namespace lfe

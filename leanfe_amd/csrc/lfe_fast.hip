// leanfe HIP engine — group sums of the demeaning loop (polars_impl.py:490-526).
//
// 1. k_sums4: the constant group sums S_f = sum_{i in g} w_i x_i in the
//    MFMA-native lane layout of lfe_gram.hip (lane = (row quad, column)): a
//    lane loads 4 consecutive rows of one column as a 32-byte vector and
//    adds them into LDS tables whose 16 lanes of a row hit 16 consecutive
//    doubles (primary FE: the 2^s-group slice of the item's bucket; small FEs:
//    whole tables).
// 2. k_sums2_raw: the same for two FEs without weights, plus the raw Gram of
//    the shifted columns on the matrix cores (the headline case).
//
// The alternating-projection sweeps of the two-FE case are in lfe_iter.hip.
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
  double* raw_part;     // RAW: [blocks][256] raw Gram tiles
  double* qpart;        // k_sums2_raw: [blocks][G_Q * p] the block's secondary-FE table (fine limbs)
  const double* fixq;   // quanta of the two-limb sums (k_fix_quanta)
  double* hi[kMaxFE];   // coarse limbs [G][p] per FE (global f64 atomics of integer values: rare)
};

// FQ: max non-primary FEs held in registers; GU: 16-row groups loaded before use;
// NT: 16-column slots per lane (p <= 16 NT); TH: threads per workgroup.
// RAW (NT = 1, p <= 15, unweighted): the same loads also feed one MFMA per 16-row
// group that accumulates the raw Gram of the kept rows' data columns, shifted by the
// first layout row (slot 15 = intercept), for the Gram-from-tables path (lfe_gram.hip).
template <int FQ, int GU, int NT, int TH, bool RAW>
__global__ __launch_bounds__(TH) void k_sums4(Sums4Args a) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int nwv = TH / 64;
  const int kq = lane >> 4, c = lane & 15;
  const int p = a.la.p, P = a.la.P, F = a.la.F;
  const int nq = a.nq < FQ ? a.nq : FQ;
  d4 racc[4];  // one per row of the quad: independent MFMA chains (issue never waits on the previous one)
#pragma unroll
  for (int s = 0; s < 4; ++s) racc[s] = d4{0.0, 0.0, 0.0, 0.0};
  const double shift = (RAW && c < p && a.la.n_items > 0) ? a.X[(int64_t)c * a.ld] : 0.0;
  // two-limb fixed point (lfe_internal.h): the fine limbs go to the tables as int64, the coarse
  // limbs of outliers to the global hi tables, so no table depends on the order of the adds
  FixCol fc[NT];
#pragma unroll
  for (int I = 0; I < NT; ++I) fc[I] = 16 * I + c < p ? fix_col(a.fixq, 16 * I + c) : FixCol{};
  typedef unsigned long long u64;
  // dst: the table entry (LDS or global), hdst: the entry's coarse limb (global)
  auto add = [&](double* dst, double* hdst, double v, int I) {
    double h;
    atomicAdd(reinterpret_cast<u64*>(dst), fix_split(v, fc[I], h));
    if (h != 0.0) atomicAdd(hdst, h);
  };
  for (int f = 0; f < F; ++f)
    if (f != P && a.tab_off[f] >= 0)
      for (int j = tid; j < a.G[f] * p; j += TH) lds[a.tab_off[f] + j] = 0.0;
  // primary slice [B][p] of the current bucket: flushed to S_P (and zeroed) on a
  // bucket change; a block owns a contiguous range of items
  auto flush = [&](int b) {
    const int lo = b << a.la.s;
    for (int j = tid; j < a.B * p; j += TH) {
      const int g = lo + j / p;
      const u64 val = reinterpret_cast<const u64*>(lds)[j];
      if (val != 0ull && g < a.G_P) atomicAdd(reinterpret_cast<u64*>(&a.S[P][(int64_t)g * p + (j % p)]), val);
      lds[j] = 0.0;
    }
  };
  if (a.slice)
    for (int j = tid; j < a.B * p; j += TH) lds[j] = 0.0;
  const BlockRows br = block_rows(a.la.items, a.la.n_items, lane);
  int cur = -1;
  for (int item = br.first; item < a.la.n_items; ++item) {
    int4 it = a.la.items[item];
    if (it.y >= br.hi) break;
    it.y = max(it.y, br.lo);
    it.z = min(it.z, br.hi);
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
        if (RAW) {
          // one MFMA per row of the quad, each followed by that row's LDS atomics, so the
          // matrix core works while the wave keeps issuing (NT = 1, unweighted, one FE besides P)
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const double z = !valid[s] ? 0.0 : (c == 15 ? 1.0 : (c < p ? xv[u][0][s] - shift : 0.0));
            racc[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(z, z, racc[s], 0, 0, 0);
            if (c < p && valid[s]) {
              const double v = xv[u][0][s];
              double* hP = &a.hi[P][(int64_t)hv[s] * p + c];
              if (a.slice) add(&lds[(hv[s] - lo) * p + c], hP, v, 0);
              else add(&a.S[P][(int64_t)hv[s] * p + c], hP, v, 0);
              const int f = a.qf[0];
              const int g = (&cq[u][0].x)[s];
              double* hQ = &a.hi[f][(int64_t)g * p + c];
              if (a.tab_off[f] >= 0) add(&lds[a.tab_off[f] + g * p + c], hQ, v, 0);
              else add(&a.S[f][(int64_t)g * p + c], hQ, v, 0);
            }
          }
          continue;
        }
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
              double* hP = &a.hi[P][(int64_t)hv[s] * p + col];
              if (a.slice) add(&lds[(hv[s] - lo) * p + col], hP, v[s], I);
              else add(&a.S[P][(int64_t)hv[s] * p + col], hP, v[s], I);
            }
#pragma unroll
            for (int q = 0; q < FQ; ++q) {
              if (q >= nq) continue;
              const int f = a.qf[q];
              const int g = (&cq[u][q].x)[s];
              double* hQ = &a.hi[f][(int64_t)g * p + col];
              if (a.tab_off[f] >= 0) add(&lds[a.tab_off[f] + g * p + col], hQ, v[s], I);
              else add(&a.S[f][(int64_t)g * p + col], hQ, v[s], I);
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
        const u64 val = reinterpret_cast<const u64*>(lds + a.tab_off[f])[j];
        if (val != 0ull) atomicAdd(reinterpret_cast<u64*>(&a.S[f][j]), val);
      }
  if (RAW) {
    // waves' raw tiles summed in LDS (lane (kq, c) holds rows kq + 4 rr of column c)
    __shared__ double rred[256];
    for (int wv = 0; wv < nwv; ++wv) {
      __syncthreads();
      if (wave == wv)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int e = (kq + 4 * rr) * 16 + c;
          const double v = (racc[0][rr] + racc[1][rr]) + (racc[2][rr] + racc[3][rr]);
          rred[e] = (wv == 0) ? v : rred[e] + v;
        }
    }
    __syncthreads();
    for (int e = tid; e < 256; e += TH) a.raw_part[(int64_t)blockIdx.x * 256 + e] = rred[e];
  }
}

// Group sums of one non-primary FE whose [G][p] table does not fit LDS but one column of it does
// (G <= kColSumsMax: config 4's third FE, 1e4 levels), one column per blockIdx.y: the block adds
// the fine limbs of its rows' column-c values into an LDS column [G] and writes it whole to
// part[c][block][G]; k_col_sums_fold adds the blocks per entry (integers: any order) into S_f.
// Per-row global int64 adds into the [G][p] table (k_sums4's path for tables that do not fit)
// ran at the chip's atomic rate, ~4.5 ms of config 4's 10 ms group sums for this FE; here every
// block rereads the codes once per column (12 B per row and column in all).
constexpr int kColSumsMax = 16384;
__global__ __launch_bounds__(1024) void k_col_sums(const int32_t* __restrict__ code, const int32_t* __restrict__ codeP,
                                                   const double* __restrict__ X, int64_t ld,
                                                   const double* __restrict__ w, int64_t n, int G, int p,
                                                   const double* __restrict__ fixq, double* __restrict__ hi,
                                                   unsigned long long* __restrict__ part) {
  extern __shared__ unsigned long long tab[];  // [G]
  const int c = blockIdx.y;
  for (int g = threadIdx.x; g < G; g += blockDim.x) tab[g] = 0ull;
  __syncthreads();
  const FixCol fc = fix_col(fixq, c);
  const double* __restrict__ xc = X + (int64_t)c * ld;
  const int64_t per = ((n + gridDim.x - 1) / gridDim.x + 3) & ~(int64_t)3;
  const int64_t r0 = (int64_t)blockIdx.x * per, r1 = min(n, r0 + per);
  for (int64_t i = r0 + threadIdx.x; i < r1; i += blockDim.x) {
    if (codeP && codeP[i] < 0) continue;  // dropped row (singleton filter)
    const int32_t g = code[i];
    double v = xc[i];
    if (w) v *= w[i];  // sum of (c * w), polars_impl.py:496
    double h;
    atomicAdd(&tab[g], fix_split(v, fc, h));
    if (h != 0.0) atomicAdd(&hi[(int64_t)g * p + c], h);
  }
  __syncthreads();
  unsigned long long* dst = part + ((int64_t)c * gridDim.x + blockIdx.x) * G;
  for (int g = threadIdx.x; g < G; g += blockDim.x) dst[g] = tab[g];
}

// S_f[g][c] fine limbs (u64 bits, as k_sums4's adds leave them) = sum over the blocks of column c
__global__ void k_col_sums_fold(const unsigned long long* __restrict__ part, int nblk, int G, int p,
                                double* __restrict__ S) {
  const int64_t m = (int64_t)G * p;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % p);
    const int64_t g = e / p;
    const unsigned long long* src = part + (int64_t)c * nblk * G + g;
    unsigned long long t = 0ull;
    for (int b = 0; b < nblk; ++b) t += src[(int64_t)b * G];
    S[e] = __longlong_as_double((long long)t);
  }
}

// The two-FE Gram-from-tables case of k_sums4 (RAW, unweighted, p <= 15, primary slice and
// secondary table both in LDS) with the per-row work cut to what the data needs: a row's
// only test is its primary code's sign (item edges are masked once per 16-row group), LDS
// byte offsets are one multiply-add per table, every pointer is hoisted out of the loop, and
// the next group pair's loads are issued before the current pair is consumed.
// BIG: some column's values may carry a coarse limb (an outlier beyond Qc / 2, or a non-finite
// value).  One launch: the kernel reads the quanta's flags (they live on the device) and runs the
// matching body, so typical data runs the fine-limb-only loop.
template <int TH, int NACC, int GU, bool BIG>
__device__ __forceinline__ void sums2_raw_body(const Sums4Args& a, double* __restrict__ lds, double* __restrict__ rred) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int nwv = TH / 64, step = nwv * GU;
  const int kq = lane >> 4, c = lane & 15;
  const int p = a.la.p, P = a.la.P, Q = a.qf[0], s = a.la.s;
  const uint32_t p8 = p * 8, c8 = c * 8;
  const bool col = c < p;
  // z = x - shift on the data lanes, 1 on lane 15 (intercept), 0 elsewhere: z = x * cm + zc
  // (lanes c >= p load column 0 so that every load is unconditional)
  const double cm = col ? 1.0 : 0.0;
  const double zc = (c == 15 ? 1.0 : 0.0) - ((col && a.la.n_items > 0) ? a.X[(int64_t)c * a.ld] : 0.0);
  const int32_t* __restrict__ hP = a.la.code[P];
  const int32_t* __restrict__ hQ = a.la.code[Q];
  const double* __restrict__ xc = a.X + (int64_t)(col ? c : 0) * a.ld;
  const int qoff = a.tab_off[Q];
  double* const qtab = lds + qoff;
  // two-limb fixed point: the fine limbs enter the LDS tables as int64 (the same whatever order
  // the waves' LDS adds and the blocks' global adds land in), the coarse limbs of outliers go to
  // the global hi tables as integer-valued f64 (exact in any order)
  const FixCol fc = col ? fix_col(a.fixq, c) : FixCol{};
  double* const hiP = a.hi[P];
  double* const hiQ = a.hi[Q];
  d4 racc[NACC];  // independent MFMA chains
#pragma unroll
  for (int r = 0; r < NACC; ++r) racc[r] = d4{0.0, 0.0, 0.0, 0.0};
  for (int j = tid; j < a.G[Q] * p; j += TH) lds[qoff + j] = 0.0;
  for (int j = tid; j < a.B * p; j += TH) lds[j] = 0.0;
  typedef unsigned long long u64;
  auto flush = [&](int b) {
    const int lo = b << s;
    for (int j = tid; j < a.B * p; j += TH) {
      const int g = lo + j / p;
      const u64 val = reinterpret_cast<const u64*>(lds)[j];
      if (val != 0ull && g < a.G_P) atomicAdd(reinterpret_cast<u64*>(&a.S[P][(int64_t)g * p + (j % p)]), val);
      lds[j] = 0.0;
    }
  };
  const BlockRows br = block_rows(a.la.items, a.la.n_items, lane);
  int cur = -1;
  for (int item = br.first; item < a.la.n_items; ++item) {
    int4 it = a.la.items[item];
    if (it.y >= br.hi) break;
    it.y = max(it.y, br.lo);
    it.z = min(it.z, br.hi);
    if (it.x != cur) {
      __syncthreads();
      if (cur >= 0) flush(cur);
      __syncthreads();
      cur = it.x;
    }
    const int lo = it.x << s;
    const int g0 = it.y >> 4, g1 = (it.z + 15) >> 4;
    int4 h0[GU], q0[GU];
    d4 x0[GU];
    // loads of groups gb, gb + 1, unconditional so that the pair in flight never forces a
    // wait for the next one (clamped into the item: a dead group is reloaded, not used)
    auto load = [&](int gb, int4 (&h)[GU], int4 (&q)[GU], d4 (&x)[GU]) {
#pragma unroll
      for (int u = 0; u < GU; ++u) {
        const int gi = min(gb + u, g1 - 1);
        const int rb = gi * 16 + kq * 4;
        h[u] = *reinterpret_cast<const int4*>(hP + rb);
        q[u] = *reinterpret_cast<const int4*>(hQ + rb);
        x[u] = ld4(xc + rb);
      }
    };
    auto consume = [&](int gb, const int4 (&h)[GU], const int4 (&q)[GU], const d4 (&x)[GU]) {
#pragma unroll
      for (int u = 0; u < GU; ++u) {
        const int gi = gb + u;
        if (gi >= g1) continue;  // wave-uniform
        int hv[4] = {h[u].x, h[u].y, h[u].z, h[u].w};
        const int gq[4] = {q[u].x, q[u].y, q[u].z, q[u].w};
        if (gi * 16 < it.y || gi * 16 + 16 > it.z) {  // an item edge cuts this group
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = gi * 16 + kq * 4 + r;
            if (row < it.y || row >= it.z) hv[r] = -1;
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool v = hv[r] >= 0;
          const double xv = x[u][r];
          const double z = v ? __builtin_fma(xv, cm, zc) : 0.0;
          racc[r % NACC] = __builtin_amdgcn_mfma_f64_16x16x4f64(z, z, racc[r % NACC], 0, 0, 0);
          if (v && col) {  // integer adds commute
            if (BIG) {
              double hh;
              const u64 xi = fix_split(xv, fc, hh);
              atomicAdd(reinterpret_cast<u64*>(lds_row_ptr(lds, hv[r] - lo, p8, c8)), xi);
              atomicAdd(reinterpret_cast<u64*>(lds_row_ptr(qtab, gq[r], p8, c8)), xi);
              if (hh != 0.0) {  // an outlier (or a non-finite value): its coarse limb
                atomicAdd(&hiP[(int64_t)hv[r] * p + c], hh);
                atomicAdd(&hiQ[(int64_t)gq[r] * p + c], hh);
              }
            } else {  // no coarse limbs: round(x sf) as the low bits of x sf + 1.5 * 2^52
              const u64 xi = (u64)__double_as_longlong(__builtin_fma(xv * fc.sf2, fc.sf, kFixMagic)) - kFixMagicBits;
              atomicAdd(reinterpret_cast<u64*>(lds_row_ptr(lds, hv[r] - lo, p8, c8)), xi);
              atomicAdd(reinterpret_cast<u64*>(lds_row_ptr(qtab, gq[r], p8, c8)), xi);
            }
          }
        }
      }
      // every register of the set is read here (a no-op), so no path leaves one of its loads
      // pending: the set's next loads then never wait for the other set's loads in flight
#pragma unroll
      for (int u = 0; u < GU; ++u)
        asm volatile("" ::"v"(h[u].x), "v"(h[u].y), "v"(h[u].z), "v"(h[u].w), "v"(q[u].x), "v"(q[u].y),
                     "v"(q[u].z), "v"(q[u].w), "v"(x[u][0]), "v"(x[u][1]), "v"(x[u][2]), "v"(x[u][3]));
    };
    // ping-pong register sets (no copies, which would wait for the loads in flight)
    int4 h1[GU], q1[GU];
    d4 x1[GU];
    int gb = g0 + wave * GU;
    load(gb, h0, q0, x0);
    while (gb < g1) {
      load(gb + step, h1, q1, x1);
      consume(gb, h0, q0, x0);
      gb += step;
      if (gb >= g1) break;
      load(gb + step, h0, q0, x0);
      consume(gb, h1, q1, x1);
      gb += step;
    }
  }
  __syncthreads();
  if (cur >= 0) flush(cur);
  // the block's secondary table goes out whole (k_qpart_reduce sums the blocks in order): every
  // block adding into the same G_Q * p entries serialised ~256 device-scope atomics per entry
  {
    const int64_t m = (int64_t)a.G[Q] * p;
    double* dst = a.qpart + (int64_t)blockIdx.x * m;
    for (int j = tid; j < m; j += TH) dst[j] = lds[qoff + j];
  }
  for (int wv = 0; wv < nwv; ++wv) {
    __syncthreads();
    if (wave == wv)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int e = (kq + 4 * rr) * 16 + c;
        double v = racc[0][rr];
#pragma unroll
        for (int r = 1; r < NACC; ++r) v += racc[r][rr];
        rred[e] = (wv == 0) ? v : rred[e] + v;
      }
  }
  __syncthreads();
  for (int e = tid; e < 256; e += TH) a.raw_part[(int64_t)blockIdx.x * 256 + e] = rred[e];
}

template <int TH, int NACC, int GU>
__global__ __launch_bounds__(TH) void k_sums2_raw(Sums4Args a) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ double rred[256];
  bool any = false;
  for (int j = 0; j < a.la.p; ++j) any = any || a.fixq[FQ_BIG * kFqCols + j] != 0.0;
  if (any) sums2_raw_body<TH, NACC, GU, true>(a, lds, rred);
  else sums2_raw_body<TH, NACC, GU, false>(a, lds, rred);
}

// ---------------------------------------------------------------------------
// two-limb fixed-point group sums (lfe_internal.h): quanta from the column statistics
// ---------------------------------------------------------------------------
// The statistics (max |x_c|, per-chunk sum of x_c^2) come from the partition, or k_col_stats when
// the rows stayed in place; both are deterministic (u64 atomicMax, chunk sums added in order).
// Non-finite values do not need a fallback: they travel in the coarse limb.

// column statistics when the partition did not run (one bucket): max |x_c| bits in st[c],
// the chunk's sum of x_c^2 in st[kColStatHead + c * nchunks + chunk] (as the partition writes them)
__global__ __launch_bounds__(256) void k_col_stats(const double* __restrict__ X, int64_t ld, int64_t n, int p,
                                                   int64_t chunk_rows, double* __restrict__ st) {
  __shared__ double ws[2][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * chunk_rows, r1 = min(n, r0 + chunk_rows);
  const auto fmaxop = [](double x, double y) { return fmax(x, y); };
  const auto addop = [](double x, double y) { return x + y; };
  for (int c = 0; c < p; ++c) {
    double m = 0.0, q = 0.0;
    for (int64_t i = r0 + tid; i < r1; i += 256) {
      const double v = X[(int64_t)c * ld + i];
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
      st[kColStatHead + (int64_t)c * gridDim.x + blockIdx.x] = ((ws[1][0] + ws[1][1]) + ws[1][2]) + ws[1][3];
      const double mm = fmax(fmax(ws[0][0], ws[0][1]), fmax(ws[0][2], ws[0][3]));
      atomicMax(reinterpret_cast<unsigned long long*>(st) + c, (unsigned long long)__double_as_longlong(mm));
    }
    __syncthreads();
  }
}

// weighted fits: the statistics of what their group sums add, in the same layout for p + 2
// "columns": c < p the products w x_c (S_f), c = p the weights (W_f), c = p + 1 the raw y (Sy_f,
// the unweighted stop test).  Rows past n read 0; dropped rows count too (a looser bound).
__global__ __launch_bounds__(256) void k_col_stats_w(const double* __restrict__ X, const double* __restrict__ w,
                                                     int64_t ld, int64_t n, int p, int64_t chunk_rows,
                                                     double* __restrict__ st) {
  __shared__ double ws[2][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * chunk_rows, r1 = min(n, r0 + chunk_rows);
  const auto fmaxop = [](double x, double y) { return fmax(x, y); };
  const auto addop = [](double x, double y) { return x + y; };
  for (int c = 0; c < p + 2; ++c) {
    double m = 0.0, q = 0.0;
    for (int64_t i = r0 + tid; i < r1; i += 256) {
      const double v = c < p ? X[(int64_t)c * ld + i] * w[i] : (c == p ? w[i] : X[i]);
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
      st[kColStatHead + (int64_t)c * gridDim.x + blockIdx.x] = ((ws[1][0] + ws[1][1]) + ws[1][2]) + ws[1][3];
      const double mm = fmax(fmax(ws[0][0], ws[0][1]), fmax(ws[0][2], ws[0][3]));
      atomicMax(reinterpret_cast<unsigned long long*>(st) + c, (unsigned long long)__double_as_longlong(mm));
    }
    __syncthreads();
  }
}

// quanta of column c = blockIdx.x (fix_quanta_col); the per-chunk squares are summed in a fixed order
__global__ __launch_bounds__(256) void k_fix_quanta(const double* __restrict__ st, int nchunks, int64_t n,
                                                    const int32_t* __restrict__ cmax, int nfe,
                                                    double* __restrict__ fq) {
  __shared__ double ws[4];
  const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const double* sq = st + kColStatHead + (int64_t)c * nchunks;
  double q = 0.0;
  for (int ch = tid; ch < nchunks; ch += 256) q += sq[ch];
  q = wave_reduce63(q, 0.0, [](double x, double y) { return x + y; });
  if (lane == 63) ws[wave] = q;
  __syncthreads();
  if (tid != 0) return;
  q = ((ws[0] + ws[1]) + ws[2]) + ws[3];
  int N = 1;
  for (int f = 0; f < nfe; ++f) N = max(N, cmax[f]);
  const double M = __longlong_as_double(reinterpret_cast<const long long*>(st)[c]);
  const double rms = n > 0 ? sqrt(q / (double)n) : 0.0;
  fix_quanta_col(M, rms, (double)N, fq, c);
}

// the entry's coarse limb (read and cleared: the hi tables stay zero between sums) when its
// column has any
__device__ __forceinline__ double take_hi(double* __restrict__ hi, int64_t e, const double* __restrict__ fq, int c) {
  if (fq[FQ_BIG * kFqCols + c] == 0.0) return 0.0;
  const double h = hi[e];
  if (h != 0.0) hi[e] = 0.0;
  return h;
}

// two-limb table entries (fine limb int64 bits in S, coarse limb in hi) -> double
__global__ void k_fix_convert(double* __restrict__ S, double* __restrict__ hi, int64_t m, int p,
                              const double* __restrict__ fq) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % p);
    S[e] = fix_value((unsigned long long)__double_as_longlong(S[e]), take_hi(hi, e, fq, c), fq, c);
  }
}

int launch_fix_quanta(lfe_ctx* c, const double* st, int nchunks, int64_t n, const int32_t* cmax, int nfe, double* fq,
                      int ncols) {
  if (ncols <= 0) return LFE_OK;
  hipLaunchKernelGGL(k_fix_quanta, dim3(ncols), dim3(256), 0, c->stream, st, nchunks, n, cmax, nfe, fq);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

int launch_fix_convert(lfe_ctx* c, double* S, double* hi, int64_t m, int p, const double* fq) {
  if (m <= 0) return LFE_OK;
  hipLaunchKernelGGL(k_fix_convert, dim3(grid_for(m)), dim3(kBlock), 0, c->stream, S, hi, m, p, fq);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

// S_Q = the blocks' fine-limb tables summed in block order (int64), plus the coarse limbs: 16
// consecutive entries x 16 block slices per workgroup
__device__ __forceinline__ void qpart_reduce_block(const double* __restrict__ part, int nblk, int64_t m,
                                                   const double* __restrict__ fq, int p, double* __restrict__ S,
                                                   double* __restrict__ hi, int blk,
                                                   double* __restrict__ alpha = nullptr,
                                                   const int32_t* __restrict__ cnt = nullptr) {
  __shared__ unsigned long long pi[16][16];
  const int ei = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int64_t e = (int64_t)blk * 16 + ei;
  unsigned long long ti = 0;
  if (e < m)
    for (int b = sl; b < nblk; b += 16) ti += (unsigned long long)__double_as_longlong(part[(int64_t)b * m + e]);
  pi[sl][ei] = ti;
  __syncthreads();
  if (sl != 0 || e >= m) return;
  unsigned long long r = 0;
  for (int k = 0; k < 16; ++k) r += pi[k][ei];
  const int c = (int)(e % p);
  const double v = fix_value(r, take_hi(hi, e, fq, c), fq, c);
  S[e] = v;
  if (alpha) {  // the first projection of the sweeps (k_fin_check with T = 0): alpha_Q = S_Q / n_Q
    const int32_t n = cnt[e / p];
    alpha[e] = n > 0 ? (v - 0.0) / (double)n : 0.0;
  }
}

__global__ __launch_bounds__(256) void k_qpart_reduce(const double* __restrict__ part, int nblk, int64_t m,
                                                      const double* __restrict__ fq, int p, double* __restrict__ S,
                                                      double* __restrict__ hi) {
  qpart_reduce_block(part, nblk, m, fq, p, S, hi, blockIdx.x);
}

// the two-FE sums' epilogue in one launch (four independent pieces, by block range): S_Q from the
// blocks' tables (k_qpart_reduce), S_P's int64 -> double (k_fix_convert), the raw Gram tiles
// summed in block order (k_reduce_partials) and the raw shift (k_raw_shift)
struct Sums2Epi {
  const double* qpart;
  int nblk;
  int64_t mq;
  const double* fq;
  int p;
  double* SQ;
  double* hiQ;
  int nbq;
  double* SP;
  double* hiP;
  int64_t mp;
  int nbp;
  const double* raw_part;
  double* raw_tile;
  const double* X;
  int64_t ld;
  int has_rows, rank;
  double* raw_shift;
  double* alphaQ;        // non-null (one rank): the sweeps' first projection alpha_Q = S_Q / n_Q here
  const int32_t* cntQ;
  double* zero2;         // non-null: two doubles zeroed (the i8 digits' guard flag)
};
__global__ __launch_bounds__(256) void k_sums2_epilogue(Sums2Epi a) {
  int b = blockIdx.x;
  if (b < a.nbq) {
    qpart_reduce_block(a.qpart, a.nblk, a.mq, a.fq, a.p, a.SQ, a.hiQ, b, a.alphaQ, a.cntQ);
    return;
  }
  b -= a.nbq;
  if (b < a.nbp) {
    for (int64_t e = (int64_t)b * 256 + threadIdx.x; e < a.mp; e += (int64_t)a.nbp * 256) {
      const int c = (int)(e % a.p);
      a.SP[e] = fix_value((unsigned long long)__double_as_longlong(a.SP[e]), take_hi(a.hiP, e, a.fq, c), a.fq, c);
    }
    return;
  }
  b -= a.nbp;
  if (b < 256) {  // entry b of the raw tile: fixed-order tree over the blocks
    __shared__ double red[256];
    double t = 0.0;
    for (int k = threadIdx.x; k < a.nblk; k += 256) t += a.raw_part[(int64_t)k * 256 + b];
    red[threadIdx.x] = t;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
      if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
      __syncthreads();
    }
    if (threadIdx.x == 0) a.raw_tile[b] = red[0];
    return;
  }
  const int j = threadIdx.x;  // the raw shift (k_raw_shift)
  if (a.zero2 && j < 2) a.zero2[j] = 0.0;
  if (j >= 16) return;
  const double own = (j < a.p && a.has_rows) ? a.X[(int64_t)j * a.ld] : 0.0;
  a.raw_shift[16 + j] = own;
  a.raw_shift[j] = a.rank == 0 ? own : 0.0;
}

// raw_shift[16 + j] = this rank's shift (first layout row; 0 for an empty shard);
// raw_shift[j] = rank 0's (summed over ranks afterwards)
__global__ void k_raw_shift(const double* __restrict__ X, int64_t ld, int p, int has_rows, int rank,
                            double* __restrict__ sh) {
  const int j = threadIdx.x;
  if (j >= 16) return;
  const double own = (j < p && has_rows) ? X[(int64_t)j * ld] : 0.0;
  sh[16 + j] = own;
  sh[j] = rank == 0 ? own : 0.0;
}

// multi-rank raw Gram: rank r's tile (relative to its own shift) and shift into slot r of a
// zeroed [world][272] buffer; after one sum over ranks every rank holds all slots
__global__ void k_raw_slot(const double* __restrict__ R, const double* __restrict__ sh, int rank,
                           double* __restrict__ slots) {
  double* s = slots + (int64_t)rank * 272;
  for (int t = threadIdx.x; t < 272; t += blockDim.x) s[t] = t < 256 ? R[t] : sh[16 + (t - 256)];
}

// the global raw tile from the slots, each re-centred from its own shift c_r to rank 0's c*,
// sum (d - c*)(d - c*)' = R + dl C' + C dl' + n dl dl', sum (d - c*) = C + n dl, dl = c_r - c*,
// and added in rank order (every rank the same bits); raw_shift: c* in both halves
__global__ void k_raw_combine(const double* __restrict__ slots, int world, int p, double* __restrict__ R,
                              double* __restrict__ sh) {
  __shared__ double C[16], dl[16];
  const int t = threadIdx.x;  // 256 threads: one tile entry each
  const int i = t / 16, j = t % 16;
  double acc = 0.0;
  for (int r = 0; r < world; ++r) {
    const double* s = slots + (int64_t)r * 272;
    __syncthreads();
    if (t < 16) {
      C[t] = s[15 * 16 + t];
      dl[t] = t < p ? s[256 + t] - slots[256 + t] : 0.0;
    }
    __syncthreads();
    const double n = s[15 * 16 + 15];
    double v = s[t];
    if (i < p && j < p) v += dl[i] * C[j] + C[i] * dl[j] + n * dl[i] * dl[j];
    else if (i == 15 && j < p) v += n * dl[j];
    else if (j == 15 && i < p) v += n * dl[i];
    acc = r == 0 ? v : acc + v;
  }
  R[t] = acc;
  if (t < 16) sh[t] = sh[16 + t] = slots[256 + t];
}

// Group sums of FEs whose primary slice and other tables do not fit LDS whole (the reference's 3-FE
// panels: 2e4 x 4e3 x 1e3 levels at p = 15, 1e4 x 2e3 x 500 at p = 21; two FEs at p > 15), by
// column groups:
// workgroup (column group cg of nc columns, row part) keeps the primary slice [B][nc] and every other
// FE's table [G_f][nc] in LDS (nc from the LDS budget), reads its nc columns and the codes of its
// rows once, and adds the fine limbs there; the slice goes to S_P at each bucket change, the tables
// at the end (integer adds: any order).  Replaces k_sums4's per-row global adds for tables that do
// not fit (~1 / 30 of the LDS rate) and k_col_sums' reread of the codes for every column.  The
// workgroups of one row part share an XCD (block i -> XCD i % 8), so its codes come from one L2.
constexpr int kCgThreads = 1024;
constexpr int kCgMaxNc = 8;
constexpr int kCgMaxF = 4;
constexpr int kCgRows = 2;  // rows per thread per round, every load issued first

struct SumsCgArgs {
  const int4* items;
  int n_items, s, P, nq;
  const int32_t* codeP;
  const int32_t* codeq[kCgMaxF - 1];
  int qf[kCgMaxF - 1];
  const double* X;
  int64_t ld;
  const double* w;
  int p, nc, ncg, nparts, B, G_P;
  int Gq[kCgMaxF - 1];
  int q_off[kCgMaxF - 1];  // u64 LDS offset of [G_q][nc] (the slice [B][nc] at 0)
  int lds_words;
  double* SP;
  double* Sq[kCgMaxF - 1];
  double* hiP;
  double* hiq[kCgMaxF - 1];
  const double* fixq;
};

__global__ __launch_bounds__(kCgThreads) void k_sums_cg(SumsCgArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long tl[];
  typedef unsigned long long u64;
  const int bid = blockIdx.x, cg = (bid >> 3) % a.ncg, part = (bid / (8 * a.ncg)) * 8 + (bid & 7);
  if (part >= a.nparts) return;  // uniform
  const int tid = threadIdx.x, lane = tid & 63, p = a.p;
  const int c0 = cg * a.nc, nc = min(a.nc, p - c0);
  for (int j = tid; j < a.lds_words; j += kCgThreads) tl[j] = 0ull;
  FixCol fc[kCgMaxNc];
#pragma unroll
  for (int cc = 0; cc < kCgMaxNc; ++cc) fc[cc] = cc < nc ? fix_col(a.fixq, c0 + cc) : FixCol{};
  auto add = [&](u64* dst, double* hdst, double v, const FixCol& q) {
    double h;
    atomicAdd(dst, fix_split(v, q, h));
    if (h != 0.0) atomicAdd(hdst, h);
  };
  auto flush = [&](int b) {
    const int lo = b << a.s;
    for (int j = tid; j < a.B * nc; j += kCgThreads) {
      const int g = lo + j / nc, cc = j - (j / nc) * nc;
      const u64 v = tl[j];
      if (v != 0ull && g < a.G_P) atomicAdd(reinterpret_cast<u64*>(&a.SP[(int64_t)g * p + c0 + cc]), v);
      tl[j] = 0ull;
    }
  };
  __syncthreads();
  const BlockRows br = block_rows(a.items, a.n_items, lane, part, a.nparts);
  int cur = -1;
  for (int item = br.first; item < a.n_items; ++item) {
    int4 it = a.items[item];
    if (it.y >= br.hi) break;
    it.y = max(it.y, br.lo);
    it.z = min(it.z, br.hi);
    if (it.x != cur) {
      __syncthreads();
      if (cur >= 0) flush(cur);
      __syncthreads();
      cur = it.x;
    }
    const int lo = it.x << a.s;
    for (int i0 = it.y + tid; i0 < it.z; i0 += kCgRows * kCgThreads) {
      int hp[kCgRows], hq[kCgRows][kCgMaxF - 1];
      double x[kCgRows][kCgMaxNc], wv[kCgRows];
#pragma unroll
      for (int r = 0; r < kCgRows; ++r) {
        const int i = i0 + r * kCgThreads;
        const bool live = i < it.z;
        hp[r] = live ? a.codeP[i] : -1;
#pragma unroll
        for (int q = 0; q < kCgMaxF - 1; ++q) hq[r][q] = (q < a.nq && live) ? a.codeq[q][i] : 0;
#pragma unroll
        for (int cc = 0; cc < kCgMaxNc; ++cc) x[r][cc] = (cc < nc && live) ? a.X[(int64_t)(c0 + cc) * a.ld + i] : 0.0;
        wv[r] = (a.w && live) ? a.w[i] : 1.0;
      }
#pragma unroll
      for (int r = 0; r < kCgRows; ++r) {
        if (hp[r] < 0) continue;  // dropped row (singleton filter) or past the item
#pragma unroll
        for (int cc = 0; cc < kCgMaxNc; ++cc) {
          if (cc >= nc) break;
          const double v = a.w ? x[r][cc] * wv[r] : x[r][cc];  // sum of (c * w), polars_impl.py:496
          add(&tl[(hp[r] - lo) * nc + cc], &a.hiP[(int64_t)hp[r] * p + c0 + cc], v, fc[cc]);
#pragma unroll
          for (int q = 0; q < kCgMaxF - 1; ++q)
            if (q < a.nq)
              add(&tl[a.q_off[q] + hq[r][q] * nc + cc], &a.hiq[q][(int64_t)hq[r][q] * p + c0 + cc], v, fc[cc]);
        }
      }
    }
  }
  __syncthreads();
  if (cur >= 0) flush(cur);
  for (int q = 0; q < a.nq; ++q)
    for (int j = tid; j < a.Gq[q] * nc; j += kCgThreads) {
      const u64 v = tl[a.q_off[q] + j];
      const int g = j / nc, cc = j - g * nc;
      if (v != 0ull) atomicAdd(reinterpret_cast<u64*>(&a.Sq[q][(int64_t)g * p + c0 + cc]), v);
    }
}

// column groups for k_sums_cg: columns per group from the LDS budget (0: the tables do not fit)
static int sums_cg_nc(const lfe_ctx* c) {
  const int P = c->L.P;
  if (c->F < 2 || c->F > kCgMaxF || P < 0) return 0;
  const char* e = knob("LFE_SUMS_CG");  // "0": off (A/B)
  if (e && e[0] == '0') return 0;
  int64_t per_col = (int64_t)1 << c->L.s;
  for (int f = 0; f < c->F; ++f)
    if (f != P) per_col += c->fe[f].G;
  const int64_t nc = std::min<int64_t>({(int64_t)kCgMaxNc, (int64_t)c->p, (150 * 1024 / 8) / per_col});
  return (int)std::max<int64_t>(nc, 0);
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
    a.hi[f] = c->fe[f].hi;
    a.tab_off[f] = -1;
    if (f != P && off + (size_t)c->fe[f].G * p <= budget) {
      a.tab_off[f] = (int)off;
      off += (size_t)c->fe[f].G * p;
    }
    if (!c->sums_zeroed) LFE_HIP(hipMemsetAsync(c->fe[f].S, 0, sizeof(double) * (size_t)c->fe[f].G * p, c->stream));
  }
  // non-primary FEs whose table does not fit LDS but one column of it does: column-split LDS sums
  // (k_col_sums) instead of k_sums4's per-row global adds
  bool colsplit[kMaxFE] = {};
  a.nq = 0;
  for (int f = 0; f < c->F; ++f) {
    if (f == P) continue;
    // (three or more FEs: a two-FE fit keeps its secondary FE in k_sums4 for the raw Gram)
    colsplit[f] = c->F >= 3 && a.tab_off[f] < 0 && c->fe[f].G <= kColSumsMax && c->n > 0;
    if (!colsplit[f]) a.qf[a.nq++] = f;
  }
  c->sums_zeroed = false;
  // three or more FEs with a table that does not fit LDS whole: the column-group sums
  int cg_nc = 0;
  {
    bool all_fit = a.slice != 0;
    for (int f = 0; f < c->F; ++f)
      if (f != P && a.tab_off[f] < 0) all_fit = false;
    if (!all_fit) cg_nc = sums_cg_nc(c);
    if (cg_nc > 0)
      for (int f = 0; f < c->F; ++f) colsplit[f] = false;
  }
  const size_t lds = off * 8;
  const int NT = (p + 15) / 16;
  const void* fn = nullptr;
#define SUMS4_FN(FQ, GU, NT_, TH_) reinterpret_cast<const void*>(&k_sums4<FQ, GU, NT_, TH_, false>)
  // the raw Gram of the shifted columns rides along when the Gram can come from the tables (not
  // in the column-group sums, which form no raw tile: the Gram then takes its own raw pass)
  const bool raw = cg_nc == 0 && c->F == 2 && P >= 0 && a.nq == 1 && p <= 15 && !a.w;
  c->raw_ready = false;
  int threads = kSumThreads;
  bool two = false;
  if (a.nq <= 1 && NT == 1) {
    // the 2-FE case: one workgroup per CU (LDS), so 16 waves of <= 128 VGPRs.  k_sums2_raw: four
    // MFMA chains, one 16-row group per load (0.925 vs 0.950 ms for 2 groups per load; 2 chains
    // measured the same)
    threads = 1024;
    two = raw && a.slice && a.tab_off[a.qf[0]] >= 0;
    fn = two   ? reinterpret_cast<const void*>(&k_sums2_raw<1024, 4, 1>)
         : raw ? reinterpret_cast<const void*>(&k_sums4<1, 2, 1, 1024, true>)
               : SUMS4_FN(1, 2, 1, 1024);
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
  LFE_HIP(set_max_lds(fn, (int)std::max<size_t>(lds, 1)));
  const int nblocks = row_blocks(c, resident_blocks(c, fn, threads, lds));
  if (raw) {
    LFE_TRY(ensure_f64(c, c->raw_part, c->raw_part_cap, (size_t)nblocks * 256));
    LFE_TRY(ensure_f64(c, c->raw_tile, c->raw_tile_cap, 256));
    a.raw_part = c->raw_part;
  }
  // two-limb fixed-point group sums for every fit: unweighted quanta from the statistics of x,
  // weighted ones from those of w x, w and the raw y (k_col_stats_w, columns p and p + 1)
  const bool wexact = a.w != nullptr;
  if (two) {
    LFE_TRY(ensure_f64(c, c->qpart, c->qpart_cap, (size_t)nblocks * c->fe[a.qf[0]].G * p));
    a.qpart = c->qpart;
  }
  LFE_TRY(ensure_f64(c, c->fixq, c->fixq_cap, (size_t)kFqRows * kFqCols));
  {
    ProfScope _ps(c, K_FIX_SUMS);
    // the column statistics (the partition wrote them unless the rows stayed in place)
    constexpr int64_t kStatRows = 16384;
    if (wexact) {
      const int nch = (int)std::max<int64_t>(1, (c->n + kStatRows - 1) / kStatRows);
      LFE_TRY(ensure_f64(c, c->colstat, c->colstat_cap, (size_t)kColStatHead + (size_t)nch * (p + 2)));
      LFE_HIP(hipMemsetAsync(c->colstat, 0, sizeof(double) * kColStatHead, c->stream));
      hipLaunchKernelGGL(k_col_stats_w, dim3(nch), dim3(256), 0, c->stream, c->L.X, c->L.w, c->ld, c->n, p,
                         kStatRows, c->colstat);
      LFE_HIP(hipGetLastError());
      hipLaunchKernelGGL(k_fix_quanta, dim3(p + 2), dim3(256), 0, c->stream, c->colstat, nch, c->n,
                         c->iscratch + kIscratchCmax, c->F, c->fixq);
      LFE_HIP(hipGetLastError());
      c->colstat_chunks = 0;  // these are the weighted statistics: an unweighted pass recomputes its own
    } else if (c->colstat_chunks == 0) {
      const int nch = (int)std::max<int64_t>(1, (c->n + kStatRows - 1) / kStatRows);
      LFE_TRY(ensure_f64(c, c->colstat, c->colstat_cap, (size_t)kColStatHead + (size_t)nch * p));
      LFE_HIP(hipMemsetAsync(c->colstat, 0, sizeof(double) * kColStatHead, c->stream));
      hipLaunchKernelGGL(k_col_stats, dim3(nch), dim3(256), 0, c->stream, c->L.X, c->ld, c->n, p, kStatRows,
                         c->colstat);
      LFE_HIP(hipGetLastError());
      c->colstat_chunks = nch;
    }
    if (!wexact && !c->fixq_ready) {  // (else k_finish_counts formed them from the same statistics)
      hipLaunchKernelGGL(k_fix_quanta, dim3(p), dim3(256), 0, c->stream, c->colstat, c->colstat_chunks, c->n,
                         c->iscratch + kIscratchCmax, c->F, c->fixq);
      LFE_HIP(hipGetLastError());
    }
    c->fixq_ready = false;
    a.fixq = c->fixq;
  }
  c->exact_sums = true;
  LFE_TRY(hi_begin(c));
  if (cg_nc > 0) {
    SumsCgArgs g{};
    g.items = reinterpret_cast<const int4*>(c->items_d);
    g.n_items = c->L.n_items;
    g.s = c->L.s;
    g.P = P;
    g.codeP = c->L.code[P];
    g.X = c->L.X;
    g.ld = c->ld;
    g.w = c->L.w;
    g.p = p;
    g.nc = cg_nc;
    g.ncg = (p + cg_nc - 1) / cg_nc;
    g.B = 1 << c->L.s;
    g.G_P = c->fe[P].G;
    g.SP = c->fe[P].S;
    g.hiP = c->fe[P].hi;
    g.fixq = c->fixq;
    int off_w = g.B * cg_nc;
    for (int f = 0; f < c->F; ++f) {
      if (f == P) continue;
      const int q = g.nq++;
      g.qf[q] = f;
      g.codeq[q] = c->L.code[f];
      g.Gq[q] = c->fe[f].G;
      g.q_off[q] = off_w;
      off_w += c->fe[f].G * cg_nc;
      g.Sq[q] = c->fe[f].S;
      g.hiq[q] = c->fe[f].hi;
    }
    g.lds_words = off_w;
    // one workgroup per CU in all (LDS), the row parts spread over the column groups
    g.nparts = std::max(1, std::min(c->L.n_items * 4, (c->n_cu + g.ncg - 1) / g.ncg));
    const size_t lds_cg = sizeof(unsigned long long) * off_w;
    LFE_HIP(set_max_lds(reinterpret_cast<const void*>(&k_sums_cg), (int)lds_cg));
    ProfScope _ps(c, K_GROUP_SUMS);
    hipLaunchKernelGGL(k_sums_cg, dim3((g.nparts + 7) / 8 * 8 * g.ncg), dim3(kCgThreads), lds_cg, c->stream, g);
  } else {
    ProfScope _ps(c, K_GROUP_SUMS);
    void* args[] = {&a};
    LFE_HIP(hipLaunchKernel(fn, dim3(nblocks), dim3(threads), args, lds, c->stream));
  }
  LFE_HIP(hipGetLastError());
  for (int f = 0; f < c->F; ++f) {
    if (!colsplit[f]) continue;
    ProfScope _ps(c, K_GROUP_SUMS);
    const int G = c->fe[f].G;
    const int nb = std::max(1, (2 * c->n_cu + p - 1) / p);  // ~2 blocks per CU over the p columns
    LFE_TRY(ensure_f64(c, c->colsum_part, c->colsum_part_cap, (size_t)p * nb * G));
    const size_t lds = sizeof(unsigned long long) * G;
    LFE_HIP(set_max_lds(reinterpret_cast<const void*>(&k_col_sums), (int)std::max<size_t>(lds, 1)));
    auto* part = reinterpret_cast<unsigned long long*>(c->colsum_part);
    hipLaunchKernelGGL(k_col_sums, dim3(nb, p), dim3(1024), lds, c->stream, c->L.code[f],
                       P >= 0 ? c->L.code[P] : nullptr, c->L.X, c->ld, c->L.w, c->n, G, p, c->fixq, c->fe[f].hi, part);
    hipLaunchKernelGGL(k_col_sums_fold, dim3(grid_for((int64_t)G * p)), dim3(kBlock), 0, c->stream, part, nb, G, p,
                       c->fe[f].S);
    LFE_HIP(hipGetLastError());
  }
  if (two) {  // two implies raw: one epilogue launch
    ProfScope _ps(c, K_FIX_SUMS);
    LFE_TRY(ensure_f64(c, c->raw_shift, c->raw_shift_cap, 32));
    Sums2Epi e{};
    e.qpart = c->qpart;
    e.nblk = nblocks;
    e.mq = (int64_t)c->fe[a.qf[0]].G * p;
    e.fq = c->fixq;
    e.p = p;
    e.SQ = c->fe[a.qf[0]].S;
    e.hiQ = c->fe[a.qf[0]].hi;
    e.nbq = (int)((e.mq + 15) / 16);
    e.SP = c->fe[P].S;
    e.hiP = c->fe[P].hi;
    e.mp = (int64_t)c->fe[P].G * p;
    e.nbp = grid_for(e.mp);
    e.raw_part = c->raw_part;
    e.raw_tile = c->raw_tile;
    e.X = c->L.X;
    e.ld = c->ld;
    e.has_rows = c->L.n_items > 0 ? 1 : 0;
    e.rank = c->rank;
    e.raw_shift = c->raw_shift;
    if (c->world == 1) {  // (several ranks all-reduce S_Q after this launch)
      LFE_TRY(ensure_f64(c, c->rflag, c->rflag_cap, 2));
      e.alphaQ = c->fe[a.qf[0]].alpha;
      e.cntQ = c->fe[a.qf[0]].cnt;
      e.zero2 = c->rflag;
      c->q_first = e.alphaQ;
    }
    hipLaunchKernelGGL(k_sums2_epilogue, dim3((unsigned)(e.nbq + e.nbp + 256 + 1)), dim3(256), 0, c->stream, e);
    LFE_HIP(hipGetLastError());
    c->raw_ready = true;
  }
  if (!two) {
    ProfScope _ps(c, K_FIX_SUMS);
    for (int f = 0; f < c->F; ++f) {
      const int64_t m = (int64_t)c->fe[f].G * p;
      hipLaunchKernelGGL(k_fix_convert, dim3(grid_for(m)), dim3(kBlock), 0, c->stream, c->fe[f].S, c->fe[f].hi, m,
                         p, c->fixq);
    }
    LFE_HIP(hipGetLastError());
  }
  hi_end(c);
  if (raw && !two) {
    reduce_tiles(c, c->raw_part, nblocks, c->raw_tile);
    LFE_TRY(ensure_f64(c, c->raw_shift, c->raw_shift_cap, 32));
    hipLaunchKernelGGL(k_raw_shift, dim3(1), dim3(64), 0, c->stream, c->L.X, c->ld, p, c->L.n_items > 0 ? 1 : 0,
                       c->rank, c->raw_shift);
    LFE_HIP(hipGetLastError());
    c->raw_ready = true;
  }
  // one grouped sum over ranks: the group tables (owner-sharded rows: the primary FE's are
  // complete on each rank) and every rank's raw tile + shift in its own slot
  std::vector<std::pair<double*, size_t>> bufs;
  for (int f = 0; f < c->F; ++f)
    if (!(c->owner_on && f == P)) bufs.push_back({c->fe[f].S, (size_t)c->fe[f].G * p});
  if (raw && c->world > 1) {
    LFE_TRY(ensure_f64(c, c->raw_slots, c->raw_slots_cap, (size_t)c->world * 272));
    LFE_HIP(hipMemsetAsync(c->raw_slots, 0, sizeof(double) * c->world * 272, c->stream));
    hipLaunchKernelGGL(k_raw_slot, dim3(1), dim3(256), 0, c->stream, c->raw_tile, c->raw_shift, c->rank,
                       c->raw_slots);
    LFE_HIP(hipGetLastError());
    bufs.push_back({c->raw_slots, (size_t)c->world * 272});
  }
  LFE_TRY(allreduce_sum_f64_many(c, bufs));
  if (raw && c->world > 1) {
    hipLaunchKernelGGL(k_raw_combine, dim3(1), dim3(256), 0, c->stream, c->raw_slots, c->world, p, c->raw_tile,
                       c->raw_shift);
    LFE_HIP(hipGetLastError());
  }
  return LFE_OK;
}

// ---------------------------------------------------------------------------
// out-of-core X: group sums and raw Gram of one streamed row chunk
// ---------------------------------------------------------------------------
// The chunk's rows in input order (no partition): lane (kq, c) holds "columns" c + 16 J (J < NJ)
// of rows 16 g + 4 kq + r as in k_sums2_raw.  Column c < p adds x_c (weighted: w x_c, polars_impl.py:496);
// weighted fits add two more: c = p the weight (W_f), c = p + 1 the raw y (Sy_f, the unweighted
// stop test).  Every FE's sums go to the chunk tables [G_f][pw] in two-limb fixed point (fine
// limbs in s64, coarse limbs in sdbl), the shifted raw Gram of the unweighted two-FE case (p <= 15,
// one column group) to one MFMA chain per row.  A row is kept iff every FE's pre-filter count of its code exceeds 1 (the
// single-pass drop, polars_impl.py:477-482).
struct StreamSumsArgs {
  const double* X;  // [p][ld] chunk columns
  int64_t ld, rows;
  int p, F, pw;                    // pw: table columns (p, or p + 2 weighted)
  const int32_t* code[kMaxFE];     // the chunk's codes (input order)
  const int32_t* cnt_pre[kMaxFE];  // pre-filter counts (all rows)
  int64_t toff[kMaxFE];            // table offset (entries) of FE f in s64 / sdbl
  const double* w;                 // the chunk's weights (null: unweighted)
  unsigned long long* s64;
  double* sdbl;
  const double* fixq;   // the chunk's quanta (k_fix_quanta, pw columns)
  const double* shift;  // [16] raw-Gram shift
  double* raw_part;     // [blocks][256]
};

template <int NJ>
__global__ __launch_bounds__(256) void k_stream_sums(StreamSumsArgs a) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kq = lane >> 4, c = lane & 15;
  const int p = a.p, pw = a.pw, F = a.F;
  bool col[NJ];
  FixCol fc[NJ];
  const double* __restrict__ xc[NJ];
#pragma unroll
  for (int J = 0; J < NJ; ++J) {
    const int cj = c + 16 * J;
    col[J] = cj < pw;
    fc[J] = col[J] ? fix_col(a.fixq, cj) : FixCol{};
    xc[J] = a.X + (int64_t)(cj < p ? cj : 0) * a.ld;  // lane p + 1 (Sy): column 0 = y
  }
  // the raw Gram (unweighted, one column group): z = x - shift on the data lanes, 1 on lane 15
  const bool dcol = c < p;
  const double cm = dcol ? 1.0 : 0.0;
  const double zc = NJ == 1 ? (c == 15 ? 1.0 : 0.0) - (dcol ? a.shift[c] : 0.0) : 0.0;
  d4 racc = d4{0.0, 0.0, 0.0, 0.0};
  const int64_t ngroups = (a.rows + 15) >> 4;
  for (int64_t g = (int64_t)blockIdx.x * 4 + wave; g < ngroups; g += (int64_t)gridDim.x * 4) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t row = g * 16 + kq * 4 + r;
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
      const double wi = (a.w && keep) ? a.w[row] : 1.0;
#pragma unroll
      for (int J = 0; J < NJ; ++J) {
        const int cj = c + 16 * J;
        const double xv = row < a.rows ? xc[J][row] : 0.0;
        if (NJ == 1) {
          const double z = keep ? __builtin_fma(xv, cm, zc) : 0.0;
          racc = __builtin_amdgcn_mfma_f64_16x16x4f64(z, z, racc, 0, 0, 0);
        }
        if (keep && col[J]) {  // two-limb fixed point: fine limbs in s64, coarse limbs in sdbl
          double v = xv;
          if (a.w) v = cj < p ? xv * wi : (cj == p ? wi : xv);
          double hh;
          const unsigned long long xi = fix_split(v, fc[J], hh);
#pragma unroll
          for (int f = 0; f < kMaxFE; ++f)
            if (f < F) atomicAdd(&a.s64[a.toff[f] + (int64_t)gc[f] * pw + cj], xi);
          if (hh != 0.0)
#pragma unroll
            for (int f = 0; f < kMaxFE; ++f)
              if (f < F) atomicAdd(&a.sdbl[a.toff[f] + (int64_t)gc[f] * pw + cj], hh);
        }
      }
    }
  }
  if (NJ > 1) return;  // no raw Gram: the caller streams the design Gram (pass 3)
  // waves' tiles summed in LDS in wave order (lane (kq, c) holds rows kq + 4 rr of column c)
  __shared__ double rred[256];
  for (int wv = 0; wv < 4; ++wv) {
    __syncthreads();
    if (wave == wv)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int e = (kq + 4 * rr) * 16 + c;
        rred[e] = (wv == 0) ? racc[rr] : rred[e] + racc[rr];
      }
  }
  __syncthreads();
  for (int e = tid; e < 256; e += 256) a.raw_part[(int64_t)blockIdx.x * 256 + e] = rred[e];
}

// S_f (W_f, Sy_f) += the chunk's sums (in chunk order: deterministic), the chunk tables cleared
// for the next; dst: per FE [0] S, [1] W, [2] Sy
__global__ void k_stream_fold(unsigned long long* __restrict__ s64, double* __restrict__ sdbl, int64_t m, int p,
                              int pw, const double* __restrict__ fq, int F, const int64_t* __restrict__ toff_end,
                              double* const* __restrict__ dst) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
    int f = 0;
    while (f + 1 < F && e >= toff_end[f]) ++f;
    const int64_t j = e - (f ? toff_end[f - 1] : 0);
    const int64_t g = j / pw;
    const int cc = (int)(j % pw);
    const double v = fix_value(s64[e], sdbl[e], fq, cc);
    if (cc < p) dst[3 * f][g * p + cc] += v;
    else dst[3 * f + (cc - p + 1)][g] += v;
    s64[e] = 0ull;
    sdbl[e] = 0.0;
  }
}

// shift of the raw Gram for streamed chunks: the first row of the first chunk (both halves,
// as k_raw_shift leaves them for one process)
__global__ void k_stream_shift(const double* __restrict__ X, int64_t ld, int p, double* __restrict__ sh) {
  const int j = threadIdx.x;
  if (j < 16) {
    const double v = j < p ? X[(int64_t)j * ld] : 0.0;
    sh[j] = v;
    sh[16 + j] = v;
  }
}

__global__ void k_tile_add(double* __restrict__ acc, const double* __restrict__ t, int m) {
  for (int e = threadIdx.x; e < m; e += blockDim.x) acc[e] += t[e];
}

void stream_tile_add(lfe_ctx* c, const double* t, int m) {
  hipLaunchKernelGGL(k_tile_add, dim3(1), dim3(256), 0, c->stream, c->sw.tile, t, m);
}

// One streamed chunk of the sums pass: [p][ld] columns on the device (rows rows starting at
// input row row0).  Column statistics and quanta of this chunk (as k_part_scatter / sums4 form
// them), then two-limb group sums into the chunk tables and their fold into S (W, Sy) in chunk
// order.
int stream_sums_chunk(lfe_ctx* c, const double* X, int64_t ld, int64_t row0, int64_t rows, bool first) {
  auto& w = c->sw;
  const int p = c->p, F = c->F;
  const bool wt = c->w != nullptr;
  const int pw = p + (wt ? 2 : 0);
  int64_t m = 0;
  std::vector<int64_t> tend(F);
  StreamSumsArgs a{};
  for (int f = 0; f < F; ++f) {
    a.toff[f] = m;
    m += (int64_t)c->fe[f].G * pw;
    tend[f] = m;
    a.code[f] = c->fe[f].code + row0;
    a.cnt_pre[f] = c->fe[f].cnt_pre;
  }
  if (first) {
    LFE_TRY(ensure_f64(c, c->raw_shift, c->raw_shift_cap, 32));
    hipLaunchKernelGGL(k_stream_shift, dim3(1), dim3(64), 0, c->stream, X, ld, p, c->raw_shift);
    LFE_HIP(hipGetLastError());
    LFE_TRY(ensure_f64(c, w.s64, w.s64_cap, (size_t)m));
    LFE_TRY(ensure_f64(c, w.sdbl, w.sdbl_cap, (size_t)m));
    LFE_HIP(hipMemsetAsync(w.s64, 0, sizeof(double) * m, c->stream));
    LFE_HIP(hipMemsetAsync(w.sdbl, 0, sizeof(double) * m, c->stream));
    LFE_TRY(ensure_f64(c, w.tile, w.tile_cap, 272));
    LFE_HIP(hipMemsetAsync(w.tile, 0, sizeof(double) * 272, c->stream));
    LFE_TRY(ensure_f64(c, w.toff, w.toff_cap, 4 * kMaxFE));
    LFE_TRY(h2d_small(c, w.toff, tend.data(), sizeof(int64_t) * F));
    std::vector<double*> dst(3 * F);
    for (int f = 0; f < F; ++f) {
      dst[3 * f] = c->fe[f].S;
      dst[3 * f + 1] = c->fe[f].W;
      dst[3 * f + 2] = c->fe[f].Sy;
      if (wt) {
        LFE_HIP(hipMemsetAsync(c->fe[f].W, 0, sizeof(double) * c->fe[f].G, c->stream));
        LFE_HIP(hipMemsetAsync(c->fe[f].Sy, 0, sizeof(double) * c->fe[f].G, c->stream));
      }
    }
    LFE_TRY(h2d_small(c, w.toff + kMaxFE, dst.data(), sizeof(double*) * 3 * F));
  }
  const double* wch = wt ? c->w + row0 : nullptr;
  {
    ProfScope _ps(c, K_FIX_SUMS);
    constexpr int64_t kStatRows = 16384;
    const int nch = (int)std::max<int64_t>(1, (rows + kStatRows - 1) / kStatRows);
    LFE_TRY(ensure_f64(c, c->colstat, c->colstat_cap, (size_t)kColStatHead + (size_t)nch * pw));
    LFE_HIP(hipMemsetAsync(c->colstat, 0, sizeof(double) * kColStatHead, c->stream));
    if (wt)
      hipLaunchKernelGGL(k_col_stats_w, dim3(nch), dim3(256), 0, c->stream, X, wch, ld, rows, p, kStatRows,
                         c->colstat);
    else
      hipLaunchKernelGGL(k_col_stats, dim3(nch), dim3(256), 0, c->stream, X, ld, rows, p, kStatRows, c->colstat);
    LFE_TRY(ensure_f64(c, c->fixq, c->fixq_cap, (size_t)kFqRows * kFqCols));
    hipLaunchKernelGGL(k_fix_quanta, dim3(pw), dim3(256), 0, c->stream, c->colstat, nch, rows,
                       c->iscratch + kIscratchCmax, c->F, c->fixq);
    LFE_HIP(hipGetLastError());
  }
  a.X = X;
  a.ld = ld;
  a.rows = rows;
  a.p = p;
  a.F = F;
  a.pw = pw;
  a.w = wch;
  a.s64 = reinterpret_cast<unsigned long long*>(w.s64);
  a.sdbl = w.sdbl;
  a.fixq = c->fixq;
  a.shift = c->raw_shift;
  const int nblocks = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)c->n_cu * 8, ((rows + 15) / 16 + 3) / 4));
  LFE_TRY(ensure_f64(c, c->raw_part, c->raw_part_cap, (size_t)nblocks * 256));
  LFE_TRY(ensure_f64(c, c->raw_tile, c->raw_tile_cap, 256));
  a.raw_part = c->raw_part;
  const int nj = (pw + 15) / 16;  // column groups per lane (one: the raw Gram rides along)
  {
    ProfScope _ps(c, K_GROUP_SUMS);
    switch (nj) {
      case 1: hipLaunchKernelGGL(k_stream_sums<1>, dim3(nblocks), dim3(256), 0, c->stream, a); break;
      case 2: hipLaunchKernelGGL(k_stream_sums<2>, dim3(nblocks), dim3(256), 0, c->stream, a); break;
      case 3: hipLaunchKernelGGL(k_stream_sums<3>, dim3(nblocks), dim3(256), 0, c->stream, a); break;
      case 4: hipLaunchKernelGGL(k_stream_sums<4>, dim3(nblocks), dim3(256), 0, c->stream, a); break;
      default: hipLaunchKernelGGL(k_stream_sums<5>, dim3(nblocks), dim3(256), 0, c->stream, a); break;
    }
    LFE_HIP(hipGetLastError());
  }
  {
    ProfScope _ps(c, K_FIX_SUMS);
    hipLaunchKernelGGL(k_stream_fold, dim3(grid_for(m)), dim3(kBlock), 0, c->stream,
                       reinterpret_cast<unsigned long long*>(w.s64), w.sdbl, m, p, pw, c->fixq, F,
                       reinterpret_cast<const int64_t*>(w.toff), reinterpret_cast<double* const*>(w.toff + kMaxFE));
    LFE_HIP(hipGetLastError());
    if (nj == 1) {
      reduce_tiles(c, c->raw_part, nblocks, c->raw_tile);
      hipLaunchKernelGGL(k_tile_add, dim3(1), dim3(256), 0, c->stream, w.tile, c->raw_tile, 256);
      LFE_HIP(hipGetLastError());
    }
  }
  return LFE_OK;
}

// after the sums pass of a weighted streamed fit: the weight column's max and rms over every row
// into the quanta table's column p (the weighted cross terms' bound, k_cross_quanta)
int stream_weight_stats(lfe_ctx* c) {
  if (!c->w) return LFE_OK;
  constexpr int64_t kStatRows = 16384;
  const int nch = (int)std::max<int64_t>(1, (c->n + kStatRows - 1) / kStatRows);
  LFE_TRY(ensure_f64(c, c->colstat, c->colstat_cap, (size_t)kColStatHead + (size_t)nch));
  LFE_HIP(hipMemsetAsync(c->colstat, 0, sizeof(double) * kColStatHead, c->stream));
  hipLaunchKernelGGL(k_col_stats, dim3(nch), dim3(256), 0, c->stream, c->w, c->ld, c->n, 1, kStatRows, c->colstat);
  // one block = column 0 of a table that starts at column p of fixq
  hipLaunchKernelGGL(k_fix_quanta, dim3(1), dim3(256), 0, c->stream, c->colstat, nch, c->n,
                     c->iscratch + kIscratchCmax, c->F, c->fixq + c->p);
  LFE_HIP(hipGetLastError());
  c->exact_sums = true;
  return LFE_OK;
}

int exact_sums_on(lfe_ctx* c, int* on) {
  *on = c->exact_sums ? 1 : 0;  // the group sums are always two-limb fixed point
  return LFE_OK;
}

int hi_begin(lfe_ctx* c) {
  if (c->hi_dirty)  // an earlier sum stopped before its conversion: clear every coarse limb
    for (auto& fe : c->fe)
      if (fe.hi) LFE_HIP(hipMemsetAsync(fe.hi, 0, sizeof(double) * (size_t)fe.G * c->p, c->stream));
  c->hi_dirty = true;
  return LFE_OK;
}

}  // namespace lfe

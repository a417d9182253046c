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
        if (RAW) {
          // one MFMA per row of the quad, each followed by that row's LDS atomics, so the
          // matrix core works while the wave keeps issuing (NT = 1, unweighted, one FE besides P)
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const double z = !valid[s] ? 0.0 : (c == 15 ? 1.0 : (c < p ? xv[u][0][s] - shift : 0.0));
            racc[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(z, z, racc[s], 0, 0, 0);
            if (c < p && valid[s]) {
              const double v = xv[u][0][s];
              if (a.slice) atomicAdd(&lds[(hv[s] - lo) * p + c], v);
              else atomicAdd(&a.S[P][(int64_t)hv[s] * p + c], v);
              const int f = a.qf[0];
              const int g = (&cq[u][0].x)[s];
              if (a.tab_off[f] >= 0) atomicAdd(&lds[a.tab_off[f] + g * p + c], v);
              else atomicAdd(&a.S[f][(int64_t)g * p + c], v);
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

// The two-FE Gram-from-tables case of k_sums4 (RAW, unweighted, p <= 15, primary slice and
// secondary table both in LDS) with the per-row work cut to what the data needs: a row's
// only test is its primary code's sign (item edges are masked once per 16-row group), LDS
// byte offsets are one multiply-add per table, every pointer is hoisted out of the loop, and
// the next group pair's loads are issued before the current pair is consumed.
template <int TH, int NACC, int GU>
__global__ __launch_bounds__(TH) void k_sums2_raw(Sums4Args a) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
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
  d4 racc[NACC];  // independent MFMA chains
#pragma unroll
  for (int r = 0; r < NACC; ++r) racc[r] = d4{0.0, 0.0, 0.0, 0.0};
  for (int j = tid; j < a.G[Q] * p; j += TH) lds[qoff + j] = 0.0;
  for (int j = tid; j < a.B * p; j += TH) lds[j] = 0.0;
  auto flush = [&](int b) {
    const int lo = b << s;
    for (int j = tid; j < a.B * p; j += TH) {
      const double val = lds[j];
      const int g = lo + j / p;
      if (val != 0.0 && g < a.G_P) atomicAdd(&a.S[P][(int64_t)g * p + (j % p)], val);
      lds[j] = 0.0;
    }
  };
  const int i0 = (int)((int64_t)blockIdx.x * a.la.n_items / gridDim.x);
  const int i1 = (int)((int64_t)(blockIdx.x + 1) * a.la.n_items / gridDim.x);
  int cur = -1;
  for (int item = i0; item < i1; ++item) {
    const int4 it = a.la.items[item];
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
          if (v && col) {
            atomicAdd(lds_row_ptr(lds, hv[r] - lo, p8, c8), xv);
            atomicAdd(lds_row_ptr(qtab, gq[r], p8, c8), xv);
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
  for (int j = tid; j < a.G[Q] * p; j += TH) {
    const double val = lds[qoff + j];
    if (val != 0.0) atomicAdd(&a.S[Q][j], val);
  }
  __shared__ double rred[256];
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

// re-centre this rank's raw tile from its own shift c_r to the common shift c*:
// sum (d - c*)(d - c*)' = R + dl C' + C dl' + n dl dl',  sum (d - c*) = C + n dl,  dl = c_r - c*
__global__ void k_raw_recenter(double* __restrict__ R, const double* __restrict__ sh, int p) {
  __shared__ double C[16], dl[16];
  const int t = threadIdx.x;
  if (t < 16) {
    C[t] = R[15 * 16 + t];
    dl[t] = t < p ? sh[16 + t] - sh[t] : 0.0;
  }
  __syncthreads();
  const double n = R[15 * 16 + 15];
  const int i = t / 16, j = t % 16;
  double v = R[t];
  if (i < p && j < p) v += dl[i] * C[j] + C[i] * dl[j] + n * dl[i] * dl[j];
  else if (i == 15 && j < p) v += n * dl[j];
  else if (j == 15 && i < p) v += n * dl[i];
  __syncthreads();
  R[t] = v;
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
    if (!c->sums_zeroed) LFE_HIP(hipMemsetAsync(c->fe[f].S, 0, sizeof(double) * (size_t)c->fe[f].G * p, c->stream));
  }
  a.nq = 0;
  for (int f = 0; f < c->F; ++f)
    if (f != P) a.qf[a.nq++] = f;
  c->sums_zeroed = false;
  const size_t lds = off * 8;
  const int NT = (p + 15) / 16;
  const void* fn = nullptr;
#define SUMS4_FN(FQ, GU, NT_, TH_) reinterpret_cast<const void*>(&k_sums4<FQ, GU, NT_, TH_, false>)
  static const int gu_env = [] {
    const char* e = getenv("LFE_SUMS_GU");  // tuning override
    return e ? atoi(e) : 0;
  }();
  static const int raw_env = [] {
    const char* e = getenv("LFE_TABLE_GRAM");  // 0: no Gram from tables (explicit design pass)
    return e ? atoi(e) : 1;
  }();
  const bool raw = raw_env != 0 && c->F == 2 && P >= 0 && a.nq == 1 && p <= 15 && !a.w && gu_env != 4;
  c->raw_ready = false;
  static const int sums2_env = [] {
    // tuning: 0 = k_sums4 for the two-FE Gram case; MFMA chains x groups per load: 1 = 4 x 2,
    // 2 = 2 x 2, 3 = 4 x 1, 4 = 2 x 1 (3: 0.925 vs 0.950 ms for 1 with 24-bit LDS addressing)
    const char* e = getenv("LFE_SUMS2");
    return e ? atoi(e) : 3;
  }();
  int threads = kSumThreads;
  if (a.nq <= 1 && NT == 1) {
    // the 2-FE case: one workgroup per CU (LDS), so 16 waves of <= 128 VGPRs (GU 2)
    threads = gu_env == 4 ? kSumThreads : 1024;
    const bool two = raw && sums2_env && a.slice && a.tab_off[a.qf[0]] >= 0;
    fn = gu_env == 4 ? SUMS4_FN(1, 4, 1, kSumThreads)
         : two       ? (sums2_env == 2   ? reinterpret_cast<const void*>(&k_sums2_raw<1024, 2, 2>)
                        : sums2_env == 3 ? reinterpret_cast<const void*>(&k_sums2_raw<1024, 4, 1>)
                        : sums2_env == 4 ? reinterpret_cast<const void*>(&k_sums2_raw<1024, 2, 1>)
                                         : reinterpret_cast<const void*>(&k_sums2_raw<1024, 4, 2>))
         : raw       ? reinterpret_cast<const void*>(&k_sums4<1, 2, 1, 1024, true>)
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
  LFE_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)std::max<size_t>(lds, 1)));
  const int nblocks = std::max(1, std::min(c->L.n_items, resident_blocks(c, fn, threads, lds)));
  if (raw) {
    LFE_TRY(ensure_f64(c, c->raw_part, c->raw_part_cap, (size_t)nblocks * 256));
    LFE_TRY(ensure_f64(c, c->raw_tile, c->raw_tile_cap, 256));
    a.raw_part = c->raw_part;
  }
  {
    ProfScope _ps(c, K_GROUP_SUMS);
    void* args[] = {&a};
    LFE_HIP(hipLaunchKernel(fn, dim3(nblocks), dim3(threads), args, lds, c->stream));
  }
  LFE_HIP(hipGetLastError());
  if (raw) {
    reduce_tiles(c, c->raw_part, nblocks, c->raw_tile);
    LFE_TRY(ensure_f64(c, c->raw_shift, c->raw_shift_cap, 32));
    hipLaunchKernelGGL(k_raw_shift, dim3(1), dim3(64), 0, c->stream, c->L.X, c->ld, p, c->L.n_items > 0 ? 1 : 0,
                       c->rank, c->raw_shift);
    LFE_HIP(hipGetLastError());
    if (c->world > 1) {
      // every rank's tile re-centred on rank 0's shift, then summed: the global raw Gram
      LFE_TRY(allreduce_sum_f64(c, c->raw_shift, 16));
      hipLaunchKernelGGL(k_raw_recenter, dim3(1), dim3(256), 0, c->stream, c->raw_tile, c->raw_shift, p);
      LFE_HIP(hipGetLastError());
      LFE_TRY(allreduce_sum_f64(c, c->raw_tile, 256));
    }
    c->raw_ready = true;
  }
  for (int f = 0; f < c->F; ++f)  // owner-sharded rows: the primary FE's sums are complete on each rank
    if (!(c->owner_on && f == P)) LFE_TRY(allreduce_sum_f64(c, c->fe[f].S, (size_t)c->fe[f].G * p));
  return LFE_OK;
}

}  // namespace lfe

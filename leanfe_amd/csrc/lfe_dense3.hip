// leanfe HIP engine — the alternating-projection sweeps (polars_impl.py:490-526) for three or more
// FEs with every cross term as a product of pair count tables on the matrix cores.
//
// The projection of FE f subtracts, per level g of f, the mean over its rows of sum_{b != f}
// alpha_b[g_b(row)] - i.e. T_f = sum_{b != f} N_fb alpha_b with N_fb[g][h] = the kept rows whose
// codes of f and b are (g, h).  The general sweeps of lfe_seg.hip gather alpha_b row by row over a
// segment layout per FE (5 ms to build at 50M rows, then ~75 ps per row and sweep); where the pair
// tables are small against the rows (the reference's 3-FE benchmark panels: 2e4 x 4e3 x 1e3 levels
// over 50M rows hold ~2 table bytes per row) one table byte per cell and pass replaces those gathers.
//
// Tables (one per ordered pair, in the K2 fragment form of the two-FE passes, lfe_dense.hip):
//   tab[a][b] = [tile t of 512 b levels][16-row block of a levels][8 k blocks of 64][1 KB], lane
//   (g, i) bytes jj = N_ab[16 rb + i][512 t + 64 kb + 16 g + jj]; a block with a count over 127 is
//   flagged, zero in the i8 table, and its counts kept as u16 in X[a][b] (16 x 64, natural order).
// The build partitions the kept rows' codes by a >> 6 (a counting sort; one partition carries the
// codes of every partner of a, up to three), counts each
// 64-level chunk of a against 2048 columns of b at a time in LDS (8-bit counters; a chunk where some
// cell passes 255 is counted again on 16-bit counters in two halves) and writes both orientations.
//
// A pass over tab[f][b] is the two-FE K2 streaming kernel (alpha_b's tiles cut into exact base-128
// digits in the workgroup, v_mfma_i32_16x16x64_i8 against the count fragments): it writes one slot
// per tile of b, and T_f = the slots of every b != f added in (b, tile) order - the same bits every
// run.  Columns go 16 at a time (p = 21: two passes per table).  The stop test (polars_impl.py:512-
// 521) follows the general sweeps: the last FE's mean from its own T, the first FE's from the next
// projection's T (kept for the next sweep), every other FE's from a y-only pass (R).
#include "lfe_internal.h"

#include <algorithm>
#include <cstdlib>
#include <vector>

namespace lfe {

constexpr int kD3Chunk = 64;     // a levels per counting chunk (= one k block of the transposed table)
constexpr int kD3W = 2048;       // b columns per counting workgroup (64 x 2048 8-bit counters: 128 KB)
constexpr int kD3Tile = 512;
constexpr int kD3MaxG = 65536;   // levels per FE (partition bins <= 1024 in LDS, 16-bit table indices)
constexpr int kD3Wgs = 1024;     // workgroups of the partition histogram / scatter

static int64_t n512(int32_t G) { return ((int64_t)G + kD3Tile - 1) / kD3Tile * kD3Tile; }
static int tiles_of(int32_t G) { return (int)(((int64_t)G + kD3Tile - 1) / kD3Tile); }

// ---------------------------------------------------------------------------
// build
// ---------------------------------------------------------------------------

// kept rows (code_P >= 0) of workgroup w's row range, counted per bin a >> 6 -> cnt[bin][w]; every
// thread keeps kD3U rows' loads in flight (one load per wave at a time left the pass latency-bound)
constexpr int kD3U = 8;
__global__ __launch_bounds__(256) void k_d3_hist(const int32_t* __restrict__ codeP, const int32_t* __restrict__ codeA,
                                                 int64_t n, int nbin, int32_t* __restrict__ cnt) {
  extern __shared__ int32_t h[];
  for (int j = threadIdx.x; j < nbin; j += blockDim.x) h[j] = 0;
  __syncthreads();
  const int64_t r0 = n * blockIdx.x / gridDim.x, r1 = n * (blockIdx.x + 1) / gridDim.x;
  for (int64_t i0 = r0 + threadIdx.x; i0 < r1; i0 += kD3U * (int64_t)blockDim.x) {
    int32_t hp[kD3U], ha[kD3U];
#pragma unroll
    for (int u = 0; u < kD3U; ++u) {
      const int64_t i = i0 + u * (int64_t)blockDim.x;
      hp[u] = i < r1 ? codeP[i] : -1;
      ha[u] = i < r1 ? codeA[i] : 0;
    }
#pragma unroll
    for (int u = 0; u < kD3U; ++u)
      if (hp[u] >= 0) atomicAdd(&h[ha[u] >> 6], 1);
  }
  __syncthreads();
  for (int j = threadIdx.x; j < nbin; j += blockDim.x) cnt[(int64_t)j * gridDim.x + blockIdx.x] = h[j];
}

// the same rows to their bin's range (bases: the scanned counts), packed as a & 63 in bits [0, 6) and
// the codes of up to three partner FEs b_j in bits [6 + 16 j, 22 + 16 j) (levels <= 65536): one
// partition serves every pair the FE with more levels forms
constexpr int kD3Slots = 3;
struct D3Codes {
  const int32_t* b[kD3Slots];
  int nb;
};
__global__ __launch_bounds__(256) void k_d3_scatter(const int32_t* __restrict__ codeP, const int32_t* __restrict__ codeA,
                                                    D3Codes cb, int64_t n, int nbin, const int32_t* __restrict__ base,
                                                    uint64_t* __restrict__ out) {
  // one row per thread and iteration (eight in flight measured slower: the returning LDS cursor adds
  // of a workgroup's few bins serialize either way, and the stores follow them)
  extern __shared__ int32_t cur[];
  for (int j = threadIdx.x; j < nbin; j += blockDim.x) cur[j] = base[(int64_t)j * gridDim.x + blockIdx.x];
  __syncthreads();
  const int64_t r0 = n * blockIdx.x / gridDim.x, r1 = n * (blockIdx.x + 1) / gridDim.x;
  for (int64_t i = r0 + threadIdx.x; i < r1; i += blockDim.x) {
    if (codeP[i] < 0) continue;
    const int32_t a = codeA[i];
    uint64_t v = (uint64_t)(a & 63);
#pragma unroll
    for (int j = 0; j < kD3Slots; ++j)
      if (j < cb.nb) v |= (uint64_t)(uint32_t)cb.b[j][i] << (6 + 16 * j);
    const int pos = atomicAdd(&cur[a >> 6], 1);
    out[pos] = v;
  }
}

struct D3Build {
  const uint64_t* part;
  int slot;              // the partner FE's 16-bit field in the packed rows
  const int32_t* base;   // scanned [bin][nwg] (+ the total): bin j's rows are [base[j nwg], base[(j + 1) nwg])
  int nwg, nbr, NA512, NB512;
  int8_t* tab_ab;        // rows a, k b: [tile of b][NA512 / 16][8][1 KB]
  uint8_t* flg_ab;
  uint16_t* X_ab;
  int8_t* tab_ba;        // rows b, k a: [tile of a][NB512 / 16][8][1 KB]
  uint8_t* flg_ba;
  uint16_t* X_ba;
};

// the chunk's rows with b in [bc0, bc0 + W) into LDS counters cnt[a & 63][b - bc0] of CT (8 or 16
// bits, packed in words); returns whether an 8-bit counter overflowed
template <typename CT>
__device__ bool d3_count(const uint64_t* __restrict__ part, int slot, uint32_t* cw, int r0, int r1, int bc0, int W) {
  constexpr int PER = 4 / sizeof(CT), SH = 8 * sizeof(CT);
  __shared__ int ovf;
  const int words = kD3Chunk * W / PER;
  for (int j = threadIdx.x; j < words; j += blockDim.x) cw[j] = 0u;
  if (threadIdx.x == 0) ovf = 0;
  __syncthreads();
  bool over = false;
  constexpr int V = 8;  // loads in flight per thread
  for (int i0 = r0 + (int)threadIdx.x; i0 < r1; i0 += V * (int)blockDim.x) {
    uint64_t v[V];
#pragma unroll
    for (int u = 0; u < V; ++u) {
      const int i = i0 + u * (int)blockDim.x;
      v[u] = i < r1 ? part[i] : 0ull;
    }
#pragma unroll
    for (int u = 0; u < V; ++u) {
      if (i0 + u * (int)blockDim.x >= r1) break;
      const uint32_t b = (uint32_t)((v[u] >> (6 + 16 * slot)) & 0xffffu) - (uint32_t)bc0;
      if (b >= (uint32_t)W) continue;
      const uint32_t idx = (uint32_t)(v[u] & 63u) * (uint32_t)W + b;
      const int sh = (int)(idx % PER) * SH;
      const uint32_t old = atomicAdd(&cw[idx / PER], 1u << sh);
      if (sizeof(CT) == 1 && ((old >> sh) & 0xffu) == 0xffu) over = true;  // carried into the next byte
    }
  }
  if (over) ovf = 1;
  __syncthreads();
  return ovf != 0;
}

// both orientations' fragments of the chunk (64 a levels) x columns [bc0, bc0 + W) from the counters
template <typename CT>
__device__ void d3_write(const D3Build& a, const CT* cnt, int bin, int bc0, int W) {
  __shared__ int ov[4 * (kD3W / 64) + kD3W / 16];
  typedef int v4 __attribute__((ext_vector_type(4)));
  const int nkl = W >> 6, na_b = 4 * nkl, nb_b = W >> 4;
  const int nrb_a = a.NA512 >> 4, nrb_b = a.NB512 >> 4;
  auto bidx_ab = [&](int j) {  // ab block j = (row block rb of the chunk, k block kl of the range)
    const int rb = j / nkl, kl = j - rb * nkl, kb = (bc0 >> 6) + kl;
    return ((int64_t)(kb >> 3) * nrb_a + bin * 4 + rb) * 8 + (kb & 7);
  };
  auto bidx_ba = [&](int j) {  // ba block j = 16-row block of b levels bc0 + 16 j (k block: the chunk)
    return ((int64_t)(bin >> 3) * nrb_b + (bc0 >> 4) + j) * 8 + (bin & 7);
  };
  for (int j = threadIdx.x; j < na_b + nb_b; j += blockDim.x) ov[j] = 0;
  __syncthreads();
  for (int e = threadIdx.x; e < na_b * 64; e += blockDim.x) {
    const int blk = e >> 6, l = e & 63, rb = blk / nkl, kl = blk - rb * nkl;
    const CT* src = cnt + (16 * rb + (l & 15)) * W + 64 * kl + 16 * (l >> 4);
    v4 w;
    bool big;
    if (sizeof(CT) == 1) {
      w = *reinterpret_cast<const v4*>(src);
      big = ((w.x | w.y | w.z | w.w) & 0x80808080) != 0;
    } else {
      const v4 u0 = reinterpret_cast<const v4*>(src)[0], u1 = reinterpret_cast<const v4*>(src)[1];
      big = ((u0.x | u0.y | u0.z | u0.w | u1.x | u1.y | u1.z | u1.w) & (int)0xff80ff80) != 0;
      auto pk = [](int x, int y) {
        const uint32_t ux = (uint32_t)x, uy = (uint32_t)y;
        return (int)((ux & 0xffu) | ((ux >> 8) & 0xff00u) | ((uy & 0xffu) << 16) | ((uy << 8) & 0xff000000u));
      };
      w = v4{pk(u0.x, u0.y), pk(u0.z, u0.w), pk(u1.x, u1.y), pk(u1.z, u1.w)};
    }
    if (big) ov[blk] = 1;
    *reinterpret_cast<v4*>(a.tab_ab + bidx_ab(blk) * 1024 + l * 16) = w;
  }
  for (int e = threadIdx.x; e < nb_b * 64; e += blockDim.x) {
    const int blk = e >> 6, l = e & 63;
    const CT* src = cnt + (16 * (l >> 4)) * W + 16 * blk + (l & 15);
    v4 w = v4{0, 0, 0, 0};
    int m = 0;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {
      const int v = (int)src[jj * W];
      m |= v;
      w[jj >> 2] |= (v & 0xff) << (8 * (jj & 3));
    }
    if (m & ~127) ov[na_b + blk] = 1;
    *reinterpret_cast<v4*>(a.tab_ba + bidx_ba(blk) * 1024 + l * 16) = w;
  }
  __syncthreads();
  for (int j = threadIdx.x; j < na_b; j += blockDim.x) a.flg_ab[bidx_ab(j)] = (uint8_t)ov[j];
  for (int j = threadIdx.x; j < nb_b; j += blockDim.x) a.flg_ba[bidx_ba(j)] = (uint8_t)ov[na_b + j];
  // flagged blocks (rare: a cell of more than 127 kept rows): the i8 block zeroed, its counts as u16
  for (int blk = 0; blk < na_b + nb_b; ++blk) {
    if (!ov[blk]) continue;  // uniform (LDS)
    if (blk < na_b) {
      const int rb = blk / nkl, kl = blk - rb * nkl;
      const int64_t bo = bidx_ab(blk) * 1024;
      for (int t = threadIdx.x; t < 1024; t += blockDim.x) {
        a.X_ab[bo + t] = (uint16_t)cnt[(16 * rb + (t >> 6)) * W + 64 * kl + (t & 63)];
        a.tab_ab[bo + t] = 0;
      }
    } else {
      const int j = blk - na_b;
      const int64_t bo = bidx_ba(j) * 1024;
      for (int t = threadIdx.x; t < 1024; t += blockDim.x) {
        a.X_ba[bo + t] = (uint16_t)cnt[(t & 63) * W + 16 * j + (t >> 6)];
        a.tab_ba[bo + t] = 0;
      }
    }
  }
}

// workgroup (bin of 64 a levels, range of kD3W b columns)
__global__ __launch_bounds__(1024) void k_d3_build(D3Build a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t cw[];
  const int bin = blockIdx.x / a.nbr, br = blockIdx.x - bin * a.nbr;
  const int r0 = a.base[(int64_t)bin * a.nwg], r1 = a.base[(int64_t)(bin + 1) * a.nwg];
  const int bc0 = br * kD3W, W = min(kD3W, a.NB512 - bc0);
  if (!d3_count<uint8_t>(a.part, a.slot, cw, r0, r1, bc0, W)) {
    d3_write<uint8_t>(a, reinterpret_cast<const uint8_t*>(cw), bin, bc0, W);
    return;
  }
  const int W2 = W / 2;  // a multiple of 256 (W is one of 512)
  for (int half = 0; half < 2; ++half) {
    __syncthreads();
    d3_count<uint16_t>(a.part, a.slot, cw, r0, r1, bc0 + half * W2, W2);
    d3_write<uint16_t>(a, reinterpret_cast<const uint16_t*>(cw), bin, bc0 + half * W2, W2);
  }
}

// ---------------------------------------------------------------------------
// sweeps
// ---------------------------------------------------------------------------

__device__ __forceinline__ void d3_max_out(double mx, unsigned long long* check) {
  for (int off = 32; off > 0; off >>= 1) {
    const double o = __shfl_down(mx, off, 64);
    mx = (isnan(o) || isnan(mx)) ? __builtin_nan("") : fmax(mx, o);
  }
  if ((threadIdx.x & 63) == 0) atomicMax(check, (unsigned long long)__double_as_longlong(fabs(mx)));
}

// T = the ns slots [ns][m] added in slot order; with out (m = G p): out = (S - T) / cnt and, with
// check, max over present groups of |out - cur| in the y column (= |mean_g(y~)| after the sweep)
__global__ __launch_bounds__(256) void k_d3_reduce(const double* __restrict__ runs, int ns, int64_t m,
                                                   double* __restrict__ T, const double* __restrict__ S,
                                                   const int32_t* __restrict__ cnt, int p, const double* cur,
                                                   double* out, unsigned long long* __restrict__ check) {
  double mx = 0.0;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
    double t = 0.0;
    int s = 0;
    for (; s + 8 <= ns; s += 8) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = runs[(int64_t)(s + u) * m + e];
#pragma unroll
      for (int u = 0; u < 8; ++u) t += v[u];
    }
    for (; s < ns; ++s) t += runs[(int64_t)s * m + e];
    if (T) T[e] = t;
    if (out) {
      const int32_t n = cnt[e / p];
      const double v = n > 0 ? (S[e] - t) / (double)n : 0.0;
      if (check && n > 0 && e % p == 0) {
        const double d = fabs(v - cur[e]);
        mx = (isnan(d) || isnan(mx)) ? __builtin_nan("") : fmax(mx, d);
      }
      out[e] = v;
    }
  }
  if (check) d3_max_out(mx, check);
}

// max over present groups of |mean_g(y~)| = |(S[g][0] - cnt alpha[g][0] - R[g]) / cnt| (R: stride rs)
__global__ __launch_bounds__(256) void k_d3_ycheck(const double* __restrict__ S, int p, const double* __restrict__ R,
                                                   int rs, const double* __restrict__ alpha,
                                                   const int32_t* __restrict__ cnt, int32_t G,
                                                   unsigned long long* __restrict__ check) {
  double mx = 0.0;
  for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x) {
    const int32_t n = cnt[g];
    if (n <= 0) continue;
    const double d = fabs((S[(int64_t)g * p] - (double)n * alpha[(int64_t)g * p] - R[(int64_t)g * rs]) / (double)n);
    mx = (isnan(d) || isnan(mx)) ? __builtin_nan("") : fmax(mx, d);
  }
  d3_max_out(mx, check);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------

bool dense3_ok(const lfe_ctx* c, const std::vector<int>& order, int check_from) {
  (void)order;
  if (c->dense_off) return false;  // the digits' range guard fired (lfe_demean)
  const char* e = knob("LFE_DENSE");  // "0": never (A/B); "1": whenever it fits
  if (e && e[0] == '0') return false;
  const bool force = e && e[0] == '1';
  const int F = c->F;
  if (F < 3 || check_from <= 0 || c->L.w || c->records || c->L.P < 0 || !c->L.permuted) return false;
  if (!(c->world == 1 || c->owner_on)) return false;
  for (int f = 0; f < F; ++f)
    if (c->fe[f].G < 1 || c->fe[f].G > kD3MaxG) return false;
  // owner-sharded ranks: the primary FE's largest level over all ranks (other FEs' counts are
  // all-reduced), and the whole panel's rows per rank, so that every rank decides alike
  const bool owner = c->owner_on && c->world > 1;
  auto cmax = [&](int f) {
    return owner && f == c->L.P ? (c->cmax_over_ranks > 0 ? 65536 : 0) : c->fe[f].cmax;
  };
  int64_t bytes = 0;
  for (int a = 0; a < F; ++a)
    for (int b = a + 1; b < F; ++b) {
      if (std::min(cmax(a), cmax(b)) > 65535) return false;  // u16 counts
      bytes += 2 * n512(c->fe[a].G) * n512(c->fe[b].G);
    }
  if (bytes > (int64_t)24 << 30) return false;
  // a pass reads a table byte per cell and 16 columns; the row gathers cost ~75 ps per row and sweep
  // against ~0.25 ps per table byte: dense from 16 table bytes per kept row
  const int64_t ncg = (c->p + 15) / 16;
  const int64_t rows = owner ? c->n_kept / c->world : c->n_kept_local;
  return force || bytes * ncg <= 16 * std::max<int64_t>(rows, 1);
}

void free_dense3(lfe_ctx* c) {
  auto& d = c->d3;
  for (int a = 0; a < kMaxFE; ++a) {
    for (int b = 0; b < kMaxFE; ++b) {
      dfree_any(d.tab[a][b]);
      dfree_any(d.flg[a][b]);
      dfree_any(d.X[a][b]);
      d.tab_cap[a][b] = d.flg_cap[a][b] = d.X_cap[a][b] = 0;
    }
    dfree_any(d.runs[a]);
    d.runs_cap[a] = 0;
  }
  dfree_any(d.part);
  dfree_any(d.hist);
  dfree_any(d.tiles);
  d.part_cap = d.hist_cap = 0;
  d.on = false;
  d.table_bytes = 0;
}

template <typename T>
static int ensure_dev(T*& p, size_t& cap, size_t elems) {
  if (p && cap >= elems) return LFE_OK;
  dfree_any(p);
  cap = 0;
  LFE_HIP(hipMalloc(reinterpret_cast<void**>(&p), sizeof(T) * std::max<size_t>(elems, 1)));
  cap = elems;
  return LFE_OK;
}

static int d3_build(lfe_ctx* c) {
  auto& d = c->d3;
  const int F = c->F;
  if (!d.tiles) {
    LFE_HIP(hipMalloc(reinterpret_cast<void**>(&d.tiles), sizeof(int32_t) * (kD3MaxG / kD3Tile)));
    std::vector<int32_t> id(kD3MaxG / kD3Tile);
    for (size_t i = 0; i < id.size(); ++i) id[i] = (int32_t)i;
    LFE_TRY(h2d_small(c, d.tiles, id.data(), sizeof(int32_t) * id.size()));  // on c->stream (pinned staging)
  }
  const int64_t n = c->n;
  LFE_TRY(ensure_dev(d.part, d.part_cap, (size_t)std::max<int64_t>(c->n_kept_local, 1)));
  d.table_bytes = 0;
  const size_t lds = (size_t)kD3Chunk * kD3W;  // 8-bit counters (16-bit: half the columns)
  LFE_HIP(set_max_lds(reinterpret_cast<const void*>(&k_d3_build), (int)lds));
  // every unordered pair is counted from the partition of its FE with more levels (more chunks):
  // one partition (histogram, scan, scatter) per such FE and up to kD3Slots partners
  std::vector<std::vector<int>> partners(F);
  for (int x = 0; x < F; ++x)
    for (int y = x + 1; y < F; ++y) {
      const int a = c->fe[x].G >= c->fe[y].G ? x : y;
      partners[a].push_back(a == x ? y : x);
    }
  const int nwg = (int)std::max<int64_t>(1, std::min<int64_t>(kD3Wgs, (n + 4095) / 4096));
  for (int a = 0; a < F; ++a) {
    if (partners[a].empty()) continue;
    const int64_t NA = n512(c->fe[a].G);
    const int nbin = (int)(NA / kD3Chunk);
    const size_t hm = (size_t)nbin * nwg;
    LFE_TRY(ensure_dev(d.hist, d.hist_cap, hm + 4));
    LFE_HIP(hipMemsetAsync(d.hist + hm, 0, sizeof(int32_t) * 4, c->stream));
    {
      ProfScope _ps(c, K_LAYOUT_HIST);
      hipLaunchKernelGGL(k_d3_hist, dim3(nwg), dim3(256), sizeof(int32_t) * nbin, c->stream, c->L.code[c->L.P],
                         c->L.code[a], n, nbin, d.hist);
      LFE_HIP(hipGetLastError());
    }
    LFE_TRY(exclusive_scan(c, d.hist, (int64_t)hm + 1));
    const auto& pb = partners[a];
    for (size_t j0 = 0; j0 < pb.size(); j0 += kD3Slots) {
      D3Codes cb{};
      cb.nb = (int)std::min<size_t>(kD3Slots, pb.size() - j0);
      for (int j = 0; j < cb.nb; ++j) cb.b[j] = c->L.code[pb[j0 + j]];
      {
        ProfScope _ps(c, K_LAYOUT_SCATTER);
        hipLaunchKernelGGL(k_d3_scatter, dim3(nwg), dim3(256), sizeof(int32_t) * nbin, c->stream, c->L.code[c->L.P],
                           c->L.code[a], cb, n, nbin, d.hist, d.part);
        LFE_HIP(hipGetLastError());
      }
      for (int j = 0; j < cb.nb; ++j) {
        const int b = pb[j0 + j];
        const int64_t NB = n512(c->fe[b].G), cells = NA * NB;
        d.table_bytes += 2 * cells;
        LFE_TRY(ensure_dev(d.tab[a][b], d.tab_cap[a][b], (size_t)cells));
        LFE_TRY(ensure_dev(d.tab[b][a], d.tab_cap[b][a], (size_t)cells));
        LFE_TRY(ensure_dev(d.flg[a][b], d.flg_cap[a][b], (size_t)cells / 1024));
        LFE_TRY(ensure_dev(d.flg[b][a], d.flg_cap[b][a], (size_t)cells / 1024));
        LFE_TRY(ensure_dev(d.X[a][b], d.X_cap[a][b], (size_t)cells));
        LFE_TRY(ensure_dev(d.X[b][a], d.X_cap[b][a], (size_t)cells));
        D3Build ba{};
        ba.part = d.part;
        ba.slot = j;
        ba.base = d.hist;
        ba.nwg = nwg;
        ba.nbr = (int)((NB + kD3W - 1) / kD3W);
        ba.NA512 = (int)NA;
        ba.NB512 = (int)NB;
        ba.tab_ab = d.tab[a][b];
        ba.flg_ab = d.flg[a][b];
        ba.X_ab = d.X[a][b];
        ba.tab_ba = d.tab[b][a];
        ba.flg_ba = d.flg[b][a];
        ba.X_ba = d.X[b][a];
        ProfScope _ps(c, K_SEG_BUILD);
        hipLaunchKernelGGL(k_d3_build, dim3(nbin * ba.nbr), dim3(1024), lds, c->stream, ba);
        LFE_HIP(hipGetLastError());
      }
    }
  }
  return LFE_OK;
}

// the slots of FE f's cross term (y_only: the y column, stride 1): every other FE's tiles in FE
// order, 16 columns per pass; returns the slot count
static int d3_cross(lfe_ctx* c, int f, bool y_only, int* ns_out) {
  auto& d = c->d3;
  const int p = c->p, pcols = y_only ? 1 : p, ldo = y_only ? 1 : p;
  const int32_t Gf = c->fe[f].G;
  int ns = 0;
  for (int b = 0; b < c->F; ++b) ns += b == f ? 0 : tiles_of(c->fe[b].G);
  LFE_TRY(ensure_dev(d.runs[f], d.runs_cap[f], (size_t)ns * Gf * p));
  ProfScope _ps(c, y_only ? K_CHECK : K_CROSS);
  int slot = 0;
  std::vector<PairPass> passes;
  for (int b = 0; b < c->F; ++b) {
    if (b == f) continue;
    for (int c0 = 0; c0 < pcols; c0 += 16) {
      PairPass pp{};
      pp.tab = d.tab[f][b];
      pp.flg = d.flg[f][b];
      pp.X = d.X[f][b];
      pp.tiles = d.tiles;
      pp.ntile_k = tiles_of(c->fe[b].G);
      pp.nrb = (int)(n512(Gf) / 16);
      pp.G_rows = Gf;
      pp.G_k = c->fe[b].G;
      pp.pc = std::min(16, pcols - c0);
      pp.lda = p;
      pp.ldo = ldo;
      pp.alpha = c->fe[b].alpha + c0;
      pp.runs = d.runs[f] + (size_t)slot * Gf * ldo + c0;
      passes.push_back(pp);
    }
    slot += tiles_of(c->fe[b].G);
  }
  // every partner and column group of the projection in one launch (LFE_D3_BATCH=0: one each, A/B)
  const bool batch = [] {
    const char* e = knob("LFE_D3_BATCH");
    return !(e && e[0] == '0');
  }();
  if (batch) {
    LFE_TRY(dn8_pair_passes(c, passes.data(), (int)passes.size()));
  } else {
    for (const auto& pp : passes) LFE_TRY(dn8_pair_pass(c, pp));
  }
  *ns_out = ns;
  return LFE_OK;
}

static int d3_reduce(lfe_ctx* c, const double* runs, int ns, int64_t m, double* T, int f, const double* cur,
                     double* out, bool check) {
  auto& fe = c->fe[f];
  ProfScope _ps(c, K_FINALIZE);
  hipLaunchKernelGGL(k_d3_reduce, dim3(grid_for(m)), dim3(256), 0, c->stream, runs, ns, m, T, fe.S, fe.cnt, c->p, cur,
                     out, check ? reinterpret_cast<unsigned long long*>(c->dred) : nullptr);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

// FE f's projection from the current effects of the others into out (check: against cur)
static int d3_project(lfe_ctx* c, int f, const double* cur, double* out, bool check) {
  auto& fe = c->fe[f];
  int ns = 0;
  LFE_TRY(d3_cross(c, f, false, &ns));
  const int64_t m = (int64_t)fe.G * c->p;
  if (c->world == 1 || (c->owner_on && f == c->L.P))  // T complete on this rank
    return d3_reduce(c, c->d3.runs[f], ns, m, fe.T, f, cur, out, check);
  LFE_TRY(d3_reduce(c, c->d3.runs[f], ns, m, fe.T, f, nullptr, nullptr, false));
  LFE_TRY(allreduce_sum_f64(c, fe.T, (size_t)m));
  return d3_reduce(c, fe.T, 1, m, nullptr, f, cur, out, check);
}

static int d3_ycheck(lfe_ctx* c, int f, const double* R, int rs) {
  auto& fe = c->fe[f];
  ProfScope _ps(c, K_CHECK_MAX);
  hipLaunchKernelGGL(k_d3_ycheck, dim3(grid_for(fe.G)), dim3(256), 0, c->stream, fe.S, c->p, R, rs, fe.alpha, fe.cnt,
                     fe.G, reinterpret_cast<unsigned long long*>(c->dred));
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

int demean_dense3(lfe_ctx* c, const std::vector<int>& order, double tol, int max_iter, int check_from,
                  int* iterations_out, double* last_out) {
  // every alpha table is zero here (lfe_demean)
  LFE_TRY(d3_build(c));
  c->d3.on = true;
  c->dense_cells = c->d3.table_bytes;  // lfe_dense_cells: the i8 cells of every ordered pair's table
  c->dn8 = true;
  const int F = c->F, p = c->p, f0 = order[0];
  LFE_TRY(ensure_f64(c, c->alpha_spare, c->alpha_spare_cap, (size_t)c->fe[f0].G * p));
  LFE_TRY(ensure_dred(c, 2));
  LFE_TRY(range_flag_reset(c));  // the digits' dynamic-range guard (lfe_dense.hip)
  int iterations = 0;
  double last = -1.0;
  bool first_ready = false;  // alpha_spare holds order[0]'s next projection (formed by the last check)
  bool checked = false;      // the last sweep ran the stop test (order[0]'s T is then from the final effects)
  c->d3.t_final = 0;
  for (int it = 1; it <= max_iter; ++it) {
    for (int k = 0; k < F; ++k) {
      const int f = order[k];
      if (k == 0 && first_ready) {
        LFE_HIP(hipMemcpyAsync(c->fe[f].alpha, c->alpha_spare, sizeof(double) * (size_t)c->fe[f].G * p,
                               hipMemcpyDeviceToDevice, c->stream));
        continue;
      }
      LFE_TRY(d3_project(c, f, c->fe[f].alpha, c->fe[f].alpha, false));
    }
    first_ready = false;
    checked = false;
    iterations = it;
    if (it < check_from) continue;
    checked = true;
    LFE_HIP(hipMemsetAsync(c->dred, 0, sizeof(double), c->stream));
    for (int k = 0; k < F; ++k) {
      const int f = order[k];
      auto& fe = c->fe[f];
      if (k == F - 1) {  // its projection used the others' final effects: T is its check term
        LFE_TRY(d3_ycheck(c, f, fe.T, p));
      } else if (k == 0) {  // the next sweep's first projection: |alpha_next - alpha| = |mean_g(y~)|
        LFE_TRY(d3_project(c, f, fe.alpha, c->alpha_spare, true));
        first_ready = true;
      } else {  // the y column's cross term from the final effects
        int ns = 0;
        LFE_TRY(d3_cross(c, f, true, &ns));
        const bool local = c->world == 1 || (c->owner_on && f == c->L.P);
        LFE_TRY(d3_reduce(c, c->d3.runs[f], ns, fe.G, fe.R, f, nullptr, nullptr, false));
        if (!local) LFE_TRY(allreduce_sum_f64(c, fe.R, (size_t)fe.G));
        LFE_TRY(d3_ycheck(c, f, fe.R, 1));
      }
    }
    // owner-sharded rows: each rank's check covers its own primary levels (and its digits flag
    // their own effects); the max over ranks of both
    LFE_HIP(hipMemcpyAsync(c->dred + 1, c->rflag, sizeof(double), hipMemcpyDeviceToDevice, c->stream));
    if (c->owner_on) LFE_TRY(allreduce_max_u64(c, reinterpret_cast<uint64_t*>(c->dred), 2));
    double rb[2];
    LFE_TRY(d2h_sync(c, rb, c->dred, sizeof(rb)));
    last = rb[0];
    if (rb[1] != 0.0) {  // a tile's digits lost precision: lfe_demean redoes the solve without them
      c->dense_coarse = true;
      break;
    }
    if (last < tol) break;
  }
  if (!c->dense_coarse && !checked) {  // the loop ended without a check
    if (c->owner_on) LFE_TRY(allreduce_max_u64(c, reinterpret_cast<uint64_t*>(c->rflag), 1));
    double f = 0.0;
    LFE_TRY(d2h_sync(c, &f, c->rflag, sizeof(double)));
    c->dense_coarse = f != 0.0;
  }
  // the last FE's T used every other FE's final effects; so did order[0]'s from the stop test
  c->d3.t_final = (1u << order[F - 1]) | (checked ? 1u << f0 : 0u);
  *iterations_out = iterations;
  *last_out = last;
  return LFE_OK;
}

int dense3_final_T(lfe_ctx* c) {
  for (int f = 0; f < c->F; ++f) {
    if (c->d3.t_final & (1u << f)) continue;
    auto& fe = c->fe[f];
    int ns = 0;
    LFE_TRY(d3_cross(c, f, false, &ns));
    const int64_t m = (int64_t)fe.G * c->p;
    LFE_TRY(d3_reduce(c, c->d3.runs[f], ns, m, fe.T, f, nullptr, nullptr, false));
    if (!(c->world == 1 || (c->owner_on && f == c->L.P))) LFE_TRY(allreduce_sum_f64(c, fe.T, (size_t)m));
    c->d3.t_final |= 1u << f;
  }
  return LFE_OK;
}

}  // namespace lfe

// leanfe HIP engine — YOCO compression on the device.
//
//   compress_polars (compress.py:282-358): group the rows by every regressor, FE
//   and cluster column; each group becomes one record with
//     _n = count (weighted: sum w),  _sum_y = sum (w) y,  _sum_y_sq = sum (w) y^2,
//     _mean_y = _sum_y / _n,  _wts = sqrt(_n)
//   and the WLS on the records with FE dummies (build_design_matrix + solve_wls,
//   :503-747) is the exact LSDV fit.
//
// Group-by: 64-bit hashes of the key columns are radix-sorted; a new record starts
// at every hash change.  Neighbours with equal hashes are compared value by value;
// if two different rows ever share a hash, those runs are split exactly into
// their distinct rows (first-appearance order) and the (record id, row) pairs are
// sorted once more, so records are always contiguous and exact.  Per-record sums
// are segmented gather-sums of (w, w y, w y^2) rows (seg_gather_sum).
//
// The records then replace the loaded rows in the context (weights = _n), so the
// rest of the engine — singleton-free layout, weighted alternating projections to
// machine precision (the FWL form of the LSDV normal equations), the weighted Gram
// and lfe_resid_yoco — runs on them unchanged.
#include "lfe_internal.h"

#include <algorithm>

namespace lfe {

static int fail(int code, const char* msg) {
  set_error(msg);
  return code;
}

constexpr int kMaxKeyCodes = kMaxFE + kMaxCl;
constexpr int kMaxSplit = 64;  // distinct rows sharing one 64-bit hash that the exact split handles

struct RecArgs {
  const double* X;  // [p][ld]; column 0 = y, columns 1..p-1 are key columns
  const double* w;  // [ld] or nullptr
  int64_t ld, n;
  int p;
  int ni;           // FE code arrays, then cluster code arrays
  const int32_t* icol[kMaxKeyCodes];
  int hash_bits;    // 64; fewer only to exercise the collision path in tests
};

__device__ __forceinline__ bool rec_equal(const RecArgs& a, int64_t i, int64_t j) {
  for (int c = 1; c < a.p; ++c)
    if (canon_bits(a.X[(int64_t)c * a.ld + i]) != canon_bits(a.X[(int64_t)c * a.ld + j])) return false;
  for (int f = 0; f < a.ni; ++f)
    if (a.icol[f][i] != a.icol[f][j]) return false;
  return true;
}

__global__ void k_rec_hash(RecArgs a, uint64_t* __restrict__ keys, int32_t* __restrict__ rows) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t h = 0x2545f4914f6cdd1dull;
    for (int c = 1; c < a.p; ++c) h = fmix64(h ^ canon_bits(a.X[(int64_t)c * a.ld + i]));
    for (int f = 0; f < a.ni; ++f) h = fmix64(h ^ (uint64_t)(uint32_t)a.icol[f][i] ^ ((uint64_t)(f + 1) << 40));
    keys[i] = a.hash_bits >= 64 ? h : (h & ((1ull << a.hash_bits) - 1));
    rows[i] = (int32_t)i;
  }
}

// flag[q] = hash change; count neighbours with equal hashes but different rows
__global__ void k_rec_heads(RecArgs a, const uint64_t* __restrict__ K, const int32_t* __restrict__ R,
                            int32_t* __restrict__ flag, int32_t* __restrict__ nmismatch) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < a.n; q += (int64_t)gridDim.x * blockDim.x) {
    const bool head = q == 0 || K[q] != K[q - 1];
    flag[q] = head ? 1 : 0;
    if (!head && !rec_equal(a, R[q], R[q - 1])) atomicAdd(nmismatch, 1);
  }
}

// Collision path.  One thread per hash run (run index h = scan[q] at its head): the
// run's rows get sub ids 0..d-1 in first-appearance order; dcount[h] = d.
__global__ void k_rec_split(RecArgs a, const uint64_t* __restrict__ K, const int32_t* __restrict__ R,
                            const int32_t* __restrict__ scan, int32_t* __restrict__ sub, int32_t* __restrict__ dcount,
                            int32_t* __restrict__ overflow) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < a.n; q += (int64_t)gridDim.x * blockDim.x) {
    if (!(q == 0 || K[q] != K[q - 1])) continue;
    int32_t rep[kMaxSplit];
    int d = 0;
    for (int64_t e = q; e < a.n && K[e] == K[q]; ++e) {
      const int32_t r = R[e];
      int s = 0;
      while (s < d && !rec_equal(a, r, rep[s])) ++s;
      if (s == d) {
        if (d == kMaxSplit) {
          atomicAdd(overflow, 1);
          s = 0;
        } else {
          rep[d++] = r;
        }
      }
      sub[e] = s;
    }
    dcount[scan[q]] = d;
  }
}

// key of position q after the split: record id = base of its run + sub id
__global__ void k_rec_ids(const uint64_t* __restrict__ K, const int32_t* __restrict__ scan,
                          const int32_t* __restrict__ base, const int32_t* __restrict__ sub, int64_t n,
                          uint64_t* __restrict__ out) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
    const bool head = q == 0 || K[q] != K[q - 1];
    const int32_t h = scan[q] + (head ? 0 : -1);
    out[q] = (uint64_t)(base[h] + sub[q]);
  }
}

__global__ void k_key_change(const uint64_t* __restrict__ K, int64_t n, int32_t* __restrict__ flag) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x)
    flag[q] = (q == 0 || K[q] != K[q - 1]) ? 1 : 0;
}

__global__ void k_rec_segoff(const uint64_t* __restrict__ K, const int32_t* __restrict__ scan, int64_t n,
                             int32_t* __restrict__ seg_off) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
    if (q == 0 || K[q] != K[q - 1]) seg_off[scan[q]] = (int32_t)q;
    if (q + 1 == n) seg_off[scan[n]] = (int32_t)n;
  }
}

// per-row sufficient statistics, row-major [n][3]: (w, w y, w y^2) (compress.py:324-337)
__global__ void k_rec_vals(const double* __restrict__ y, const double* __restrict__ w, int64_t n,
                           double* __restrict__ vals) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double wi = w ? w[i] : 1.0, yi = y[i];
    vals[3 * i + 0] = wi;
    vals[3 * i + 1] = yi * wi;
    vals[3 * i + 2] = yi * yi * wi;
  }
}

struct RecOut {
  double* X;        // [p][ldr]
  int64_t ldr;
  int32_t* icol[kMaxKeyCodes];  // [ni][ldr]
  double* wn;       // [ldr] _n
  double* sy;       // [ldr] _sum_y
  double* syy;      // [ldr] _sum_y_sq
};

// record g from its first row: key columns copied, _mean_y = _sum_y / _n (compress.py:343-346)
__global__ void k_rec_build(RecArgs a, const int32_t* __restrict__ R, const int32_t* __restrict__ seg_off,
                            const double* __restrict__ agg, int32_t G, RecOut o) {
  for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x) {
    const int64_t r0 = R[seg_off[g]];
    const double n = agg[3 * (int64_t)g], s1 = agg[3 * (int64_t)g + 1], s2 = agg[3 * (int64_t)g + 2];
    o.X[g] = s1 / n;
    for (int c = 1; c < a.p; ++c) o.X[(int64_t)c * o.ldr + g] = a.X[(int64_t)c * a.ld + r0];
    for (int f = 0; f < a.ni; ++f) o.icol[f][g] = a.icol[f][r0];
    o.wn[g] = n;
    o.sy[g] = s1;
    o.syy[g] = s2;
  }
}

template <typename T>
static int tmp_alloc(T** p, size_t elems) {
  LFE_HIP(hipMalloc(reinterpret_cast<void**>(p), sizeof(T) * std::max<size_t>(elems, 1)));
  return LFE_OK;
}

struct TmpBufs {
  std::vector<void*> v;
  ~TmpBufs() {
    for (void* p : v) (void)hipFree(p);
  }
  template <typename T>
  int get(T** p, size_t elems) {
    LFE_TRY(tmp_alloc(p, elems));
    v.push_back(*p);
    return LFE_OK;
  }
};

// permuted copy of a record array into layout order (rec_lay), identity when unpermuted
__global__ void k_gather_lay(const double* __restrict__ src, const int32_t* __restrict__ orig, int64_t n,
                             double* __restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[orig ? orig[i] : i];
}

int records_layout(lfe_ctx* c) {
  const int64_t n = c->n;
  LFE_TRY(ensure_f64(c, c->rec_lay, c->rec_lay_cap, 2 * (size_t)c->ld));
  LFE_TRY(ensure_layout_orig(c));
  if (n > 0) {
    hipLaunchKernelGGL(k_gather_lay, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, c->rec_sy,
                       c->L.orig, n, c->rec_lay);
    hipLaunchKernelGGL(k_gather_lay, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, c->rec_syy,
                       c->L.orig, n, c->rec_lay + c->ld);
  }
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

}  // namespace lfe

using namespace lfe;

int lfe_compress(lfe_ctx* c, int64_t* n_records_out) {
  if (c && c->sw.on) {
    set_error("not available with streamed X (lfe_load_codes)");
    return LFE_ESTATE;
  }
  if (!c) return fail(LFE_EINVAL, "null context");
  if (!n_records_out) return fail(LFE_EINVAL, "null pointer");
  if (!c->loaded) return fail(LFE_ESTATE, "lfe_load first");
  if (c->records) return fail(LFE_ESTATE, "the loaded rows are already compressed records");
  if (c->world > 1) return fail(LFE_EINVAL, "lfe_compress groups one process's rows only");
  if ((int)c->cl.size() > kMaxCl) return fail(LFE_EINVAL, "too many cluster columns to compress on");
  LFE_HIP(hipSetDevice(c->device));
  const int64_t n = c->n;
  const int p = c->p, F = c->F, m = (int)c->cl.size();
  RecArgs a{};
  a.X = c->X;
  a.w = c->w;
  a.ld = c->ld;
  a.n = n;
  a.p = p;
  for (int f = 0; f < F; ++f) a.icol[a.ni++] = c->fe[f].code;
  for (int j = 0; j < m; ++j) a.icol[a.ni++] = c->cl[j];
  const char* hb_env = knob("LFE_ROW_HASH_BITS");  // tests: a short hash forces collisions
  const int hb = hb_env ? atoi(hb_env) : 64;
  a.hash_bits = hb >= 4 && hb <= 64 ? hb : 64;

  TmpBufs tmp;
  int32_t G = 0;
  const int32_t* R = nullptr;
  const uint64_t* K = nullptr;
  auto& W = c->clw;
  if (n > 0) {
    LFE_TRY(ensure_sort_ws(c, (size_t)n));
    hipLaunchKernelGGL(k_rec_hash, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, a, W.keys[0],
                       W.rows[0]);
    LFE_HIP(hipGetLastError());
    int buf = 0;
    LFE_TRY(radix_sort(c, n, a.hash_bits, &buf));
    K = W.keys[buf];
    R = W.rows[buf];
    LFE_TRY(ensure_iscratch(c, 4));
    LFE_HIP(hipMemsetAsync(c->iscratch, 0, 4 * sizeof(int32_t), c->stream));
    LFE_HIP(hipMemsetAsync(W.flag + n, 0, sizeof(int32_t), c->stream));
    hipLaunchKernelGGL(k_rec_heads, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, a, K, R, W.flag,
                       c->iscratch);
    LFE_HIP(hipGetLastError());
    LFE_TRY(exclusive_scan(c, W.flag, n + 1));
    int32_t nmis = 0;
    LFE_TRY(d2h_sync(c, &nmis, c->iscratch, sizeof(int32_t)));
    if (nmis > 0) {
      // different rows share a hash: split those runs exactly, re-key by record id, sort again
      int32_t runs = 0;
      LFE_TRY(d2h_sync(c, &runs, W.flag + n, sizeof(int32_t)));
      int32_t *sub = nullptr, *dcount = nullptr;
      LFE_TRY(tmp.get(&sub, (size_t)n));
      LFE_TRY(tmp.get(&dcount, (size_t)runs + 1));
      hipLaunchKernelGGL(k_rec_split, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, a, K, R, W.flag,
                         sub, dcount, c->iscratch + 1);
      LFE_HIP(hipGetLastError());
      LFE_TRY(exclusive_scan(c, dcount, (int64_t)runs + 1));
      int32_t hov[2] = {0, 0};
      LFE_TRY(d2h_sync(c, hov, c->iscratch, 2 * sizeof(int32_t)));
      if (hov[1] > 0) return fail(LFE_EINVAL, "more than 64 distinct rows share one row hash");
      int32_t nrec = 0;
      LFE_TRY(d2h_sync(c, &nrec, dcount + runs, sizeof(int32_t)));
      // (record id, row) pairs into the other buffer, then a stable sort by record id
      const int other = 1 - buf;
      hipLaunchKernelGGL(k_rec_ids, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, K, W.flag, dcount,
                         sub, n, W.keys[other]);
      LFE_HIP(hipGetLastError());
      // radix_sort sorts buffer 0: move the pairs there
      if (other != 0) {
        LFE_HIP(hipMemcpyAsync(W.keys[0], W.keys[other], sizeof(uint64_t) * n, hipMemcpyDeviceToDevice, c->stream));
        LFE_HIP(hipMemcpyAsync(W.rows[0], R, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, c->stream));
      } else {
        LFE_HIP(hipMemcpyAsync(W.rows[0], R, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, c->stream));
      }
      LFE_TRY(radix_sort(c, n, bit_length((uint64_t)std::max(nrec - 1, 1)), &buf));
      K = W.keys[buf];
      R = W.rows[buf];
      LFE_HIP(hipMemsetAsync(W.flag + n, 0, sizeof(int32_t), c->stream));
      hipLaunchKernelGGL(k_key_change, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, K, n, W.flag);
      LFE_HIP(hipGetLastError());
      LFE_TRY(exclusive_scan(c, W.flag, n + 1));
    }
    LFE_TRY(d2h_sync(c, &G, W.flag + n, sizeof(int32_t)));
  }

  // per-record sums over contiguous segments, then the record arrays
  const int64_t ldr = std::max<int64_t>(((int64_t)G + 63) / 64 * 64, 64);
  RecOut o{};
  o.ldr = ldr;
  LFE_TRY(tmp.get(&o.X, (size_t)p * ldr));
  for (int f = 0; f < a.ni; ++f) LFE_TRY(tmp.get(&o.icol[f], (size_t)ldr));
  LFE_TRY(tmp.get(&o.wn, (size_t)ldr));
  LFE_TRY(tmp.get(&o.sy, (size_t)ldr));
  LFE_TRY(tmp.get(&o.syy, (size_t)ldr));
  if (n > 0) {
    int32_t *seg_off = nullptr, *ufirst = nullptr;
    double *vals = nullptr, *agg = nullptr;
    LFE_TRY(tmp.get(&seg_off, (size_t)G + 1));
    LFE_TRY(tmp.get(&ufirst, (size_t)seg_units_needed(n)));
    LFE_TRY(tmp.get(&vals, 3 * (size_t)n));
    LFE_TRY(tmp.get(&agg, 3 * (size_t)G));
    hipLaunchKernelGGL(k_rec_segoff, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, K, W.flag, n,
                       seg_off);
    hipLaunchKernelGGL(k_rec_vals, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, c->X, c->w, n, vals);
    LFE_HIP(hipGetLastError());
    LFE_TRY(seg_gather_sum(c, seg_off, G, ufirst, n, R, vals, 3, 3, agg, K_MISC));
    hipLaunchKernelGGL(k_rec_build, dim3(grid_for(G, kBlock, 8192)), dim3(kBlock), 0, c->stream, a, R, seg_off, agg,
                       G, o);
    LFE_HIP(hipGetLastError());
  }
  // the records replace the rows (device-to-device load; weights = _n)
  std::vector<int32_t> fe_levels(F), cl_levels(c->cl_levels);
  for (int f = 0; f < F; ++f) fe_levels[f] = c->fe[f].G;
  std::vector<const double*> cols(p);
  for (int j = 0; j < p; ++j) cols[j] = o.X + (size_t)j * ldr;
  std::vector<const int32_t*> fcodes(F), ccodes(m);
  for (int f = 0; f < F; ++f) fcodes[f] = o.icol[f];
  for (int j = 0; j < m; ++j) ccodes[j] = o.icol[F + j];
  LFE_HIP(hipStreamSynchronize(c->stream));
  LFE_TRY(lfe_load(c, G, p, cols.data(), F, fcodes.data(), fe_levels.data(), o.wn, LFE_DEVICE));
  if (m > 0) LFE_TRY(lfe_load_clusters(c, m, ccodes.data(), cl_levels.data(), LFE_DEVICE));
  LFE_TRY(ensure_f64(c, c->rec_sy, c->rec_sy_cap, (size_t)c->ld));
  LFE_TRY(ensure_f64(c, c->rec_syy, c->rec_syy_cap, (size_t)c->ld));
  if (G > 0) {
    LFE_HIP(hipMemcpyAsync(c->rec_sy, o.sy, sizeof(double) * G, hipMemcpyDeviceToDevice, c->stream));
    LFE_HIP(hipMemcpyAsync(c->rec_syy, o.syy, sizeof(double) * G, hipMemcpyDeviceToDevice, c->stream));
  }
  LFE_HIP(hipStreamSynchronize(c->stream));
  c->records = true;
  c->rows_in = n;
  *n_records_out = G;
  return LFE_OK;
}

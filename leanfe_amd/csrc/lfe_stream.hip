// leanfe HIP engine — clustered standard errors of out-of-core fits (data larger than HBM).
//
// The cluster scores S_c = sum_{i in c} u_i r_i (w_i) (std_errors.py:289-441, the one-hot SpMM
// W_C'(X (.) e) of compress.py:817-851) need the residual of every row, which a streamed fit
// only has chunk by chunk.  The cluster structure itself lives in the resident codes:
//   1. lfe_stream_clusters: for every subset (a mask over the loaded cluster columns, the
//      intersections of std_errors.py:399-408) the rows' keys are radix-sorted and grouped once
//      (lfe_keys.hip / lfe_cluster.hip), and every input row gets its dense cluster id
//      (-1: a dropped singleton);
//   2. every residual chunk (pass 2, or the IV pass 4) writes its score rows; per subset they
//      are sorted by cluster id inside the chunk (stable), summed per cluster in that order and
//      added into the subset's table S[G][k] in chunk order - one add per cluster and chunk, so
//      the sums do not depend on scheduling;
//   3. lfe_stream_cluster_meats: S'S per subset (the table Gram of lfe_gram.hip) and the counts.
//      A sharded engine (every rank streams its own rows; cluster codes are global) keeps each local
//      cluster's intersection key, and the per-cluster sums go through the owner-partitioned exchange
//      of the resident fits (owner_meat, lfe_cluster.hip): a cluster split across ranks is merged by
//      its owner, and only the k x k meats and the cluster counts are all-reduced.
#include "lfe_internal.h"

#include <algorithm>

namespace lfe {

struct SclKeyArgs {
  int m, F;
  const int32_t* cl[kMaxCl];     // cluster codes (input order)
  uint64_t mult[kMaxCl];
  const int32_t* code[kMaxFE];   // FE codes (input order) and pre-filter counts: the singleton drop
  const int32_t* cnt_pre[kMaxFE];
  int64_t n;
  uint64_t drop;
  uint64_t* keys;
  int32_t* rows;
};

__global__ void k_scl_keys(SclKeyArgs a) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
    bool keep = true;
    for (int f = 0; f < a.F; ++f) keep = keep && a.cnt_pre[f][a.code[f][i]] > 1;
    uint64_t key = 0;
    for (int j = 0; j < a.m; ++j) key += (uint64_t)(uint32_t)a.cl[j][i] * a.mult[j];
    a.keys[i] = keep ? key : a.drop;
    a.rows[i] = (int32_t)i;
  }
}

// dense cluster id of every row from the sorted keys and the scan of their segment heads
__global__ void k_scl_cid(const uint64_t* __restrict__ K, const int32_t* __restrict__ R,
                          const int32_t* __restrict__ scan, int64_t n, uint64_t drop, int32_t* __restrict__ cid) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
    const bool head = q == 0 || K[q] != K[q - 1];
    cid[R[q]] = K[q] == drop ? -1 : scan[q] - (head ? 0 : 1);
  }
}

// the chunk's rows as (cluster id, chunk row) pairs; dropped rows carry key = G (sorted last)
__global__ void k_scl_chunk_keys(const int32_t* __restrict__ cid, int64_t rows, int32_t G, uint64_t* __restrict__ keys,
                                 int32_t* __restrict__ idx) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t h = cid[i];
    keys[i] = h < 0 ? (uint64_t)G : (uint64_t)h;
    idx[i] = (int32_t)i;
  }
}

// S[key(h)] += the chunk's sum of cluster h (each key once per chunk: no two adds meet)
__global__ void k_scl_accum(const uint64_t* __restrict__ K, const int32_t* __restrict__ seg_off, int32_t Gc,
                            const double* __restrict__ part, int k, double* __restrict__ S) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < (int64_t)Gc * k;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t h = e / k;
    const int j = (int)(e % k);
    S[(int64_t)K[seg_off[h]] * k + j] += part[e];
  }
}

// the key of every local cluster (the first row of its sorted segment)
__global__ void k_scl_ukey(const uint64_t* __restrict__ K, const int32_t* __restrict__ seg_off, int32_t G,
                           uint64_t* __restrict__ ukey) {
  for (int h = blockIdx.x * blockDim.x + threadIdx.x; h < G; h += gridDim.x * blockDim.x) ukey[h] = K[seg_off[h]];
}

void free_stream_clusters(lfe_ctx* c) {
  auto& w = c->sw;
  for (auto& p : w.cid) dfree_any(p);
  for (auto& p : w.S) dfree_any(p);
  for (auto& p : w.ukey) dfree_any(p);
  w.cid.clear();
  w.S.clear();
  w.ukey.clear();
  w.span.clear();
  w.S_cap.clear();
  w.G.clear();
  w.masks.clear();
  w.ks = 0;
  dfree_any(w.sc);
  w.sc_cap = 0;
}

int stream_clusters_prep(lfe_ctx* c, int n_subsets, const int32_t* masks) {
  auto& w = c->sw;
  const int m = (int)c->cl.size();
  for (int s = 0; s < n_subsets; ++s)
    if (masks[s] <= 0 || masks[s] >= (1 << m)) {
      set_error("subset mask must select loaded cluster columns");
      return LFE_EINVAL;
    }
  free_stream_clusters(c);
  const int64_t n = c->n;
  LFE_TRY(ensure_sort_ws(c, (size_t)std::max<int64_t>(n, 1)));
  auto& W = c->clw;
  for (int s = 0; s < n_subsets; ++s) {
    SclKeyArgs ka{};
    uint64_t span = 1;
    for (int j = 0; j < m; ++j) {
      if (!(masks[s] >> j & 1)) continue;
      if (ka.m == kMaxCl) {
        set_error("too many cluster columns in one subset");
        return LFE_EINVAL;
      }
      const uint64_t g = (uint64_t)c->cl_levels[j];
      if (span > ((1ull << 62) / g)) {
        set_error("cluster intersection span exceeds 2^62");
        return LFE_EINVAL;
      }
      ka.cl[ka.m] = c->cl[j];
      ka.mult[ka.m] = span;
      ++ka.m;
      span *= g;
    }
    ka.F = c->F;
    for (int f = 0; f < c->F; ++f) {
      ka.code[f] = c->fe[f].code;
      ka.cnt_pre[f] = c->fe[f].cnt_pre;
    }
    ka.n = n;
    ka.drop = span;
    ka.keys = W.keys[0];
    ka.rows = W.rows[0];
    int32_t* cid = nullptr;
    LFE_HIP(hipMalloc(reinterpret_cast<void**>(&cid), sizeof(int32_t) * (size_t)std::max<int64_t>(n, 1)));
    w.cid.push_back(cid);
    w.masks.push_back(masks[s]);
    int32_t G = 0;
    int buf = 0;
    if (n > 0) {
      {
        ProfScope _ps(c, K_CLUSTER_SORT);
        hipLaunchKernelGGL(k_scl_keys, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, ka);
      }
      LFE_HIP(hipGetLastError());
      LFE_TRY(radix_sort(c, n, bit_length(span), &buf));
      LFE_TRY(group_sorted(c, n, span, W.keys[buf], W.rows[buf], nullptr, 0, &G));
      hipLaunchKernelGGL(k_scl_cid, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, W.keys[buf],
                         W.rows[buf], W.flag, n, span, cid);
      LFE_HIP(hipGetLastError());
    }
    uint64_t* ukey = nullptr;
    if (c->world > 1) {  // sharded: the owner exchange needs every local cluster's key
      LFE_HIP(hipMalloc(reinterpret_cast<void**>(&ukey), sizeof(uint64_t) * (size_t)std::max(G, 1)));
      if (G > 0)
        hipLaunchKernelGGL(k_scl_ukey, dim3(grid_for(G)), dim3(kBlock), 0, c->stream, W.keys[buf], W.seg_off, G, ukey);
      LFE_HIP(hipGetLastError());
    }
    w.ukey.push_back(ukey);
    w.span.push_back(span);
    w.G.push_back(G);
    w.S.push_back(nullptr);
    w.S_cap.push_back(0);
  }
  return LFE_OK;
}

// the current chunk's score rows (w.sc, [rows][ks]) into every subset's cluster sums
int stream_clusters_chunk(lfe_ctx* c, int64_t row0, int64_t rows) {
  auto& w = c->sw;
  auto& W = c->clw;
  const int k = w.ks;
  LFE_TRY(ensure_sort_ws(c, (size_t)std::max<int64_t>(rows, 1)));
  for (size_t s = 0; s < w.cid.size(); ++s) {
    const int32_t G = w.G[s];
    if (G == 0 || rows == 0) continue;
    hipLaunchKernelGGL(k_scl_chunk_keys, dim3(grid_for(rows, kBlock, 8192)), dim3(kBlock), 0, c->stream,
                       w.cid[s] + row0, rows, G, W.keys[0], W.rows[0]);
    LFE_HIP(hipGetLastError());
    int buf = 0;
    LFE_TRY(radix_sort(c, rows, bit_length((uint64_t)G), &buf));
    int32_t Gc = 0;
    LFE_TRY(group_sorted(c, rows, (uint64_t)G, W.keys[buf], W.rows[buf], w.sc, k, &Gc));
    if (Gc > 0) {
      ProfScope _ps(c, K_CLUSTER_SCATTER);
      hipLaunchKernelGGL(k_scl_accum, dim3(grid_for((int64_t)Gc * k)), dim3(kBlock), 0, c->stream, W.keys[buf],
                         W.seg_off, Gc, c->clS, k, w.S[s]);
    }
    LFE_HIP(hipGetLastError());
  }
  return LFE_OK;
}

int stream_cluster_meats(lfe_ctx* c, double* meats, int64_t* G_out) {
  auto& w = c->sw;
  const int k = w.ks;
  for (size_t s = 0; s < w.cid.size(); ++s) {
    G_out[s] = w.G[s];
    double* meat = meats + s * (size_t)k * k;
    if (c->world > 1) {  // every rank takes part, whatever its local cluster count
      LFE_TRY(owner_meat(c, w.ukey[s], nullptr, w.S[s], w.G[s], k, w.span[s], meat, G_out + s));
      continue;
    }
    if (w.G[s] == 0 || k == 0) {
      std::fill(meat, meat + (size_t)k * k, 0.0);
      continue;
    }
    LFE_TRY(launch_table_gram(c, w.S[s], w.G[s], k, meat));
  }
  return LFE_OK;
}

}  // namespace lfe

// leanfe HIP engine — owner re-shard of loaded row blocks (multi-GPU).
//
// The reference's loop (polars_impl.py:490-526) has no notion of shards.  Across GPUs the
// cheapest schedule for two FEs gives each rank every row of a contiguous range of the
// primary FE's levels ("owner-sharded rows"): the primary FE's counts, group sums, cross
// term and effects are then complete on every rank, and a sweep all-reduces only the
// secondary FE's table (88 KB at config 3 instead of the primary's 8.8 MB).
//
// A caller that loads contiguous row blocks (lfe_load on every rank) gets there with one
// all-to-all:
//   1. level counts of the owner FE, all-reduced (int32) -> every rank computes the same
//      level ranges [lo_r, hi_r), cut where the running row count crosses r N / world, so
//      ranks hold equal rows (up to one level's rows), not equal levels;
//   2. every local row's destination rank, a stable LSD radix sort of (dest, row) pairs
//      (the row order within a destination stays the input order);
//   3. every column (X, w, FE codes, loaded cluster columns) gathered in that order into a
//      staging buffer, the shard re-allocated for the rows it will receive, and one grouped
//      ncclSend / ncclRecv set per column moves the blocks (received in source-rank order);
//   4. lfe_ctx_set_owner(fe, lo_r, hi_r).
// Everything is deterministic: the counts are integers, the sort is stable and the received
// order is (source rank, source row).  The data crosses the fabric once per load, not per solve.
#include "lfe_internal.h"

#include <algorithm>
#include <cstdlib>

namespace lfe {

__global__ void k_level_counts(const int32_t* __restrict__ code, int64_t n, int32_t* __restrict__ cnt) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(&cnt[code[i]], 1);
}

// destination rank of every row (bounds[r] = lo_r, bounds[world] = G) as a sort key, rows = iota,
// and the rows per destination
__global__ void k_dest_keys(const int32_t* __restrict__ code, int64_t n, const int32_t* __restrict__ bounds,
                            int world, uint64_t* __restrict__ keys, int32_t* __restrict__ rows,
                            int32_t* __restrict__ per_dest) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t g = code[i];
    int lo = 0, hi = world;  // the rank r with bounds[r] <= g < bounds[r + 1]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (bounds[mid] <= g) lo = mid;
      else hi = mid;
    }
    keys[i] = (uint64_t)lo;
    rows[i] = (int32_t)i;
    atomicAdd(&per_dest[lo], 1);
  }
}

template <typename T>
__global__ void k_gather_rows(const T* __restrict__ src, const int32_t* __restrict__ rows, int64_t n,
                              T* __restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[rows[i]];
}

int reshard_owner(lfe_ctx* c, int fe, int32_t* lo_out, int32_t* hi_out) {
  if (fe < 0 || fe >= c->F) {
    set_error("bad owner FE");
    return LFE_EINVAL;
  }
  if (c->sw.on || c->records || c->loading) {
    set_error("owner re-shard needs resident columns (not streamed X, records or an unfinished chunked load)");
    return LFE_ESTATE;
  }
  const int world = c->world, rank = c->rank;
  const int32_t G = c->fe[fe].G;
  const int64_t n = c->n;
  const int p = c->p, F = c->F, m = (int)c->cl.size();
  const bool weighted = c->w != nullptr;
  // 1. global level counts -> level ranges balanced by rows
  int32_t* cnt = nullptr;
  LFE_TRY(ensure_i32(c, c->pcounts, c->pcounts_elems, (size_t)G + 2 * world + 2));
  cnt = c->pcounts;
  LFE_HIP(hipMemsetAsync(cnt, 0, sizeof(int32_t) * ((size_t)G + 2 * world + 2), c->stream));
  if (n > 0)
    hipLaunchKernelGGL(k_level_counts, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, c->fe[fe].code,
                       n, cnt);
  LFE_HIP(hipGetLastError());
  LFE_TRY(allreduce_sum_i32(c, cnt, (size_t)G));
  std::vector<int32_t> hc(G);
  LFE_TRY(d2h_sync(c, hc.data(), cnt, sizeof(int32_t) * G));
  int64_t total = 0;
  for (int32_t v : hc) total += v;
  std::vector<int32_t> bounds(world + 1, G);
  {
    int64_t run = 0;
    int g = 0;
    for (int r = 0; r < world; ++r) {
      const int64_t target = total * r / world;  // the first level whose preceding rows reach it
      while (g < G && run < target) run += hc[g++];
      bounds[r] = g;
    }
    bounds[world] = G;
  }
  std::vector<int64_t> rank_rows(world, 0);
  for (int r = 0; r < world; ++r)
    for (int g = bounds[r]; g < bounds[r + 1]; ++g) rank_rows[r] += hc[g];
  // every refusal before the data moves is decided from the same all-reduced counts on every rank,
  // so all ranks return the same code and keep their blocks (nothing has moved yet)
  for (int r = 0; r < world; ++r)
    if (rank_rows[r] == 0) {
      set_error("owner re-shard: a rank would hold no rows (fewer populated levels than ranks)");
      return LFE_EINVAL;
    }
  if (*std::max_element(rank_rows.begin(), rank_rows.end()) >= (int64_t)INT32_MAX) {
    set_error("owner re-shard: a rank would hold 2^31 rows or more");
    return LFE_EINVAL;
  }
  *lo_out = bounds[rank];
  *hi_out = bounds[rank + 1];
  if (world == 1) return LFE_OK;

  // 2. destinations, stable sort by destination
  int32_t* dbounds = cnt + G;          // [world + 1]
  int32_t* per_dest = dbounds + world + 1;  // [world]
  LFE_TRY(h2d_small(c, dbounds, bounds.data(), sizeof(int32_t) * (world + 1)));
  LFE_TRY(ensure_sort_ws(c, (size_t)std::max<int64_t>(n, 1)));
  auto& W = c->clw;
  if (n > 0)
    hipLaunchKernelGGL(k_dest_keys, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, c->fe[fe].code, n,
                       dbounds, world, W.keys[0], W.rows[0], per_dest);
  LFE_HIP(hipGetLastError());
  int buf = 0;
  if (n > 0) LFE_TRY(radix_sort(c, n, bit_length((uint64_t)(world - 1)), &buf));
  std::vector<int32_t> send_rows(world);
  LFE_TRY(d2h_sync(c, send_rows.data(), per_dest, sizeof(int32_t) * world));
  // who sends how many rows to whom
  std::vector<int32_t> mat((size_t)world * world, 0);
  {
    LFE_TRY(ensure_i32(c, W.ocnt, W.ocnt_cap, (size_t)world * world));
    int32_t* dmat = W.ocnt;
    for (int q = 0; q < world; ++q) mat[(size_t)rank * world + q] = send_rows[q];
    LFE_TRY(h2d_small(c, dmat, mat.data(), sizeof(int32_t) * world * world));
    LFE_TRY(allreduce_sum_i32(c, dmat, (size_t)world * world));
    LFE_TRY(d2h_sync(c, mat.data(), dmat, sizeof(int32_t) * world * world));
  }
  std::vector<int64_t> soff(world + 1, 0), roff(world + 1, 0);
  for (int q = 0; q < world; ++q) {
    soff[q + 1] = soff[q] + send_rows[q];
    roff[q + 1] = roff[q] + mat[(size_t)q * world + rank];
  }
  const int64_t n_new = roff[world];

  // 3. gather every column in destination order into staging (f64 columns, then int32 columns).
  // The staging copy and the re-allocated shard coexist: every rank checks that both fit (the old
  // shard's columns are freed in between) and the ranks agree on the outcome before anything moves,
  // so a rank short of memory makes every rank return LFE_ENOMEM with its block in place.
  const int nf64 = p + (weighted ? 1 : 0), ni32 = F + m;
  const size_t ldn = (size_t)std::max<int64_t>(n, 1);
  const size_t row_bytes = sizeof(double) * nf64 + sizeof(int32_t) * std::max(ni32, 1);
  double* sf = nullptr;
  int32_t* si = nullptr;
  int32_t short_mem = 0;
  if (hipMalloc(reinterpret_cast<void**>(&sf), sizeof(double) * ldn * nf64) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&si), sizeof(int32_t) * ldn * std::max(ni32, 1)) != hipSuccess) {
    short_mem = 1;
  } else {
    size_t free_b = 0, total_b = 0;
    const size_t need = row_bytes * (size_t)std::max<int64_t>(n_new, 1), have_old = row_bytes * ldn;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess || free_b + have_old < need + ((size_t)256 << 20))
      short_mem = 1;
  }
  (void)hipGetLastError();  // a failed allocation is decided below, with the other ranks
  if (c->test_hooks & LFE_TEST_SHORT_MEMORY) short_mem = 1;  // tests: this rank short of memory
  {
    int32_t* dflag = W.ocnt;  // [world * world] is free again after the counts above
    LFE_TRY(h2d_small(c, dflag, &short_mem, sizeof(int32_t)));
    LFE_TRY(allreduce_sum_i32(c, dflag, 1));
    int32_t any_short = 0;
    LFE_TRY(d2h_sync(c, &any_short, dflag, sizeof(int32_t)));
    if (any_short) {
      if (sf) (void)hipFree(sf);
      if (si) (void)hipFree(si);
      set_error("owner re-shard: a rank lacks device memory for the staging copy and the new shard "
                "(every rank keeps its row block)");
      return LFE_ENOMEM;
    }
  }
  struct Staging {
    double* f;
    int32_t* i;
    ~Staging() {
      if (f) (void)hipFree(f);
      if (i) (void)hipFree(i);
    }
  } stage{sf, si};
  const int32_t* perm = W.rows[buf];
  if (n > 0) {
    const dim3 grid(grid_for(n, kBlock, 8192));
    for (int j = 0; j < p; ++j)
      hipLaunchKernelGGL(k_gather_rows<double>, grid, dim3(kBlock), 0, c->stream, c->X + (size_t)j * c->ld, perm, n,
                         sf + (size_t)j * ldn);
    if (weighted)
      hipLaunchKernelGGL(k_gather_rows<double>, grid, dim3(kBlock), 0, c->stream, c->w, perm, n, sf + (size_t)p * ldn);
    for (int f = 0; f < F; ++f)
      hipLaunchKernelGGL(k_gather_rows<int32_t>, grid, dim3(kBlock), 0, c->stream, c->fe[f].code, perm, n,
                         si + (size_t)f * ldn);
    for (int j = 0; j < m; ++j)
      hipLaunchKernelGGL(k_gather_rows<int32_t>, grid, dim3(kBlock), 0, c->stream, c->cl[j], perm, n,
                         si + (size_t)(F + j) * ldn);
    LFE_HIP(hipGetLastError());
  }
  // the shard re-allocated for the rows it receives (every derived table is rebuilt by the
  // next lfe_drop_singletons)
  std::vector<int32_t> levels(F), cl_levels(c->cl_levels);
  for (int f = 0; f < F; ++f) levels[f] = c->fe[f].G;
  LFE_HIP(hipStreamSynchronize(c->stream));
  LFE_TRY(alloc_shard(c, n_new, p, F, levels.data(), weighted));
  c->cl.assign(m, nullptr);
  c->cl_levels = cl_levels;
  for (int j = 0; j < m; ++j) LFE_HIP(hipMalloc(reinterpret_cast<void**>(&c->cl[j]), sizeof(int32_t) * c->ld));
  // 4. one grouped send / receive set per column
  std::vector<size_t> so(world), sb(world), ro(world), rb(world);
  auto move = [&](const char* send, size_t esize, char* recv) -> int {
    for (int q = 0; q < world; ++q) {
      so[q] = (size_t)soff[q] * esize;
      sb[q] = (size_t)send_rows[q] * esize;
      ro[q] = (size_t)roff[q] * esize;
      rb[q] = (size_t)(roff[q + 1] - roff[q]) * esize;
    }
    return alltoallv_bytes(c, send, so.data(), sb.data(), recv, ro.data(), rb.data());
  };
  for (int j = 0; j < p; ++j)
    LFE_TRY(move(reinterpret_cast<const char*>(sf + (size_t)j * ldn), 8, reinterpret_cast<char*>(c->X + (size_t)j * c->ld)));
  if (weighted)
    LFE_TRY(move(reinterpret_cast<const char*>(sf + (size_t)p * ldn), 8, reinterpret_cast<char*>(c->w)));
  for (int f = 0; f < F; ++f)
    LFE_TRY(move(reinterpret_cast<const char*>(si + (size_t)f * ldn), 4, reinterpret_cast<char*>(c->fe[f].code)));
  for (int j = 0; j < m; ++j)
    LFE_TRY(move(reinterpret_cast<const char*>(si + (size_t)(F + j) * ldn), 4, reinterpret_cast<char*>(c->cl[j])));
  LFE_HIP(hipStreamSynchronize(c->stream));  // the staging buffers are freed on return
  c->loaded = true;
  return LFE_OK;
}

}  // namespace lfe

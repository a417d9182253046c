// leanfe HIP engine — device keys: a stable LSD radix sort of (u64 key, int32 row)
// pairs, and the two host-prep steps built on it:
//   - lfe_factorize_ids: integer id column -> dense codes in sorted-unique order,
//     i.e. np.unique(..., return_inverse=True) (the code values do not affect any
//     result, polars_impl.py:118-139; only group membership does);
//   - lfe_count_distinct_rows: the exact number of distinct (x, FE) rows,
//     estimate_compression_ratio's numerator (compress.py:187-253, the
//     `lf.select(key_cols).unique()` count, key_cols = x_cols + fe_cols,
//     compress.py:249-250), over all loaded rows.
// Distinct rows: 64-bit row hashes are sorted; equal rows have equal hashes, so a
// new row starts at every hash change.  Neighbours with equal hashes are compared
// value by value; if two different rows ever share a hash (about 1e-4 odds per 50M
// rows) the affected runs are recounted exactly, so the count is exact.
// Float values compare as in a group-by: -0.0 == 0.0 and every NaN equal.
#include "lfe_internal.h"

#include <algorithm>

namespace lfe {

static int fail(int code, const char* msg) {
  set_error(msg);
  return code;
}

constexpr int kRsThreads = 512;
constexpr int kRsWaves = kRsThreads / 64;
constexpr int kRsPer = 16;                       // items per thread
constexpr int kRsItems = kRsThreads * kRsPer;    // items per block (a tile)
constexpr int kRsBits = 8;
constexpr int kRsBins = 1 << kRsBits;

// digit counts of tile b: counts[d * nblk + b]
__global__ __launch_bounds__(kRsThreads) void k_rs_hist(const uint64_t* __restrict__ keys, int64_t n, int shift,
                                                        int nblk, int32_t* __restrict__ counts) {
  __shared__ int32_t h[kRsBins];
  const int tid = threadIdx.x;
  for (int j = tid; j < kRsBins; j += kRsThreads) h[j] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kRsItems;
#pragma unroll 4
  for (int s = 0; s < kRsPer; ++s) {
    const int64_t i = base + s * kRsThreads + tid;
    if (i < n) atomicAdd(&h[(int)((keys[i] >> shift) & (kRsBins - 1))], 1);
  }
  __syncthreads();
  for (int j = tid; j < kRsBins; j += kRsThreads) counts[(int64_t)j * nblk + blockIdx.x] = h[j];
}

// Stable scatter of one tile.  Wave w owns items [b*8192 + w*1024, +1024) in 16 steps of 64;
// within a step, lanes with equal digits are matched by 8 ballots and ranked by lane; per-wave
// running counts in LDS carry the rank across steps.  The tile is then sorted by digit in LDS
// (position = the digit's start in the tile + the waves before + the rank) and written out by
// consecutive threads, so every digit's run of the tile (~32 items) leaves as one contiguous
// store sequence instead of 32 scattered ones (the partial lines at the runs' ends are the
// only ones the L2 has to merge).
__global__ __launch_bounds__(kRsThreads) void k_rs_scatter(const uint64_t* __restrict__ kin,
                                                           const int32_t* __restrict__ vin,
                                                           uint64_t* __restrict__ kout, int32_t* __restrict__ vout,
                                                           int64_t n, int shift, int nblk,
                                                           const int32_t* __restrict__ scanned) {
  __shared__ int32_t cnt[kRsWaves][kRsBins];
  __shared__ int32_t dstart[kRsBins + 1];  // digit starts in the tile
  __shared__ int32_t gbase[kRsBins];       // digit starts in the output, minus dstart
  __shared__ uint64_t skey[kRsItems];
  __shared__ int32_t sval[kRsItems];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int j = tid; j < kRsWaves * kRsBins; j += kRsThreads) (&cnt[0][0])[j] = 0;
  __syncthreads();
  const int64_t t0 = (int64_t)blockIdx.x * kRsItems;
  const int64_t b0 = t0 + (int64_t)w * (kRsItems / kRsWaves);
  const int tlen = (int)min((int64_t)kRsItems, n - t0);
  const uint64_t lt = (1ull << lane) - 1ull;
  uint64_t key[kRsPer];
  int32_t val[kRsPer];
  int rank[kRsPer];
#pragma unroll
  for (int s = 0; s < kRsPer; ++s) {
    const int64_t i = b0 + s * 64 + lane;
    const bool valid = i < n;
    key[s] = valid ? kin[i] : 0ull;
    val[s] = valid ? vin[i] : 0;
  }
#pragma unroll
  for (int s = 0; s < kRsPer; ++s) {
    const bool valid = b0 + s * 64 + lane < n;
    const int d = (int)((key[s] >> shift) & (kRsBins - 1));
    uint64_t m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < kRsBits; ++b) {
      const bool bit = (d >> b) & 1;
      const uint64_t bb = __ballot(bit);
      m &= bit ? bb : ~bb;
    }
    const int before = __popcll(m & lt);
    rank[s] = cnt[w][d] + before;  // every lane reads before the leader below writes
    if (valid && before == 0) cnt[w][d] += __popcll(m);
  }
  __syncthreads();
  if (tid < kRsBins) {  // per digit: exclusive prefix over waves, the digit's tile total
    int run = 0;
#pragma unroll
    for (int w2 = 0; w2 < kRsWaves; ++w2) {
      const int t = cnt[w2][tid];
      cnt[w2][tid] = run;
      run += t;
    }
    dstart[tid] = run;  // total for now
  }
  __syncthreads();
  if (tid < 64) {  // exclusive scan of the digit totals (4 digits per lane, then the wave)
    int v[4], sum = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[q] = dstart[tid * 4 + q];
      sum += v[q];
    }
    int x = sum;
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(x, off, 64);
      if (lane >= off) x += y;
    }
    int run = x - sum;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int d = tid * 4 + q;
      gbase[d] = scanned[(int64_t)d * nblk + blockIdx.x] - run;
      dstart[d] = run;
      run += v[q];
    }
  }
  __syncthreads();
#pragma unroll
  for (int s = 0; s < kRsPer; ++s) {
    if (b0 + s * 64 + lane >= n) continue;
    const int d = (int)((key[s] >> shift) & (kRsBins - 1));
    const int q = dstart[d] + cnt[w][d] + rank[s];
    skey[q] = key[s];
    sval[q] = val[s];
  }
  __syncthreads();
  for (int q = tid; q < tlen; q += kRsThreads) {
    const uint64_t k = skey[q];
    const int64_t pos = (int64_t)gbase[(int)((k >> shift) & (kRsBins - 1))] + q;
    kout[pos] = k;
    vout[pos] = sval[q];
  }
}


int bit_length(uint64_t v) {
  int b = 0;
  while (v) {
    ++b;
    v >>= 1;
  }
  return b;
}

int ensure_sort_ws(lfe_ctx* c, size_t n) {
  auto& W = c->clw;
  for (int b = 0; b < 2; ++b) {
    LFE_TRY(ensure_u64(c, W.keys[b], W.keys_cap[b], std::max<size_t>(n, 1)));
    LFE_TRY(ensure_i32(c, W.rows[b], W.rows_cap[b], std::max<size_t>(n, 1)));
  }
  LFE_TRY(ensure_i32(c, W.flag, W.flag_cap, n + 1));
  return LFE_OK;
}

// one stable pass of the workspace's (keys, rows) [0, n) from buffer cur to 1 - cur by the 8-bit
// digit at `shift`
int radix_pass(lfe_ctx* c, int64_t n, int shift, int cur, int kid) {
  auto& W = c->clw;
  if (n <= 0) return LFE_OK;
  const int nblk = (int)((n + kRsItems - 1) / kRsItems);
  LFE_TRY(ensure_i32(c, W.counts, W.counts_cap, (size_t)kRsBins * std::max(nblk, 1)));
  {
    ProfScope _ps(c, kid);
    hipLaunchKernelGGL(k_rs_hist, dim3(nblk), dim3(kRsThreads), 0, c->stream, W.keys[cur], n, shift, nblk, W.counts);
  }
  LFE_HIP(hipGetLastError());
  LFE_TRY(exclusive_scan(c, W.counts, (int64_t)kRsBins * nblk));
  {
    ProfScope _ps(c, kid);
    hipLaunchKernelGGL(k_rs_scatter, dim3(nblk), dim3(kRsThreads), 0, c->stream, W.keys[cur], W.rows[cur],
                       W.keys[1 - cur], W.rows[1 - cur], n, shift, nblk, W.counts);
  }
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

// sort (keys, rows) [0, n) of the workspace by the low `bits` bits; *out_buf = the
// buffer (0/1) holding the result
int radix_sort(lfe_ctx* c, int64_t n, int bits, int* out_buf) {
  int cur = 0;
  for (int shift = 0; shift < bits && n > 0; shift += kRsBits) {
    LFE_TRY(radix_pass(c, n, shift, cur, K_CLUSTER_SORT));
    cur = 1 - cur;
  }
  *out_buf = cur;
  return LFE_OK;
}

// ---------------------------------------------------------------------------
// factorization of integer ids
// ---------------------------------------------------------------------------

__global__ void k_minmax_i64(const int64_t* __restrict__ v, int64_t n, unsigned long long* __restrict__ out) {
  // out[0] = min, out[1] = max, as order-preserving unsigned (sign bit flipped)
  unsigned long long lo = ~0ull, hi = 0ull;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long u = (unsigned long long)v[i] ^ (1ull << 63);
    lo = u < lo ? u : lo;
    hi = u > hi ? u : hi;
  }
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long a = __shfl_down(lo, off, 64), b = __shfl_down(hi, off, 64);
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMin(&out[0], lo);
    atomicMax(&out[1], hi);
  }
}

__global__ void k_fz_keys(const int64_t* __restrict__ ids, int64_t n, unsigned long long lo_biased,
                          uint64_t* __restrict__ keys, int32_t* __restrict__ rows) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    keys[i] = ((unsigned long long)ids[i] ^ (1ull << 63)) - lo_biased;
    rows[i] = (int32_t)i;
  }
}

__global__ void k_key_heads(const uint64_t* __restrict__ K, int64_t n, int32_t* __restrict__ flag) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x)
    flag[q] = (q == 0 || K[q] != K[q - 1]) ? 1 : 0;
}

// code of row R[q] = rank of its key among the distinct keys
__global__ void k_fz_codes(const uint64_t* __restrict__ K, const int32_t* __restrict__ scan,
                           const int32_t* __restrict__ R, int64_t n, int32_t* __restrict__ codes) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
    const bool head = q == 0 || K[q] != K[q - 1];
    codes[R[q]] = scan[q] + (head ? 0 : -1);
  }
}

// ---------------------------------------------------------------------------
// factorization of strings (Arrow layout: int64 offsets [n + 1] + one byte buffer)
// ---------------------------------------------------------------------------
// 64-bit string hashes are radix-sorted; equal strings have equal hashes, so a new
// group starts at every hash change.  Neighbours with equal hashes are compared byte
// by byte; a hash run that holds different strings (about 1e-8 odds for 1e6 distinct
// strings) is split exactly by k_str_exact, so the grouping is always exact.

struct StrArgs {
  const int64_t* off;   // [n + 1]
  const uint8_t* data;  // off[n] bytes
  int64_t n;
  int hash_bits;        // 64; fewer only to exercise the collision path in tests
};

__device__ __forceinline__ uint64_t str_hash(const uint8_t* s, int64_t len) {
  uint64_t h = fmix64(0x9e3779b97f4a7c15ull ^ (uint64_t)len);
  int64_t i = 0;
  for (; i + 8 <= len; i += 8) {
    uint64_t w = 0;
#pragma unroll
    for (int b = 0; b < 8; ++b) w |= (uint64_t)s[i + b] << (8 * b);
    h = fmix64(h ^ w);
  }
  uint64_t w = 0;
  for (int b = 0; i + b < len; ++b) w |= (uint64_t)s[i + b] << (8 * b);
  return fmix64(h ^ w ^ 0x5bd1e995ull);
}

__device__ __forceinline__ bool str_equal(const StrArgs& a, int64_t i, int64_t j) {
  const int64_t li = a.off[i + 1] - a.off[i], lj = a.off[j + 1] - a.off[j];
  if (li != lj) return false;
  const uint8_t* si = a.data + a.off[i];
  const uint8_t* sj = a.data + a.off[j];
  for (int64_t b = 0; b < li; ++b)
    if (si[b] != sj[b]) return false;
  return true;
}

__global__ void k_str_keys(StrArgs a, uint64_t* __restrict__ keys, int32_t* __restrict__ rows) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t h = str_hash(a.data + a.off[i], a.off[i + 1] - a.off[i]);
    keys[i] = a.hash_bits >= 64 ? h : (h & ((1ull << a.hash_bits) - 1));
    rows[i] = (int32_t)i;
  }
}

// flag[q] = hash change; mm[q] = 1 where a neighbour has an equal hash but a different string
// (counted into nmismatch)
__global__ void k_str_heads(StrArgs a, const uint64_t* __restrict__ K, const int32_t* __restrict__ R,
                            int32_t* __restrict__ flag, int32_t* __restrict__ nmismatch, int32_t* __restrict__ mm) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < a.n; q += (int64_t)gridDim.x * blockDim.x) {
    const bool head = q == 0 || K[q] != K[q - 1];
    flag[q] = head ? 1 : 0;
    const bool mis = !head && !str_equal(a, R[q], R[q - 1]);
    mm[q] = mis ? 1 : 0;
    if (mis) atomicAdd(nmismatch, 1);
  }
}

// Collision path, step 1: adj = 0 at every run head, -1 elsewhere (a run of one string), and the
// head of every run holding a mismatch is marked flag = -1 (the mismatching position walks back
// to its head: collisions are rare, so are these walks)
__global__ void k_str_mark(const uint64_t* __restrict__ K, const int32_t* __restrict__ mm, int64_t n,
                           int32_t* __restrict__ flag, int32_t* __restrict__ adj) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
    const bool head = q == 0 || K[q] != K[q - 1];
    adj[q] = head ? 0 : -1;
    if (mm[q]) {
      int64_t h = q;
      while (h > 0 && K[h - 1] == K[q]) --h;
      flag[h] = -1;  // (every writer stores the same value)
    }
  }
}

// Step 2: exact split of the marked runs (one thread per marked head).  A run of d distinct
// strings sets flag[head] = d, and adj[i] = local index of member i's string (first-occurrence
// order in the run) minus d for every member but the head, so that after the exclusive scan of
// flag code(i) = scan[i] + adj[i] (k_str_codes).  Runs of one string keep step 1's adj and are not
// walked (a frequent string with no colliding neighbour costs nothing here).
__global__ void k_str_exact(StrArgs a, const uint64_t* __restrict__ K, const int32_t* __restrict__ R,
                            int32_t* __restrict__ flag, int32_t* __restrict__ adj) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < a.n; q += (int64_t)gridDim.x * blockDim.x) {
    if (flag[q] != -1) continue;
    int64_t e = q + 1;
    while (e < a.n && K[e] == K[q]) ++e;
    int32_t d = 0;
    for (int64_t i = q; i < e; ++i) {  // adj[i] = local index (first occurrence order)
      int64_t j = q;
      while (j < i && !str_equal(a, R[j], R[i])) ++j;
      adj[i] = j == i ? d++ : adj[j];
    }
    flag[q] = d;
    for (int64_t i = q + 1; i < e; ++i) adj[i] -= d;
  }
}

__global__ void k_str_codes(const int32_t* __restrict__ scan, const int32_t* __restrict__ adj,
                            const int32_t* __restrict__ R, int64_t n, int32_t* __restrict__ codes) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x)
    codes[R[q]] = scan[q] + adj[q];
}

// ---------------------------------------------------------------------------
// distinct rows
// ---------------------------------------------------------------------------

struct RowArgs {
  const double* X;   // [p][ld]; columns 1..p-1 are the regressors
  int64_t ld, n;
  int p, F;
  const int32_t* code[kMaxFE];
  int hash_bits;     // 64; fewer only to exercise the collision path in tests
};

__global__ void k_row_hash(RowArgs a, uint64_t* __restrict__ keys, int32_t* __restrict__ rows) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t h = 0x9e3779b97f4a7c15ull;
    for (int c = 1; c < a.p; ++c) h = fmix64(h ^ canon_bits(a.X[(int64_t)c * a.ld + i]));
    for (int f = 0; f < a.F; ++f) h = fmix64(h ^ (uint64_t)(uint32_t)a.code[f][i] ^ 0x5bd1e995ull);
    keys[i] = a.hash_bits >= 64 ? h : (h & ((1ull << a.hash_bits) - 1));
    rows[i] = (int32_t)i;
  }
}

__device__ __forceinline__ bool rows_equal(const RowArgs& a, int64_t i, int64_t j) {
  for (int c = 1; c < a.p; ++c)
    if (canon_bits(a.X[(int64_t)c * a.ld + i]) != canon_bits(a.X[(int64_t)c * a.ld + j])) return false;
  for (int f = 0; f < a.F; ++f)
    if (a.code[f][i] != a.code[f][j]) return false;
  return true;
}

// flag[q] = hash change; count neighbours with equal hashes but different rows
__global__ void k_dr_heads(RowArgs a, const uint64_t* __restrict__ K, const int32_t* __restrict__ R,
                           int32_t* __restrict__ flag, int32_t* __restrict__ nmismatch) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < a.n; q += (int64_t)gridDim.x * blockDim.x) {
    const bool head = q == 0 || K[q] != K[q - 1];
    flag[q] = head ? 1 : 0;
    if (!head && !rows_equal(a, R[q], R[q - 1])) atomicAdd(nmismatch, 1);
  }
}

// exact recount of hash runs holding different rows: one thread per run head;
// a run with mismatching neighbours counts its distinct rows by pairwise
// comparison and adds (distinct - 1) (the run was counted once)
__global__ void k_dr_exact(RowArgs a, const uint64_t* __restrict__ K, const int32_t* __restrict__ R,
                           unsigned long long* __restrict__ extra) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < a.n; q += (int64_t)gridDim.x * blockDim.x) {
    if (!(q == 0 || K[q] != K[q - 1])) continue;
    int64_t e = q + 1;
    bool mixed = false;
    while (e < a.n && K[e] == K[q]) {
      mixed = mixed || !rows_equal(a, R[e], R[e - 1]);
      ++e;
    }
    if (!mixed) continue;
    unsigned long long distinct = 0;
    for (int64_t i = q; i < e; ++i) {
      bool seen = false;
      for (int64_t j = q; j < i && !seen; ++j) seen = rows_equal(a, R[i], R[j]);
      distinct += seen ? 0 : 1;
    }
    atomicAdd(extra, distinct - 1);
  }
}

}  // namespace lfe

using namespace lfe;

int lfe_factorize_ids(lfe_ctx* c, int64_t n, const int64_t* ids, int32_t* codes_out, int32_t* n_levels_out) {
  if (!c) return fail(LFE_EINVAL, "null context");
  if (n < 0 || n >= (int64_t)INT32_MAX || (n > 0 && (!ids || !codes_out)) || !n_levels_out)
    return fail(LFE_EINVAL, "bad arguments");
  if (n == 0) {
    *n_levels_out = 0;
    return LFE_OK;
  }
  LFE_HIP(hipSetDevice(c->device));
  LFE_TRY(ensure_sort_ws(c, (size_t)n));
  auto& W = c->clw;
  int64_t* dids = reinterpret_cast<int64_t*>(W.keys[1]);  // raw ids staged in the second key buffer
  LFE_HIP(hipMemcpyAsync(dids, ids, sizeof(int64_t) * n, hipMemcpyHostToDevice, c->stream));
  LFE_TRY(ensure_dred(c, 2));
  unsigned long long* mm = reinterpret_cast<unsigned long long*>(c->dred);
  const unsigned long long init[2] = {~0ull, 0ull};
  LFE_TRY(h2d_small(c, mm, init, sizeof(init)));
  hipLaunchKernelGGL(k_minmax_i64, dim3(grid_for(n, kBlock, 1024)), dim3(kBlock), 0, c->stream, dids, n, mm);
  LFE_HIP(hipGetLastError());
  unsigned long long h[2];
  LFE_TRY(d2h_sync(c, h, mm, sizeof(h)));
  hipLaunchKernelGGL(k_fz_keys, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, dids, n, h[0], W.keys[0],
                     W.rows[0]);
  LFE_HIP(hipGetLastError());
  int buf = 0;
  LFE_TRY(radix_sort(c, n, bit_length(h[1] - h[0]), &buf));
  const uint64_t* K = W.keys[buf];
  const int32_t* R = W.rows[buf];
  LFE_HIP(hipMemsetAsync(W.flag + n, 0, sizeof(int32_t), c->stream));
  hipLaunchKernelGGL(k_key_heads, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, K, n, W.flag);
  LFE_HIP(hipGetLastError());
  LFE_TRY(exclusive_scan(c, W.flag, n + 1));
  // codes go to the other row buffer (free now), then to the host
  int32_t* dcodes = W.rows[1 - buf];
  hipLaunchKernelGGL(k_fz_codes, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, K, W.flag, R, n, dcodes);
  LFE_HIP(hipGetLastError());
  LFE_HIP(hipMemcpyAsync(codes_out, dcodes, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->stream));
  int32_t G = 0;
  LFE_TRY(d2h_sync(c, &G, W.flag + n, sizeof(int32_t)));
  *n_levels_out = G;
  return LFE_OK;
}

namespace {
// one-call device scratch (string offsets / bytes); hipFree waits for the device
struct ScratchBuf {
  void* p = nullptr;
  ~ScratchBuf() {
    if (p) (void)hipFree(p);
  }
};
}  // namespace

int lfe_factorize_strings(lfe_ctx* c, int64_t n, const int64_t* offsets, const uint8_t* data, int32_t* codes_out,
                          int32_t* n_levels_out) {
  if (!c) return fail(LFE_EINVAL, "null context");
  if (n < 0 || n >= (int64_t)INT32_MAX || !n_levels_out || (n > 0 && (!offsets || !codes_out)))
    return fail(LFE_EINVAL, "bad arguments");
  if (n == 0) {
    *n_levels_out = 0;
    return LFE_OK;
  }
  // the kernels index data with these offsets: they must start at 0 and never decrease
  if (offsets[0] != 0) return fail(LFE_EINVAL, "offsets[0] must be 0");
  for (int64_t i = 0; i < n; ++i)
    if (offsets[i + 1] < offsets[i]) return fail(LFE_EINVAL, "offsets must be non-decreasing");
  const int64_t nbytes = offsets[n];
  if (nbytes > 0 && !data) return fail(LFE_EINVAL, "null string data");
  LFE_HIP(hipSetDevice(c->device));
  ScratchBuf boff, bdata;
  LFE_HIP(hipMalloc(&boff.p, sizeof(int64_t) * (size_t)(n + 1)));
  LFE_HIP(hipMalloc(&bdata.p, (size_t)std::max<int64_t>(nbytes, 1)));
  StrArgs a{};
  a.off = static_cast<const int64_t*>(boff.p);
  a.data = static_cast<const uint8_t*>(bdata.p);
  a.n = n;
  const char* hb_env = knob("LFE_STR_HASH_BITS");  // tests: a short hash forces collisions
  const int hb = hb_env ? atoi(hb_env) : 64;
  a.hash_bits = hb >= 4 && hb <= 64 ? hb : 64;
  LFE_HIP(hipMemcpyAsync(boff.p, offsets, sizeof(int64_t) * (size_t)(n + 1), hipMemcpyHostToDevice, c->stream));
  if (nbytes > 0) LFE_HIP(hipMemcpyAsync(bdata.p, data, (size_t)nbytes, hipMemcpyHostToDevice, c->stream));
  LFE_TRY(ensure_sort_ws(c, (size_t)n));
  auto& W = c->clw;
  hipLaunchKernelGGL(k_str_keys, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, a, W.keys[0],
                     W.rows[0]);
  LFE_HIP(hipGetLastError());
  int buf = 0;
  LFE_TRY(radix_sort(c, n, a.hash_bits, &buf));
  const uint64_t* K = W.keys[buf];
  const int32_t* R = W.rows[buf];
  LFE_TRY(ensure_dred(c, 1));
  LFE_HIP(hipMemsetAsync(c->dred, 0, sizeof(double), c->stream));
  int32_t* nmis = reinterpret_cast<int32_t*>(c->dred);
  LFE_HIP(hipMemsetAsync(W.flag + n, 0, sizeof(int32_t), c->stream));
  // the sort's spare key buffer (n x u64): adj [n] and the mismatch marks [n]
  int32_t* adj = reinterpret_cast<int32_t*>(W.keys[1 - buf]);
  int32_t* mm = adj + n;
  hipLaunchKernelGGL(k_str_heads, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, a, K, R, W.flag,
                     nmis, mm);
  LFE_HIP(hipGetLastError());
  int32_t mismatches = 0;
  LFE_TRY(d2h_sync(c, &mismatches, nmis, sizeof(int32_t)));
  if (mismatches > 0) {
    hipLaunchKernelGGL(k_str_mark, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, K, mm, n, W.flag,
                       adj);
    LFE_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_str_exact, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, a, K, R, W.flag,
                       adj);
    LFE_HIP(hipGetLastError());
  }
  LFE_TRY(exclusive_scan(c, W.flag, n + 1));
  int32_t* dcodes = W.rows[1 - buf];
  if (mismatches > 0)
    hipLaunchKernelGGL(k_str_codes, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, W.flag, adj, R, n,
                       dcodes);
  else
    hipLaunchKernelGGL(k_fz_codes, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, K, W.flag, R, n,
                       dcodes);
  LFE_HIP(hipGetLastError());
  LFE_HIP(hipMemcpyAsync(codes_out, dcodes, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->stream));
  int32_t G = 0;
  LFE_TRY(d2h_sync(c, &G, W.flag + n, sizeof(int32_t)));
  *n_levels_out = G;
  return LFE_OK;
}

int lfe_count_distinct_rows(lfe_ctx* c, int n_x, int64_t* n_distinct_out) {
  if (c && c->sw.on) {
    set_error("not available with streamed X (lfe_load_codes)");
    return LFE_ESTATE;
  }
  if (!c) return fail(LFE_EINVAL, "null context");
  if (!n_distinct_out) return fail(LFE_EINVAL, "null pointer");
  if (!c->loaded) return fail(LFE_ESTATE, "lfe_load first");
  if (n_x >= c->p) return fail(LFE_EINVAL, "n_x exceeds the loaded regressor columns");
  if (c->world > 1) return fail(LFE_EINVAL, "lfe_count_distinct_rows counts one process's rows only");
  LFE_HIP(hipSetDevice(c->device));
  const int64_t n = c->n;
  if (n == 0) {
    *n_distinct_out = 0;
    return LFE_OK;
  }
  LFE_TRY(ensure_sort_ws(c, (size_t)n));
  auto& W = c->clw;
  RowArgs a{};
  a.X = c->X;
  a.ld = c->ld;
  a.n = n;
  a.p = n_x < 0 ? c->p : 1 + n_x;  // key: x columns 1..n_x (instruments after them are not keyed)
  a.F = c->F;
  for (int f = 0; f < c->F; ++f) a.code[f] = c->fe[f].code;
  const char* hb_env = knob("LFE_ROW_HASH_BITS");  // tests: a short hash forces collisions
  const int hb = hb_env ? atoi(hb_env) : 64;
  a.hash_bits = hb >= 4 && hb <= 64 ? hb : 64;
  hipLaunchKernelGGL(k_row_hash, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, a, W.keys[0], W.rows[0]);
  LFE_HIP(hipGetLastError());
  int buf = 0;
  LFE_TRY(radix_sort(c, n, a.hash_bits, &buf));
  const uint64_t* K = W.keys[buf];
  const int32_t* R = W.rows[buf];
  LFE_TRY(ensure_dred(c, 2));
  LFE_HIP(hipMemsetAsync(c->dred, 0, 2 * sizeof(double), c->stream));
  int32_t* nmis = reinterpret_cast<int32_t*>(c->dred);
  LFE_HIP(hipMemsetAsync(W.flag + n, 0, sizeof(int32_t), c->stream));
  hipLaunchKernelGGL(k_dr_heads, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, a, K, R, W.flag, nmis);
  LFE_HIP(hipGetLastError());
  LFE_TRY(exclusive_scan(c, W.flag, n + 1));
  int32_t hres[2] = {0, 0};
  LFE_TRY(d2h_sync(c, &hres[0], nmis, sizeof(int32_t)));
  LFE_TRY(d2h_sync(c, &hres[1], W.flag + n, sizeof(int32_t)));
  int64_t distinct = hres[1];
  if (hres[0] > 0) {
    unsigned long long* extra = reinterpret_cast<unsigned long long*>(c->dred) + 1;
    hipLaunchKernelGGL(k_dr_exact, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, c->stream, a, K, R, extra);
    LFE_HIP(hipGetLastError());
    unsigned long long ex = 0;
    LFE_TRY(d2h_sync(c, &ex, extra, sizeof(ex)));
    distinct += (int64_t)ex;
  }
  *n_distinct_out = distinct;
  return LFE_OK;
}

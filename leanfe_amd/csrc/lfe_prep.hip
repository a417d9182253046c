// leanfe HIP engine — row layout + singleton drop (polars_impl.py:477-482).
//
// Every later pass runs on a bucketed row layout: rows are grouped by
// buckets of the primary (highest-cardinality) FE P, bucket b holding the
// codes [b << s, (b+1) << s).  A group table slice of one bucket (2^s groups x
// a few columns) then fits in LDS, so group sums over P become LDS-privatised
// reductions instead of global atomics over a G_P x p table.
//
// Partition = stable counting sort by bucket, one wavefront per row chunk:
//   k_part_hist    per-wave bucket histogram -> counts[bucket][wave]
//   scan           exclusive scan of counts (bucket-major) -> destinations
//   k_part_scatter per-wave LDS cursors; rows written to their bucket slot
// Within one wave instruction same-bucket lanes are ranked in lane order by
// ballots, so the layout is a pure function of the codes and the geometry.
#include "lfe_internal.h"


#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace lfe {

#define GRID_STRIDE(i, n)                                                      \
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (n);   \
       i += (int64_t)gridDim.x * blockDim.x)

// ---------------------------------------------------------------------------
// histograms
// ---------------------------------------------------------------------------

// LDS-privatised histogram for G <= kLdsHistMax; flush of non-zero bins
__global__ __launch_bounds__(256) void k_hist_lds(const int32_t* __restrict__ code, int64_t n, int32_t G,
                                                  int32_t* __restrict__ cnt) {
  extern __shared__ int32_t h[];
  for (int g = threadIdx.x; g < G; g += blockDim.x) h[g] = 0;
  __syncthreads();
  // 4 rows per thread per trip (one 16-byte load); the tail n % 4 rows one by one
  const int64_t n4 = n >> 2;
  const int4* c4 = reinterpret_cast<const int4*>(code);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const int4 v = c4[i];
    atomicAdd(&h[v.x], 1);
    atomicAdd(&h[v.y], 1);
    atomicAdd(&h[v.z], 1);
    atomicAdd(&h[v.w], 1);
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(&h[code[i]], 1);
  __syncthreads();
  for (int g = threadIdx.x; g < G; g += blockDim.x)
    if (h[g]) atomicAdd(&cnt[g], h[g]);
}

// Key ranges of kHistRange counters (128 KB of LDS) for G > kLdsHistMax: block (x, y) counts the
// codes in [y R, (y + 1) R) of its rows in LDS and flushes its non-zero bins with coalesced adds.
// Per-row global atomics into a 1e5-level table (config 4's second FE) ran at ~25 G adds/s:
// 1.96 ms for 50M rows; the ranges read the codes once per range instead.
constexpr int kHistRange = 32768;
constexpr int kHistMaxRanges = 8;
__global__ __launch_bounds__(1024) void k_hist_lds_range(const int32_t* __restrict__ code, int64_t n, int32_t G,
                                                         int32_t* __restrict__ cnt) {
  extern __shared__ int32_t h[];
  const int32_t k0 = (int32_t)blockIdx.y * kHistRange, nk = min(kHistRange, G - k0);
  for (int g = threadIdx.x; g < nk; g += blockDim.x) h[g] = 0;
  __syncthreads();
  const int64_t n4 = n >> 2;
  const int4* c4 = reinterpret_cast<const int4*>(code);
  auto one = [&](int32_t v) {
    const uint32_t d = (uint32_t)(v - k0);
    if (d < (uint32_t)nk) atomicAdd(&h[d], 1);
  };
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const int4 v = c4[i];
    one(v.x);
    one(v.y);
    one(v.z);
    one(v.w);
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    one(code[i]);
  __syncthreads();
  for (int g = threadIdx.x; g < nk; g += blockDim.x)
    if (h[g]) atomicAdd(&cnt[k0 + g], h[g]);
}

__global__ void k_hist_global(const int32_t* __restrict__ code, int64_t n, int32_t* __restrict__ cnt) {
  GRID_STRIDE(i, n) atomicAdd(&cnt[code[i]], 1);
}

// per-chunk bucket histogram, chunk = rows [w*cw, (w+1)*cw) -> counts[bucket][chunk]
// (z: the drop's tables and counters zeroed by the same grid, one launch fewer; n == 0 ranges: none)
__global__ __launch_bounds__(256) void k_part_hist(const int32_t* __restrict__ code, int64_t n, int s, int nb,
                                                   int64_t cw, int nw, int32_t* __restrict__ counts, ZeroArgs z) {
  extern __shared__ int32_t h[];
  const int w = blockIdx.x;
  zero_ranges_part(z, (int64_t)w * blockDim.x + threadIdx.x, (int64_t)gridDim.x * blockDim.x);
  for (int b = threadIdx.x; b < nb; b += blockDim.x) h[b] = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)w * cw, r1 = min(n, r0 + cw);
  // 16-byte code loads (chunk starts are multiples of 4 rows; the shard's tail is scalar)
  const int64_t v1 = r0 + ((r1 - r0) & ~(int64_t)3);
  for (int64_t i = r0 + 4 * (int64_t)threadIdx.x; i < v1; i += 4 * (int64_t)blockDim.x) {
    const int4 g = *reinterpret_cast<const int4*>(code + i);
    atomicAdd(&h[g.x >> s], 1);
    atomicAdd(&h[g.y >> s], 1);
    atomicAdd(&h[g.z >> s], 1);
    atomicAdd(&h[g.w >> s], 1);
  }
  for (int64_t i = v1 + threadIdx.x; i < r1; i += blockDim.x) atomicAdd(&h[code[i] >> s], 1);
  __syncthreads();
  for (int b = threadIdx.x; b < nb; b += blockDim.x) counts[(int64_t)b * nw + w] = h[b];
}

// ---------------------------------------------------------------------------
// exclusive scan of int32 (3 kernels: block scan, scan of block sums, add)
// ---------------------------------------------------------------------------

constexpr int kScanPer = 8;                 // elements per thread
constexpr int kScanBlock = 256 * kScanPer;  // elements per block

__device__ __forceinline__ int32_t block_excl_scan(int32_t v, int32_t* tmp, int32_t* total) {
  // wave inclusive scan
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int32_t x = v;
  for (int off = 1; off < 64; off <<= 1) {
    int32_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) tmp[wave] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t acc = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) {
      int32_t t = tmp[k];
      tmp[k] = acc;
      acc += t;
    }
    *total = acc;
  }
  __syncthreads();
  return x - v + tmp[wave];
}

// Up to two independent arrays per launch: blocks [0, nb1) scan a1[0, m1), the rest a2[0, m2).
struct ScanPair {
  int32_t* a1;
  int64_t m1;
  int64_t nb1;
  int32_t* a2;
  int64_t m2;
  __device__ __forceinline__ int32_t* arr(int64_t& blk, int64_t& m) const {
    if (blk < nb1) {
      m = m1;
      return a1;
    }
    blk -= nb1;
    m = m2;
    return a2;
  }
};

// a thread's kScanPer consecutive elements: two 16-byte accesses when all lie inside the array
// (base is a multiple of 8 elements; element-wise 4-byte accesses put the lanes of one
// instruction 32 bytes apart, eight instructions per 2 KB: 0.5 TB/s on config 4's 49M-entry scans)
static_assert(kScanPer == 8, "two int4 per thread");
__device__ __forceinline__ void scan_load8(const int32_t* a, int64_t base, int64_t m, int32_t (&v)[8]) {
  if (base + 8 <= m) {
    const int4 x = *reinterpret_cast<const int4*>(a + base), y = *reinterpret_cast<const int4*>(a + base + 4);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
    v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = base + k < m ? a[base + k] : 0;
  }
}
__device__ __forceinline__ void scan_store8(int32_t* a, int64_t base, int64_t m, const int32_t (&v)[8]) {
  if (base + 8 <= m) {
    *reinterpret_cast<int4*>(a + base) = int4{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<int4*>(a + base + 4) = int4{v[4], v[5], v[6], v[7]};
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (base + k < m) a[base + k] = v[k];
  }
}

__global__ __launch_bounds__(256) void k_scan_blocks(ScanPair sp, int32_t* __restrict__ sums) {
  __shared__ int32_t tmp[8];
  __shared__ int32_t total;
  int64_t blk = blockIdx.x, m;
  int32_t* __restrict__ a = sp.arr(blk, m);
  const int64_t base = blk * kScanBlock + (int64_t)threadIdx.x * kScanPer;
  int32_t v[kScanPer];
  scan_load8(a, base, m, v);
  int32_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) s += v[k];
  int32_t off = block_excl_scan(s, tmp, &total);
  int32_t o[kScanPer];
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    o[k] = off;
    off += v[k];
  }
  scan_store8(a, base, m, o);
  if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

// block sums of both arrays: [0, nb1) and [nb1, nb1 + nb2), each scanned from 0
__global__ __launch_bounds__(1024) void k_scan_top(int32_t* __restrict__ sums, int nb1, int nb2) {
  __shared__ int32_t tmp[16];
  __shared__ int32_t total;
  for (int seg = 0; seg < 2; ++seg) {
    int32_t* sg = sums + (seg ? nb1 : 0);
    const int nblocks = seg ? nb2 : nb1;
    int32_t carry = 0;
    for (int base = 0; base < nblocks; base += blockDim.x) {
      const int i = base + threadIdx.x;
      const int32_t v = i < nblocks ? sg[i] : 0;
      const int32_t ex = block_excl_scan(v, tmp, &total);
      if (i < nblocks) sg[i] = ex + carry;
      __syncthreads();
      carry += total;
      __syncthreads();
    }
  }
}

__global__ __launch_bounds__(256) void k_scan_add(ScanPair sp, const int32_t* __restrict__ sums) {
  int64_t blk = blockIdx.x, m;
  int32_t* __restrict__ a = sp.arr(blk, m);
  const int64_t base = blk * kScanBlock + (int64_t)threadIdx.x * kScanPer;
  const int32_t add = sums[blockIdx.x];
  int32_t v[kScanPer];
  scan_load8(a, base, m, v);
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) v[k] += add;
  scan_store8(a, base, m, v);
}

__global__ void k_gather_bstart(const int32_t* __restrict__ scanned, int nb, int nw, int32_t* __restrict__ out) {
  for (int b = blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += gridDim.x * blockDim.x)
    out[b] = scanned[(int64_t)b * nw];
}

// k_scan_add for few blocks (<= kScanFewBlocks): every block forms its own offset, the sum of the
// block sums before it in its array (integer adds: any order), so k_scan_top's launch goes.
// gather: out[b] = a1[b * gstride] for b < gn after the add (the partition's bucket starts).
constexpr int kScanFewBlocks = 2048;
__global__ __launch_bounds__(256) void k_scan_add_few(ScanPair sp, const int32_t* __restrict__ sums,
                                                      int32_t* __restrict__ gout, int64_t gstride, int gn) {
  __shared__ int32_t ws[4];
  int64_t blk = blockIdx.x, m;
  const int64_t first = blk < sp.nb1 ? 0 : sp.nb1;  // this array's first block
  int32_t* __restrict__ a = sp.arr(blk, m);
  int32_t part = 0;
  for (int64_t j = first + threadIdx.x; j < (int64_t)blockIdx.x; j += 256) part += sums[j];
  for (int off = 32; off > 0; off >>= 1) part += __shfl_down(part, off, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = part;
  __syncthreads();
  const int32_t add = (ws[0] + ws[1]) + (ws[2] + ws[3]);
  const int64_t base = blk * kScanBlock + (int64_t)threadIdx.x * kScanPer;
  const bool g = gout != nullptr && blockIdx.x < sp.nb1;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k)
    if (base + k < m) {
      const int32_t v = a[base + k] + add;
      a[base + k] = v;
      if (g && (base + k) % gstride == 0 && (base + k) / gstride < gn) gout[(base + k) / gstride] = v;
    }
}

constexpr int64_t kScanFusedMax = 96;  // blocks of the one-launch ticketed scan (k_scan_fused)

// Up to kScanFusedMax blocks in one launch: a block takes the next ticket (the dispatch order, so
// it waits only on blocks that are running), scans its 2048 elements, publishes its sum tagged with
// the launch's epoch, then adds the published sums of the blocks before it in its array (integer
// adds: any order) - k_scan_blocks + k_scan_add_few without the kernel boundary.  status needs no
// zeroing between launches: a word of another epoch reads as not yet published.
__global__ __launch_bounds__(256) void k_scan_fused(ScanPair sp, unsigned long long* __restrict__ status,
                                                    unsigned int* __restrict__ ticket, unsigned int epoch, int nblocks,
                                                    int32_t* __restrict__ gout, int64_t gstride, int gn,
                                                    unsigned int* __restrict__ done, unsigned long long* __restrict__ msg,
                                                    unsigned long long seq) {
  __shared__ int32_t tmp[8];
  __shared__ int32_t total;
  __shared__ int id_s;
  __shared__ int32_t ws[4];
  if (threadIdx.x == 0) {
    const unsigned int t = atomicAdd(ticket, 1u);
    if (t == (unsigned int)nblocks - 1) atomicExch(ticket, 0u);  // the last ticket: reset for the next launch
    id_s = (int)t;
  }
  __syncthreads();
  const int id = id_s;
  int64_t blk = id, m;
  const int64_t first = blk < sp.nb1 ? 0 : sp.nb1;  // this array's first block
  int32_t* __restrict__ a = sp.arr(blk, m);
  const int64_t base = blk * kScanBlock + (int64_t)threadIdx.x * kScanPer;
  int32_t v[kScanPer];
  scan_load8(a, base, m, v);
  int32_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) s += v[k];
  int32_t off = block_excl_scan(s, tmp, &total);
  if (threadIdx.x == 0)
    __hip_atomic_store(&status[id], ((unsigned long long)epoch << 32) | (unsigned int)total, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_AGENT);
  int32_t part = 0;
  for (int64_t j = first + threadIdx.x; j < (int64_t)id; j += 256) {
    unsigned long long w;
    int spin = 0;  // bounded: a lost publication would give a wrong scan, never a hung queue
    do {
      w = __hip_atomic_load(&status[j], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    } while ((unsigned int)(w >> 32) != epoch && ++spin < (1 << 22));
    part += (int32_t)(unsigned int)w;
  }
  for (int o = 32; o > 0; o >>= 1) part += __shfl_down(part, o, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = part;
  __syncthreads();
  off += (ws[0] + ws[1]) + (ws[2] + ws[3]);
  int32_t o8[kScanPer];
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    o8[k] = off;
    off += v[k];
  }
  scan_store8(a, base, m, o8);
  if (gout && id < sp.nb1)
#pragma unroll
    for (int k = 0; k < kScanPer; ++k)
      if (base + k < m && (base + k) % gstride == 0 && (base + k) / gstride < gn) gout[(base + k) / gstride] = o8[k];
  // the gathered values (the partition's bucket starts) to the host message by the last block
  if (msg && last_block_done(done) && threadIdx.x == 0) host_msg_publish_i32(msg, seq, gout, gn);
}

static int exclusive_scan_g(lfe_ctx* c, int32_t* a1, int64_t m1, int32_t* a2, int64_t m2, int32_t* gout,
                            int64_t gstride, int gn, unsigned long long* gout_seq = nullptr) {
  const int64_t nb1 = (m1 + kScanBlock - 1) / kScanBlock, nb2 = a2 ? (m2 + kScanBlock - 1) / kScanBlock : 0;
  const int64_t nblocks = nb1 + nb2;
  if (nblocks == 0) return LFE_OK;
  LFE_TRY(ensure_pcounts(c, 0, (size_t)nblocks + 1));
  if (((uintptr_t)a1 | (uintptr_t)a2) & 15) {  // scan_load8 / scan_store8: 16-byte accesses
    set_error("exclusive_scan: arrays must be 16-byte aligned");
    return LFE_EINVAL;
  }
  const ScanPair sp{a1, m1, nb1, a2, m2};
  ProfScope _ps(c, K_SCAN);
  // one launch for few blocks: every block reads the published sums of all blocks before it, so the
  // reads grow with the square of the blocks (292 blocks, the headline's partition scan: 28 us against
  // 13 us for k_scan_blocks + k_scan_add_few; 37 blocks, the 8-rank shard's: 11 against 14 us)
  if (nblocks <= kScanFusedMax) {
    if (!c->scan_status) {
      LFE_HIP(hipMalloc(reinterpret_cast<void**>(&c->scan_status), sizeof(unsigned long long) * kScanFewBlocks));
      LFE_HIP(hipMemsetAsync(c->scan_status, 0, sizeof(unsigned long long) * kScanFewBlocks, c->stream));
      c->scan_epoch = 0;
    }
    if (++c->scan_epoch == 0) c->scan_epoch = 1;  // (0 is the zeroed buffer's tag)
    // gout_seq: the gathered values to the host message (one rank, fits the message)
    const bool msg = gout_seq && gout && host_msg_on(c) && (size_t)gn <= kHostMsgBytes / 8;
    if (msg) *gout_seq = next_msg_seq(c);
    hipLaunchKernelGGL(k_scan_fused, dim3((unsigned)nblocks), dim3(256), 0, c->stream, sp, c->scan_status,
                       c->gsync + GS_SCAN, c->scan_epoch, (int)nblocks, gout, gstride, gn, c->gsync + GS_SCAN_DONE,
                       msg ? c->dmsg : nullptr, msg ? *gout_seq : 0ull);
    LFE_HIP(hipGetLastError());
    return LFE_OK;
  }
  hipLaunchKernelGGL(k_scan_blocks, dim3((unsigned)nblocks), dim3(256), 0, c->stream, sp, c->psums);
  if (nblocks <= kScanFewBlocks) {
    hipLaunchKernelGGL(k_scan_add_few, dim3((unsigned)nblocks), dim3(256), 0, c->stream, sp, c->psums, gout, gstride,
                       gn);
  } else {
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(1024), 0, c->stream, c->psums, (int)nb1, (int)nb2);
    hipLaunchKernelGGL(k_scan_add, dim3((unsigned)nblocks), dim3(256), 0, c->stream, sp, c->psums);
    if (gout) hipLaunchKernelGGL(k_gather_bstart, dim3(grid_for(gn)), dim3(kBlock), 0, c->stream, a1, gn,
                                 (int)gstride, gout);
  }
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

int exclusive_scan2(lfe_ctx* c, int32_t* a1, int64_t m1, int32_t* a2, int64_t m2) {
  return exclusive_scan_g(c, a1, m1, a2, m2, nullptr, 1, 0);
}

int exclusive_scan(lfe_ctx* c, int32_t* a, int64_t m) { return exclusive_scan2(c, a, m, nullptr, 0); }

// ---------------------------------------------------------------------------
// partition scatter
// ---------------------------------------------------------------------------

// the work items from the mapped staging (host memory, coherent) into the device buffer
__global__ __launch_bounds__(256) void k_copy_staged(const int4* __restrict__ src, int4* __restrict__ dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

// LDS-staged scatter.  A workgroup owns a chunk of kPartThreads*PER rows
// (wave w: PER*64 consecutive rows).  It ranks its rows by bucket in LDS, then
// moves every column through an LDS stage in bucket order, so consecutive
// threads write consecutive addresses of one bucket run (~chunk/nb rows per run)
// instead of 8-byte scatters.
//
// Ranking is deterministic by construction: every wave owns its own cursor per
// bucket, and within one wave instruction the lanes of one bucket are ranked in
// lane order from ballots of the bucket's bits (no returning atomics), so a later
// launch of the same geometry reproduces the layout exactly (ensure_layout_orig).
//
// Column c + 1's loads are issued as soon as column c is staged, so they are in
// flight during column c's write-out.

struct ScatterArgs {
  int p, F, P, s, nb, nbits, nchunks;
  int64_t n, ld;
  const double* X;
  const double* w;
  const int32_t* code[kMaxFE];
  double* Xo;
  double* wo;
  int32_t* codeo[kMaxFE];
  int32_t* orig;
  const int32_t* scanned;  // [nb][nchunks] exclusive destinations
  int cols;                // move the X / w columns and the codes
  int want_orig;           // write the input row index of each layout row
  int ncl;                 // with cols: loaded cluster columns moved into layout order too
  const int32_t* cl[kMaxCl];
  int32_t* clo[kMaxCl];
  double* colstat;         // with cols: max |x_c| (u64 bits, atomicMax) and per-chunk sums of x_c^2
};

// a global-memory byte pointer the compiler keeps in SGPRs (it is the same in every lane), so
// loads and stores use the saddr + 32-bit voffset forms
typedef __attribute__((address_space(1))) char gchar;
__device__ __forceinline__ gchar* uniform_gptr(const void* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<gchar*>(((uint64_t)hi << 32) | lo);
}

// block i -> chunk: XCD x = i % 8 walks its contiguous eighth of the chunks, so the adjacent
// runs that consecutive chunks write into every bucket region meet in one L2
__device__ __forceinline__ int xcd_chunk(int i, int nw) {
  const int x = i & 7, r = i >> 3;
  const int per = (nw + 7) >> 3;          // chunks per XCD (the last XCD may have fewer)
  return x * per + r;                      // may be >= nw: the caller's r0 >= n then
}

// O32: every column is < 4 GiB (ld * 8 < 2^32), so loads and stores address it with 32-bit
// byte offsets from a uniform base (the saddr + 32-bit voffset forms: one VGPR per address)
template <int PER, int NTH, bool O32>
__global__ __launch_bounds__(NTH) void k_part_scatter(ScatterArgs a) {
  using off_t = typename std::conditional<O32, uint32_t, int64_t>::type;
  constexpr int kWaves = NTH / 64;
  constexpr int R = NTH * PER;
  static_assert(R <= 32768, "stage slots are kept as 16-bit values");
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* stage = smem;                                           // [R] (doubles or two int32 halves)
  // [waves][nb] 16-bit cursors (< R <= 32768): half the LDS of 32-bit ones, so 16 waves' cursors
  // fit beside the 128 KB stage up to ~700 buckets (a wide fit's 391)
  uint16_t* cur = reinterpret_cast<uint16_t*>(stage + R);
  const int ncur = (kWaves * a.nb + 1) & ~1;
  int32_t* delta = reinterpret_cast<int32_t*>(cur + ncur);        // [nb]
  int32_t* tot = delta + a.nb;                                    // [nb + 1]
  __shared__ int32_t wsum[16];
  __shared__ double wstat[2][16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int chunk = xcd_chunk(blockIdx.x, a.nchunks);
  const int64_t r0 = (int64_t)chunk * R, r1 = min(a.n, r0 + R);
  if (chunk >= a.nchunks) return;
  const int64_t wbase = r0 + (int64_t)wave * PER * 64;
  // slot k of a lane holds row wbase + (k / 2) * 128 + 2 lane + (k % 2): pairs of consecutive
  // rows, so every column is read with 16-byte loads (the guide's streaming-read shape)
  auto row_of = [&](int k) -> int64_t { return wbase + (k >> 1) * 128 + 2 * lane + (k & 1); };
  for (int j = tid; j < kWaves * a.nb; j += NTH) cur[j] = 0;
  __syncthreads();
  int32_t bk[PER];
#pragma unroll
  for (int k = 0; k < PER; k += 2) {
    const int64_t i = row_of(k);  // even: an 8-byte code pair (i + 1 < ld)
    const int2 g = i < r1 ? *reinterpret_cast<const int2*>(a.code[a.P] + i) : int2{0, 0};
    bk[k] = i < r1 ? (g.x >> a.s) : -1;
    bk[k + 1] = i + 1 < r1 ? (g.y >> a.s) : -1;
  }
  // per-wave bucket counts (integer adds commute: the counts do not depend on their order)
#pragma unroll
  for (int k = 0; k < PER; ++k)
    if (bk[k] >= 0) {  // 32-bit adds into the cursor pair (a wave counts <= PER * 64 rows: no carry)
      const int idx = wave * a.nb + bk[k];
      atomicAdd(reinterpret_cast<uint32_t*>(cur) + (idx >> 1), 1u << (16 * (idx & 1)));
    }
  __syncthreads();
  // per bucket: exclusive scan over waves, total
  for (int b = tid; b < a.nb; b += NTH) {
    int32_t t = 0;
    for (int w2 = 0; w2 < kWaves; ++w2) {
      const int32_t h = cur[w2 * a.nb + b];
      cur[w2 * a.nb + b] = t;
      t += h;
    }
    tot[b] = t;
  }
  __syncthreads();
  // exclusive scan of tot over buckets (one thread per `per` buckets, then waves)
  {
    const int per = (a.nb + NTH - 1) / NTH;
    const int b0 = tid * per;
    int32_t sacc = 0;
    for (int q = 0; q < per; ++q)
      if (b0 + q < a.nb) sacc += tot[b0 + q];
    int32_t x = sacc;  // wave inclusive scan
    for (int off = 1; off < 64; off <<= 1) {
      const int32_t y = __shfl_up(x, off, 64);
      if (lane >= off) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    int32_t wofs = 0;
    for (int w2 = 0; w2 < wave; ++w2) wofs += wsum[w2];
    int32_t run = x - sacc + wofs;
    __syncthreads();
    for (int q = 0; q < per; ++q)
      if (b0 + q < a.nb) {
        const int32_t t = tot[b0 + q];
        tot[b0 + q] = run;  // now: local offset of bucket
        run += t;
      }
  }
  __syncthreads();
  for (int b = tid; b < a.nb; b += NTH) {
    const int32_t boff = tot[b];
    delta[b] = a.scanned[(int64_t)b * a.nchunks + chunk] - boff;
    for (int w2 = 0; w2 < kWaves; ++w2) cur[w2 * a.nb + b] += boff;
  }
  __syncthreads();
  // stage slot of every row: the wave's cursor of its bucket + its rank among the lanes of this
  // instruction with the same bucket (lane order, from the ballots of the bucket's bits); the
  // first such lane advances the cursor.  The slot's bucket goes to the (not yet used) stage.
  int32_t* sb = reinterpret_cast<int32_t*>(stage);
  const uint64_t lanes_below = lane ? (~0ull >> (64 - lane)) : 0ull;
  uint32_t posp[PER / 2];  // two 16-bit slots per register (0xffff: no row)
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int b = bk[k];
    const bool act = b >= 0;
    uint32_t slot = 0xffffu;
    uint64_t same = __ballot(act);
    for (int bit = 0; bit < a.nbits; ++bit) {
      const bool one = act && ((b >> bit) & 1);
      const uint64_t m = __ballot(one);
      same &= one ? m : ~m;
    }
    if (act) {
      uint16_t* cw = &cur[wave * a.nb + b];
      const int base = *cw;
      const int rank = __popcll(same & lanes_below);
      if (rank == 0) *cw = (uint16_t)(base + __popcll(same));
      slot = (uint32_t)(base + rank);
      sb[slot] = b;
    }
    if (k & 1) posp[k >> 1] |= slot << 16;
    else posp[k >> 1] = slot;
  }
  auto pos_of = [&](int k) -> int {
    const uint32_t v = (k & 1) ? (posp[k >> 1] >> 16) : (posp[k >> 1] & 0xffffu);
    return v == 0xffffu ? -1 : (int)v;
  };
  __syncthreads();
  const int len = (int)(r1 - r0);
  // write-out slot k of a thread: consecutive threads read consecutive stage slots
  auto slot_of = [&](int k) -> int { return tid + k * NTH; };
  int32_t dd[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int j = slot_of(k);
    dd[k] = j < len ? delta[sb[j]] + j : -1;
  }
  __syncthreads();
  // ---- move columns through the stage: gather in row order, store in bucket order ----
  // cols 1: X (and w) and the codes; cols 2 (streamed X): the codes and w only
  const int ncol = a.cols == 1 ? a.p + (a.w ? 1 : 0) : (a.cols == 2 && a.w ? 1 : 0);
  const int cbase = a.cols == 2 ? a.p : 0;  // column id of the first moved column (p: w)
  typedef double d2v __attribute__((ext_vector_type(2)));
  // rows i < n are loaded in 16-byte pairs: i is even and the columns are padded to a multiple
  // of 64 rows, so row i + 1 lies inside the column even when i + 1 == n.  A full chunk (every
  // chunk but the last) runs without per-row predicates.
  const bool full = len == R;
  auto move_cols = [&](auto full_c) {
    constexpr bool FULL = decltype(full_c)::value;
    // the wave's rows start at wbase: the column base moves by wbase rows (uniform), a lane's
    // offset is then 16 * lane + 1024 * (k / 2) bytes (one VGPR plus immediates)
    const uint32_t lane_off = 16u * (uint32_t)lane;
    auto load_col = [&](int c, double (&v)[PER]) {
      const gchar* src = uniform_gptr(reinterpret_cast<const char*>(c < a.p ? a.X + (int64_t)c * a.ld : a.w) +
                                      wbase * 8);
      uint32_t lo = lane_off;
      asm volatile("" : "+v"(lo));  // the per-row offsets are formed here, not hoisted as 64-bit pairs
#pragma unroll
      for (int k = 0; k < PER; k += 2) {
        d2v t = d2v{0.0, 0.0};
        if (FULL || row_of(k) < r1)
          t = *reinterpret_cast<const __attribute__((address_space(1))) d2v*>(
              src + (off_t)(lo + 1024u * (uint32_t)(k >> 1)));
        v[k] = t.x;
        v[k + 1] = t.y;
      }
    };
    auto stage_col = [&](const double (&v)[PER]) {
      // the packed slots are decoded here, per column, instead of living unpacked in 16 more
      // registers across the loop (the empty asm keeps the compiler from hoisting the decode)
#pragma unroll
      for (int k = 0; k < PER / 2; ++k) asm volatile("" : "+v"(posp[k]));
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int q = pos_of(k);
        if (FULL || q >= 0) stage[q] = v[k];
      }
    };
    auto write_col = [&](int c) {
      gchar* dst = uniform_gptr(c < a.p ? a.Xo + (int64_t)c * a.ld : a.wo);
#pragma unroll
      for (int k = 0; k < PER; ++k) asm volatile("" : "+v"(dd[k]));  // no hoisted 64-bit addresses
      // four stage reads in flight before their stores (not one LDS round trip per store)
#pragma unroll
      for (int k0 = 0; k0 < PER; k0 += 4) {
        double t[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) t[u] = stage[slot_of(k0 + u)];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (FULL || dd[k0 + u] >= 0)
            *reinterpret_cast<__attribute__((address_space(1))) double*>(dst + (off_t)dd[k0 + u] * 8) = t[u];
      }
    };
    // column statistics for the exact group sums (lfe_fast.hip): max |x| and sum x^2 of this
    // chunk's rows (rows past the end load as 0).  Each wave reduces its values over DPP lane
    // moves (VALU only: the stage keeps the LDS busy); after the barrier, lanes 0-15 of wave
    // c % 16 combine the 16 waves the same way and lane 15 writes the chunk's figures.
    const auto fmaxop = [](double x, double y) { return fmax(x, y); };
    const auto addop = [](double x, double y) { return x + y; };
    auto col_stats = [&](const double (&v)[PER]) {
      double m = 0.0, q = 0.0;
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        m = fmax(m, fabs(v[k]));
        q = __builtin_fma(v[k], v[k], q);
      }
      // (fmax drops a NaN; the sum of squares keeps it, and the guard tests that sum)
      m = wave_reduce63(m, 0.0, fmaxop);
      q = wave_reduce63(q, 0.0, addop);
      if (lane == 63) {
        wstat[0][wave] = m;
        wstat[1][wave] = q;
      }
    };
    auto col_stats_out = [&](int c) {  // after the barrier that follows col_stats
      if (wave != (c & (kWaves - 1)) || lane >= 16) return;
      double m = lane < kWaves ? wstat[0][lane] : 0.0, q = lane < kWaves ? wstat[1][lane] : 0.0;
      m = row16_reduce15(m, 0.0, fmaxop);
      q = row16_reduce15(q, 0.0, addop);
      if (lane == 15) {
        a.colstat[kColStatHead + (int64_t)c * a.nchunks + chunk] = q;
        atomicMax(reinterpret_cast<unsigned long long*>(a.colstat) + c, (unsigned long long)__double_as_longlong(m));
      }
    };
    // one register set: column c + 1 is loaded while column c is written out (two register
    // sets, loading c + 2 during c + 1's staging, measured 2.12 vs 2.09 ms)
    double v[PER];
    if (ncol > 0) load_col(cbase, v);
    for (int c = cbase; c < cbase + ncol; ++c) {
      stage_col(v);
#ifndef LFE_NO_COLSTAT
      if (c < a.p) col_stats(v);
#endif
      asm volatile("" ::: "memory");  // the next loads stay after the stage writes
      if (c + 1 < cbase + ncol) load_col(c + 1, v);
      __syncthreads();
#ifndef LFE_NO_COLSTAT
      if (c < a.p) col_stats_out(c);
#endif
      write_col(c);
      __syncthreads();
    }
  };
  if (full) move_cols(std::true_type{});
  else move_cols(std::false_type{});
  int32_t* istage0 = reinterpret_cast<int32_t*>(stage);
  const int ic0 = a.cols ? 0 : a.F + a.ncl;
  // F code arrays, the cluster columns, then the input row index
  for (int c = ic0; c < a.F + a.ncl + a.want_orig; ++c) {
    const int32_t* src = c < a.F ? a.code[c] : c < a.F + a.ncl ? a.cl[c - a.F] : nullptr;
    int32_t* dst = c < a.F ? a.codeo[c] : c < a.F + a.ncl ? a.clo[c - a.F] : a.orig;
    int32_t* istage = istage0 + ((c - ic0) & 1) * R;  // two int32 halves of the double stage
#pragma unroll
    for (int k = 0; k < PER; k += 2) {
      const int64_t i = row_of(k);
      int2 g = int2{(int32_t)i, (int32_t)i + 1};
      const int q0 = pos_of(k), q1 = pos_of(k + 1);
      if (src && q0 >= 0) g = *reinterpret_cast<const int2*>(src + i);
      if (q0 >= 0) istage[q0] = g.x;
      if (q1 >= 0) istage[q1] = g.y;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER; ++k)
      if (dd[k] >= 0) dst[dd[k]] = istage[slot_of(k)];
  }
}


// ---------------------------------------------------------------------------
// counts on the layout + singleton marks
// ---------------------------------------------------------------------------

// pre-filter counts from the per-item histograms of the two-FE layouts: primary group h sums
// its bucket's items (cnt1[item][h - lo]); secondary level q sums a 1/256 slice of all items
// both in one launch: blocks [0, nbp) the primary FE (one group per thread), then the secondary
// levels in 256 item slices (block nbp + y * nqx + x: levels 256 x.., slice y)
// any / done (one rank): the singleton test of k_any_singleton folded in - a primary count of 1 as
// it is written, the secondary counts (summed by atomics) by the last workgroup
__global__ void k_cnt_from_items(const int32_t* __restrict__ cnt1, const int32_t* __restrict__ cnt2,
                                 const int32_t* __restrict__ bitems, int s, int32_t G_P, int32_t* __restrict__ cntP,
                                 int n_items, int32_t G_Q, int32_t* __restrict__ cntQ, int nbp, int nqx,
                                 int32_t* __restrict__ any) {
  int found = 0;
  if ((int)blockIdx.x < nbp) {
    const int B = 1 << s;
    const int h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h < G_P) {
      const int b = h >> s, j = h & (B - 1);
      int32_t t = 0;
#pragma unroll 4
      for (int i = bitems[b]; i < bitems[b + 1]; ++i) t += cnt1[(int64_t)i * B + j];
      cntP[h] = t;
      found = t == 1;
    }
  } else {
    const int lin = blockIdx.x - nbp, x = lin % nqx, y = lin / nqx;
    const int q = x * blockDim.x + threadIdx.x;
    if (q < G_Q) {
      const int i0 = (int)((int64_t)y * n_items / 256), i1 = (int)((int64_t)(y + 1) * n_items / 256);
      int32_t t = 0;
#pragma unroll 4
      for (int i = i0; i < i1; ++i) t += cnt2[(int64_t)i * G_Q + q];
      if (t) atomicAdd(&cntQ[q], t);
    }
  }
  // the primary FE's singleton levels counted here (its counts are final per thread); the secondary
  // FE's, whose counts the blocks add up, by k_any_eq1 after the launch.  (Folding that check into
  // the last block to finish cost every block a fence and a counter add: +9 to +44 us at 1-15M rows.)
  if (any && __any(found) && (threadIdx.x & 63) == 0) atomicAdd(any, 1);
}

// any level with a count of one -> *any += 1 (per wave)
__global__ void k_any_eq1(const int32_t* __restrict__ cnt, int32_t G, int32_t* __restrict__ any) {
  int found = 0;
  for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x) found |= cnt[g] == 1;
  if (__any(found) && (threadIdx.x & 63) == 0) atomicAdd(any, 1);
}

int launch_any_eq1(lfe_ctx* c, const int32_t* cnt, int32_t G, int32_t* any) {
  if (G > 0)
    hipLaunchKernelGGL(k_any_eq1, dim3((unsigned)std::min(64, (G + 255) / 256)), dim3(256), 0, c->stream, cnt, G, any);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

// primary-FE counts: per work item an LDS slice of 2^s bins
__global__ __launch_bounds__(256) void k_count_items(const int4* __restrict__ items, const int32_t* __restrict__ code,
                                                     int s, int32_t G, int32_t* __restrict__ cnt) {
  extern __shared__ int32_t h[];
  const int4 it = items[blockIdx.x];
  const int B = 1 << s;
  for (int j = threadIdx.x; j < B; j += blockDim.x) h[j] = 0;
  __syncthreads();
  const int32_t lo = it.x << s;
  for (int64_t i = it.y + threadIdx.x; i < it.z; i += blockDim.x) atomicAdd(&h[code[i] - lo], 1);
  __syncthreads();
  for (int j = threadIdx.x; j < B; j += blockDim.x)
    if (h[j] && lo + j < G) atomicAdd(&cnt[lo + j], h[j]);
}

struct MarkArgs {
  int F, P;
  int32_t* code[kMaxFE];
  const int32_t* cnt_pre[kMaxFE];
  int32_t* drops[kMaxFE];
  int32_t* ndropped;
  const int32_t* any;   // number of singleton groups (k_any_singleton); 0: nothing to mark
  int G[kMaxFE];
};

// singleton groups over every FE (pre-filter counts of 1): k_mark returns at once without any
__global__ void k_any_singleton(MarkArgs a, int32_t* __restrict__ out) {
  int found = 0;
  for (int f = 0; f < a.F; ++f)
    for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < a.G[f]; g += gridDim.x * blockDim.x)
      found |= a.cnt_pre[f][g] == 1;
  if (__any(found) && (threadIdx.x & 63) == 0) atomicAdd(out, 1);
}

// single-pass singleton marks (polars_impl.py:477-482): a row is dropped when any
// of its FE groups has a pre-filter count of 1.  F is a template parameter and a
// thread handles 4 consecutive rows (16-byte code loads; the layout is padded to ld).
template <int F>
__global__ __launch_bounds__(256) void k_mark(MarkArgs a, int64_t n) {
  if (*a.any == 0) return;  // no group has a single row: nothing is dropped
  const int64_t n4 = (n + 3) >> 2;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n4; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i0 = t << 2;
    int4 g[F];
#pragma unroll
    for (int f = 0; f < F; ++f) g[f] = reinterpret_cast<const int4*>(a.code[f])[t];
    bool ok[4] = {true, true, true, true};
#pragma unroll
    for (int f = 0; f < F; ++f) {
      const int gv[4] = {g[f].x, g[f].y, g[f].z, g[f].w};
#pragma unroll
      for (int s = 0; s < 4; ++s)
        if (i0 + s < n) ok[s] = ok[s] && a.cnt_pre[f][gv[s]] > 1;
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (ok[s] || i0 + s >= n) continue;
#pragma unroll
      for (int f = 0; f < F; ++f) atomicAdd(&a.drops[f][(&g[f].x)[s]], 1);
      a.code[a.P][i0 + s] = -1;
      atomicAdd(a.ndropped, 1);
    }
  }
}

// every FE at once (blockIdx.y = f): cnt = pre - drops, and the number of levels present
// before and after the drop (one atomic per wave into two counters per FE)
struct FinishCountsArgs {
  const int32_t* pre[kMaxFE];
  const int32_t* drops[kMaxFE];
  int32_t* cnt[kMaxFE];
  int32_t G[kMaxFE];
  int32_t* out;  // [2 F]: (levels kept, levels present) per FE
  int32_t* cmax;  // [F]: largest kept count per FE (the exact group sums' bound, lfe_fast.hip)
  // the group sums' quanta in the same launch (k_fix_quanta of lfe_fast.hip): the workgroups of row
  // blockIdx.y == F sum the partition's per-chunk squares of one column each, and the last
  // workgroup of the grid forms every column's quanta from them and the kept counts' maximum
  const double* st;  // the partition's column statistics (null: no quanta here)
  int nchunks, p;
  int64_t n;
  double* colq;      // [p] the columns' sums of squares
  double* fq;
  unsigned int* done;
  // one rank: the last workgroup publishes the count scratch (iscratch[0, kIscratchInts)) to the
  // host message - no copy kernel and no event between the drop and the group sums
  const int32_t* is;
  unsigned long long* msg;
  unsigned long long seq;
};

__global__ void k_finish_counts(FinishCountsArgs a, int F) {
  const int f = blockIdx.y;
  if (f < F) {
    const int32_t G = a.G[f];
    int la = 0, lb = 0, mx = 0;
    for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x) {
      const int32_t pre = a.pre[f][g], c = pre - a.drops[f][g];
      a.cnt[f][g] = c;
      la += c > 0;
      lb += pre > 0;
      mx = max(mx, c);
    }
    for (int off = 32; off > 0; off >>= 1) {
      la += __shfl_down(la, off, 64);
      lb += __shfl_down(lb, off, 64);
      mx = max(mx, __shfl_down(mx, off, 64));
    }
    if ((threadIdx.x & 63) == 0) {
      if (la) atomicAdd(&a.out[2 * f], la);
      if (lb) atomicAdd(&a.out[2 * f + 1], lb);
      if (mx) atomicMax(&a.cmax[f], mx);
    }
  } else {
    // column c's sum of the per-chunk squares, in k_fix_quanta's order (256 threads, DPP wave sums,
    // the four waves in order)
    __shared__ double ws[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int c = blockIdx.x; c < a.p; c += gridDim.x) {
      const double* sq = a.st + kColStatHead + (int64_t)c * a.nchunks;
      double q = 0.0;
      for (int ch = tid; ch < a.nchunks; ch += 256) q += sq[ch];
      q = wave_reduce63(q, 0.0, [](double x, double y) { return x + y; });
      if (lane == 63) ws[wave] = q;
      __syncthreads();
      if (tid == 0) a.colq[c] = ((ws[0] + ws[1]) + ws[2]) + ws[3];
      __syncthreads();
    }
  }
  if (!a.done || !last_block_done(a.done)) return;
  if (a.st) {
    int N = 1;
    for (int g = 0; g < F; ++g) N = max(N, __hip_atomic_load(&a.cmax[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    for (int c = threadIdx.x; c < a.p; c += blockDim.x) {
      const double M = __longlong_as_double(reinterpret_cast<const long long*>(a.st)[c]);
      const double rms = a.n > 0 ? sqrt(a.colq[c] / (double)a.n) : 0.0;
      fix_quanta_col(M, rms, (double)N, a.fq, c);
    }
  }
  if (a.msg && threadIdx.x == 0) host_msg_publish_i32(a.msg, a.seq, a.is, kIscratchInts);
}

// multi-rank: the kept rows and (owner-sharded) the primary FE's level counts summed over ranks
// on the device, so the host reads them with the other counts (no extra round trip)
constexpr int kIsKept = 2 * kMaxFE + 2;  // iscratch: kept rows (lo, hi int32 halves), primary dims, card
__global__ void k_kept_pack(const int32_t* __restrict__ is, int64_t n, int P, int owner, double* __restrict__ d) {
  if (threadIdx.x != 0) return;
  d[0] = (double)(n - is[2 * kMaxFE]);
  d[1] = owner ? (double)is[2 * P] : 0.0;
  d[2] = owner ? (double)is[2 * P + 1] : 0.0;
  d[3] = owner && is[kIscratchCmax + P] > 65535 ? 1.0 : 0.0;  // the dense paths' u16 counts (dense_ok)
}
__global__ void k_kept_unpack(const double* __restrict__ d, int owner, int32_t* __restrict__ is) {
  if (threadIdx.x != 0) return;
  const int64_t k = (int64_t)d[0];
  is[kIsCmaxOver] = owner ? (int32_t)d[3] : 0;
  is[kIsKept] = (int32_t)(uint32_t)(k & 0xffffffffll);
  is[kIsKept + 1] = (int32_t)(k >> 32);
  is[kIsKept + 2] = (int32_t)d[1];
  is[kIsKept + 3] = (int32_t)d[2];
}

// ---------------------------------------------------------------------------
// driver
// ---------------------------------------------------------------------------

// Bucket = 2^s primary groups.  Larger buckets give the partition longer runs per
// chunk (512-group buckets: 3.1 vs 3.5 ms at 50M rows) and the run layout longer
// runs; the bucket's alpha slice must still fit in LDS beside the secondary table
// (Gram, group sums: (2^s + G_Q) p 8 bytes <= 150 KB), so 512 only for two FEs.
static int choose_shift(int32_t G, int smin) {
  int s = 0;
  while ((1ll << s) < G && s < 8) ++s;       // small FE: one bucket
  if ((1ll << s) >= G) return s;
  s = smin;
  while (((int64_t)G + (1ll << s) - 1) >> s > 2048) ++s;  // <= 2048 buckets (LDS cursors of the scatter)
  return s;
}

// side: upload on up_stream after up_ev0 (recorded before the partition scatter), the main
// stream waiting for it, so the copy overlaps the scatter instead of following it
static int build_items(lfe_ctx* c, bool side) {
  auto& L = c->L;
  L.hitems.clear();
  std::vector<int32_t> bfirst(L.nb + 1, 0);
  for (int b = 0; b < L.nb; ++b) {
    const int32_t lo = L.bstart[b], hi = L.bstart[b + 1];
    const int32_t len = hi - lo;
    bfirst[b] = (int32_t)(L.hitems.size() / 4);
    if (len <= 0) continue;
    const int32_t k = (len + kItemRows - 1) / kItemRows;
    for (int32_t q = 0; q < k; ++q) {
      const int32_t r0 = lo + (int32_t)((int64_t)len * q / k), r1 = lo + (int32_t)((int64_t)len * (q + 1) / k);
      L.hitems.insert(L.hitems.end(), {b, r0, r1, 0});
    }
  }
  bfirst[L.nb] = (int32_t)(L.hitems.size() / 4);
  if (L.hitems.empty()) L.hitems.insert(L.hitems.end(), {0, 0, 0, 0});
  L.n_items = (int)(L.hitems.size() / 4);
  // XCD-grouped block order: workgroups are dispatched round-robin over the 8 XCDs
  // (block i on XCD i % 8), so block r * 8 + x takes the r-th item of the buckets
  // b with b % 8 == x.  All items of a bucket then share one L2, where the short
  // per-item pieces they write into the bucket's key regions merge into full
  // lines.  Speed only: any mapping is correct.
  std::vector<int32_t> xg;
  {
    constexpr int kX = 8;
    std::vector<std::vector<int32_t>> per(kX);
    for (int b = 0; b < L.nb; ++b)
      for (int i = bfirst[b]; i < bfirst[b + 1]; ++i) per[b % kX].push_back(i);
    size_t rounds = 0;
    for (auto& v : per) rounds = std::max(rounds, v.size());
    xg.assign(rounds * kX, -1);
    for (int x = 0; x < kX; ++x)
      for (size_t r = 0; r < per[x].size(); ++r) xg[r * kX + x] = per[x][r];
    if (xg.empty()) xg.push_back(0);
    c->n_xgrid = (int)xg.size();
  }
  // the buckets that hold rows, in order: the secondary cross term (K2) runs over these only.  An
  // owner shard of N ranks holds ~1/N of the primary FE's buckets; the rest are empty
  std::vector<int32_t> bl;
  for (int b = 0; b < L.nb; ++b)
    if (L.bstart[b + 1] > L.bstart[b]) bl.push_back(b);
  c->nbe = (int)bl.size();
  if (bl.empty()) bl.push_back(0);
  // items, bucket firsts, the XCD order and the bucket list share one device buffer and one upload
  // through pinned staging, asynchronously (the staging buffer is next written only after later
  // stream synchronizations); bitems_d / xitems_d / blist_d point into it
  const size_t ni = L.hitems.size(), nbf = bfirst.size(), nx = xg.size(), nl = bl.size();
  LFE_TRY(ensure_items(c, (ni + nbf + nx + nl + 3) / 4));
  c->bitems_d = c->items_d + ni;
  c->xitems_d = c->items_d + ni + nbf;
  c->blist_d = c->items_d + ni + nbf + nx;
  const size_t ib = sizeof(int32_t) * ni, bb = sizeof(int32_t) * nbf, xb = sizeof(int32_t) * nx,
               lb = sizeof(int32_t) * nl;
  LFE_TRY(ensure_pinned_items(c, ib + bb + xb + lb));
  memcpy(c->hpin_items, L.hitems.data(), ib);
  memcpy(c->hpin_items + ib, bfirst.data(), bb);
  memcpy(c->hpin_items + ib + bb, xg.data(), xb);
  memcpy(c->hpin_items + ib + bb + xb, bl.data(), lb);
  // on the main stream, behind the partition scatter (a few KB: the copy that follows the scatter
  // costs less than the cross-stream wait that let it overlap, ~10 us of barrier at small shards),
  // by a kernel reading the mapped staging (an SDMA copy there left the GPU idle ~15-20 us)
  (void)side;
  const int64_t words = (int64_t)((ib + bb + xb + lb + 15) / 16);
  hipLaunchKernelGGL(k_copy_staged, dim3((unsigned)std::min<int64_t>(64, (words + 255) / 256)), dim3(256), 0,
                     c->stream, reinterpret_cast<const int4*>(c->hpin_items_dev), reinterpret_cast<int4*>(c->items_d),
                     words);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

// Partition scatter of the current layout geometry (L.part, the scanned destinations in
// c->pcounts): cols = X / w columns and codes, orig = the input row index of each layout row.
// The ranking is deterministic, so an orig-only launch later reproduces the same layout.
static int launch_part_scatter(lfe_ctx* c, int cols, int orig) {
  auto& L = c->L;
  const PartGeom& g = L.part;
  ScatterArgs a{};
  a.p = c->p;
  a.F = c->F;
  a.P = L.P;
  a.s = L.s;
  a.nb = L.nb;
  a.nchunks = g.nw;
  a.n = c->n;
  a.ld = c->ld;
  a.X = c->X;
  a.w = c->w;
  a.Xo = c->Xp;
  a.wo = c->wp;
  for (int f = 0; f < c->F; ++f) {
    a.code[f] = c->fe[f].code;
    a.codeo[f] = c->codes_p + (size_t)f * c->ld;
  }
  a.orig = c->origp;
  a.scanned = c->pcounts;
  a.cols = cols;
  a.want_orig = orig;
  // the cluster columns ride along with the codes when their layout copies are wanted now
  a.ncl = 0;
  if (cols && c->clw.lay_move) {
    a.ncl = (int)c->cl.size();
    for (int j = 0; j < a.ncl; ++j) {
      a.cl[j] = c->cl[j];
      a.clo[j] = c->clw.lay[j];
    }
  }
  a.colstat = c->colstat;
  a.nbits = 0;  // bits of a bucket id (ballot ranking)
  while ((1 << a.nbits) < L.nb) ++a.nbits;
  const int pgrid = ((g.nw + 7) / 8) * 8;  // xcd_chunk: a multiple of the 8 XCDs
  // dynamic LDS above 64 KB must be opted in (static LDS + dynamic <= 160 KB)
  using Fn = void (*)(ScatterArgs);
  const bool o32 = (uint64_t)c->ld * 8 <= 0xffffffffull;
#define PART_FN(PER, NTH) (o32 ? &k_part_scatter<PER, NTH, true> : &k_part_scatter<PER, NTH, false>)
  Fn fn = g.nth == 1024 ? (g.per == 16 ? PART_FN(16, 1024) : g.per == 8 ? PART_FN(8, 1024) : PART_FN(4, 1024))
        : g.per == 16   ? PART_FN(16, 512)
                        : PART_FN(8, 512);
#undef PART_FN
  LFE_HIP(set_max_lds(reinterpret_cast<const void*>(fn), (int)g.lds));
  {
    ProfScope _ps(c, cols ? K_PART_SCATTER : K_MISC);
    hipLaunchKernelGGL(fn, dim3(pgrid), dim3(g.nth), g.lds, c->stream, a);
  }
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

int ensure_layout_orig(lfe_ctx* c) {
  if (!c->L.orig_pending) return LFE_OK;
  LFE_TRY(launch_part_scatter(c, /*cols=*/0, /*orig=*/1));
  c->L.orig = c->origp;
  c->L.orig_pending = false;
  return LFE_OK;
}

int prepare_layout(lfe_ctx* c) {
  auto& L = c->L;
  const int64_t n = c->n;
  c->sums_ready = false;
  c->q_first = nullptr;
  c->any_ready = false;
  c->fixq_ready = false;
  c->seg_ready = false;
  c->colstat_chunks = 0;  // the partition (or sums4's k_col_stats) writes them again
  c->gram_spec = false;
  c->clw.lay_valid = false;  // cluster columns follow the new layout
  // primary FE: most levels (ties -> first)
  L.P = -1;
  for (int f = 0; f < c->F; ++f)
    if (L.P < 0 || c->fe[f].G > c->fe[L.P].G) L.P = f;
  int smin = 8;
  // 512-group buckets where the row passes' LDS tables (alpha_Q + the primary slice) fit them; else
  // 256 (a wide fit's residual pass stages the primary slice of 256 groups: three workgroups per CU
  // where 512 allow one - measured 3.7 vs 5.8 ms at p = 21, against 0.7 ms more partition)
  if (c->F == 2 && L.P >= 0 && ((int64_t)512 + c->fe[1 - L.P].G) * c->p * 8 <= 150 * 1024) smin = 9;
  L.s = L.P >= 0 ? choose_shift(c->fe[L.P].G, smin) : 0;
  L.nb = L.P >= 0 ? (int)(((int64_t)c->fe[L.P].G + (1ll << L.s) - 1) >> L.s) : 1;
  L.permuted = L.nb > 1 && n > 0;

  // two-FE fast layouts: both FEs' pre-filter counts come from the layouts' per-item
  // histograms (formed after the partition, reused by build_layouts when nothing is dropped)
  c->hists_kept = false;
  L.w = c->w;  // fast_layout_ok reads it before the layout pointers are set below
  const bool item_counts = L.permuted && fast_layout_ok(c);
  // owner-sharded rows: every row of the primary FE's groups [owner_lo, owner_hi) is on this rank,
  // so its counts, drops, group sums (W, Sy), cross term and effects are complete without an
  // all-reduce - in the two-FE sweeps and in the general sweeps (any F, weights) alike
  c->owner_on = c->world > 1 && c->owner_fe >= 0 && c->owner_fe == L.P && !c->records;
  // every count / drop / group-sum table and the scratch counters zeroed in one launch
  LFE_TRY(ensure_iscratch(c, kIscratchAll));
  ZeroArgs zpart{};  // zeroed by k_part_hist instead (the two-FE fast layout)
  {
    std::vector<std::pair<void*, size_t>> z;
    for (int f = 0; f < c->F; ++f) {
      auto& fe = c->fe[f];
      z.push_back({fe.cnt_pre, sizeof(int32_t) * fe.G});
      z.push_back({fe.drops, sizeof(int32_t) * fe.G});
      z.push_back({fe.S, sizeof(double) * (size_t)fe.G * c->p});
    }
    // the primary FE's effects: the two-FE sweeps' K1 writes only the levels with rows on this
    // shard (an owner shard's other levels, levels whose rows were all dropped stay 0)
    if (L.P >= 0) z.push_back({c->fe[L.P].alpha, sizeof(double) * (size_t)c->fe[L.P].G * c->p});
    z.push_back({c->iscratch, sizeof(int32_t) * kIscratchInts});
    if (L.permuted && item_counts && n > 0) {
      // nothing reads these before the partition histogram: it zeroes them (colstat's head too)
      LFE_TRY(ensure_f64(c, c->colstat, c->colstat_cap, (size_t)kColStatHead));
      z.push_back({c->colstat, sizeof(double) * kColStatHead});
      LFE_TRY(build_zero_args(z, &zpart, nullptr));
    } else {
      LFE_TRY(zero_ranges(c, z));
    }
    c->sums_zeroed = true;
  }
  // pre-filter counts of every FE (on input codes, except P when bucketed)
  for (int f = 0; f < c->F; ++f) {
    auto& fe = c->fe[f];
    if (n == 0 || (f == L.P && L.permuted) || item_counts) continue;
    ProfScope _ps(c, K_COUNT);
    const int nr = (fe.G + kHistRange - 1) / kHistRange;
    if (fe.G <= kLdsHistMax) {
      hipLaunchKernelGGL(k_hist_lds, dim3(grid_for((n + 3) / 4, 256, 2048)), dim3(256), sizeof(int32_t) * fe.G, c->stream,
                         fe.code, n, fe.G, fe.cnt_pre);
    } else if (nr <= kHistMaxRanges) {
      // about two blocks per CU over all ranges, and at least ~64K rows per block
      const int bx = (int)std::max<int64_t>(1, std::min<int64_t>((2 * (int64_t)c->n_cu + nr - 1) / nr, n / 65536 + 1));
      const size_t lds = sizeof(int32_t) * kHistRange;
      LFE_HIP(set_max_lds(reinterpret_cast<const void*>(&k_hist_lds_range), (int)lds));
      hipLaunchKernelGGL(k_hist_lds_range, dim3(bx, nr), dim3(1024), lds, c->stream, fe.code, n, fe.G, fe.cnt_pre);
    } else
      hipLaunchKernelGGL(k_hist_global, dim3(grid_for(n)), dim3(kBlock), 0, c->stream, fe.code, n, fe.cnt_pre);
    LFE_HIP(hipGetLastError());
  }

  if (L.permuted) {
    // ---- partition by bucket of P ----
    const int nb = L.nb;
    // Chunk geometry, measured at 50M rows x 196 buckets (s = 9): 16384-row chunks on
    // 1024-thread workgroups (16 rows per thread), one workgroup per CU, 2.06 ms; 8192-row
    // chunks on 512 threads 2.28 ms.  Earlier: 4096-row chunks, several chunks per
    // workgroup and register scatter without the LDS stage were all slower.
    // one 16-wave workgroup per CU: with two per CU (32 waves) twice as many chunks write into
    // every bucket region at once and the scatter ran 13 % slower (measured); pad the LDS request
    constexpr size_t kLdsMin = 82 * 1024;
    // 16K-row chunks: ~84-row runs per bucket at s = 9.  One workgroup per CU: a shard of few
    // chunks (the 8-GPU shard: 382 for 256 CUs) leaves CUs idle in the last round, so the chunk
    // halves (down to 4K rows) while that fills the rounds markedly better
    // (more buckets: 8192-row chunks while the per-wave cursors of 8 waves fit beside the stage,
    // config 4's 1954 buckets 0.35 ms faster than 4096-row chunks; else 4096)
    int64_t cw = nb <= 512 ? 16384 : 8192;
    if (cw == 16384) {
      auto fill = [&](int64_t w) {
        const int64_t k = (n + w - 1) / w, r = (k + c->n_cu - 1) / c->n_cu;
        return (double)k / (double)(std::max<int64_t>(r, 1) * c->n_cu);
      };
      for (int64_t w = 8192; w >= 4096; w /= 2)
        if (fill(w) > fill(cw) + 0.1) cw = w;
    }
    if (const char* e = knob("LFE_PART_CW")) cw = atoll(e);  // A/B only
    auto part_lds = [&](int nth) {  // stage, 16-bit per-wave cursors, deltas and totals
      return sizeof(double) * cw + sizeof(uint16_t) * (((size_t)(nth / 64) * nb + 1) & ~(size_t)1) +
             sizeof(int32_t) * (2 * (size_t)nb + 1);
    };
    // 16 waves per chunk when their per-wave bucket cursors fit (nb <= ~1500)
    const int nth = part_lds(1024) <= 150 * 1024 ? 1024 : 512;
    if (cw == 16384 && nth != 1024) cw = 8192;
    if (part_lds(nth) > 150 * 1024) cw = 4096;
    const int per = (int)(cw / nth);
    const int nw = (int)((n + cw - 1) / cw);
    // column statistics of the exact group sums, written by the scatter (max |x| by atomicMax)
    if (zpart.n == 0 || c->colstat_cap < (size_t)kColStatHead + (size_t)nw * c->p) {
      // (a larger colstat moves: its head zeroed here, and the ranges' copy of the old pointer
      // dropped - the ranges are zeroed now by their own launch)
      LFE_TRY(ensure_f64(c, c->colstat, c->colstat_cap, (size_t)kColStatHead + (size_t)nw * c->p));
      if (zpart.n > 0) {
        std::vector<std::pair<void*, size_t>> z2;
        for (int j = 0; j < zpart.n; ++j) {
          const int64_t len = zpart.end[j] - (j ? zpart.end[j - 1] : 0);
          z2.push_back({zpart.p[j], (size_t)len * 4});
        }
        z2.pop_back();  // the old colstat head
        LFE_TRY(zero_ranges(c, z2));
        zpart = ZeroArgs{};
      }
      LFE_HIP(hipMemsetAsync(c->colstat, 0, sizeof(double) * kColStatHead, c->stream));
    }
    c->colstat_chunks = nw;
    const int64_t m = (int64_t)nb * nw;
    LFE_TRY(ensure_pcounts(c, (size_t)m + nb + 1, 0));
    {
      ProfScope _ps(c, K_PART_HIST);
      hipLaunchKernelGGL(k_part_hist, dim3(nw), dim3(256), sizeof(int32_t) * nb, c->stream, c->fe[L.P].code, n, L.s,
                         nb, cw, nw, c->pcounts, zpart);
    }
    LFE_HIP(hipGetLastError());
    // bucket starts depend on the scan only (gathered by its last kernel): fetch them now and
    // build the work items on the host while the GPU runs the scatter
    int32_t* dbstart = c->pcounts + m;
    unsigned long long bseq = 0;  // the scan's last block publishes the bucket starts (one rank)
    LFE_TRY(exclusive_scan_g(c, c->pcounts, m, nullptr, 0, dbstart, nw, nb, &bseq));
    // (else read on the side stream below, after the scatter is enqueued: no copy enqueue between
    // the scan and the scatter on the main stream, whose GPU time it was - unless the scatter is
    // short: the side stream's wait for the scan took ~20 us at 1M rows, longer than the host then
    // needs to build the items, so up to 16M rows the copy goes on the main stream before the
    // scatter; same-box A/B, profiles/r06/ab_bstart.txt: 1-10M rows equal or slightly faster)
    const char* kb = knob("LFE_BSTART_MAIN_ROWS");
    const bool bs_main = !bseq && n <= (kb ? std::atoll(kb) : (int64_t)(16 << 20));
    if (bs_main) {
      LFE_HIP(hipMemcpyAsync(c->hpin, dbstart, sizeof(int32_t) * nb, hipMemcpyDeviceToHost, c->stream));
      LFE_HIP(hipEventRecord(c->aux_ev, c->stream));
    } else if (!bseq) {
      LFE_HIP(hipEventRecord(c->up_ev0, c->stream));
    }
    const size_t lds = std::min<size_t>(std::max(part_lds(nth), kLdsMin), 160 * 1024);
    L.part = PartGeom{nth, per, nw, lds};
    // the input row index of each layout row is written only when a caller needs it
    // (ensure_layout_orig: cluster, records and demeaned-column export paths)
    // loaded cluster columns (clustered SEs follow this solve) move with the codes: no later
    // orig-only launch and row-index gathers (lfe_cluster.hip launch_cluster_subsets)
    auto& W = c->clw;
    W.lay_move = !c->sw.on && !c->cl.empty() && (int)c->cl.size() <= kMaxCl;
    if (W.lay_move) {
      const int m = (int)c->cl.size();
      W.lay.resize(m, nullptr);
      W.lay_cap.resize(m, 0);
      for (int j = 0; j < m; ++j) LFE_TRY(ensure_i32(c, W.lay[j], W.lay_cap[j], (size_t)c->ld));
    }
    LFE_TRY(launch_part_scatter(c, /*cols=*/c->sw.on ? 2 : 1, /*orig=*/0));
    if (!bseq && !bs_main) {
      LFE_HIP(hipStreamWaitEvent(c->up_stream, c->up_ev0, 0));  // the scan is done
      LFE_HIP(hipMemcpyAsync(c->hpin, dbstart, sizeof(int32_t) * nb, hipMemcpyDeviceToHost, c->up_stream));
      LFE_HIP(hipEventRecord(c->aux_ev, c->up_stream));
    }
    W.lay_valid = W.lay_move;
    W.lay_move = false;
    L.orig_pending = true;
    LFE_HIP(hipGetLastError());
    L.bstart.assign(nb + 1, 0);
    if (bseq) LFE_TRY(host_msg_wait_i32(c, bseq, L.bstart.data(), nb));
    else LFE_TRY(d2h_wait(c, L.bstart.data(), sizeof(int32_t) * nb));
    L.bstart[nb] = (int32_t)n;
    L.X = c->sw.on ? nullptr : c->Xp;
    L.w = c->w ? c->wp : nullptr;
    for (int f = 0; f < c->F; ++f) L.code[f] = c->codes_p + (size_t)f * c->ld;
    L.orig = nullptr;
  } else {
    L.orig_pending = false;
    L.bstart = {0, (int32_t)n};
    L.X = c->X;
    L.w = c->w;
    for (int f = 0; f < c->F; ++f) {
      L.code[f] = c->codes_p + (size_t)f * c->ld;
      if (n) LFE_HIP(hipMemcpyAsync(L.code[f], c->fe[f].code, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, c->stream));
    }
    L.orig = nullptr;
  }
  LFE_TRY(build_items(c, L.permuted));

  c->dn_pre = c->dn_pre_valid = false;
  if (item_counts && dense_pre_ok(c)) {
    // the dense cross terms will run: their count tables, built on every row now, give both FEs'
    // pre-filter counts (row / column sums) in place of the layout histograms, and serve the sweeps
    // as they are when no row is dropped
    LFE_TRY(dense_build(c, true));
    c->dn_pre = true;
  } else if (item_counts) {
    const int Q = 1 - L.P, B = 1 << L.s;
    LFE_TRY(layout_hists(c, Q));
    ProfScope _ps(c, K_COUNT);
    const int32_t* c1 = c->seg_aux;
    const int32_t* c2 = c->seg_aux + (size_t)L.n_items * B;
    const int nbp = (c->fe[L.P].G + 255) / 256, nqx = (c->fe[Q].G + 255) / 256;
    const bool one = c->world == 1;  // (several ranks sum the counts afterwards: k_any_singleton then)
    hipLaunchKernelGGL(k_cnt_from_items, dim3(nbp + nqx * 256), dim3(256), 0, c->stream, c1, c2, c->bitems_d, L.s,
                       c->fe[L.P].G, c->fe[L.P].cnt_pre, L.n_items, c->fe[Q].G, c->fe[Q].cnt_pre, nbp, nqx,
                       one ? c->iscratch + kIsAny : nullptr);
    if (one) LFE_TRY(launch_any_eq1(c, c->fe[Q].cnt_pre, c->fe[Q].G, c->iscratch + kIsAny));
    c->any_ready = one;
    LFE_HIP(hipGetLastError());
  } else if (L.permuted) {
    ProfScope _ps(c, K_COUNT);
    auto& fe = c->fe[L.P];
    hipLaunchKernelGGL(k_count_items, dim3(L.n_items), dim3(256), sizeof(int32_t) << L.s, c->stream,
                       reinterpret_cast<const int4*>(c->items_d), L.code[L.P], L.s, fe.G, fe.cnt_pre);
    LFE_HIP(hipGetLastError());
  }
  for (int f = 0; f < c->F; ++f)
    if (!(c->owner_on && f == L.P)) LFE_TRY(allreduce_sum_i32(c, c->fe[f].cnt_pre, c->fe[f].G));

  unsigned long long is_seq = 0;  // the counts published to the host message (k_finish_counts)
  // ---- single-pass singleton drop: mark, then kept counts = pre - drops ----
  int32_t* ndropped = c->iscratch + 2 * kMaxFE;
  if (c->F > 0) {
    MarkArgs a{};
    a.F = c->F;
    a.P = L.P;
    for (int f = 0; f < c->F; ++f) {
      auto& fe = c->fe[f];
      a.code[f] = L.code[f];
      a.cnt_pre[f] = fe.cnt_pre;
      a.drops[f] = fe.drops;
    }
    a.ndropped = ndropped;
    a.any = ndropped + 1;
    int gmax = 1;
    for (int f = 0; f < c->F; ++f) {
      a.G[f] = c->fe[f].G;
      gmax = std::max(gmax, c->fe[f].G);
    }
    if (!c->any_ready)  // (else the count kernel above counted the singleton groups)
      hipLaunchKernelGGL(k_any_singleton, dim3(grid_for(gmax, kBlock, 256)), dim3(kBlock), 0, c->stream, a,
                         ndropped + 1);
    LFE_HIP(hipGetLastError());
    // YOCO records keep every record: compress has no singleton drop (compress.py:1049-1175);
    // a record alone in its level is fitted exactly by its own dummy
    if (n && !c->records) {
      ProfScope _ps(c, K_MARK);
      const int grid = grid_for((n + 3) / 4, kBlock, 8192);
      switch (c->F) {
#define MARK_CASE(FF) \
  case FF: hipLaunchKernelGGL(k_mark<FF>, dim3(grid), dim3(kBlock), 0, c->stream, a, n); break;
        MARK_CASE(1) MARK_CASE(2) MARK_CASE(3) MARK_CASE(4) MARK_CASE(5) MARK_CASE(6) MARK_CASE(7) MARK_CASE(8)
#undef MARK_CASE
        default: break;
      }
    }
    LFE_HIP(hipGetLastError());
    FinishCountsArgs fa{};
    for (int f = 0; f < c->F; ++f) {
      auto& fe = c->fe[f];
      if (!(c->owner_on && f == L.P)) LFE_TRY(allreduce_sum_i32(c, fe.drops, fe.G));
      fa.pre[f] = fe.cnt_pre;
      fa.drops[f] = fe.drops;
      fa.cnt[f] = fe.cnt;
      fa.G[f] = fe.G;
    }
    fa.out = c->iscratch;
    fa.cmax = c->iscratch + kIscratchCmax;
    // the unweighted group sums' quanta from the partition's column statistics in this launch too
    // (sums4 then launches no k_fix_quanta)
    c->fixq_ready = false;
    if (!c->w && !c->sw.on && L.permuted && c->colstat_chunks > 0 && n > 0) {
      LFE_TRY(ensure_f64(c, c->fixq, c->fixq_cap, (size_t)kFqRows * kFqCols));
      LFE_TRY(ensure_f64(c, c->colq, c->colq_cap, (size_t)kMaxCols + 1));
      fa.st = c->colstat;
      fa.nchunks = c->colstat_chunks;
      fa.p = c->p;
      fa.n = n;
      fa.colq = c->colq;
      fa.fq = c->fixq;
      fa.done = c->gsync + GS_FINISH;
      c->fixq_ready = true;
    }
    if (host_msg_on(c)) {  // the counts to the host by the last workgroup
      fa.is = c->iscratch;
      fa.msg = c->dmsg;
      fa.seq = is_seq = next_msg_seq(c);
      fa.done = c->gsync + GS_FINISH;
    }
    if (c->F > 0) {
      // few blocks: thousands of same-address adds would serialize
      hipLaunchKernelGGL(k_finish_counts, dim3(grid_for(gmax, kBlock, 32), c->F + (fa.st ? 1 : 0)), dim3(kBlock), 0,
                         c->stream, fa, c->F);
      LFE_HIP(hipGetLastError());
    }
  }
  if (c->world > 1) {
    LFE_TRY(ensure_dred(c, 4));
    hipLaunchKernelGGL(k_kept_pack, dim3(1), dim3(64), 0, c->stream, c->iscratch, n, L.P, c->owner_on ? 1 : 0,
                       c->dred);
    LFE_HIP(hipGetLastError());
    LFE_TRY(allreduce_sum_f64(c, c->dred, c->owner_on ? 4 : 1));
    hipLaunchKernelGGL(k_kept_unpack, dim3(1), dim3(64), 0, c->stream, c->dred, c->owner_on ? 1 : 0, c->iscratch);
    LFE_HIP(hipGetLastError());
  }
  int32_t h[kIscratchInts];  // dims / card per FE, dropped rows, kept sums, largest kept counts
  if (!is_seq) LFE_TRY(d2h_async(c, c->iscratch, sizeof(h)));
  // the constant group sums S_f do not depend on the FE order: enqueue them now so the
  // GPU keeps working while the host reads the counts and returns (lfe_demean skips them)
  if (c->F > 0 && c->n > 0 && !c->sw.on) {  // streamed X: the sums come from lfe_stream pass 1
    LFE_TRY(sweep_group_sums(c));
    c->sums_ready = true;
  }
  if (is_seq) LFE_TRY(host_msg_wait_i32(c, is_seq, h, kIscratchInts));
  else LFE_TRY(d2h_wait(c, h, sizeof(h)));
  for (int f = 0; f < c->F; ++f) {
    c->fe[f].dims = h[2 * f];
    c->fe[f].card = h[2 * f + 1];
    c->fe[f].cmax = h[kIscratchCmax + f];
  }
  c->hists_kept = item_counts && !c->dn_pre && h[2 * kMaxFE] == 0;
  c->dn_pre_valid = c->dn_pre && h[2 * kMaxFE] == 0 && h[kIsDnPre] == 0;
  // kept rows over all ranks (owner-sharded: with the primary FE's level counts, which each
  // rank has for its own levels only; integers < 2^53 are exact in f64)
  double kept[3] = {(double)(n - h[2 * kMaxFE]), 0.0, 0.0};
  if (c->owner_on) {
    kept[1] = c->fe[L.P].dims;
    kept[2] = c->fe[L.P].card;
  }
  if (c->world > 1) {  // summed over ranks on the device (k_kept_pack / k_kept_unpack)
    kept[0] = (double)(((int64_t)h[kIsKept + 1] << 32) | (int64_t)(uint32_t)h[kIsKept]);
    kept[1] = h[kIsKept + 2];
    kept[2] = h[kIsKept + 3];
  }
  if (c->owner_on) {
    c->fe[L.P].dims = (int32_t)kept[1];
    c->fe[L.P].card = (int32_t)kept[2];
  }
  c->n_kept = (int64_t)kept[0];
  c->n_kept_local = n - h[2 * kMaxFE];
  c->cmax_over_ranks = c->world > 1 && c->owner_on ? h[kIsCmaxOver] : 0;
  return LFE_OK;
}

}  // namespace lfe

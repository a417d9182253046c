// Counter-based synthetic HDFE panel on the device.
//
// Bit-identical to leanfe_amd/synth.py: integer splitmix64, exact u64 -> f64
// conversion, and every floating-point expression evaluated in the same order
// with contraction disabled (no FMA), so a row generated here equals the NumPy
// row bit for bit and any row shard of any GPU count sees the same data.
#include "lfe_internal.h"

#pragma clang fp contract(off)

namespace lfe {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ double uni(uint64_t i, uint64_t s, uint64_t seed) {
  const uint64_t key = seed ^ (s << 40) ^ i;
  const double v = (double)(splitmix64(key) >> 12);
  return (v + 0.5) * 0x1p-52;
}

__device__ __forceinline__ double nrm(uint64_t i, uint64_t s, uint64_t seed) {
  double acc = uni(i, 16 * s, seed);
#pragma unroll
  for (uint64_t j = 1; j < 12; ++j) acc = acc + uni(i, 16 * s + j, seed);
  return acc - 6.0;
}

// eff[f][g] = 0.5^f * z(g, 101 + f)
__global__ void k_synth_effects(double* __restrict__ eff, int32_t G, int f, double scale, uint64_t seed) {
  for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x)
    eff[g] = scale * nrm((uint64_t)g, 101 + f, seed);
}

struct SynthArgs {
  int F, k;
  int32_t L[kMaxFE];
  int32_t* code[kMaxFE];
  const double* eff[kMaxFE];
  double beta[kMaxCols];
};

// code of FE f for global row i (bit-identical to synth.py: floor(u * L), clamped to L - 1)
__device__ __forceinline__ int32_t synth_code(uint64_t i, int f, int32_t L, uint64_t seed) {
  double c = floor(uni(i, (uint64_t)f, seed) * (double)L);
  c = fmin(c, (double)(L - 1));
  return (int32_t)c;
}

// rows r of the shard: global row index row_offset + r, or idx[r] (owner-sharded shards)
__global__ void k_synth_rows(SynthArgs a, double* __restrict__ X, int64_t ld, int64_t n, uint64_t seed,
                             int64_t row_offset, const int64_t* __restrict__ idx) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t i = idx ? (uint64_t)idx[r] : (uint64_t)(row_offset + r);
    int32_t g[kMaxFE];
    for (int f = 0; f < a.F; ++f) {
      g[f] = synth_code(i, f, a.L[f], seed);
      if (a.code[f]) a.code[f][r] = g[f];
    }
    if (!X) continue;  // codes only (streamed X keeps the codes resident, lfe_synth_load_codes)
    const double a0 = a.F > 0 ? a.eff[0][g[0]] : 0.0;
    double y = 0.0;
    for (int j = 0; j < a.k; ++j) {
      const double x = nrm(i, 200 + j, seed) + 0.5 * a0;
      X[(int64_t)(1 + j) * ld + r] = x;
      const double t = a.beta[j] * x;
      y = (j == 0) ? t : y + t;
    }
    for (int f = 0; f < a.F; ++f) y = y + a.eff[f][g[f]];
    y = y + nrm(i, 300, seed);
    X[r] = y;
  }
}

// owner-sharded shard: the global rows whose code of FE f lies in [lo, hi), in row order.
// Block b owns rows [b * kOwnChunk, (b + 1) * kOwnChunk): pass 1 counts them, pass 2 writes
// their indices at the block's offset, ranked in row order (wave ballots, waves in order).
constexpr int64_t kOwnChunk = 1 << 16;

__global__ __launch_bounds__(256) void k_own_count(int64_t n_total, int f, int32_t L, int32_t lo, int32_t hi,
                                                   uint64_t seed, int32_t* __restrict__ cnt) {
  __shared__ int32_t wsum[4];
  const int64_t r0 = (int64_t)blockIdx.x * kOwnChunk, r1 = min(n_total, r0 + kOwnChunk);
  int32_t c = 0;
  for (int64_t i = r0 + threadIdx.x; i < r1; i += blockDim.x) {
    const int32_t g = synth_code((uint64_t)i, f, L, seed);
    c += (g >= lo && g < hi) ? 1 : 0;
  }
  for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

__global__ __launch_bounds__(256) void k_own_index(int64_t n_total, int f, int32_t L, int32_t lo, int32_t hi,
                                                   uint64_t seed, const int64_t* __restrict__ base,
                                                   int64_t* __restrict__ idx) {
  __shared__ int32_t wcnt[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * kOwnChunk, r1 = min(n_total, r0 + kOwnChunk);
  int64_t out = base[blockIdx.x];
  for (int64_t t0 = r0; t0 < r1; t0 += blockDim.x) {
    const int64_t i = t0 + threadIdx.x;
    bool own = false;
    if (i < r1) {
      const int32_t g = synth_code((uint64_t)i, f, L, seed);
      own = g >= lo && g < hi;
    }
    const uint64_t m = __ballot(own);
    const int before = __popcll(m & ((lane ? (~0ull >> (64 - lane)) : 0ull)));
    if (lane == 0) wcnt[wave] = __popcll(m);
    __syncthreads();
    int32_t wofs = 0, tot = 0;
    for (int w = 0; w < 4; ++w) {
      wofs += w < wave ? wcnt[w] : 0;
      tot += wcnt[w];
    }
    if (own) idx[out + wofs + before] = i;
    out += tot;
    __syncthreads();
  }
}

static int synth_fill(lfe_ctx* c, int k, const int32_t* levels, const double* beta, uint64_t seed,
                      int64_t row_offset, const int64_t* idx) {
  SynthArgs a{};
  a.F = c->F;
  a.k = k;
  std::vector<double*> eff(c->F, nullptr);
  double scale = 1.0;
  for (int f = 0; f < c->F; ++f) {
    a.L[f] = levels[f];
    a.code[f] = c->fe[f].code;
    LFE_HIP(hipMalloc(&eff[f], sizeof(double) * (size_t)levels[f]));
    hipLaunchKernelGGL(k_synth_effects, dim3(grid_for(levels[f])), dim3(kBlock), 0, c->stream, eff[f], levels[f],
                       f, scale, seed);
    LFE_HIP(hipGetLastError());
    a.eff[f] = eff[f];
    scale *= 0.5;
  }
  for (int j = 0; j < k; ++j) a.beta[j] = beta[j];
  if (c->n)
    hipLaunchKernelGGL(k_synth_rows, dim3(grid_for(c->n, kBlock, 256 * 16)), dim3(kBlock), 0, c->stream, a, c->X,
                       c->ld, c->n, seed, row_offset, idx);
  LFE_HIP(hipGetLastError());
  LFE_HIP(hipStreamSynchronize(c->stream));
  for (int f = 0; f < c->F; ++f) LFE_HIP(hipFree(eff[f]));
  return LFE_OK;
}

int launch_synth(lfe_ctx* c, int k, const int32_t* levels, const double* beta, uint64_t seed, int64_t row_offset) {
  return synth_fill(c, k, levels, beta, seed, row_offset, nullptr);
}

// streamed X on the synthetic panel: the [p][ld] columns of global rows [row0, row0 + rows)
// into X (codes not written: they are resident), as lfe_synth_load would hold them
int synth_chunk(lfe_ctx* c, int k, const int32_t* levels, const double* beta, uint64_t seed, int64_t row0,
                int64_t rows, double* X, int64_t ld) {
  SynthArgs a{};
  a.F = c->F;
  a.k = k;
  std::vector<double*> eff(c->F, nullptr);
  double scale = 1.0;
  for (int f = 0; f < c->F; ++f) {
    a.L[f] = levels[f];
    a.code[f] = nullptr;
    LFE_HIP(hipMalloc(&eff[f], sizeof(double) * (size_t)levels[f]));
    hipLaunchKernelGGL(k_synth_effects, dim3(grid_for(levels[f])), dim3(kBlock), 0, c->stream, eff[f], levels[f],
                       f, scale, seed);
    LFE_HIP(hipGetLastError());
    a.eff[f] = eff[f];
    scale *= 0.5;
  }
  for (int j = 0; j < k; ++j) a.beta[j] = beta[j];
  if (rows)
    hipLaunchKernelGGL(k_synth_rows, dim3(grid_for(rows, kBlock, 256 * 16)), dim3(kBlock), 0, c->stream, a, X, ld,
                       rows, seed, row0, nullptr);
  LFE_HIP(hipGetLastError());
  LFE_HIP(hipStreamSynchronize(c->stream));
  for (int f = 0; f < c->F; ++f) LFE_HIP(hipFree(eff[f]));
  return LFE_OK;
}

// Columns [c_lo, c_lo + pc) of the K-regressor panel (global column 0 = y, j >= 1 = x_j) for global
// rows row0 + r: a wide fit's column block (k_synth_rows for K > 62; y needs every x of the row, so
// a block holding y evaluates all K, in k_synth_rows' order).  beta: K device doubles.
__global__ void k_synth_cols(SynthArgs a, int K, int c_lo, int pc, const double* __restrict__ beta,
                             double* __restrict__ X, int64_t ld, int64_t n, uint64_t seed, int64_t row0) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t i = (uint64_t)(row0 + r);
    int32_t g[kMaxFE];
    for (int f = 0; f < a.F; ++f) g[f] = synth_code(i, f, a.L[f], seed);
    const double a0 = a.F > 0 ? a.eff[0][g[0]] : 0.0;
    if (c_lo == 0) {
      double y = 0.0;
      for (int j = 0; j < K; ++j) {
        const double x = nrm(i, 200 + j, seed) + 0.5 * a0;
        if (1 + j < pc) X[(int64_t)(1 + j) * ld + r] = x;
        const double t = beta[j] * x;
        y = (j == 0) ? t : y + t;
      }
      for (int f = 0; f < a.F; ++f) y = y + a.eff[f][g[f]];
      y = y + nrm(i, 300, seed);
      X[r] = y;
    } else {
      for (int c = 0; c < pc; ++c) {
        const int j = c_lo + c - 1;  // x_{j+1}
        X[(int64_t)c * ld + r] = nrm(i, 200 + (uint64_t)j, seed) + 0.5 * a0;
      }
    }
  }
}

int synth_cols_chunk(lfe_ctx* c, int K, int c_lo, const int32_t* levels, const double* beta, uint64_t seed,
                     int64_t row0, int64_t rows, double* X, int64_t ld) {
  SynthArgs a{};
  a.F = c->F;
  a.k = 0;
  std::vector<double*> eff(c->F, nullptr);
  double* dbeta = nullptr;
  double scale = 1.0;
  int rc = LFE_OK;
  for (int f = 0; f < c->F && rc == LFE_OK; ++f) {
    a.L[f] = levels[f];
    if (hipMalloc(&eff[f], sizeof(double) * (size_t)levels[f]) != hipSuccess) {
      rc = LFE_ENOMEM;
      break;
    }
    hipLaunchKernelGGL(k_synth_effects, dim3(grid_for(levels[f])), dim3(kBlock), 0, c->stream, eff[f], levels[f], f,
                       scale, seed);
    a.eff[f] = eff[f];
    scale *= 0.5;
  }
  if (rc == LFE_OK && hipMalloc(&dbeta, sizeof(double) * (size_t)std::max(K, 1)) != hipSuccess) rc = LFE_ENOMEM;
  if (rc == LFE_OK && K > 0 &&
      hipMemcpyAsync(dbeta, beta, sizeof(double) * (size_t)K, hipMemcpyHostToDevice, c->stream) != hipSuccess)
    rc = LFE_EHIP;
  if (rc == LFE_OK && rows)
    hipLaunchKernelGGL(k_synth_cols, dim3(grid_for(rows, kBlock, 256 * 16)), dim3(kBlock), 0, c->stream, a, K, c_lo,
                       c->p, dbeta, X, ld, rows, seed, row0);
  if (rc == LFE_OK && hipGetLastError() != hipSuccess) rc = LFE_EHIP;
  (void)hipStreamSynchronize(c->stream);
  for (auto* e : eff)
    if (e) (void)hipFree(e);
  if (dbeta) (void)hipFree(dbeta);
  if (rc != LFE_OK) set_error("synthetic column block: allocation or launch failed");
  return rc;
}

int synth_codes(lfe_ctx* c, const int32_t* levels, uint64_t seed, int64_t row0) {
  SynthArgs a{};
  a.F = c->F;
  a.k = 0;
  for (int f = 0; f < c->F; ++f) {
    a.L[f] = levels[f];
    a.code[f] = c->fe[f].code;
  }
  if (c->n)
    hipLaunchKernelGGL(k_synth_rows, dim3(grid_for(c->n, kBlock, 256 * 16)), dim3(kBlock), 0, c->stream, a,
                       static_cast<double*>(nullptr), c->ld, c->n, seed, row0, nullptr);
  LFE_HIP(hipGetLastError());
  LFE_HIP(hipStreamSynchronize(c->stream));
  return LFE_OK;
}

int synth_count_owned(lfe_ctx* c, int64_t n_total, int f, int32_t L, int32_t lo, int32_t hi, uint64_t seed,
                      std::vector<int64_t>& base, int64_t* n_local) {
  const int64_t nblk = std::max<int64_t>(1, (n_total + kOwnChunk - 1) / kOwnChunk);
  int32_t* cnt = nullptr;
  LFE_HIP(hipMalloc(&cnt, sizeof(int32_t) * (size_t)nblk));
  hipLaunchKernelGGL(k_own_count, dim3((unsigned)nblk), dim3(256), 0, c->stream, n_total, f, L, lo, hi, seed, cnt);
  std::vector<int32_t> h((size_t)nblk);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(h.data(), cnt, sizeof(int32_t) * (size_t)nblk, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(cnt);
  LFE_HIP(e);
  base.assign((size_t)nblk + 1, 0);
  for (int64_t b = 0; b < nblk; ++b) base[b + 1] = base[b] + h[b];
  *n_local = base[nblk];
  return LFE_OK;
}

int launch_synth_owned(lfe_ctx* c, int64_t n_total, int k, const int32_t* levels, const double* beta, uint64_t seed,
                       int f, int32_t lo, int32_t hi, const std::vector<int64_t>& base) {
  const int64_t nblk = (int64_t)base.size() - 1;
  int64_t* dbase = nullptr;
  int64_t* idx = nullptr;
  hipError_t e = hipMalloc(&dbase, sizeof(int64_t) * base.size());
  if (e == hipSuccess) e = hipMalloc(&idx, sizeof(int64_t) * (size_t)std::max<int64_t>(c->n, 1));
  if (e == hipSuccess)
    e = hipMemcpyAsync(dbase, base.data(), sizeof(int64_t) * base.size(), hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_own_index, dim3((unsigned)nblk), dim3(256), 0, c->stream, n_total, f, levels[f], lo, hi,
                       seed, dbase, idx);
    e = hipGetLastError();
  }
  int rc = LFE_OK;
  if (e == hipSuccess) rc = synth_fill(c, k, levels, beta, seed, 0, idx);
  else (void)hipStreamSynchronize(c->stream);
  if (dbase) (void)hipFree(dbase);
  if (idx) (void)hipFree(idx);
  LFE_HIP(e);
  return rc;
}

}  // namespace lfe

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

__global__ void k_synth_rows(SynthArgs a, double* __restrict__ X, int64_t ld, int64_t n, uint64_t seed,
                             int64_t row_offset) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t i = (uint64_t)(row_offset + r);
    int32_t g[kMaxFE];
    for (int f = 0; f < a.F; ++f) {
      double c = floor(uni(i, (uint64_t)f, seed) * (double)a.L[f]);
      c = fmin(c, (double)(a.L[f] - 1));
      g[f] = (int32_t)c;
      a.code[f][r] = g[f];
    }
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

int launch_synth(lfe_ctx* c, int k, const int32_t* levels, const double* beta, uint64_t seed, int64_t row_offset) {
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
                       c->ld, c->n, seed, row_offset);
  LFE_HIP(hipGetLastError());
  LFE_HIP(hipStreamSynchronize(c->stream));
  for (int f = 0; f < c->F; ++f) LFE_HIP(hipFree(eff[f]));
  return LFE_OK;
}

}  // namespace lfe

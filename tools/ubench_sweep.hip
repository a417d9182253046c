// Microbenchmarks for the sweep design: LDS f64 atomics, row gathers from L2 vs LDS.
// hipcc --offload-arch=gfx950 -O3 -munsafe-fp-atomics tools/ubench_sweep.hip -o /tmp/ubench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int P = 11;

// per row: W LDS f64 atomics into a [256][P] slice at random rows
__global__ __launch_bounds__(512) void lds_atomic(const int* __restrict__ h, int64_t n, double* out) {
  __shared__ double t[256 * P];
  for (int j = threadIdx.x; j < 256 * P; j += 512) t[j] = 0;
  __syncthreads();
  for (int64_t i = blockIdx.x * 512ll + threadIdx.x; i < n; i += gridDim.x * 512ll) {
    const int g = h[i] & 255;
#pragma unroll
    for (int c = 0; c < P; ++c) atomicAdd(&t[g * P + c], 1.0);
  }
  __syncthreads();
  for (int j = threadIdx.x; j < 256 * P; j += 512) atomicAdd(&out[j], t[j]);
}

// per row: gather a P-double row from a global table [G][P] (L2 resident), dwordx2 loads
__global__ __launch_bounds__(512) void gather_global(const int* __restrict__ g, int64_t n, const double* __restrict__ tab,
                                                     int G, double* out) {
  double acc = 0;
  for (int64_t i = blockIdx.x * 512ll + threadIdx.x; i < n; i += gridDim.x * 512ll) {
    const double* r = tab + (int64_t)(g[i] % G) * P;
#pragma unroll
    for (int c = 0; c < P; ++c) acc += r[c];
  }
  if (acc == 123.456) out[0] = acc;
}

// same with a 16-B aligned padded row (12 doubles) read as 6 x dwordx4
__global__ __launch_bounds__(512) void gather_global_v4(const int* __restrict__ g, int64_t n, const double2* __restrict__ tab,
                                                        int G, double* out) {
  double acc = 0;
  for (int64_t i = blockIdx.x * 512ll + threadIdx.x; i < n; i += gridDim.x * 512ll) {
    const double2* r = tab + (int64_t)(g[i] % G) * 6;
#pragma unroll
    for (int c = 0; c < 6; ++c) { double2 v = r[c]; acc += v.x + v.y; }
  }
  if (acc == 123.456) out[0] = acc;
}

// per row: gather a P-double row from an LDS table of G rows (G*P*8 <= 96 KB)
__global__ __launch_bounds__(512) void gather_lds(const int* __restrict__ g, int64_t n, const double* __restrict__ tab,
                                                  int G, double* out) {
  extern __shared__ double t[];
  for (int j = threadIdx.x; j < G * P; j += 512) t[j] = tab[j];
  __syncthreads();
  double acc = 0;
  for (int64_t i = blockIdx.x * 512ll + threadIdx.x; i < n; i += gridDim.x * 512ll) {
    const double* r = t + (g[i] % G) * P;
#pragma unroll
    for (int c = 0; c < P; ++c) acc += r[c];
  }
  if (acc == 123.456) out[0] = acc;
}

// stream codes only
__global__ __launch_bounds__(512) void codes_only(const int* __restrict__ g, int64_t n, double* out) {
  int acc = 0;
  for (int64_t i = blockIdx.x * 512ll + threadIdx.x; i < n; i += gridDim.x * 512ll) acc += g[i];
  if (acc == 123456) out[0] = acc;
}

int main() {
  const int64_t n = 50000000;
  std::vector<int> hh(n), hg(n);
  uint64_t s = 1;
  for (int64_t i = 0; i < n; ++i) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    hh[i] = (int)(s >> 33) % 100000;
    hg[i] = (int)((s >> 13) % 1000);
  }
  int *dh, *dg;
  double *tab, *out;
  CK(hipMalloc(&dh, n * 4)); CK(hipMalloc(&dg, n * 4));
  CK(hipMalloc(&tab, 100000 * 12 * 8)); CK(hipMalloc(&out, 1 << 20));
  CK(hipMemcpy(dh, hh.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dg, hg.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemset(tab, 0, 100000 * 12 * 8));
  CK(hipFuncSetAttribute((const void*)gather_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 1000 * P * 8));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto run = [&](const char* name, auto fn) {
    fn();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < 5; ++r) fn();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    printf("%-36s %8.3f ms  (%.1f Grows/s)\n", name, ms / 5, n / (ms / 5) / 1e6);
    return 0;
  };
  for (int grid : {512, 1024, 2048}) {
    printf("grid %d\n", grid);
    run("codes_only", [&] { codes_only<<<grid, 512>>>(dg, n, out); });
    run("lds_atomic f64 x11", [&] { lds_atomic<<<grid, 512>>>(dh, n, out); });
    run("gather_global 1000 rows dwordx2", [&] { gather_global<<<grid, 512>>>(dg, n, tab, 1000, out); });
    run("gather_global_v4 1000 rows dwordx4", [&] { gather_global_v4<<<grid, 512>>>(dg, n, (const double2*)tab, 1000, out); });
    run("gather_global 100000 rows dwordx2", [&] { gather_global<<<grid, 512>>>(dh, n, tab, 100000, out); });
    run("gather_lds 1000 rows", [&] { gather_lds<<<grid, 512, 1000 * P * 8>>>(dg, n, tab, 1000, out); });
  }
  return 0;
}

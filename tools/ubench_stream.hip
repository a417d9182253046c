// Microbenchmark: streaming P column-major f64 columns (the Gram/sums access
// pattern) under different work distributions.
// hipcc --offload-arch=gfx950 -O3 tools/ubench_stream.hip -o tools/ubench_stream
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));
constexpr int P = 11;

// 1. thread per row, grid-stride, one f64 per column
__global__ __launch_bounds__(256) void k_row(const double* __restrict__ X, int64_t ld, int64_t n, double* out) {
  double acc = 0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += gridDim.x * 256ll)
#pragma unroll
    for (int c = 0; c < P; ++c) acc += X[c * ld + i];
  if (acc == 123.456) out[0] = acc;
}

// 2. thread per 2 rows (d2), grid-stride
__global__ __launch_bounds__(256) void k_row2(const double* __restrict__ X, int64_t ld, int64_t n, double* out) {
  double acc = 0;
  for (int64_t i = (blockIdx.x * 256ll + threadIdx.x) * 2; i < n; i += gridDim.x * 512ll)
#pragma unroll
    for (int c = 0; c < P; ++c) { d2 v = *(const d2*)(X + c * ld + i); acc += v.x + v.y; }
  if (acc == 123.456) out[0] = acc;
}

// 3. lane layout (lane = 4 rows of column l&15), groups of 16 rows strided over all waves
template <int GU>
__global__ __launch_bounds__(256) void k_lane_inter(const double* __restrict__ X, int64_t ld, int64_t n, double* out) {
  const int lane = threadIdx.x & 63, c = lane & 15, kq = lane >> 4;
  const int64_t ngr = n / 16;
  const int64_t wid = blockIdx.x * 4ll + (threadIdx.x >> 6), nw = gridDim.x * 4ll;
  double acc = 0;
  for (int64_t g = wid * GU; g < ngr; g += nw * GU) {
    d4 v[GU];
#pragma unroll
    for (int u = 0; u < GU; ++u) v[u] = (c < P && g + u < ngr) ? *(const d4*)(X + c * ld + (g + u) * 16 + kq * 4) : d4{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < GU; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
  }
  if (acc == 123.456) out[0] = acc;
}

// 4. lane layout, each block owns a contiguous chunk of `chunk` rows (waves interleaved inside)
template <int GU>
__global__ __launch_bounds__(256) void k_lane_chunk(const double* __restrict__ X, int64_t ld, int64_t n, int64_t chunk,
                                                    double* out) {
  const int lane = threadIdx.x & 63, c = lane & 15, kq = lane >> 4, wave = threadIdx.x >> 6;
  double acc = 0;
  const int64_t nchunks = (n + chunk - 1) / chunk;
  for (int64_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const int64_t g0 = ch * chunk / 16, g1 = std::min(n, (ch + 1) * chunk) / 16;
    for (int64_t g = g0 + wave * GU; g < g1; g += 4 * GU) {
      d4 v[GU];
#pragma unroll
      for (int u = 0; u < GU; ++u) v[u] = (c < P && g + u < g1) ? *(const d4*)(X + c * ld + (g + u) * 16 + kq * 4) : d4{0, 0, 0, 0};
#pragma unroll
      for (int u = 0; u < GU; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
    }
  }
  if (acc == 123.456) out[0] = acc;
}

// 5. column-outer: each wave reads 64 consecutive rows x d2 of one column at a time (fully coalesced 1 KB)
__global__ __launch_bounds__(256) void k_colwave(const double* __restrict__ X, int64_t ld, int64_t n, double* out) {
  const int lane = threadIdx.x & 63;
  const int64_t wid = blockIdx.x * 4ll + (threadIdx.x >> 6), nw = gridDim.x * 4ll;
  double acc = 0;
  for (int64_t r = wid * 128; r < n; r += nw * 128) {
    d2 v[P];
#pragma unroll
    for (int c = 0; c < P; ++c) v[c] = *(const d2*)(X + c * ld + r + lane * 2);
#pragma unroll
    for (int c = 0; c < P; ++c) acc += v[c].x + v[c].y;
  }
  if (acc == 123.456) out[0] = acc;
}

// 6. lane layout with write: read P cols, write P-1 cols (resid scores pattern), interleaved
__global__ __launch_bounds__(256) void k_lane_rw(const double* __restrict__ X, double* __restrict__ Y, int64_t ld,
                                                 int64_t n) {
  const int lane = threadIdx.x & 63, c = lane & 15, kq = lane >> 4;
  const int64_t ngr = n / 16;
  const int64_t wid = blockIdx.x * 4ll + (threadIdx.x >> 6), nw = gridDim.x * 4ll;
  for (int64_t g = wid * 2; g < ngr; g += nw * 2) {
    d4 v[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) v[u] = (c < P && g + u < ngr) ? *(const d4*)(X + c * ld + (g + u) * 16 + kq * 4) : d4{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < 2; ++u)
      if (c >= 1 && c < P && g + u < ngr) *(d4*)(Y + (c - 1) * ld + (g + u) * 16 + kq * 4) = v[u] * 2.0;
  }
}

int main() {
  const int64_t n = 50000000, ld = n;
  double *X, *Y, *out;
  CK(hipMalloc(&X, sizeof(double) * P * ld));
  CK(hipMalloc(&Y, sizeof(double) * P * ld));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(X, 0, sizeof(double) * P * ld));
  CK(hipMemset(Y, 0, sizeof(double) * P * ld));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const double bytes = 8.0 * P * n;
  auto run = [&](const char* name, double nbytes, auto launch) -> int {
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e9;
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipEventRecord(a));
      launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      if (ms < best) best = ms;
    }
    printf("%-40s %8.3f ms  %7.0f GB/s\n", name, best, nbytes / best / 1e6);
    return 0;
  };
  for (int grid : {1024, 2048, 4096, 8192}) {
    char nm[64];
    snprintf(nm, 64, "row grid=%d", grid);
    run(nm, bytes, [&] { hipLaunchKernelGGL(k_row, dim3(grid), dim3(256), 0, 0, X, ld, n, out); });
    snprintf(nm, 64, "row2 grid=%d", grid);
    run(nm, bytes, [&] { hipLaunchKernelGGL(k_row2, dim3(grid), dim3(256), 0, 0, X, ld, n, out); });
    snprintf(nm, 64, "colwave grid=%d", grid);
    run(nm, bytes, [&] { hipLaunchKernelGGL(k_colwave, dim3(grid), dim3(256), 0, 0, X, ld, n, out); });
    snprintf(nm, 64, "lane_inter GU=1 grid=%d", grid);
    run(nm, bytes, [&] { hipLaunchKernelGGL(k_lane_inter<1>, dim3(grid), dim3(256), 0, 0, X, ld, n, out); });
    snprintf(nm, 64, "lane_inter GU=4 grid=%d", grid);
    run(nm, bytes, [&] { hipLaunchKernelGGL(k_lane_inter<4>, dim3(grid), dim3(256), 0, 0, X, ld, n, out); });
    snprintf(nm, 64, "lane_rw grid=%d", grid);
    run(nm, bytes * 2 * (P - 0.5) / P, [&] { hipLaunchKernelGGL(k_lane_rw, dim3(grid), dim3(256), 0, 0, X, Y, ld, n); });
  }
  for (int64_t chunk : {4096ll, 16384ll, 65536ll}) {
    for (int grid : {782, 2048, 4096}) {
      char nm[64];
      snprintf(nm, 64, "lane_chunk GU=4 chunk=%lld grid=%d", (long long)chunk, grid);
      run(nm, bytes, [&] { hipLaunchKernelGGL(k_lane_chunk<4>, dim3(grid), dim3(256), 0, 0, X, ld, n, chunk, out); });
    }
  }
  return 0;
}

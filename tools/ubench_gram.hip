// Ablation of the Gram pass's ingredients on the MFMA lane layout (50M rows,
// p = 11 columns, 1e5 x 1e3 groups): what each one costs in bandwidth.
// hipcc --offload-arch=gfx950 -O3 tools/ubench_gram.hip -o tools/ubench_gram
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int P = 11;
enum { F_CODES = 1, F_GQ = 2, F_LDS = 4, F_MFMA = 8 };

template <int FL, int GU>
__global__ __launch_bounds__(256) void k_abl(const double* __restrict__ X, const int* __restrict__ h,
                                             const int* __restrict__ q, const double* __restrict__ aQ,
                                             const double* __restrict__ aP, int64_t ld, int n, double* out) {
  __shared__ double slice[256 * P];
  const int lane = threadIdx.x & 63, c = lane & 15, kq = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int xl = c < P ? c : 0;
  const double* xb = X + (int64_t)xl * ld;
  // blocks own contiguous ranges of 16-row groups; slice = alpha_P of 256 groups
  const int ng = n / 16;
  const int g0 = (int)((int64_t)blockIdx.x * ng / gridDim.x), g1 = (int)((int64_t)(blockIdx.x + 1) * ng / gridDim.x);
  if (FL & F_LDS) {
    for (int j = threadIdx.x; j < 256 * P; j += 256) slice[j] = aP[j];
    __syncthreads();
  }
  d4 acc = {0, 0, 0, 0};
  double sink = 0;
  for (int gb = g0 + wave * GU; gb < g1; gb += 4 * GU) {
    d4 xv[GU];
    int4 hv[GU], qv[GU];
#pragma unroll
    for (int u = 0; u < GU; ++u) {
      const int r = (gb + u) * 16 + kq * 4;
      const bool live = gb + u < g1;
      xv[u] = live ? *(const d4*)(xb + r) : d4{0, 0, 0, 0};
      if (FL & F_CODES) {
        hv[u] = live ? *(const int4*)(h + r) : int4{0, 0, 0, 0};
        qv[u] = live ? *(const int4*)(q + r) : int4{0, 0, 0, 0};
      }
    }
    double ga[GU][4];
#pragma unroll
    for (int u = 0; u < GU; ++u)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int hh = (&hv[u].x)[s], qq = (&qv[u].x)[s];
        double v = 0;
        if (FL & F_GQ) v = aQ[(uint32_t)qq * P + xl];
        if (FL & F_LDS) v += slice[(uint32_t)(hh & 255) * P + xl];
        ga[u][s] = v;
      }
#pragma unroll
    for (int u = 0; u < GU; ++u) {
      double z[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) z[s] = xv[u][s] - ga[u][s];
      if (FL & F_MFMA) {
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(z[s], z[s], acc, 0, 0, 0);
      } else {
        sink += z[0] + z[1] + z[2] + z[3];
      }
    }
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] + sink == 123.456) out[0] = 1;
}

int main() {
  const int n = 50000000;
  const int64_t ld = n;
  double *X, *aQ, *aP, *out;
  int *h, *q;
  CK(hipMalloc(&X, sizeof(double) * P * ld));
  CK(hipMalloc(&h, sizeof(int) * n));
  CK(hipMalloc(&q, sizeof(int) * n));
  CK(hipMalloc(&aQ, sizeof(double) * 1000 * P));
  CK(hipMalloc(&aP, sizeof(double) * 100000 * P));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(X, 0, sizeof(double) * P * ld));
  CK(hipMemset(aQ, 0, sizeof(double) * 1000 * P));
  CK(hipMemset(aP, 0, sizeof(double) * 100000 * P));
  {
    std::vector<int> hh(n), qq(n);
    uint64_t s = 88172645463325252ull;
    for (int i = 0; i < n; ++i) {
      s ^= s << 13; s ^= s >> 7; s ^= s << 17;
      hh[i] = (int)(s % 100000); qq[i] = (int)((s >> 20) % 1000);
    }
    CK(hipMemcpy(h, hh.data(), sizeof(int) * n, hipMemcpyHostToDevice));
    CK(hipMemcpy(q, qq.data(), sizeof(int) * n, hipMemcpyHostToDevice));
  }
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const double bytes = (8.0 * P + 8) * n;
  auto run = [&](const char* name, auto kern, int grid) -> int {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, X, h, q, aQ, aP, ld, n, out);
    CK(hipDeviceSynchronize());
    float best = 1e9;
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipEventRecord(a));
      hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, X, h, q, aQ, aP, ld, n, out);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      if (ms < best) best = ms;
    }
    printf("%-34s grid=%5d %8.3f ms  %7.0f GB/s\n", name, grid, best, bytes / best / 1e6);
    return 0;
  };
#define RUN(FL, GU, G) run(#FL " GU=" #GU, k_abl<FL, GU>, G)
  for (int G : {1024, 2048}) {
    RUN(0, 2, G);
    RUN(1, 2, G);
    RUN(3, 2, G);
    RUN(5, 2, G);
    RUN(7, 2, G);
    RUN(15, 2, G);
    RUN(9, 2, G);
    RUN(15, 4, G);
    RUN(15, 1, G);
  }
  return 0;
}

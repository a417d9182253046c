// Checks the semantics of DPP row_newbcast:N on this GPU: lane l must receive
// lane (l & ~15) + N of the source (broadcast within each 16-lane row).
// hipcc --offload-arch=gfx950 -O3 tools/dpp_check.hip -o tools/dpp_check
#include <hip/hip_runtime.h>
#include <cstdio>
template <int N>
__global__ void k(int* out, const int* in) {
  const int v = in[threadIdx.x];
  out[threadIdx.x] = __builtin_amdgcn_update_dpp(0, v, 0x150 + N, 0xF, 0xF, false);
}
int main() {
  int *in, *out, h[64];
  hipMalloc(&in, 256); hipMalloc(&out, 256);
  for (int i = 0; i < 64; ++i) h[i] = 1000 + i;
  hipMemcpy(in, h, 256, hipMemcpyHostToDevice);
  int bad = 0;
#define T(N) hipLaunchKernelGGL(k<N>, 1, 64, 0, 0, out, in); hipMemcpy(h, out, 256, hipMemcpyDeviceToHost); \
  for (int l = 0; l < 64; ++l) if (h[l] != 1000 + (l & ~15) + N) { if (bad < 8) printf("N=%d lane %d got %d\n", N, l, h[l]); ++bad; }
  T(0) T(1) T(3) T(7) T(15)
  printf("row_newbcast check: %s\n", bad ? "MISMATCH" : "ok");
  return bad != 0;
}

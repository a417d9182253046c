// Probe of the v_mfma_i32_16x16x64_i8 operand maps (cdna_hip_programming.md: "check the map with
// exact integer data before relying on it").  Each lane loads 16 i8 values of A and of B as
// A[row l&15][k = 16 (l >> 4) + j], B[k = 16 (l >> 4) + j][col l&15] (the bf16 16x16x32 pattern
// widened to 16 elements), the product is compared with a host GEMM of the same asymmetric data,
// and the C/D map col = l&15, row = 4 (l >> 4) + r is checked at the same time.
//   hipcc --offload-arch=gfx950 -O2 tools/mfma_i8_probe.hip -o tools/mfma_i8_probe && tools/mfma_i8_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void k_probe(const signed char* A, const signed char* B, int* D) {
  const int l = threadIdx.x, i = l & 15, g = l >> 4;
  v4i a, b;
  signed char* ap = reinterpret_cast<signed char*>(&a);
  signed char* bp = reinterpret_cast<signed char*>(&b);
  for (int j = 0; j < 16; ++j) {
    ap[j] = A[i * 64 + 16 * g + j];   // A [16][64] row-major
    bp[j] = B[(16 * g + j) * 16 + i]; // B [64][16] row-major
  }
  v4i acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(4 * g + r) * 16 + i] = acc[r];
}

int main() {
  signed char hA[16 * 64], hB[64 * 16];
  for (int i = 0; i < 16 * 64; ++i) hA[i] = (signed char)((i * 37 + 11) % 255 - 127);
  for (int i = 0; i < 64 * 16; ++i) hB[i] = (signed char)((i * 53 + 5) % 251 - 125);
  int ref[256];
  for (int r = 0; r < 16; ++r)
    for (int c = 0; c < 16; ++c) {
      int s = 0;
      for (int k = 0; k < 64; ++k) s += (int)hA[r * 64 + k] * (int)hB[k * 16 + c];
      ref[r * 16 + c] = s;
    }
  signed char *dA, *dB;
  int* dD;
  if (hipMalloc(&dA, sizeof(hA)) || hipMalloc(&dB, sizeof(hB)) || hipMalloc(&dD, 256 * sizeof(int))) return 2;
  hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof(hB), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  int hD[256];
  hipMemcpy(hD, dD, sizeof(hD), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int e = 0; e < 256; ++e) bad += hD[e] != ref[e];
  printf("mfma_i32_16x16x64_i8 map A[l&15][16(l>>4)+j], B[16(l>>4)+j][l&15], D row 4(l>>4)+r: %s (%d of 256 wrong)\n",
         bad ? "MISMATCH" : "OK", bad);
  if (bad) {
    for (int e = 0; e < 8; ++e) printf("  D[%d] = %d ref %d\n", e, hD[e], ref[e]);
  }
  hipFree(dA);
  hipFree(dB);
  hipFree(dD);
  return bad ? 1 : 0;
}

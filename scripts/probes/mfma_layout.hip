#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f16v __attribute__((ext_vector_type(16)));
__global__ void k(const float* A, const float* B, float* D, unsigned* P) {
  int l = threadIdx.x;
  // A: 32x2 (row l%32, k l/32); B: 2x32 (col l%32, k l/32)
  float a = A[(l % 32) * 2 + l / 32];
  float b = B[(l / 32) * 32 + l % 32];
  f16v c = {0};
  c = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  for (int v = 0; v < 16; v++) D[l * 16 + v] = c[v];
  auto r = __builtin_amdgcn_permlane32_swap((unsigned)l, (unsigned)(100 + l), false, false);
  P[l * 2] = r[0]; P[l * 2 + 1] = r[1];
}
int main() {
  float hA[64], hB[64]; for (int i = 0; i < 64; i++) { hA[i] = i % 7 + 1; hB[i] = (i * 3) % 5 + 1; }
  float *dA, *dB, *dD; unsigned* dP;
  hipMalloc(&dA, 256); hipMalloc(&dB, 256); hipMalloc(&dD, 64 * 16 * 4); hipMalloc(&dP, 512);
  hipMemcpy(dA, hA, 256, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 256, hipMemcpyHostToDevice);
  k<<<1, 64>>>(dA, dB, dD, dP);
  float hD[1024]; unsigned hP[128];
  hipMemcpy(hD, dD, 4096, hipMemcpyDeviceToHost); hipMemcpy(hP, dP, 512, hipMemcpyDeviceToHost);
  // check hypothesis: lane l, vgpr v -> D[i][j], j = l%32, i = 8*(v/4) + 4*(l/32) + v%4
  int bad = 0;
  for (int l = 0; l < 64; l++) for (int v = 0; v < 16; v++) {
    int j = l % 32, i = 8 * (v / 4) + 4 * (l / 32) + v % 4;
    float ref = hA[i * 2] * hB[j] + hA[i * 2 + 1] * hB[32 + j];
    if (ref != hD[l * 16 + v]) bad++;
  }
  printf("layout mismatches %d\n", bad);
  printf("swap lane0 %u %u lane31 %u %u lane32 %u %u lane63 %u %u\n", hP[0], hP[1], hP[62], hP[63], hP[64], hP[65], hP[126], hP[127]);
  return 0;
}

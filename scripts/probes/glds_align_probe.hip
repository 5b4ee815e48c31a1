// Does global_load_lds (16 bytes per lane) accept 4-byte-aligned global sources on gfx950?
// Each lane copies 16 B from src + 4*(offset + 4*lane) bytes into LDS (lane-linear), then the wave
// writes LDS back to dst; the host compares with the expected floats.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_probe(const float* src, float* dst, int offset) {
  __shared__ __attribute__((aligned(16))) float lds[256];
  const int lane = threadIdx.x;
  const float* p = src + offset + 4 * lane;
  __builtin_amdgcn_global_load_lds(p, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = 0; i < 4; i++) dst[4 * lane + i] = lds[4 * lane + i];
}

int main() {
  const int n = 1024;
  std::vector<float> h(n);
  for (int i = 0; i < n; i++) h[i] = (float)i;
  float *s, *d;
  hipMalloc(&s, n * 4);
  hipMalloc(&d, 256 * 4);
  hipMemcpy(s, h.data(), n * 4, hipMemcpyHostToDevice);
  for (int off = 0; off < 4; off++) {
    hipMemset(d, 0, 256 * 4);
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, s, d, off);
    hipError_t e = hipDeviceSynchronize();
    std::vector<float> o(256);
    hipMemcpy(o.data(), d, 256 * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; i++) bad += o[i] != (float)(off + i);
    printf("offset %d floats (%d-byte aligned): %s, %d of 256 wrong, first %g %g %g %g\n", off, off ? 4 : 16,
           hipGetErrorString(e), bad, o[0], o[1], o[2], o[3]);
  }
  return 0;
}

// Where does the dispatcher put K_step's blocks?  A kernel with K_step's launch shape (2048 blocks
// of one 64-lane wave, 19.5 KB of LDS per block, amdgpu_waves_per_eu(2, 2)) records per block its
// HW_ID (wave slot, SIMD, CU, shader array / engine) and XCC_ID hardware registers and a start
// timestamp, then holds the wave for a while so every block is resident at once.  Printed as one
// line per block: block xcc se sh cu simd wave t_start.  Development probe (scripts/probes/).
//
//   hipcc --offload-arch=gfx950 -O3 scripts/probes/placement_probe.hip -o scripts/probes/placement_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2))) k_place(unsigned* out, float* sink,
                                                                                       int spin) {
  __shared__ float lds[4992];  // 19.5 KB, as K_step's two EnvSh
  unsigned hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  const unsigned long long t = __builtin_amdgcn_s_memrealtime();
  float acc = threadIdx.x;
  for (int i = threadIdx.x; i < 4992; i += 64) lds[i] = acc + i;
  __syncthreads();
  for (int k = 0; k < spin; k++) acc = acc * 0.999f + lds[(threadIdx.x * 7 + k) % 4992];
  if (threadIdx.x == 0) {
    out[4 * blockIdx.x + 0] = hw;
    out[4 * blockIdx.x + 1] = xcc;
    out[4 * blockIdx.x + 2] = (unsigned)(t & 0xffffffffu);
    out[4 * blockIdx.x + 3] = (unsigned)(t >> 32);
  }
  if (acc == 12345.f) sink[blockIdx.x] = acc;  // keeps the loop
}

int main() {
  const int nb = 2048;
  unsigned* d;
  float* sink;
  hipMalloc(&d, nb * 16);
  hipMalloc(&sink, nb * 4);
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_place, dim3(nb), dim3(64), 0, 0, d, sink, 20000);
    hipDeviceSynchronize();
  }
  std::vector<unsigned> h(nb * 4);
  hipMemcpy(h.data(), d, nb * 16, hipMemcpyDeviceToHost);
  unsigned long long t0 = ~0ull;
  for (int b = 0; b < nb; b++) {
    unsigned long long t = ((unsigned long long)h[4 * b + 3] << 32) | h[4 * b + 2];
    if (t < t0) t0 = t;
  }
  for (int b = 0; b < nb; b++) {
    const unsigned hw = h[4 * b];
    unsigned long long t = ((unsigned long long)h[4 * b + 3] << 32) | h[4 * b + 2];
    // gfx9 HW_ID: wave_id [3:0], simd_id [5:4], pipe_id [7:6], cu_id [11:8], sh_id [12], se_id [15:13]
    printf("%d %u %u %u %u %u %u %llu\n", b, h[4 * b + 1] & 0xf, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 0xf,
           (hw >> 4) & 3, hw & 0xf, t - t0);
  }
  hipFree(d);
  hipFree(sink);
  return 0;
}

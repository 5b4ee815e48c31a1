// Probe: half-wave lane broadcast via row_newbcast + v_permlane16_swap (gfx950), checked against
// the readlane definition for every source lane.  hipcc --offload-arch=gfx950 -O2 -o /tmp/bp bcast_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int R, int SEL>
__device__ __forceinline__ float bcast32(float x) {
  constexpr int n = R & 15;
  const int v = __builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x150 + n, 0xF, 0xF, false);
  auto sw = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  const int s = SEL ? (int)sw[1] : (int)sw[0];
  const bool odd_row = (__lane_id() >> 4) & 1;
  const int out = (R < 16) ? (odd_row ? s : v) : (odd_row ? v : s);
  return __int_as_float(out);
}

template <int R>
__device__ void one(float x, float* out) {
  out[(R * 2 + 0) * 64 + threadIdx.x] = bcast32<R, 0>(x);
  out[(R * 2 + 1) * 64 + threadIdx.x] = bcast32<R, 1>(x);
}
template <int... Rs>
__device__ void all(float x, float* out, std::integer_sequence<int, Rs...>) { (one<Rs>(x, out), ...); }

__global__ void k(float* out) {
  const float x = (float)threadIdx.x;
  all(x, out, std::make_integer_sequence<int, 32>{});
}

int main() {
  float* d;
  hipMalloc(&d, 64 * 64 * sizeof(float));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  float h[64 * 64];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int sel = 0; sel < 2; sel++) {
    int bad = 0;
    for (int r = 0; r < 32; r++)
      for (int l = 0; l < 64; l++) {
        const float want = (float)((l < 32 ? 0 : 32) + r);
        if (h[(r * 2 + sel) * 64 + l] != want) bad++;
      }
    printf("sel %d: %d mismatches\n", sel, bad);
    for (int r : {3, 21}) {
      printf("R=%d sel=%d:", r, sel);
      for (int l = 0; l < 64; l += 4) printf(" %g", h[(r * 2 + sel) * 64 + l]);
      printf("\n");
    }
  }
  return 0;
}

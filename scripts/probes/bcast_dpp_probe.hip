// Checks the half-wave broadcast built from DPP row_newbcast + v_permlane16_swap against the
// ds_swizzle form K_step uses (lane R of this lane's 32-lane half), for every R.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int R>
__device__ __forceinline__ float bc_dpp(float x) {
  int y = __builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x150 | (R & 15), 0xF, 0xF, false);
  auto p = __builtin_amdgcn_permlane16_swap(y, y, false, false);
  return __int_as_float(R < 16 ? p[0] : p[1]);
}
template <int R>
__device__ __forceinline__ float bc_swz(float x) {
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(x), R << 5));
}
template <int R>
__device__ void check(float x, int* bad) {
  if (bc_dpp<R>(x) != bc_swz<R>(x)) atomicAdd(bad, 1);
  if constexpr (R < 31) check<R + 1>(x, bad);
}
__global__ void k(int* bad) {
  float x = 1000.f + threadIdx.x;
  check<0>(x, bad);
}
int main() {
  int* d; hipMalloc(&d, 4); hipMemset(d, 0, 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  int h = -1; hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
  printf("bcast_dpp_probe mismatches: %d\n", h);
  return h != 0;
}

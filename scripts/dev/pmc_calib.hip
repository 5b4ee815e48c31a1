// FETCH_SIZE / WRITE_SIZE calibration for the access widths the env-logic kernels use (development
// tool).  Each kernel moves a known byte count; rocprofv3 --pmc FETCH_SIZE (or WRITE_SIZE) over
// this binary gives counter bytes per launch, and the ratio is the correction for that pattern.
//   rd_dword_row64 : 4 B/lane, 64 consecutive lanes -> 256 B contiguous (SoA row of 64 envs)
//   rd_dword_row16 : 4 B/lane, 16-lane groups reading 64 B of a row (SoA row of a 16-env block)
//   rd_x4          : 16 B/lane streaming (the guide's calibrated case: FETCH = 1/2 bytes)
//   wr_dword_row16 : 4 B/lane stores, 16-lane groups (64 B)
//   wr_x4          : 16 B/lane streaming stores
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int N = 1 << 24;  // 64 MiB of floats per buffer (past L2; read once)

__global__ void rd_dword_row64(const float* __restrict__ a, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float v = a[i];
  if (v == 12345.f) out[0] = v;  // keep the load
}
__global__ void rd_dword_row16(const float* __restrict__ a, float* __restrict__ out) {
  // block of 256 threads = 16 rows x 16 lanes; row r of the block reads 16 floats at r * (N / 16) + blk * 16
  const int lane = threadIdx.x & 15, r = threadIdx.x >> 4;
  const size_t idx = (size_t)r * (N / 16) + (size_t)blockIdx.x * 16 + lane;
  float v = a[idx];
  if (v == 12345.f) out[0] = v;
}
__global__ void rd_x4(const float4* __restrict__ a, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float4 v = a[i];
  if (v.x + v.y + v.z + v.w == 12345.f) out[0] = v.x;
}
__global__ void wr_dword_row16(float* __restrict__ a) {
  const int lane = threadIdx.x & 15, r = threadIdx.x >> 4;
  const size_t idx = (size_t)r * (N / 16) + (size_t)blockIdx.x * 16 + lane;
  a[idx] = 1.f;
}
__global__ void wr_x4(float4* __restrict__ a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  a[i] = make_float4(1.f, 1.f, 1.f, 1.f);
}

int main() {
  float *a, *b, *out;
  hipMalloc(&a, (size_t)N * 4);
  hipMalloc(&b, (size_t)N * 4);
  hipMalloc(&out, 64);
  hipMemset(a, 0, (size_t)N * 4);
  hipMemset(b, 0, (size_t)N * 4);
  // flush between launches: stream a third 256 MiB+ buffer so the Infinity Cache holds nothing of a / b
  float* flush;
  const size_t FL = (size_t)80 << 20;  // 320 MiB
  hipMalloc(&flush, FL * 4);
  auto fl = [&]() { hipMemset(flush, 1, FL * 4); hipDeviceSynchronize(); };
  for (int rep = 0; rep < 2; rep++) {
    fl(); hipLaunchKernelGGL(rd_dword_row64, dim3(N / 256), dim3(256), 0, 0, a, out); hipDeviceSynchronize();
    fl(); hipLaunchKernelGGL(rd_dword_row16, dim3(N / 256), dim3(256), 0, 0, a, out); hipDeviceSynchronize();
    fl(); hipLaunchKernelGGL(rd_x4, dim3(N / 4 / 256), dim3(256), 0, 0, (const float4*)a, out); hipDeviceSynchronize();
    fl(); hipLaunchKernelGGL(wr_dword_row16, dim3(N / 256), dim3(256), 0, 0, b); hipDeviceSynchronize();
    fl(); hipLaunchKernelGGL(wr_x4, dim3(N / 4 / 256), dim3(256), 0, 0, (float4*)b); hipDeviceSynchronize();
  }
  printf("bytes per launch: %zu\n", (size_t)N * 4);
  return 0;
}

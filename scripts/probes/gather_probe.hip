// Variants of the minibatch gather of frame-only rollout storage (hg_gather_stacked's f32 path with
// two plain tables, csrc/hg_rollout.hip) at the bench's shapes: N = 4096 envs, T = 24, a 15 x 47
// frame stack (705), the 219-wide critic rows and a 43-wide packed per-sample table, 24576 rows
// gathered by a random permutation.  Every variant's output is compared with V0's; time per call
// from HIP events (200 calls after 20 warm-up, three interleaved rounds).  Development probe.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/probes/gather_probe.hip -o scripts/probes/gather_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);          \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));
constexpr int TPB = 256;

struct Args {
  const int64_t* idx;
  int64_t rows;
  const float* frames;
  const float* init;
  const uint8_t* dones;  // env-major [N][T]
  int T, N, F, W;
  float* dst;
  const float* tsrc[2];
  float* tdst[2];
  int tw[2];
};

// the plain tables: lane l moves elements 4l .. 4l + 3 (width <= 256)
__device__ __forceinline__ void tab_load(const Args& A, int64_t s, f32x4u pv[2]) {
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const float* src = A.tsrc[q] + s * A.tw[q];
    const int w = A.tw[q], c = 4 * (threadIdx.x & 63);
    if (c + 3 < w) pv[q] = *reinterpret_cast<const f32x4u*>(src + c);
    else
      for (int k = 0; k < 4; k++) pv[q][k] = c + k < w ? src[c + k] : 0.f;
  }
}
__device__ __forceinline__ void tab_store(const Args& A, int64_t i, const f32x4u pv[2]) {
#pragma unroll
  for (int q = 0; q < 2; q++) {
    float* d = A.tdst[q] + i * A.tw[q];
    const int w = A.tw[q], c = 4 * (threadIdx.x & 63);
    if (c + 3 < w) *reinterpret_cast<f32x4u*>(d + c) = pv[q];
    else
      for (int k = 0; k < 4; k++)
        if (c + k < w) d[c + k] = pv[q][k];
  }
}

// V0: the shipped kernel's f32 path (int64 index math)
__global__ void __launch_bounds__(TPB) k_v0(Args A) {
  const int64_t i = (int64_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= A.rows) return;
  const int64_t total = (int64_t)A.T * A.N;
  int64_t s = A.idx[i];
  s = s < 0 ? 0 : (s >= total ? total - 1 : s);
  const int t = (int)(s / A.N), e = (int)(s - (int64_t)t * A.N);
  f32x4u pv[2];
  tab_load(A, s, pv);
  const int F = A.F, W = A.W, T = A.T;
  const int back = t - 1 - lane;
  const bool scan = lane < F - 1 && back >= 0;
  uint32_t dz = A.dones[(int64_t)max(back, 0) * 1 + (int64_t)e * T];
  const int row = F * W;
  const int Bnd = (t < F - 1 ? F - 1 - t : 0) * W;
  const float* srcA = A.init + (int64_t)e * row + (int64_t)t * W;
  const int64_t offB = ((int64_t)e * T + t - (F - 1)) * W;
  float* out = A.dst + i * (int64_t)row;
  constexpr int KD = 12;
  for (int base = 0; base < row; base += 64 * KD) {
    float v[KD];
#pragma unroll
    for (int k = 0; k < KD; k++) {
      const int c = min(base + lane + 64 * k, row - 1);
      const uintptr_t a = c < Bnd ? (uintptr_t)(srcA + c) : (uintptr_t)(A.frames + offB + c);
      v[k] = *reinterpret_cast<const __attribute__((address_space(1))) float*>(a);
    }
    asm volatile("" : "+v"(dz));
    const uint64_t m = __ballot(scan && dz != 0);
    const int Z = (m ? F - 1 - (__ffsll((unsigned long long)m) - 1) : 0) * W;
#pragma unroll
    for (int k = 0; k < KD; k++) {
      const int c = base + lane + 64 * k;
      if (c < row) out[c] = c < Z ? 0.f : v[k];
    }
  }
  tab_store(A, i, pv);
}

// V1: 32-bit index math (T N < 2^31), otherwise V0
__global__ void __launch_bounds__(TPB) k_v1(Args A) {
  const int64_t i = (int64_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= A.rows) return;
  const int total = A.T * A.N;
  int s = (int)min<int64_t>(max<int64_t>(A.idx[i], 0), total - 1);
  const int t = s / A.N, e = s - t * A.N;
  f32x4u pv[2];
  tab_load(A, s, pv);
  const int F = A.F, W = A.W, T = A.T;
  const int back = t - 1 - lane;
  const bool scan = lane < F - 1 && back >= 0;
  uint32_t dz = A.dones[max(back, 0) + e * T];
  const int row = F * W;
  const int Bnd = (t < F - 1 ? F - 1 - t : 0) * W;
  const float* srcA = A.init + (int64_t)e * row + t * W;
  const float* srcB = A.frames + ((int64_t)e * T + t - (F - 1)) * W;
  float* out = A.dst + i * (int64_t)row;
  constexpr int KD = 12;
  for (int base = 0; base < row; base += 64 * KD) {
    float v[KD];
#pragma unroll
    for (int k = 0; k < KD; k++) {
      const int c = min(base + lane + 64 * k, row - 1);
      const uintptr_t a = c < Bnd ? (uintptr_t)(srcA + c) : (uintptr_t)(srcB + c);
      v[k] = *reinterpret_cast<const __attribute__((address_space(1))) float*>(a);
    }
    asm volatile("" : "+v"(dz));
    const uint64_t m = __ballot(scan && dz != 0);
    const int Z = (m ? F - 1 - (__ffsll((unsigned long long)m) - 1) : 0) * W;
#pragma unroll
    for (int k = 0; k < KD; k++) {
      const int c = base + lane + 64 * k;
      if (c < row) out[c] = c < Z ? 0.f : v[k];
    }
  }
  tab_store(A, i, pv);
}

// V2: V1 with 16-byte frame loads and stores (4-byte aligned vector accesses) on the rows whose
// stack is all in the frame table (Bnd == 0, a wave-uniform branch); V1's dword path otherwise
__global__ void __launch_bounds__(TPB) k_v2(Args A) {
  const int64_t i = (int64_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= A.rows) return;
  const int total = A.T * A.N;
  int s = (int)min<int64_t>(max<int64_t>(A.idx[i], 0), total - 1);
  const int t = s / A.N, e = s - t * A.N;
  f32x4u pv[2];
  tab_load(A, s, pv);
  const int F = A.F, W = A.W, T = A.T;
  const int back = t - 1 - lane;
  const bool scan = lane < F - 1 && back >= 0;
  uint32_t dz = A.dones[max(back, 0) + e * T];
  const int row = F * W;
  const int Bnd = (t < F - 1 ? F - 1 - t : 0) * W;
  const float* srcA = A.init + (int64_t)e * row + t * W;
  const float* srcB = A.frames + ((int64_t)e * T + t - (F - 1)) * W;
  float* out = A.dst + i * (int64_t)row;
  if (Bnd == 0 && row <= 1024) {
    constexpr int KV = 4;  // 4 x 256 elements
    f32x4u v[KV];
#pragma unroll
    for (int k = 0; k < KV; k++) {
      const int c = min(4 * (lane + 64 * k), row - 4);
      v[k] = *reinterpret_cast<const f32x4u*>(srcB + c);
    }
    asm volatile("" : "+v"(dz));
    const uint64_t m = __ballot(scan && dz != 0);
    const int Z = (m ? F - 1 - (__ffsll((unsigned long long)m) - 1) : 0) * W;
#pragma unroll
    for (int k = 0; k < KV; k++) {
      const int c = 4 * (lane + 64 * k);
      for (int q = 0; q < 4; q++)
        if (c + q < Z) v[k][q] = 0.f;
      if (c + 3 < row) {
        *reinterpret_cast<f32x4u*>(out + c) = v[k];
      } else if (c < row) {
        // the row's tail: reload the last 4 from the clamped start (c0 = row - 4) already held by
        // this lane only if c == row - 4 -- handled element by element
        for (int q = 0; q < 4; q++)
          if (c + q < row) out[c + q] = (c + q < Z) ? 0.f : srcB[c + q];
      }
    }
  } else {
    constexpr int KD = 12;
    for (int base = 0; base < row; base += 64 * KD) {
      float v[KD];
#pragma unroll
      for (int k = 0; k < KD; k++) {
        const int c = min(base + lane + 64 * k, row - 1);
        const uintptr_t a = c < Bnd ? (uintptr_t)(srcA + c) : (uintptr_t)(srcB + c);
        v[k] = *reinterpret_cast<const __attribute__((address_space(1))) float*>(a);
      }
      asm volatile("" : "+v"(dz));
      const uint64_t m = __ballot(scan && dz != 0);
      const int Z = (m ? F - 1 - (__ffsll((unsigned long long)m) - 1) : 0) * W;
#pragma unroll
      for (int k = 0; k < KD; k++) {
        const int c = base + lane + 64 * k;
        if (c < row) out[c] = c < Z ? 0.f : v[k];
      }
    }
  }
  tab_store(A, i, pv);
}

// V3: V1 with two rows per wave (rows i and i + half; all loads of both issued before either's
// stores)
__global__ void __launch_bounds__(TPB) k_v3(Args A) {
  const int64_t half = (A.rows + 1) / 2;
  const int64_t i0 = (int64_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i0 >= half) return;
  const int total = A.T * A.N;
  const int F = A.F, W = A.W, T = A.T, row = F * W;
  constexpr int KD = 12;
  int64_t ii[2] = {i0, i0 + half};
  bool ok[2] = {true, i0 + half < A.rows};
  float v[2][KD];
  f32x4u pv[2][2];
  uint32_t dz[2];
  bool scan[2];
  const float* src[2][2];
  int Bnd[2];
#pragma unroll
  for (int r = 0; r < 2; r++) {
    const int64_t i = ok[r] ? ii[r] : ii[0];
    int s = (int)min<int64_t>(max<int64_t>(A.idx[i], 0), total - 1);
    const int t = s / A.N, e = s - t * A.N;
    tab_load(A, s, pv[r]);
    const int back = t - 1 - lane;
    scan[r] = lane < F - 1 && back >= 0;
    dz[r] = A.dones[max(back, 0) + e * T];
    Bnd[r] = (t < F - 1 ? F - 1 - t : 0) * W;
    src[r][0] = A.init + (int64_t)e * row + t * W;
    src[r][1] = A.frames + ((int64_t)e * T + t - (F - 1)) * W;
#pragma unroll
    for (int k = 0; k < KD; k++) {
      const int c = min(lane + 64 * k, row - 1);
      const uintptr_t a = c < Bnd[r] ? (uintptr_t)(src[r][0] + c) : (uintptr_t)(src[r][1] + c);
      v[r][k] = *reinterpret_cast<const __attribute__((address_space(1))) float*>(a);
    }
  }
#pragma unroll
  for (int r = 0; r < 2; r++) {
    asm volatile("" : "+v"(dz[r]));
    const uint64_t m = __ballot(scan[r] && dz[r] != 0);
    const int Z = (m ? F - 1 - (__ffsll((unsigned long long)m) - 1) : 0) * W;
    if (!ok[r]) continue;
    float* out = A.dst + ii[r] * (int64_t)row;
#pragma unroll
    for (int k = 0; k < KD; k++) {
      const int c = lane + 64 * k;
      if (c < row) out[c] = c < Z ? 0.f : v[r][k];
    }
    tab_store(A, ii[r], pv[r]);
  }
}

int main() {
  const int N = 4096, T = 24, F = 15, W = 47, row = F * W;
  const int64_t rows = 24576;
  const int tw[2] = {219, 43};
  std::mt19937 rng(1);
  std::vector<float> h_frames((size_t)N * T * W), h_init((size_t)N * row), h_t0((size_t)T * N * tw[0]),
      h_t1((size_t)T * N * tw[1]);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  for (auto& x : h_frames) x = U(rng);
  for (auto& x : h_init) x = U(rng);
  for (auto& x : h_t0) x = U(rng);
  for (auto& x : h_t1) x = U(rng);
  std::vector<uint8_t> h_dones((size_t)N * T);
  for (auto& d : h_dones) d = (rng() % 100) < 2;  // 2 % resets
  std::vector<int64_t> perm((size_t)T * N);
  std::iota(perm.begin(), perm.end(), 0);
  std::shuffle(perm.begin(), perm.end(), rng);
  perm.resize(rows);
  float *frames, *init, *t0, *t1;
  uint8_t* dones;
  int64_t* idx;
  CK(hipMalloc(&frames, h_frames.size() * 4));
  CK(hipMalloc(&init, h_init.size() * 4));
  CK(hipMalloc(&t0, h_t0.size() * 4));
  CK(hipMalloc(&t1, h_t1.size() * 4));
  CK(hipMalloc(&dones, h_dones.size()));
  CK(hipMalloc(&idx, rows * 8));
  CK(hipMemcpy(frames, h_frames.data(), h_frames.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(init, h_init.data(), h_init.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(t0, h_t0.data(), h_t0.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(t1, h_t1.data(), h_t1.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dones, h_dones.data(), h_dones.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(idx, perm.data(), rows * 8, hipMemcpyHostToDevice));
  const int NV = 4;
  float *dst[NV], *d0[NV], *d1[NV];
  for (int v = 0; v < NV; v++) {
    CK(hipMalloc(&dst[v], rows * row * 4));
    CK(hipMalloc(&d0[v], rows * tw[0] * 4));
    CK(hipMalloc(&d1[v], rows * tw[1] * 4));
  }
  auto args = [&](int v) {
    Args A;
    A.idx = idx; A.rows = rows; A.frames = frames; A.init = init; A.dones = dones;
    A.T = T; A.N = N; A.F = F; A.W = W; A.dst = dst[v];
    A.tsrc[0] = t0; A.tsrc[1] = t1; A.tdst[0] = d0[v]; A.tdst[1] = d1[v]; A.tw[0] = tw[0]; A.tw[1] = tw[1];
    return A;
  };
  const int blocks = (int)((rows + 3) / 4), blocks2 = (int)(((rows + 1) / 2 + 3) / 4);
  auto launch = [&](int v) {
    Args A = args(v);
    if (v == 0) hipLaunchKernelGGL(k_v0, dim3(blocks), dim3(TPB), 0, 0, A);
    if (v == 1) hipLaunchKernelGGL(k_v1, dim3(blocks), dim3(TPB), 0, 0, A);
    if (v == 2) hipLaunchKernelGGL(k_v2, dim3(blocks), dim3(TPB), 0, 0, A);
    if (v == 3) hipLaunchKernelGGL(k_v3, dim3(blocks2), dim3(TPB), 0, 0, A);
  };
  for (int v = 0; v < NV; v++) launch(v);
  CK(hipDeviceSynchronize());
  std::vector<float> ref((size_t)rows * row), got((size_t)rows * row), r0(rows * tw[0]), g0(rows * tw[0]),
      r1(rows * tw[1]), g1(rows * tw[1]);
  CK(hipMemcpy(ref.data(), dst[0], ref.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(r0.data(), d0[0], r0.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(r1.data(), d1[0], r1.size() * 4, hipMemcpyDeviceToHost));
  for (int v = 1; v < NV; v++) {
    CK(hipMemcpy(got.data(), dst[v], got.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(g0.data(), d0[v], g0.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(g1.data(), d1[v], g1.size() * 4, hipMemcpyDeviceToHost));
    const bool same = !memcmp(ref.data(), got.data(), ref.size() * 4) && !memcmp(r0.data(), g0.data(), r0.size() * 4) &&
                      !memcmp(r1.data(), g1.data(), r1.size() * 4);
    printf("V%d equal to V0: %s\n", v, same ? "yes" : "NO");
  }
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int round = 0; round < 3; round++) {
    for (int v = 0; v < NV; v++) {
      for (int k = 0; k < 20; k++) launch(v);
      CK(hipEventRecord(a));
      for (int k = 0; k < 200; k++) launch(v);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("round %d V%d %.2f us\n", round, v, ms * 1000.f / 200);
    }
  }
  return 0;
}

// hg_gae.hip — K_gae: fused reverse-time GAE scan + advantage normalisation over the rollout
// buffer.  Replaces RolloutStorage.compute_returns (humanoid/algo/ppo/rollout_storage.py:122-143),
// which runs T tiny torch kernels per iteration plus mean/std reductions.
//
// Pass 1 (k_gae_scan): one lane per env walks t = T-1..0 with the carry in a register; every
// [t, :] row it touches is a contiguous 4*N-byte stream, so the wave's loads/stores coalesce.
// The op order of the reference is kept and FMA contraction is disabled (clang fp contract(off);
// plus -ffp-contract=off for this file), so returns match the reference bitwise.
// Per-block (sum A, sum A^2) partials are written in fp64 to stats[2 + 2b .. 3 + 2b] and a
// one-wave final kernel adds them to stats[0..1] in block order: the statistics, and so the
// normalised advantages, are bitwise reproducible run to run (no atomics).
// Pass 2 (k_gae_norm): A = (A - mean) / (std_unbiased + 1e-8), elementwise, float4-vectorised.
// Roofline: HBM.  Algorithmic bytes: 17 B per (t, env) in pass 1 (r 4 + done 1 + V 4 + R 4 +
// A 4) + 8 B per env (last V read) ; 8 B per element in pass 2.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void __launch_bounds__(256) k_gae_scan(const float* __restrict__ rewards, const uint8_t* __restrict__ dones,
                                                  const float* __restrict__ values,
                                                  const float* __restrict__ last_values, float* __restrict__ returns,
                                                  float* __restrict__ advantages, double* __restrict__ stats, int T,
                                                  int N, float gamma, float lam) {
#pragma clang fp contract(off)
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  double s1 = 0.0, s2 = 0.0;
  if (e < N) {
    float adv = 0.f;
    float next_v = last_values[e];
    for (int t = T - 1; t >= 0; t--) {
      const size_t i = (size_t)t * N + e;
      const float v = values[i];
      const float nnt = 1.0f - (float)dones[i];
      // delta = r + nnt*gamma*next_v - v
      const float g = nnt * gamma;
      const float delta = (rewards[i] + g * next_v) - v;
      // adv = delta + nnt*gamma*lam*adv
      adv = delta + (g * lam) * adv;
      const float ret = adv + v;
      returns[i] = ret;
      const float a = ret - v;  // advantages = returns - values
      advantages[i] = a;
      s1 += (double)a;
      s2 += (double)a * (double)a;
      next_v = v;
    }
  }
  // wave reduction, then the block's partial pair (fixed order, no atomics)
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s1 += __shfl_down(s1, off, 64);
    s2 += __shfl_down(s2, off, 64);
  }
  __shared__ double red[2][4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { red[0][wid] = s1; red[1][wid] = s2; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, b = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); w++) { a += red[0][w]; b += red[1][w]; }
    stats[2 + 2 * blockIdx.x] = a;
    stats[3 + 2 * blockIdx.x] = b;
  }
}

// fixed-order sum of the block partials: lane i sums blocks i, i+64, ... in order, then a
// fixed butterfly over the 64 lanes; added to stats[0..1] (zeroed first when zero_stats)
__global__ void __launch_bounds__(64) k_gae_stats_final(double* __restrict__ stats, int nblocks, int zero_stats) {
  double a = 0.0, b = 0.0;
  for (int k = threadIdx.x; k < nblocks; k += 64) { a += stats[2 + 2 * k]; b += stats[3 + 2 * k]; }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    a += __shfl_xor(a, off, 64);
    b += __shfl_xor(b, off, 64);
  }
  if (threadIdx.x == 0) {
    stats[0] = (zero_stats ? 0.0 : stats[0]) + a;
    stats[1] = (zero_stats ? 0.0 : stats[1]) + b;
  }
}

__global__ void __launch_bounds__(256) k_gae_norm(float* __restrict__ adv, const double* __restrict__ stats,
                                                  int64_t count, int64_t n) {
  const double mean = stats[0] / (double)count;
  const double var = (stats[1] - stats[0] * mean) / (double)(count - 1);
  const float m = (float)mean;
  const float d = (float)sqrt(var > 0.0 ? var : 0.0) + 1e-8f;  // (A - mean) / (std + 1e-8), as torch
  const int64_t n4 = n / 4;
  float4* a4 = reinterpret_cast<float4*>(adv);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 v = a4[i];
    v.x = (v.x - m) / d; v.y = (v.y - m) / d; v.z = (v.z - m) / d; v.w = (v.w - m) / d;
    a4[i] = v;
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    adv[i] = (adv[i] - m) / d;
}

extern "C" int hg_gae_scan(const float* rewards, const uint8_t* dones, const float* values, const float* last_values,
                           float* returns, float* advantages, double* stats, int64_t stats_len, int T, int N,
                           float gamma, float lam, int zero_stats, void* stream) {
  if (T <= 0 || N <= 0 || !rewards || !dones || !values || !last_values || !returns || !advantages || !stats) return 1;
  const int nblocks = (N + 255) / 256;
  if (stats_len < 2 + 2 * (int64_t)nblocks) return 1;  // the block partials would not fit
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_gae_scan, dim3(nblocks), dim3(256), 0, s, rewards, dones, values, last_values, returns,
                     advantages, stats, T, N, gamma, lam);
  hipLaunchKernelGGL(k_gae_stats_final, dim3(1), dim3(64), 0, s, stats, nblocks, zero_stats);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int64_t hg_gae_stats_len(int N) { return N > 0 ? 2 + 2 * (int64_t)((N + 255) / 256) : 0; }

extern "C" int hg_gae_normalize(float* advantages, const double* stats, int64_t count, int64_t n_local, void* stream) {
  if (!advantages || !stats || count < 2 || n_local <= 0) return 1;
  if (((uintptr_t)advantages & 15) != 0) return 1;
  int64_t blocks = (n_local / 4 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(k_gae_norm, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, advantages, stats, count,
                     n_local);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

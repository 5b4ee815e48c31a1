// hg_mlp.hip — fused activation-backward + bias-gradient pass of the policy MLPs (gfx950).
//
// The actor / lin-vel / critic networks are Linear/ELU chains (actor_critic.py:36-149).  In the
// backward of a Linear(+ELU) layer torch runs, per layer, an ELU-backward elementwise kernel and a
// separate column reduction for the bias gradient (grad_bias = grad_h.sum(0)), i.e. it reads the
// [rows, width] gradient twice.  hg_mlp_act_backward does both in one pass:
//   gh = gy * elu'(h)        elu'(h) = 1 (h > 0), exp(h) = y + 1 (h <= 0), from the layer OUTPUT y
//   gb = sum_rows gh          (deterministic: per-row-tile partials, then fixed-order column sums)
// y == NULL means an identity activation (the output layer): gh is gy itself (nothing written),
// only gb is produced.  HBM per layer: read gy, y; write gh — 12 B per element (4 B when y is
// NULL) + the per-tile partials (4 B per column per 32 rows).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hg_common.h"

namespace {

constexpr int TPB = 256;
constexpr int RT = 32;   // rows per tile: 768 tiles at the 24576-row minibatch (>= 3 blocks per CU)

// width % 4 == 0, width >= 128: float4 columns; W4 = min(width/4, 64) column groups per block,
// L = TPB / W4 row lanes
__global__ void __launch_bounds__(TPB) k_act_bwd_vec(const float* __restrict__ gy, const float* __restrict__ y,
                                                    float* __restrict__ gh, int64_t rows, int width,
                                                    float* __restrict__ partial) {
  const int W4 = min(width >> 2, 64);
  const int L = TPB / W4;
  const int g = threadIdx.x % W4, rho = threadIdx.x / W4;
  const int col = (blockIdx.y * W4 + g) * 4;
  const int64_t r0 = (int64_t)blockIdx.x * RT;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  const bool colok = col < width;
  if (colok) {
    for (int64_t r = r0 + rho; r < r0 + RT && r < rows; r += L) {
      const int64_t i = r * width + col;
      float4 v = *reinterpret_cast<const float4*>(gy + i);
      if (y) {
        const float4 o = *reinterpret_cast<const float4*>(y + i);
        v.x = o.x > 0.f ? v.x : v.x * (o.x + 1.0f);
        v.y = o.y > 0.f ? v.y : v.y * (o.y + 1.0f);
        v.z = o.z > 0.f ? v.z : v.z * (o.z + 1.0f);
        v.w = o.w > 0.f ? v.w : v.w * (o.w + 1.0f);
        *reinterpret_cast<float4*>(gh + i) = v;
      }
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
  }
  __shared__ float4 red[TPB];
  red[threadIdx.x] = acc;
  __syncthreads();
  if (rho == 0 && colok) {
    float4 s = red[g];
    for (int k = 1; k < L; k++) {
      const float4 t = red[k * W4 + g];
      s.x += t.x;
      s.y += t.y;
      s.z += t.z;
      s.w += t.w;
    }
    *reinterpret_cast<float4*>(partial + (int64_t)blockIdx.x * width + col) = s;
  }
}

// any width <= TPB: thread t -> column t % width, row lane t / width (lanes beyond the last full
// group idle)
__global__ void __launch_bounds__(TPB) k_act_bwd_small(const float* __restrict__ gy, const float* __restrict__ y,
                                                      float* __restrict__ gh, int64_t rows, int width,
                                                      float* __restrict__ partial) {
  const int L = TPB / width;
  const int c = threadIdx.x % width, rho = threadIdx.x / width;
  const int64_t r0 = (int64_t)blockIdx.x * RT;
  float acc = 0.f;
  if (rho < L) {
    for (int64_t r = r0 + rho; r < r0 + RT && r < rows; r += L) {
      const int64_t i = r * width + c;
      float v = gy[i];
      if (y) {
        const float o = y[i];
        v = o > 0.f ? v : v * (o + 1.0f);
        gh[i] = v;
      }
      acc += v;
    }
  }
  __shared__ float red[TPB];
  red[threadIdx.x] = acc;
  __syncthreads();
  if (rho == 0) {
    float s = red[c];
    for (int k = 1; k < L; k++) s += red[k * width + c];
    partial[(int64_t)blockIdx.x * width + c] = s;
  }
}

// column sums of the per-tile partials: a block covers 16 columns with 16 tile lanes; lane k sums
// tiles k, k+16, ... (8 independent loads in flight), then a fixed-order sum over the lanes
constexpr int FC = 16, FL = TPB / FC;
__global__ void __launch_bounds__(TPB) k_colsum_final(const float* __restrict__ partial, int tiles, int width,
                                                     float* __restrict__ gb) {
  const int cl = threadIdx.x % FC, lane = threadIdx.x / FC;
  const int c = blockIdx.x * FC + cl;
  float acc = 0.f;
  if (c < width) {
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int t = lane;
    for (; t + 7 * FL < tiles; t += 8 * FL) {
#pragma unroll
      for (int u = 0; u < 8; u++) s[u] += partial[(int64_t)(t + u * FL) * width + c];
    }
    for (; t < tiles; t += FL) s[0] += partial[(int64_t)t * width + c];
    acc = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  }
  __shared__ float red[TPB];
  red[threadIdx.x] = acc;
  __syncthreads();
  if (lane == 0 && c < width) {
    float r = red[cl];
    for (int k = 1; k < FL; k++) r += red[k * FC + cl];
    gb[c] = r;
  }
}

}  // namespace

extern "C" int64_t hg_mlp_act_backward_scratch(int64_t rows, int width) {
  return ((rows + RT - 1) / RT) * (int64_t)width;
}

extern "C" int hg_mlp_act_backward(const float* gy, const float* y, float* gh, int64_t rows, int width,
                                   float* grad_bias, float* scratch, void* stream) {
  if (!gy || !grad_bias || !scratch || rows <= 0 || width <= 0 || (y && !gh)) return HG_ERR_ARG;
  const int64_t tiles64 = (rows + RT - 1) / RT;
  if (tiles64 > 65535 * 16) return HG_ERR_ARG;
  const int tiles = (int)tiles64;
  hipStream_t s = (hipStream_t)stream;
  const bool vec = (width % 4 == 0) && width >= 128 && ((uintptr_t)gy % 16 == 0) && (!y || (uintptr_t)y % 16 == 0) &&
                   (!gh || (uintptr_t)gh % 16 == 0);
  if (vec) {
    const int W4 = width / 4 < 64 ? width / 4 : 64;
    const int ct = (width / 4 + W4 - 1) / W4;
    hipLaunchKernelGGL(k_act_bwd_vec, dim3(tiles, ct), dim3(TPB), 0, s, gy, y, gh, rows, width, scratch);
  } else if (width <= TPB) {
    hipLaunchKernelGGL(k_act_bwd_small, dim3(tiles), dim3(TPB), 0, s, gy, y, gh, rows, width, scratch);
  } else {
    return HG_ERR_ARG;
  }
  hipLaunchKernelGGL(k_colsum_final, dim3((width + FC - 1) / FC), dim3(TPB), 0, s, scratch, tiles, width,
                     grad_bias);
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}

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

// Element access for the fp32 and bf16 (config 5 policy) variants: bf16 is stored as __bf16,
// widened to fp32 for all arithmetic, narrowed with round-to-nearest-even (v_cvt_pk_bf16_f32).
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__device__ inline float bf_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ inline float bf_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ inline uint32_t bf_pack(float a, float b) {
  const bf16x2 v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}
template <typename T> __device__ inline float4 ld4(const T* p);
template <> __device__ inline float4 ld4<float>(const float* p) { return *reinterpret_cast<const float4*>(p); }
template <> __device__ inline float4 ld4<__bf16>(const __bf16* p) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  return make_float4(bf_lo(u.x), bf_hi(u.x), bf_lo(u.y), bf_hi(u.y));
}
template <typename T> __device__ inline void st4(T* p, float4 v);
template <> __device__ inline void st4<float>(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
template <> __device__ inline void st4<__bf16>(__bf16* p, float4 v) {
  *reinterpret_cast<uint2*>(p) = make_uint2(bf_pack(v.x, v.y), bf_pack(v.z, v.w));
}
template <typename T> __device__ inline float2 ld2(const T* p);
template <> __device__ inline float2 ld2<float>(const float* p) { return *reinterpret_cast<const float2*>(p); }
template <> __device__ inline float2 ld2<__bf16>(const __bf16* p) {
  const uint32_t u = *reinterpret_cast<const uint32_t*>(p);
  return make_float2(bf_lo(u), bf_hi(u));
}
template <typename T> __device__ inline void st2(T* p, float2 v);
template <> __device__ inline void st2<float>(float* p, float2 v) { *reinterpret_cast<float2*>(p) = v; }
template <> __device__ inline void st2<__bf16>(__bf16* p, float2 v) {
  *reinterpret_cast<uint32_t*>(p) = bf_pack(v.x, v.y);
}
// 8 consecutive elements (16-byte aligned)
template <typename T> __device__ inline void ld8(const T* p, float v[8]);
template <> __device__ inline void ld8<float>(const float* p, float v[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 c = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = c.x; v[5] = c.y; v[6] = c.z; v[7] = c.w;
}
template <> __device__ inline void ld8<__bf16>(const __bf16* p, float v[8]) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  v[0] = bf_lo(u.x); v[1] = bf_hi(u.x); v[2] = bf_lo(u.y); v[3] = bf_hi(u.y);
  v[4] = bf_lo(u.z); v[5] = bf_hi(u.z); v[6] = bf_lo(u.w); v[7] = bf_hi(u.w);
}
__device__ inline float ld1(const float* p) { return *p; }
__device__ inline float ld1(const __bf16* p) { return (float)*p; }
__device__ inline void st1(float* p, float v) { *p = v; }
__device__ inline void st1(__bf16* p, float v) { *p = (__bf16)v; }

constexpr int TPB = 256;
constexpr int RT = 32;   // rows per tile: 768 tiles at the 24576-row minibatch (>= 3 blocks per CU)

// width % 4 == 0, width >= 128: float4 columns; W4 = min(width/4, 64) column groups per block,
// L = TPB / W4 row lanes
template <typename T>
__global__ void __launch_bounds__(TPB) k_act_bwd_vec(const T* __restrict__ gy, const T* __restrict__ y,
                                                    T* __restrict__ gh, int64_t rows, int width,
                                                    float* __restrict__ partial) {
  const int W4 = min(width >> 2, 64);
  const int L = TPB / W4;
  const int g = threadIdx.x % W4, rho = threadIdx.x / W4;
  const int col = (blockIdx.y * W4 + g) * 4;
  const int64_t r0 = (int64_t)blockIdx.x * RT;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  const bool colok = col < width;
  const int nr = RT / L;  // rows per lane of a full tile (L = 4..8)
  if (colok && r0 + RT <= rows && RT % L == 0 && nr <= 8) {
    // full tile: every load of the lane's rows issued before the first store (one memory latency
    // per tile instead of one per row), rows summed in the same order as the loop below
    float4 a[8], o[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      if (u < nr) {
        const int64_t i = (r0 + rho + (int64_t)u * L) * width + col;
        a[u] = ld4(gy + i);
        if (y) o[u] = ld4(y + i);
      }
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      if (u < nr) {
        float4 v = a[u];
        if (y) {
          v.x = o[u].x > 0.f ? v.x : v.x * (o[u].x + 1.0f);
          v.y = o[u].y > 0.f ? v.y : v.y * (o[u].y + 1.0f);
          v.z = o[u].z > 0.f ? v.z : v.z * (o[u].z + 1.0f);
          v.w = o[u].w > 0.f ? v.w : v.w * (o[u].w + 1.0f);
          st4(gh + (r0 + rho + (int64_t)u * L) * width + col, v);
        }
        acc.x += v.x;
        acc.y += v.y;
        acc.z += v.z;
        acc.w += v.w;
      }
    }
  } else if (colok) {
    for (int64_t r = r0 + rho; r < r0 + RT && r < rows; r += L) {
      const int64_t i = r * width + col;
      float4 v = ld4(gy + i);
      if (y) {
        const float4 o = ld4(y + i);
        v.x = o.x > 0.f ? v.x : v.x * (o.x + 1.0f);
        v.y = o.y > 0.f ? v.y : v.y * (o.y + 1.0f);
        v.z = o.z > 0.f ? v.z : v.z * (o.z + 1.0f);
        v.w = o.w > 0.f ? v.w : v.w * (o.w + 1.0f);
        st4(gh + i, v);
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
template <typename T>
__global__ void __launch_bounds__(TPB) k_act_bwd_small(const T* __restrict__ gy, const T* __restrict__ y,
                                                      T* __restrict__ gh, int64_t rows, int width,
                                                      float* __restrict__ partial) {
  const int L = TPB / width;
  const int c = threadIdx.x % width, rho = threadIdx.x / width;
  const int64_t r0 = (int64_t)blockIdx.x * RT;
  float acc = 0.f;
  if (rho < L) {
    for (int64_t r = r0 + rho; r < r0 + RT && r < rows; r += L) {
      const int64_t i = r * width + c;
      float v = ld1(gy + i);
      if (y) {
        const float o = ld1(y + i);
        v = o > 0.f ? v : v * (o + 1.0f);
        st1(gh + i, v);
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

namespace {
template <typename T>
int act_backward(const T* gy, const T* y, T* gh, int64_t rows, int width, float* grad_bias, float* scratch,
                 void* stream) {
  if (!gy || !scratch || rows <= 0 || width <= 0 || (y && !gh)) return HG_ERR_ARG;
  const int64_t tiles64 = (rows + RT - 1) / RT;
  if (tiles64 > 65535 * 16) return HG_ERR_ARG;
  const int tiles = (int)tiles64;
  hipStream_t s = (hipStream_t)stream;
  const uintptr_t al = 4 * sizeof(T);  // one 4-element vector per lane
  const bool vec = (width % 4 == 0) && width >= 128 && ((uintptr_t)gy % al == 0) && (!y || (uintptr_t)y % al == 0) &&
                   (!gh || (uintptr_t)gh % al == 0);
  if (vec) {
    const int W4 = width / 4 < 64 ? width / 4 : 64;
    const int ct = (width / 4 + W4 - 1) / W4;
    hipLaunchKernelGGL(k_act_bwd_vec<T>, dim3(tiles, ct), dim3(TPB), 0, s, gy, y, gh, rows, width, scratch);
  } else if (width <= TPB) {
    hipLaunchKernelGGL(k_act_bwd_small<T>, dim3(tiles), dim3(TPB), 0, s, gy, y, gh, rows, width, scratch);
  } else {
    return HG_ERR_ARG;
  }
  // grad_bias NULL: the per-tile partials stay in scratch for a later hg_colsum_jobs launch
  if (grad_bias)
    hipLaunchKernelGGL(k_colsum_final, dim3((width + FC - 1) / FC), dim3(TPB), 0, s, scratch, tiles, width,
                       grad_bias);
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}
}  // namespace

extern "C" int hg_mlp_act_backward(const float* gy, const float* y, float* gh, int64_t rows, int width,
                                   float* grad_bias, float* scratch, void* stream) {
  return act_backward<float>(gy, y, gh, rows, width, grad_bias, scratch, stream);
}

extern "C" int hg_mlp_act_backward_bf16(const uint16_t* gy, const uint16_t* y, uint16_t* gh, int64_t rows, int width,
                                        float* grad_bias, float* scratch, void* stream) {
  return act_backward<__bf16>(reinterpret_cast<const __bf16*>(gy), reinterpret_cast<const __bf16*>(y),
                              reinterpret_cast<__bf16*>(gh), rows, width, grad_bias, scratch, stream);
}

// ---------------------------------------------------------------------------------------------
// Skinny output layers (width N <= 16 over K = 128 inputs: the actor's 12 actions, the lin-vel
// head's 3, the critic's single value): y = x W^T + b and its backward.  BLAS runs these
// [rows, 128] x [128, N] products at a few TFLOP/s (latency and tile-shape bound); here each is a
// streaming pass over the [rows, 128] activation:
//   forward: 16 lanes per row (8 inputs each, two float4 loads = one coalesced 512-B row per
//            16-lane group), the lane's W slice in registers, a 4-step xor reduction per output;
//   dX:      lanes along K (2 columns each), the tile's gh rows staged in LDS (broadcast reads);
//   dW, db:  same mapping, per-64-row-tile partials of gh^T h and of gh, then the fixed-order
//            column sums of k_colsum_final over the N*K + N partial columns.
// ---------------------------------------------------------------------------------------------
namespace {
constexpr int SK_K = 128;
constexpr int SK_ROWS = 64;

template <int N, typename TX>
__global__ void __launch_bounds__(256) k_skinny_fwd(const TX* __restrict__ x, int64_t ldx,
                                                   const float* __restrict__ W, const float* __restrict__ b,
                                                   float* __restrict__ y, int64_t rows) {
  const int q = threadIdx.x & 15;  // lane within the row's 16-lane group
  const int k0 = 8 * q;
  float w[N][8];
#pragma unroll
  for (int n = 0; n < N; n++) {
    const float4 a = *reinterpret_cast<const float4*>(W + n * SK_K + k0);
    const float4 c = *reinterpret_cast<const float4*>(W + n * SK_K + k0 + 4);
    w[n][0] = a.x; w[n][1] = a.y; w[n][2] = a.z; w[n][3] = a.w;
    w[n][4] = c.x; w[n][5] = c.y; w[n][6] = c.z; w[n][7] = c.w;
  }
  const float bq = q < N ? b[q] : 0.f;
  const int64_t groups = (rows + 15) / 16;
  for (int64_t gi = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4); gi < rows; gi += (int64_t)gridDim.x * 16) {
    float v[8];
    ld8(x + gi * ldx + k0, v);
    float out = 0.f;
#pragma unroll
    for (int n = 0; n < N; n++) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 8; j++) s = fmaf(v[j], w[n][j], s);
      s += __shfl_xor(s, 8, 16);
      s += __shfl_xor(s, 4, 16);
      s += __shfl_xor(s, 2, 16);
      s += __shfl_xor(s, 1, 16);
      out = (q == n) ? s : out;
    }
    if (q < N) y[gi * N + q] = out + bq;
  }
  (void)groups;
}

// dX and dW/db of a 64-row tile run on 4 waves (16 rows each): the per-lane serial chains are 4x
// shorter than one wave walking all 64 rows (skinny dW 17 -> ? us at 24576 rows).
constexpr int SK_WAVES = 4;
constexpr int SK_WROWS = SK_ROWS / SK_WAVES;

// ACT: the layer below's ELU backward fused in — dx becomes that layer's pre-activation gradient
// dx * elu'(h) (h = this layer's input = the layer below's ELU output; elu' = 1 for h > 0, h + 1
// otherwise) and the block's column sums of it (that layer's bias-gradient partials, one row per
// 64-row tile: each wave sums its 16 rows in order, then waves 0 + 1 + 2 + 3).
template <int N, typename TD, bool ACT>
__device__ __forceinline__ void skinny_dx_body(int bx, float* __restrict__ g_s, float2 (*red)[64],
                                               const float* __restrict__ gh, const float* __restrict__ W,
                                               TD* __restrict__ dx, int64_t rows, const float* __restrict__ h,
                                               int64_t ldh, float* __restrict__ colpart) {
  const int64_t r0 = (int64_t)bx * SK_ROWS;
  const int nr = (int)min<int64_t>(SK_ROWS, rows - r0);
  for (int i = threadIdx.x; i < nr * N; i += 64 * SK_WAVES) g_s[i] = gh[r0 * N + i];
  const int c = 2 * (threadIdx.x & 63);
  const int wv = threadIdx.x >> 6;
  float w0[N], w1[N];
#pragma unroll
  for (int n = 0; n < N; n++) {
    const float2 t = *reinterpret_cast<const float2*>(W + n * SK_K + c);
    w0[n] = t.x;
    w1[n] = t.y;
  }
  __syncthreads();
  const int re = min(nr, SK_WROWS * (wv + 1));
  float s0 = 0.f, s1 = 0.f;
  for (int r = SK_WROWS * wv; r < re; r++) {
    float a0 = 0.f, a1 = 0.f;
#pragma unroll
    for (int n = 0; n < N; n++) {
      const float g = g_s[r * N + n];
      a0 = fmaf(g, w0[n], a0);
      a1 = fmaf(g, w1[n], a1);
    }
    if (ACT) {
      const float2 y = *reinterpret_cast<const float2*>(h + (r0 + r) * ldh + c);
      a0 = y.x > 0.f ? a0 : a0 * (y.x + 1.f);
      a1 = y.y > 0.f ? a1 : a1 * (y.y + 1.f);
      s0 += a0;
      s1 += a1;
    }
    st2(dx + (r0 + r) * SK_K + c, make_float2(a0, a1));
  }
  if (ACT) {
    if (wv > 0) red[wv - 1][threadIdx.x & 63] = make_float2(s0, s1);
    __syncthreads();
    if (wv == 0) {
#pragma unroll
      for (int q = 0; q < SK_WAVES - 1; q++) {
        const float2 t = red[q][threadIdx.x];
        s0 += t.x;
        s1 += t.y;
      }
      *reinterpret_cast<float2*>(colpart + (int64_t)bx * SK_K + c) = make_float2(s0, s1);
    }
  }
}

template <int N, typename TD, bool ACT = false>
__global__ void __launch_bounds__(64 * SK_WAVES) k_skinny_dx(const float* __restrict__ gh, const float* __restrict__ W,
                                                             TD* __restrict__ dx, int64_t rows,
                                                             const float* __restrict__ h = nullptr, int64_t ldh = 0,
                                                             float* __restrict__ colpart = nullptr) {
  __shared__ float g_s[SK_ROWS * N];
  __shared__ float2 red[ACT ? SK_WAVES - 1 : 1][64];
  skinny_dx_body<N, TD, ACT>(blockIdx.x, g_s, red, gh, W, dx, rows, h, ldh, colpart);
}

template <int N, typename TH>
__device__ __forceinline__ void skinny_dw_body(int bx, float* __restrict__ g_s, float2 (*red)[N][64],
                                               const float* __restrict__ gh, const TH* __restrict__ h, int64_t ldh,
                                               float* __restrict__ partial, int64_t rows) {
  const int64_t r0 = (int64_t)bx * SK_ROWS;
  const int nr = (int)min<int64_t>(SK_ROWS, rows - r0);
  for (int i = threadIdx.x; i < nr * N; i += 64 * SK_WAVES) g_s[i] = gh[r0 * N + i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int c = 2 * lane;
  float a0[N], a1[N];
#pragma unroll
  for (int n = 0; n < N; n++) a0[n] = a1[n] = 0.f;
  const int rb = SK_WROWS * wv, re = min(nr, rb + SK_WROWS);
  const TH* hr = h + r0 * ldh + c;
  int r = rb;
  for (; r + 8 <= re; r += 8) {
    float2 v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) v[u] = ld2(hr + (int64_t)(r + u) * ldh);
#pragma unroll
    for (int u = 0; u < 8; u++) {
#pragma unroll
      for (int n = 0; n < N; n++) {
        const float g = g_s[(r + u) * N + n];
        a0[n] = fmaf(g, v[u].x, a0[n]);
        a1[n] = fmaf(g, v[u].y, a1[n]);
      }
    }
  }
  for (; r < re; r++) {
    const float2 v = ld2(hr + (int64_t)r * ldh);
#pragma unroll
    for (int n = 0; n < N; n++) {
      const float g = g_s[r * N + n];
      a0[n] = fmaf(g, v.x, a0[n]);
      a1[n] = fmaf(g, v.y, a1[n]);
    }
  }
  // fixed-order sum of the 4 waves' 16-row partials (wave 0 + 1 + 2 + 3)
  if (wv > 0) {
#pragma unroll
    for (int n = 0; n < N; n++) red[wv - 1][n][lane] = make_float2(a0[n], a1[n]);
  }
  __syncthreads();
  if (wv != 0) return;
#pragma unroll
  for (int q = 0; q < SK_WAVES - 1; q++) {
#pragma unroll
    for (int n = 0; n < N; n++) {
      const float2 t = red[q][n][lane];
      a0[n] += t.x;
      a1[n] += t.y;
    }
  }
  float* out = partial + (int64_t)bx * (N * SK_K + N);
#pragma unroll
  for (int n = 0; n < N; n++) *reinterpret_cast<float2*>(out + n * SK_K + c) = make_float2(a0[n], a1[n]);
  if (lane < N) {
    float gb = 0.f;
    for (int rr = 0; rr < nr; rr++) gb += g_s[rr * N + lane];
    out[N * SK_K + lane] = gb;
  }
}

template <int N, typename TH>
__global__ void __launch_bounds__(64 * SK_WAVES) k_skinny_dw(const float* __restrict__ gh, const TH* __restrict__ h,
                                                             int64_t ldh, float* __restrict__ partial, int64_t rows) {
  __shared__ float g_s[SK_ROWS * N];
  __shared__ float2 red[SK_WAVES - 1][N][64];
  skinny_dw_body<N, TH>(blockIdx.x, g_s, red, gh, h, ldh, partial, rows);
}

// dW / db partials (blocks [0, tiles)) and the ELU-fused input gradient (blocks [tiles, 2 tiles))
// of hg_linear_skinny_backward_act in ONE launch: the two bodies unchanged (the same bits), one
// launch ramp / tail instead of two
template <int N>
__global__ void __launch_bounds__(64 * SK_WAVES) k_skinny_bwd_act(const float* __restrict__ gh, const float* __restrict__ h,
                                                                  int64_t ldh, const float* __restrict__ W,
                                                                  float* __restrict__ partial, float* __restrict__ dx,
                                                                  float* __restrict__ colpart, int64_t rows, int tiles) {
  __shared__ float g_s[SK_ROWS * N];
  __shared__ float2 red[SK_WAVES - 1][N][64];
  if ((int)blockIdx.x < tiles) {
    skinny_dw_body<N, float>(blockIdx.x, g_s, red, gh, h, ldh, partial, rows);
  } else {
    // the dx body's [SK_WAVES - 1][64] view over the whole buffer (>= that size for every N >= 1),
    // not red[0], whose [N][64] bound is one row for the critic head
    float2 (*red_dx)[64] = reinterpret_cast<float2 (*)[64]>(&red[0][0][0]);
    skinny_dx_body<N, float, true>(blockIdx.x - tiles, g_s, red_dx, gh, W, dx, rows, h, ldh, colpart);
  }
}
}  // namespace

#define HG_SKINNY_SWITCH(N, CALL) \
  switch (N) {                    \
    case 1: CALL(1); break;       \
    case 2: CALL(2); break;       \
    case 3: CALL(3); break;       \
    case 4: CALL(4); break;       \
    case 6: CALL(6); break;       \
    case 8: CALL(8); break;       \
    case 12: CALL(12); break;     \
    case 16: CALL(16); break;     \
    default: return HG_ERR_ARG;   \
  }

extern "C" int hg_linear_skinny_supported(int n, int k) {
  return (n == 1 || n == 2 || n == 3 || n == 4 || n == 6 || n == 8 || n == 12 || n == 16) && k == SK_K;
}

namespace {
template <typename TX>
int skinny_forward(const TX* x, int64_t ldx, const float* W, const float* b, float* y, int64_t rows, int n, int k,
                   void* stream) {
  // 8 elements of x per lane: 16-byte aligned rows
  const int64_t vec = 16 / sizeof(TX);
  if (!x || !W || !b || !y || rows <= 0 || !hg_linear_skinny_supported(n, k) || ldx < k || ldx % vec != 0 ||
      (uintptr_t)x % 16 != 0 || (uintptr_t)W % 16 != 0)
    return HG_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int64_t want = (rows + 15) / 16;  // one 16-row group per block pass
  const dim3 grid((unsigned)(want < 1024 ? want : 1024));
#define HG_SK_FWD(NN) hipLaunchKernelGGL((k_skinny_fwd<NN, TX>), grid, dim3(256), 0, s, x, ldx, W, b, y, rows)
  HG_SKINNY_SWITCH(n, HG_SK_FWD)
#undef HG_SK_FWD
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}

template <typename TH>
int skinny_backward(const float* gh, const TH* h, int64_t ldh, const float* W, TH* dx, float* grad_wb, int64_t rows,
                    int n, int k, float* scratch, void* stream) {
  // two elements of h / dx per lane
  if (!gh || !h || !W || !scratch || rows <= 0 || !hg_linear_skinny_supported(n, k) || ldh < k ||
      ldh % 2 != 0 || (uintptr_t)h % (2 * sizeof(TH)) != 0 || (uintptr_t)W % 8 != 0 ||
      (dx && (uintptr_t)dx % (2 * sizeof(TH)) != 0))
    return HG_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int tiles = (int)((rows + SK_ROWS - 1) / SK_ROWS);
  const dim3 grid((unsigned)tiles);
#define HG_SK_DW(NN) hipLaunchKernelGGL((k_skinny_dw<NN, TH>), grid, dim3(64 * SK_WAVES), 0, s, gh, h, ldh, scratch, rows)
  HG_SKINNY_SWITCH(n, HG_SK_DW)
#undef HG_SK_DW
  const int width = n * k + n;
  // grad_wb NULL: partials stay in scratch ([tiles, n*k + n]) for a later hg_colsum_jobs launch
  if (grad_wb)
    hipLaunchKernelGGL(k_colsum_final, dim3((width + FC - 1) / FC), dim3(TPB), 0, s, scratch, tiles, width, grad_wb);
  if (dx) {
#define HG_SK_DX(NN) hipLaunchKernelGGL((k_skinny_dx<NN, TH>), grid, dim3(64 * SK_WAVES), 0, s, gh, W, dx, rows)
    HG_SKINNY_SWITCH(n, HG_SK_DX)
#undef HG_SK_DX
  }
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}
}  // namespace

extern "C" int hg_linear_skinny_forward(const float* x, int64_t ldx, const float* W, const float* b, float* y,
                                        int64_t rows, int n, int k, void* stream) {
  return skinny_forward<float>(x, ldx, W, b, y, rows, n, k, stream);
}

extern "C" int hg_linear_skinny_forward_bf16(const uint16_t* x, int64_t ldx, const float* W, const float* b, float* y,
                                             int64_t rows, int n, int k, void* stream) {
  return skinny_forward<__bf16>(reinterpret_cast<const __bf16*>(x), ldx, W, b, y, rows, n, k, stream);
}

extern "C" int64_t hg_linear_skinny_backward_scratch(int64_t rows, int n, int k) {
  return ((rows + SK_ROWS - 1) / SK_ROWS) * (int64_t)(n * k + n);
}

// gh [rows, n] (the output gradient), h [rows, k] (the layer input, row stride ldh), W [n, k].
// grad_wb [n*k + n]: dW (row-major [n, k]) followed by db.  dx [rows, k] (contiguous) may be NULL.
extern "C" int hg_linear_skinny_backward(const float* gh, const float* h, int64_t ldh, const float* W, float* dx,
                                         float* grad_wb, int64_t rows, int n, int k, float* scratch, void* stream) {
  return skinny_backward<float>(gh, h, ldh, W, dx, grad_wb, rows, n, k, scratch, stream);
}

extern "C" int64_t hg_linear_skinny_colpart_rows(int64_t rows) { return (rows + SK_ROWS - 1) / SK_ROWS; }

extern "C" int hg_linear_skinny_backward_act(const float* gh, const float* h, int64_t ldh, const float* W,
                                             float* gh_prev, float* colpart, int64_t rows, int n, int k,
                                             float* scratch, void* stream) {
  // dW / db partials as hg_linear_skinny_backward (left in scratch), then the fused input gradient
  if (!gh_prev || !colpart || ldh % 2 != 0 || (uintptr_t)h % 8 != 0 || (uintptr_t)gh_prev % 8 != 0 ||
      (uintptr_t)colpart % 8 != 0)
    return HG_ERR_ARG;
  if (!gh || !h || !W || !scratch || rows <= 0 || !hg_linear_skinny_supported(n, k) || ldh < k ||
      (uintptr_t)W % 8 != 0 || rows > ((int64_t)1 << 36))
    return HG_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int tiles = (int)((rows + SK_ROWS - 1) / SK_ROWS);
  const dim3 grid((unsigned)(2 * tiles));
#define HG_SK_BWDA(NN) \
  hipLaunchKernelGGL((k_skinny_bwd_act<NN>), grid, dim3(64 * SK_WAVES), 0, s, gh, h, ldh, W, scratch, gh_prev, colpart, rows, tiles)
  HG_SKINNY_SWITCH(n, HG_SK_BWDA)
#undef HG_SK_BWDA
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}

extern "C" int hg_linear_skinny_backward_bf16(const float* gh, const uint16_t* h, int64_t ldh, const float* W,
                                              uint16_t* dx, float* grad_wb, int64_t rows, int n, int k,
                                              float* scratch, void* stream) {
  return skinny_backward<__bf16>(gh, reinterpret_cast<const __bf16*>(h), ldh, W, reinterpret_cast<__bf16*>(dx),
                                 grad_wb, rows, n, k, scratch, stream);
}

// ---------------------------------------------------------------------------------------------
// Batched column sums: the deferred reductions of one MLP backward in ONE launch.  Each job sums a
// row-major [parts, width] block of partials over its parts into out[width]:
//   the per-row-tile bias-gradient partials of hg_mlp_act_backward / hg_linear_skinny_backward
//   (parts = row tiles, hundreds): the k_colsum_final reduction, same order, so the same bits;
//   the split-K weight-gradient chunks (parts = S row chunks of the minibatch, width = n k):
//   S <= 16 one thread per element, p = 0 .. S-1 in order; wide jobs (width >= CJ_WIDE, a
//   multiple of 4, 16-byte aligned) four columns per thread with 16-byte loads — each part row
//   read as whole 1 KB runs per wave (the 16-column blocks below read it as 64-byte pieces) — and
//   for S > 16 eight interleaved accumulators (part p into p % 8), combined as a fixed tree.
// Saves the 4-6 us launch of every per-layer reduction (20 per PPO minibatch -> 3).
// ---------------------------------------------------------------------------------------------
namespace {
constexpr int CJ_MAX = 16;
constexpr int CJ_SEQ_MAXPARTS = 16;
constexpr int64_t CJ_WIDE = 4096;  // bias partials are at most a layer wide (<= 768 columns)
struct ColsumJobs {
  const float* src[CJ_MAX];
  float* dst[CJ_MAX];
  int64_t width[CJ_MAX];
  int parts[CJ_MAX];
  int wide[CJ_MAX];        // 1: four columns per thread; 2: eight threads per four columns (see above)
  int block0[CJ_MAX + 1];  // first block of each job; block0[njobs] = grid size
  int njobs;
};

__global__ void __launch_bounds__(TPB) k_colsum_jobs(ColsumJobs J) {
  const int bid = blockIdx.x;
  int j = 0;
  while (j + 1 < J.njobs && bid >= J.block0[j + 1]) j++;
  const float* __restrict__ src = J.src[j];
  const int64_t width = J.width[j];
  const int parts = J.parts[j];
  const int lb = bid - J.block0[j];
  if (J.wide[j] == 2) {
    // many parts: eight threads per four columns, thread u summing parts u, u + 8, u + 16, .. in
    // order (its loads all in flight at once), the eight sums combined in LDS by the fixed tree —
    // the interleaved-accumulator order below, so the same bits, with 8x the waves in flight
    constexpr int CW = TPB / 8;  // float4 columns per block
    const int u = threadIdx.x / CW, cl = threadIdx.x % CW;
    const int64_t c4 = (int64_t)lb * CW + cl;
    const int64_t w4 = width / 4;
    const float4* __restrict__ s4 = reinterpret_cast<const float4*>(src) + c4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c4 < w4) {
      int p = u;
      for (; p + 56 < parts; p += 64) {  // eight loads per round, issued together
        float4 x[8];
#pragma unroll
        for (int q = 0; q < 8; q++) x[q] = s4[(int64_t)(p + 8 * q) * w4];
#pragma unroll
        for (int q = 0; q < 8; q++) { acc.x += x[q].x; acc.y += x[q].y; acc.z += x[q].z; acc.w += x[q].w; }
      }
      for (; p < parts; p += 8) {
        const float4 x = s4[(int64_t)p * w4];
        acc.x += x.x; acc.y += x.y; acc.z += x.z; acc.w += x.w;
      }
    }
    __shared__ float4 red4[8][CW];
    red4[u][cl] = acc;
    __syncthreads();
    if (u == 0 && c4 < w4) {
      auto tree = [&](int k) {
        const float* r0 = &red4[0][cl].x;
        const int st = CW * 4;
        return ((r0[k] + r0[st + k]) + (r0[2 * st + k] + r0[3 * st + k])) +
               ((r0[4 * st + k] + r0[5 * st + k]) + (r0[6 * st + k] + r0[7 * st + k]));
      };
      reinterpret_cast<float4*>(J.dst[j])[c4] = make_float4(tree(0), tree(1), tree(2), tree(3));
    }
    return;
  }
  if (J.wide[j]) {
    const int64_t c4 = (int64_t)lb * TPB + threadIdx.x;
    if (4 * c4 >= width) return;
    const float4* __restrict__ s4 = reinterpret_cast<const float4*>(src) + c4;
    const int64_t w4 = width / 4;
    float4 acc;
    if (parts <= CJ_SEQ_MAXPARTS) {
      acc = s4[0];
      for (int p = 1; p < parts; p++) {
        const float4 x = s4[p * w4];
        acc.x += x.x; acc.y += x.y; acc.z += x.z; acc.w += x.w;
      }
    } else {
      float4 s8[8];
#pragma unroll
      for (int u = 0; u < 8; u++) s8[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      int p = 0;
      for (; p + 8 <= parts; p += 8) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
          const float4 x = s4[(int64_t)(p + u) * w4];
          s8[u].x += x.x; s8[u].y += x.y; s8[u].z += x.z; s8[u].w += x.w;
        }
      }
      for (; p < parts; p++) {
        const float4 x = s4[(int64_t)p * w4];
        s8[p & 7].x += x.x; s8[p & 7].y += x.y; s8[p & 7].z += x.z; s8[p & 7].w += x.w;
      }
      auto tree = [&](float a0, float a1, float a2, float a3, float a4, float a5, float a6, float a7) {
        return ((a0 + a1) + (a2 + a3)) + ((a4 + a5) + (a6 + a7));
      };
      acc.x = tree(s8[0].x, s8[1].x, s8[2].x, s8[3].x, s8[4].x, s8[5].x, s8[6].x, s8[7].x);
      acc.y = tree(s8[0].y, s8[1].y, s8[2].y, s8[3].y, s8[4].y, s8[5].y, s8[6].y, s8[7].y);
      acc.z = tree(s8[0].z, s8[1].z, s8[2].z, s8[3].z, s8[4].z, s8[5].z, s8[6].z, s8[7].z);
      acc.w = tree(s8[0].w, s8[1].w, s8[2].w, s8[3].w, s8[4].w, s8[5].w, s8[6].w, s8[7].w);
    }
    reinterpret_cast<float4*>(J.dst[j])[c4] = acc;
    return;
  }
  if (parts <= CJ_SEQ_MAXPARTS) {
    const int64_t c = (int64_t)lb * TPB + threadIdx.x;
    if (c < width) {
      float acc = src[c];
      for (int p = 1; p < parts; p++) acc += src[(int64_t)p * width + c];
      J.dst[j][c] = acc;
    }
    return;
  }
  // k_colsum_final's mapping and order: 16 columns x 16 part lanes, 8 accumulators per lane
  const int cl = threadIdx.x % FC, lane = threadIdx.x / FC;
  const int64_t c = (int64_t)lb * FC + cl;
  float acc = 0.f;
  if (c < width) {
    float s8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int t = lane;
    for (; t + 7 * FL < parts; t += 8 * FL) {
#pragma unroll
      for (int u = 0; u < 8; u++) s8[u] += src[(int64_t)(t + u * FL) * width + c];
    }
    for (; t < parts; t += FL) s8[0] += src[(int64_t)t * width + c];
    acc = ((s8[0] + s8[1]) + (s8[2] + s8[3])) + ((s8[4] + s8[5]) + (s8[6] + s8[7]));
  }
  __shared__ float red[TPB];
  red[threadIdx.x] = acc;
  __syncthreads();
  if (lane == 0 && c < width) {
    float r = red[cl];
    for (int k = 1; k < FL; k++) r += red[k * FC + cl];
    J.dst[j][c] = r;
  }
}
}  // namespace

extern "C" int hg_colsum_jobs(const float* const* src, float* const* dst, const int64_t* width, const int* parts,
                              int njobs, void* stream) {
  if (njobs <= 0) return HG_OK;
  if (njobs > CJ_MAX || !src || !dst || !width || !parts) return HG_ERR_ARG;
  ColsumJobs J;
  J.njobs = njobs;
  int64_t blocks = 0;
  for (int j = 0; j < njobs; j++) {
    if (!src[j] || !dst[j] || width[j] <= 0 || parts[j] <= 0) return HG_ERR_ARG;
    J.src[j] = src[j];
    J.dst[j] = dst[j];
    J.width[j] = width[j];
    J.parts[j] = parts[j];
    J.wide[j] = width[j] >= CJ_WIDE && width[j] % 4 == 0 && (uintptr_t)src[j] % 16 == 0 && (uintptr_t)dst[j] % 16 == 0;
    if (J.wide[j] && parts[j] > CJ_SEQ_MAXPARTS) J.wide[j] = 2;  // eight threads per four columns
    J.block0[j] = (int)blocks;
    blocks += J.wide[j] == 2 ? (width[j] / 4 + TPB / 8 - 1) / (TPB / 8)
              : J.wide[j] ? (width[j] / 4 + TPB - 1) / TPB
                          : parts[j] <= CJ_SEQ_MAXPARTS ? (width[j] + TPB - 1) / TPB : (width[j] + FC - 1) / FC;
    if (blocks > (int64_t)1 << 30) return HG_ERR_ARG;
  }
  J.block0[njobs] = (int)blocks;
  hipLaunchKernelGGL(k_colsum_jobs, dim3((unsigned)blocks), dim3(TPB), 0, (hipStream_t)stream, J);
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}

// ---------------------------------------------------------------------------------------------
// bf16 policy (config 5): fp32 -> bf16 copies of a list of tensors in ONE launch — the hidden
// layers' weights and biases before a bf16 forward (master weights, gradients and Adam stay fp32).
// Block b belongs to the job whose [block0[j], block0[j+1]) range holds it; 4 elements per thread
// (float4 in, two packed bf16 pairs out) when the job is 16-byte aligned with count % 4 == 0,
// element-wise otherwise.
// ---------------------------------------------------------------------------------------------
namespace {
constexpr int CAST_MAX = 32;
struct CastJobs {
  const float* src[CAST_MAX];
  __bf16* dst[CAST_MAX];
  int64_t count[CAST_MAX];
  int block0[CAST_MAX + 1];
  int njobs;
};

__global__ void __launch_bounds__(TPB) k_cast_bf16_jobs(CastJobs J) {
  const int bid = blockIdx.x;
  int j = 0;
  while (j + 1 < J.njobs && bid >= J.block0[j + 1]) j++;
  const float* __restrict__ src = J.src[j];
  __bf16* __restrict__ dst = J.dst[j];
  const int64_t n = J.count[j];
  const int64_t e = ((int64_t)(bid - J.block0[j]) * TPB + threadIdx.x) * 4;
  if (e >= n) return;
  if (n % 4 == 0 && (uintptr_t)src % 16 == 0 && (uintptr_t)dst % 8 == 0) {
    st4(dst + e, ld4(src + e));
  } else {
    for (int64_t i = e; i < e + 4 && i < n; i++) dst[i] = (__bf16)src[i];
  }
}
}  // namespace

extern "C" int hg_cast_bf16_jobs(const float* const* src, uint16_t* const* dst, const int64_t* count, int njobs,
                                 void* stream) {
  if (njobs <= 0) return HG_OK;
  if (njobs > CAST_MAX || !src || !dst || !count) return HG_ERR_ARG;
  CastJobs J;
  J.njobs = njobs;
  int64_t blocks = 0;
  for (int j = 0; j < njobs; j++) {
    if (!src[j] || !dst[j] || count[j] <= 0) return HG_ERR_ARG;
    J.src[j] = src[j];
    J.dst[j] = reinterpret_cast<__bf16*>(dst[j]);
    J.count[j] = count[j];
    J.block0[j] = (int)blocks;
    blocks += (count[j] + 4 * TPB - 1) / (4 * TPB);
    if (blocks > (int64_t)1 << 30) return HG_ERR_ARG;
  }
  J.block0[njobs] = (int)blocks;
  hipLaunchKernelGGL(k_cast_bf16_jobs, dim3((unsigned)blocks), dim3(TPB), 0, (hipStream_t)stream, J);
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}

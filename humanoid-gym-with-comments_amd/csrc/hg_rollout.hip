// hg_rollout.hip — fused rollout-storage writes of the PPO collection loop (gfx950).
//
// Replaces, per policy step, the elementwise tail of PPO.act + RolloutStorage.add_transitions
// (humanoid/algo/ppo/ppo.py:116-138, rollout_storage.py:83-100): ~25 small launches become two.
//   hg_rollout_act (before env.step): a = mu + sigma * z, z ~ N(0,1) (Philox, Box–Muller);
//     log p(a) = sum_j [ -(a_j - mu_j)^2 / (2 sigma_j^2) - log sigma_j - log sqrt(2 pi) ]
//     (torch.distributions.Normal.log_prob summed over actions); writes actions, log-prob, mu,
//     sigma, value into slot t of the storage, and copies the observation / critic observation
//     rows into slot t (fp32 or fp16 storage) in the same launch — for the actor observation
//     optionally only a column range (the newest frame of the stack: frame-only storage).
//   hg_rollout_env (after env.step): rewards[t] = r + gamma * V * time_out (the time-out
//     bootstrap of ppo.py:132-133), dones[t] = reset; with values == NULL the bootstrap is
//     deferred: rewards[t] = r and time_outs[t] is kept for the batched value pass.
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "hg_common.h"

namespace {

constexpr int TPB = 256;
constexpr uint32_t RNG_ACTION_SAMPLE = 9;
constexpr int ACT_LANES = 16;  // lanes per env in the sampling blocks (num_actions <= 16)

__device__ inline u4 philox_key(uint64_t seed, uint32_t env, uint64_t step, uint32_t block) {
  u4 c = {env, (uint32_t)step, (block & 0xFFFFu) | ((uint32_t)(step >> 32) << 16), RNG_ACTION_SAMPLE};
  return philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}

template <typename OT>
__device__ inline void store_obs(OT* dst, float v);
template <>
__device__ inline void store_obs<float>(float* dst, float v) { *dst = v; }
template <>
__device__ inline void store_obs<__half>(__half* dst, float v) { *dst = __float2half(v); }

// the fused output layer (hg_rollout_act_head): HEAD_N outputs over HEAD_K = 128 inputs, lane j of
// an env's 16-lane group holding inputs 8j .. 8j + 7 (k_skinny_fwd's layout and arithmetic)
constexpr int HEAD_N = 12, HEAD_K = 128;
struct ActHead {
  const float* h;
  int64_t ld;
  const float* W;
  const float* b;
};

// mean of the row h (HEAD_K values; global memory or LDS) = W h + b for lane j of the env's 16-lane
// group, as k_skinny_fwd<12> computes it (same fma chain, the same xor-shuffle tree, the bias added
// last), so bitwise the two-launch result
__device__ __forceinline__ float act_head_mean(const float* __restrict__ hrow, const float* __restrict__ W,
                                               const float* __restrict__ b, int j) {
  const int k0 = 8 * j;
  const float4 xa = *reinterpret_cast<const float4*>(hrow + k0);
  const float4 xb = *reinterpret_cast<const float4*>(hrow + k0 + 4);
  const float v[8] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
  float out = 0.f;
#pragma unroll
  for (int q = 0; q < HEAD_N; q++) {
    const float4 wa = *reinterpret_cast<const float4*>(W + q * HEAD_K + k0);
    const float4 wb = *reinterpret_cast<const float4*>(W + q * HEAD_K + k0 + 4);
    const float w[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) s = fmaf(v[i], w[i], s);
    s += __shfl_xor(s, 8, 16);
    s += __shfl_xor(s, 4, 16);
    s += __shfl_xor(s, 2, 16);
    s += __shfl_xor(s, 1, 16);
    out = (j == q) ? s : out;
  }
  return out + (j < HEAD_N ? b[j] : 0.f);
}

// one env's sample / log-prob / storage writes by its 16-lane group, one lane per action (its Philox
// block computed by each of the group's lanes); the log-prob terms are summed in action order by
// every lane of the group (the same additions as the one-thread-per-env loop of k_act)
__device__ __forceinline__ void act_env16(int e, int j, int A, float m, const float* __restrict__ std,
                                          const float* __restrict__ value, float* __restrict__ act_out,
                                          float* __restrict__ logp_out, float* __restrict__ mu_out,
                                          float* __restrict__ sigma_out, float* __restrict__ value_out,
                                          int row_offset, uint64_t seed, uint64_t counter) {
  const float c = 0.91893853320467274178f;  // log(sqrt(2 pi))
  float term = 0.f;
  if (j < A) {
    float z4[4];
    normals4(philox_key(seed, (uint32_t)(e + row_offset), counter, (uint32_t)(j >> 2)), z4);
    const float z = (j & 3) == 0 ? z4[0] : (j & 3) == 1 ? z4[1] : (j & 3) == 2 ? z4[2] : z4[3];
    const float s = std[j];
    const float a = m + s * z;
    const float d = a - m;
    term = -(d * d) / (2.0f * (s * s)) - logf(s) - c;
    act_out[(size_t)e * A + j] = a;
    mu_out[(size_t)e * A + j] = m;
    sigma_out[(size_t)e * A + j] = s;
  }
  float lp = 0.f;
  for (int jj = 0; jj < A; jj++) lp += __shfl(term, jj, ACT_LANES);
  if (j == 0) {
    logp_out[e] = lp;
    if (value) value_out[e] = value[e];
  }
}

// observation rows -> storage slot: one wave per (table, row), lanes along the row; source rows
// strided (the env's stacks are column slices of its history windows), storage rows packed.  Wave
// w0 of the copy waves (nw of them) takes rows w0, w0 + nw, ..
template <typename OT>
__device__ __forceinline__ void act_copy_obs(int64_t w0, int64_t nw, const float* __restrict__ obs,
                                             const float* __restrict__ cobs, int n, int64_t obs_w, int64_t cobs_w,
                                             int64_t obs_ld, int64_t obs_c0, int64_t cobs_ld, int64_t obs_out_ld,
                                             OT* __restrict__ obs_out, OT* __restrict__ cobs_out) {
  const int64_t rows = cobs_w > 0 ? 2 * (int64_t)n : n;
  const int lane = threadIdx.x & 63;
  for (int64_t q = w0; q < rows; q += nw) {
    const bool o = q < n;
    const int64_t r = o ? q : q - n;
    const int64_t w = o ? obs_w : cobs_w;
    const float* __restrict__ src = o ? obs + r * obs_ld + obs_c0 : cobs + r * cobs_ld;
    OT* __restrict__ dst = o ? obs_out + r * obs_out_ld : cobs_out + r * w;
    int64_t c = lane;
    for (; c + 192 < w; c += 256) {
      const float a = src[c], b = src[c + 64], d = src[c + 128], e = src[c + 192];
      store_obs<OT>(dst + c, a);
      store_obs<OT>(dst + c + 64, b);
      store_obs<OT>(dst + c + 128, d);
      store_obs<OT>(dst + c + 192, e);
    }
    for (; c < w; c += 64) store_obs<OT>(dst + c, src[c]);
  }
}

template <typename OT, bool HEAD>
__global__ void __launch_bounds__(TPB) k_act(const float* __restrict__ mean, ActHead hd, const float* __restrict__ std,
                                            const float* __restrict__ value, const float* __restrict__ obs,
                                            const float* __restrict__ cobs, int n, int A, int64_t obs_w,
                                            int64_t cobs_w, int64_t obs_ld, int64_t obs_c0, int64_t cobs_ld,
                                            float* __restrict__ act_out, float* __restrict__ logp_out,
                                            float* __restrict__ mu_out, float* __restrict__ sigma_out,
                                            float* __restrict__ value_out, int64_t obs_out_ld, OT* __restrict__ obs_out,
                                            OT* __restrict__ cobs_out, int row_offset, uint64_t seed,
                                            uint64_t counter, int env_blocks) {
  if ((int)blockIdx.x < env_blocks) {
    if (A <= ACT_LANES) {
      const int e = (int)(((int64_t)blockIdx.x * TPB + threadIdx.x) / ACT_LANES);
      const int j = threadIdx.x % ACT_LANES;
      if (e >= n) return;  // whole groups leave together
      const float m = HEAD ? act_head_mean(hd.h + (int64_t)e * hd.ld, hd.W, hd.b, j)
                           : (j < A ? mean[(size_t)e * A + j] : 0.f);
      act_env16(e, j, A, m, std, value, act_out, logp_out, mu_out, sigma_out, value_out, row_offset, seed, counter);
      return;
    }
    const float c = 0.91893853320467274178f;  // log(sqrt(2 pi))
    const int e = blockIdx.x * TPB + threadIdx.x;
    if (e >= n) return;
    float lp = 0.f;
    float z4[4];
    for (int j = 0; j < A; j++) {
      if ((j & 3) == 0) normals4(philox_key(seed, (uint32_t)(e + row_offset), counter, (uint32_t)(j >> 2)), z4);
      const float m = mean[(size_t)e * A + j], s = std[j];
      const float a = m + s * z4[j & 3];
      const float d = a - m;
      lp += -(d * d) / (2.0f * (s * s)) - logf(s) - c;
      act_out[(size_t)e * A + j] = a;
      mu_out[(size_t)e * A + j] = m;
      sigma_out[(size_t)e * A + j] = s;
    }
    logp_out[e] = lp;
    if (value) value_out[e] = value[e];
    return;
  }
  act_copy_obs<OT>((int64_t)(blockIdx.x - env_blocks) * (TPB / 64) + (threadIdx.x >> 6),
                   (int64_t)(gridDim.x - env_blocks) * (TPB / 64), obs, cobs, n, obs_w, cobs_w, obs_ld, obs_c0,
                   cobs_ld, obs_out_ld, obs_out, cobs_out);
}

// The actor's last hidden layer and its output layer in the sampling launch
// (hg_rollout_act_tail): a block of TAIL_WAVES waves owns 16 rows — wave w computes the 16 x 16
// tile of columns 16 w .. 16 w + 15 of y = elu(x W3^T + b3) exactly as k_linear_act16 does
// (hg_lin16_acc, the same epilogue) into LDS, and the block's first 256 threads then run the
// head and the sampling of its 16 envs from those rows (k_act's HEAD path).  Bitwise the
// linear_act + hg_rollout_act_head pair; one launch and no global round trip of the hidden row.
constexpr int TAIL_WAVES = HEAD_K / 16;
struct ActTail {
  const float* x;
  int64_t ldx;
  const float* W3;
  const float* b3;
  int K;
  const float* W;
  const float* b;
};

template <typename OT>
__global__ void __launch_bounds__(64 * TAIL_WAVES) k_act_tail(ActTail tl, const float* __restrict__ std,
                                                              const float* __restrict__ value,
                                                              const float* __restrict__ obs,
                                                              const float* __restrict__ cobs, int n, int A,
                                                              int64_t obs_w, int64_t cobs_w, int64_t obs_ld,
                                                              int64_t obs_c0, int64_t cobs_ld,
                                                              float* __restrict__ act_out, float* __restrict__ logp_out,
                                                              float* __restrict__ mu_out, float* __restrict__ sigma_out,
                                                              float* __restrict__ value_out, int64_t obs_out_ld,
                                                              OT* __restrict__ obs_out, OT* __restrict__ cobs_out,
                                                              int row_offset, uint64_t seed, uint64_t counter,
                                                              int env_blocks) {
  if ((int)blockIdx.x < env_blocks) {
    __shared__ __attribute__((aligned(16))) float hs[16][HEAD_K + 4];  // 528-byte rows: 16-byte aligned
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int i = lane & 15, g = lane >> 4;
    const int64_t r0 = (int64_t)blockIdx.x * 16;
    const int c = wv * 16 + i;
    {
      const float* xr = tl.x + (int64_t)min((int)r0 + i, n - 1) * tl.ldx + 8 * g;
      const float* wr = tl.W3 + (int64_t)c * tl.K + 8 * g;
      hg_f32x4 acc0, acc1;
      hg_lin16_acc<true>(xr, wr, tl.K, g, acc0, acc1);
      const float bc = tl.b3[c];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        float v = acc0[q] + acc1[q] + bc;
        v = v > 0.f ? v : expm1f(v);
        hs[4 * g + q][c] = v;
      }
    }
    __syncthreads();
    if (threadIdx.x >= 16 * ACT_LANES) return;
    const int el = threadIdx.x / ACT_LANES, j = threadIdx.x % ACT_LANES;
    const int e = (int)r0 + el;
    if (e >= n) return;  // whole groups leave together
    const float m = act_head_mean(&hs[el][0], tl.W, tl.b, j);
    act_env16(e, j, A, m, std, value, act_out, logp_out, mu_out, sigma_out, value_out, row_offset, seed, counter);
    return;
  }
  act_copy_obs<OT>((int64_t)(blockIdx.x - env_blocks) * TAIL_WAVES + (threadIdx.x >> 6),
                   (int64_t)(gridDim.x - env_blocks) * TAIL_WAVES, obs, cobs, n, obs_w, cobs_w, obs_ld, obs_c0,
                   cobs_ld, obs_out_ld, obs_out, cobs_out);
}

__global__ void __launch_bounds__(TPB) k_env(const float* __restrict__ rew, const uint8_t* __restrict__ reset,
                                            const uint8_t* __restrict__ time_out, const float* __restrict__ values,
                                            int n, float gamma, float* __restrict__ rew_out,
                                            uint8_t* __restrict__ dones_out, uint8_t* __restrict__ time_out_out) {
  const int e = blockIdx.x * TPB + threadIdx.x;
  if (e >= n) return;
  float r = rew[e];
  if (time_out && values) r += gamma * (values[e] * (float)time_out[e]);
  rew_out[e] = r;
  dones_out[e] = reset[e];
  if (time_out_out) time_out_out[e] = time_out ? time_out[e] : (uint8_t)0;
}

int launch_act(const float* mean, ActHead hd, const float* std, const float* value, const float* obs,
               const float* critic_obs, int num_envs, int num_actions, int64_t obs_width, int64_t critic_obs_width,
               int64_t obs_ld, int64_t obs_col0, int64_t critic_obs_ld, float* actions_out, float* logp_out,
               float* mu_out, float* sigma_out, float* value_out, void* obs_out, int64_t obs_out_ld,
               void* critic_obs_out, int obs_fp16, int row_offset, uint64_t seed, uint64_t counter, void* stream) {
  if ((!mean && !hd.h) || !std || (value && !value_out) || !obs || !actions_out || !logp_out || !mu_out || !sigma_out ||
      !obs_out || num_envs <= 0 || num_actions <= 0 || num_actions > 64 || obs_width <= 0 || obs_col0 < 0 ||
      (obs_out_ld != 0 && obs_out_ld < obs_width) ||
      obs_ld < obs_col0 + obs_width || (critic_obs_width > 0 && (!critic_obs || !critic_obs_out ||
                                                                 critic_obs_ld < critic_obs_width)))
    return HG_ERR_ARG;
  const int64_t env_threads = (int64_t)num_envs * (num_actions <= ACT_LANES ? ACT_LANES : 1);
  const int env_blocks = (int)((env_threads + TPB - 1) / TPB);
  const int64_t copy_rows = critic_obs_width > 0 ? 2 * (int64_t)num_envs : num_envs;
  const int copy_blocks = (int)std::min<int64_t>((copy_rows + TPB / 64 - 1) / (TPB / 64), 2048);
  const int64_t cw = critic_obs_width > 0 ? critic_obs_width : 0;
  const int64_t old = obs_out_ld ? obs_out_ld : obs_width;
  hipStream_t s = (hipStream_t)stream;
#define HG_ACT(OT, H) hipLaunchKernelGGL((k_act<OT, H>), dim3(env_blocks + copy_blocks), dim3(TPB), 0, s, mean, hd, std,  \
                                         value, obs, critic_obs, num_envs, num_actions, obs_width, cw, obs_ld, obs_col0, \
                                         critic_obs_ld, actions_out, logp_out, mu_out, sigma_out, value_out, old,       \
                                         (OT*)obs_out, (OT*)critic_obs_out, row_offset, seed, counter, env_blocks)
  const bool head = hd.h != nullptr;
  if (obs_fp16) {
    if (head) HG_ACT(__half, true);
    else HG_ACT(__half, false);
  } else {
    if (head) HG_ACT(float, true);
    else HG_ACT(float, false);
  }
#undef HG_ACT
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}

int launch_act_tail(ActTail tl, const float* std, const float* value, const float* obs, const float* critic_obs,
                    int num_envs, int num_actions, int64_t obs_width, int64_t critic_obs_width, int64_t obs_ld,
                    int64_t obs_col0, int64_t critic_obs_ld, float* actions_out, float* logp_out, float* mu_out,
                    float* sigma_out, float* value_out, void* obs_out, int64_t obs_out_ld, void* critic_obs_out,
                    int obs_fp16, int row_offset, uint64_t seed, uint64_t counter, void* stream) {
  if (!std || (value && !value_out) || !obs || !actions_out || !logp_out || !mu_out || !sigma_out || !obs_out ||
      num_envs <= 0 || num_actions != HEAD_N || obs_width <= 0 || obs_col0 < 0 ||
      (obs_out_ld != 0 && obs_out_ld < obs_width) || obs_ld < obs_col0 + obs_width ||
      (critic_obs_width > 0 && (!critic_obs || !critic_obs_out || critic_obs_ld < critic_obs_width)))
    return HG_ERR_ARG;
  const int env_blocks = (num_envs + 15) / 16;
  const int64_t copy_rows = critic_obs_width > 0 ? 2 * (int64_t)num_envs : num_envs;
  const int copy_blocks = (int)std::min<int64_t>((copy_rows + TAIL_WAVES - 1) / TAIL_WAVES, 1024);
  const int64_t cw = critic_obs_width > 0 ? critic_obs_width : 0;
  const int64_t old = obs_out_ld ? obs_out_ld : obs_width;
  hipStream_t s = (hipStream_t)stream;
#define HG_ACTT(OT) hipLaunchKernelGGL((k_act_tail<OT>), dim3(env_blocks + copy_blocks), dim3(64 * TAIL_WAVES), 0, s, tl, \
                                       std, value, obs, critic_obs, num_envs, num_actions, obs_width, cw, obs_ld,        \
                                       obs_col0, critic_obs_ld, actions_out, logp_out, mu_out, sigma_out, value_out, old, \
                                       (OT*)obs_out, (OT*)critic_obs_out, row_offset, seed, counter, env_blocks)
  if (obs_fp16) HG_ACTT(__half);
  else HG_ACTT(float);
#undef HG_ACTT
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}
}  // namespace

extern "C" int hg_rollout_act(const float* mean, const float* std, const float* value, const float* obs,
                              const float* critic_obs, int num_envs, int num_actions, int64_t obs_width,
                              int64_t critic_obs_width, int64_t obs_ld, int64_t obs_col0, int64_t critic_obs_ld,
                              float* actions_out, float* logp_out, float* mu_out, float* sigma_out, float* value_out,
                              void* obs_out, int64_t obs_out_ld, void* critic_obs_out, int obs_fp16, int row_offset,
                              uint64_t seed, uint64_t counter, void* stream) {
  if (!mean) return HG_ERR_ARG;
  return launch_act(mean, ActHead{nullptr, 0, nullptr, nullptr}, std, value, obs, critic_obs, num_envs, num_actions,
                    obs_width, critic_obs_width, obs_ld, obs_col0, critic_obs_ld, actions_out, logp_out, mu_out,
                    sigma_out, value_out, obs_out, obs_out_ld, critic_obs_out, obs_fp16, row_offset, seed, counter,
                    stream);
}

extern "C" int hg_rollout_act_head(const float* h, int64_t h_ld, const float* W, const float* b, int head_k,
                                   const float* std, const float* value, const float* obs, const float* critic_obs,
                                   int num_envs, int num_actions, int64_t obs_width, int64_t critic_obs_width,
                                   int64_t obs_ld, int64_t obs_col0, int64_t critic_obs_ld, float* actions_out,
                                   float* logp_out, float* mu_out, float* sigma_out, float* value_out, void* obs_out,
                                   int64_t obs_out_ld, void* critic_obs_out, int obs_fp16, int row_offset,
                                   uint64_t seed, uint64_t counter, void* stream) {
  if (!h || !W || !b || num_actions != HEAD_N || head_k != HEAD_K || h_ld < HEAD_K || h_ld % 4 != 0 ||
      (uintptr_t)h % 16 != 0 || (uintptr_t)W % 16 != 0)
    return HG_ERR_ARG;
  return launch_act(nullptr, ActHead{h, h_ld, W, b}, std, value, obs, critic_obs, num_envs, num_actions, obs_width,
                    critic_obs_width, obs_ld, obs_col0, critic_obs_ld, actions_out, logp_out, mu_out, sigma_out,
                    value_out, obs_out, obs_out_ld, critic_obs_out, obs_fp16, row_offset, seed, counter, stream);
}

// hg_rollout_act_head with the actor's last hidden layer folded in (k_act_tail): x [num_envs, tail_k]
// (row stride x_ld) is that layer's input, W3 [HEAD_K, tail_k] / b3 its weight and bias (ELU), W / b
// the output layer.  Bitwise hg_linear_act_forward (16 x 16 tile, hg_linear_act_tile's choice at the
// rollout's row counts) followed by hg_rollout_act_head.  16-byte aligned rows required.
extern "C" int hg_rollout_act_tail(const float* x, int64_t x_ld, const float* W3, const float* b3, int tail_k,
                                   const float* W, const float* b, const float* std, const float* value,
                                   const float* obs, const float* critic_obs, int num_envs, int num_actions,
                                   int64_t obs_width, int64_t critic_obs_width, int64_t obs_ld, int64_t obs_col0,
                                   int64_t critic_obs_ld, float* actions_out, float* logp_out, float* mu_out,
                                   float* sigma_out, float* value_out, void* obs_out, int64_t obs_out_ld,
                                   void* critic_obs_out, int obs_fp16, int row_offset, uint64_t seed, uint64_t counter,
                                   void* stream) {
  if (!x || !W3 || !b3 || !W || !b || tail_k <= 0 || tail_k % 4 != 0 || x_ld < tail_k || x_ld % 4 != 0 ||
      (uintptr_t)x % 16 != 0 || (uintptr_t)W3 % 16 != 0 || (uintptr_t)W % 16 != 0)
    return HG_ERR_ARG;
  return launch_act_tail(ActTail{x, x_ld, W3, b3, tail_k, W, b}, std, value, obs, critic_obs, num_envs, num_actions,
                         obs_width, critic_obs_width, obs_ld, obs_col0, critic_obs_ld, actions_out, logp_out, mu_out,
                         sigma_out, value_out, obs_out, obs_out_ld, critic_obs_out, obs_fp16, row_offset, seed, counter,
                         stream);
}
extern "C" int hg_rollout_env(const float* rewards, const uint8_t* reset, const uint8_t* time_outs,
                              const float* values, int num_envs, float gamma, float* rewards_out,
                              uint8_t* dones_out, uint8_t* time_outs_out, void* stream) {
  if (!rewards || !reset || !rewards_out || !dones_out || num_envs <= 0) return HG_ERR_ARG;
  hipLaunchKernelGGL(k_env, dim3((num_envs + TPB - 1) / TPB), dim3(TPB), 0, (hipStream_t)stream, rewards, reset,
                     time_outs, values, num_envs, gamma, rewards_out, dones_out, time_outs_out);
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}

// ---------------------------------------------------------------------------------------------
// Minibatch gather (RolloutStorage.mini_batch_generator, rollout_storage.py:153-191:
// observations[batch_idx], critic_observations[batch_idx], ... ): one launch copies row idx[i]
// of up to three row-major tables into row i of their minibatch buffers.  One wave per output
// row, lanes along the row with 4 independent element loads in flight per lane; 4-byte or
// 2-byte elements (the 705-wide fp32 observation rows are not 16-byte aligned, fp16 storage
// rows not 4-byte aligned).  torch's index kernel ran these at ~2.2 TB/s with per-element 64-bit
// index arithmetic.
namespace {

struct GatherTab {
  const void* src;
  void* dst;
  int64_t width;  // elements per row
  int es;         // element bytes: 4 or 2 (cvt == 0)
  int cvt;        // 0: copy; 1: fp16 -> bf16; 2: fp32 -> bf16 (the bf16 policy's minibatch inputs)
};
struct GatherArgs {
  GatherTab t[3];
  int ntab;
  int short_rows;  // every table 4-byte elements and <= 1024 wide: the all-loads-first path
};

template <typename E>
__device__ inline void gather_row(const E* __restrict__ src, E* __restrict__ dst, int64_t w, int lane) {
  int64_t j = lane;
  for (; j + 192 < w; j += 256) {
    const E a = src[j], b = src[j + 64], c = src[j + 128], d = src[j + 192];
    dst[j] = a;
    dst[j + 64] = b;
    dst[j + 128] = c;
    dst[j + 192] = d;
  }
  for (; j < w; j += 64) dst[j] = src[j];
}

// gathered row converted to bf16 on the way (round-to-nearest-even)
template <typename S>
__device__ inline void gather_row_bf16(const S* __restrict__ src, __bf16* __restrict__ dst, int64_t w, int lane) {
  int64_t j = lane;
  for (; j + 192 < w; j += 256) {
    const float a = (float)src[j], b = (float)src[j + 64], c = (float)src[j + 128], d = (float)src[j + 192];
    dst[j] = (__bf16)a;
    dst[j + 64] = (__bf16)b;
    dst[j + 128] = (__bf16)c;
    dst[j + 192] = (__bf16)d;
  }
  for (; j < w; j += 64) dst[j] = (__bf16)(float)src[j];
}

// rows up to 16 x 64 elements: every load of the row's three tables is issued before the first
// store (up to 48 loads in flight per lane instead of 4)
constexpr int GK = 16;
template <typename E>
__device__ inline void gather_load(const E* __restrict__ src, int64_t w, int lane, E* v) {
#pragma unroll
  for (int k = 0; k < GK; k++) {
    const int64_t j = lane + 64 * k;
    v[k] = j < w ? src[j] : E(0);
  }
}
template <typename E>
__device__ inline void gather_store(E* __restrict__ dst, int64_t w, int lane, const E* v) {
#pragma unroll
  for (int k = 0; k < GK; k++) {
    const int64_t j = lane + 64 * k;
    if (j < w) dst[j] = v[k];
  }
}

__global__ void __launch_bounds__(TPB) k_gather_rows(const int64_t* __restrict__ idx, int64_t rows,
                                                     int64_t src_rows, GatherArgs A) {
  const int64_t i = (int64_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= rows) return;
  int64_t s = idx[i];
  s = s < 0 ? 0 : (s >= src_rows ? src_rows - 1 : s);  // never read out of bounds
  if (A.short_rows) {
    uint32_t v[3][GK];
#pragma unroll
    for (int t = 0; t < 3; t++)
      if (t < A.ntab) gather_load<uint32_t>((const uint32_t*)A.t[t].src + s * A.t[t].width, A.t[t].width, lane, v[t]);
#pragma unroll
    for (int t = 0; t < 3; t++)
      if (t < A.ntab) gather_store<uint32_t>((uint32_t*)A.t[t].dst + i * A.t[t].width, A.t[t].width, lane, v[t]);
    return;
  }
  for (int t = 0; t < A.ntab; t++) {
    const GatherTab& T = A.t[t];
    if (T.cvt == 1)
      gather_row_bf16<_Float16>((const _Float16*)T.src + s * T.width, (__bf16*)T.dst + i * T.width, T.width, lane);
    else if (T.cvt == 2)
      gather_row_bf16<float>((const float*)T.src + s * T.width, (__bf16*)T.dst + i * T.width, T.width, lane);
    else if (T.es == 4)
      gather_row<uint32_t>((const uint32_t*)T.src + s * T.width, (uint32_t*)T.dst + i * T.width, T.width, lane);
    else
      gather_row<uint16_t>((const uint16_t*)T.src + s * T.width, (uint16_t*)T.dst + i * T.width, T.width, lane);
  }
}

}  // namespace

extern "C" int hg_gather_rows(const int64_t* idx, int64_t rows, int64_t src_rows, const void* src0, void* dst0,
                              int64_t width0, int es0, const void* src1, void* dst1, int64_t width1, int es1,
                              const void* src2, void* dst2, int64_t width2, int es2, void* stream) {
  hg_gather_table T[3];
  const void* src[3] = {src0, src1, src2};
  void* dst[3] = {dst0, dst1, dst2};
  const int64_t w[3] = {width0, width1, width2};
  const int es[3] = {es0, es1, es2};
  if (!src0) return HG_ERR_ARG;
  int n = 0;
  for (int t = 0; t < 3; t++) {
    if (!src[t]) continue;
    if (es[t] != 4 && es[t] != 2) return HG_ERR_ARG;
    const int ty = es[t] == 4 ? HG_DTYPE_F32 : HG_DTYPE_F16;  // a 2-byte copy is type-agnostic
    T[n++] = hg_gather_table{src[t], dst[t], w[t], ty, ty};
  }
  return hg_gather_rows_ex(idx, rows, src_rows, T, n, stream);
}

extern "C" int hg_gather_rows_ex(const int64_t* idx, int64_t rows, int64_t src_rows, const hg_gather_table* tabs,
                                 int ntab, void* stream) {
  if (!idx || rows <= 0 || src_rows <= 0 || !tabs || ntab < 1 || ntab > 3) return HG_ERR_ARG;
  GatherArgs A;
  A.ntab = 0;
  for (int t = 0; t < ntab; t++) {
    const hg_gather_table& g = tabs[t];
    if (!g.src || !g.dst || g.width <= 0) return HG_ERR_ARG;
    const auto bytes = [](int ty) { return ty == HG_DTYPE_F32 ? 4 : (ty == HG_DTYPE_F16 || ty == HG_DTYPE_BF16) ? 2 : 0; };
    const int sb = bytes(g.src_dtype), db = bytes(g.dst_dtype);
    if (!sb || !db) return HG_ERR_ARG;
    int cvt = 0;
    if (g.src_dtype != g.dst_dtype) {
      if (g.dst_dtype != HG_DTYPE_BF16) return HG_ERR_ARG;
      cvt = g.src_dtype == HG_DTYPE_F16 ? 1 : 2;
    }
    A.t[A.ntab++] = GatherTab{g.src, g.dst, g.width, sb, cvt};
  }
  A.short_rows = 1;
  for (int t = 0; t < A.ntab; t++) A.short_rows &= (A.t[t].cvt == 0 && A.t[t].es == 4 && A.t[t].width <= 64 * GK);
  const int64_t blocks = (rows + TPB / 64 - 1) / (TPB / 64);
  hipLaunchKernelGGL(k_gather_rows, dim3((unsigned)blocks), dim3(TPB), 0, (hipStream_t)stream, idx, rows, src_rows, A);
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}

// ---------------------------------------------------------------------------------------------
// Minibatch rows of a frame-only observation storage (RolloutStorage with obs_frames): slot t of
// the rollout keeps only the newest W-element frame of the stacked observation the policy saw,
// env-major ([N, T, W]: a row's frames are one contiguous run), slot 0 also the whole stack (init).  The stack of storage row s = t N + e is rebuilt as the
// reference's deque would have held it (humanoid_env.py:880-887): position j < F holds the
// newest frame of slot tau = t - (F - 1 - j) (tau < 0: position j + t of init), zero when the env
// was reset by a post step r with tau <= r <= t - 1 (dones[r][e]; the reset zeroes the history
// before its new frame).  One wave per output row; lane l < F - 1 tests dones[t - 1 - l][e] and
// one ballot gives the latest reset.
// ---------------------------------------------------------------------------------------------
namespace {

// up to two plain tables gathered by the same waves (the critic observations and the packed
// per-sample table of the minibatch): one launch and one index load per row for all of them
struct PlainTabs {
  GatherTab t[2];
  int ntab;
  int early;  // every table 4-byte, no conversion, <= 256 wide: its loads are issued with the frames'
};
constexpr int PK = 4;  // plain-table elements per lane on the early path (256 / 64): one 16-byte access
typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));  // 4-byte-aligned 16-byte accesses
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(4)));

template <typename S, typename D, bool EARLY>
__global__ void __launch_bounds__(TPB) k_gather_stacked(const int64_t* __restrict__ idx, int64_t rows,
                                                        const S* __restrict__ frames, const S* __restrict__ init,
                                                        const uint8_t* __restrict__ dones, int64_t dts, int64_t des,
                                                        int T, int N, int F, int W, D* __restrict__ dst, PlainTabs P) {
  const int64_t i = (int64_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= rows) return;
  const int64_t total = (int64_t)T * N;
  int64_t s = idx[i];
  s = s < 0 ? 0 : (s >= total ? total - 1 : s);  // never read out of bounds
  const int t = (int)(s / N), e = (int)(s - (int64_t)t * N);
  // the plain tables' row loads first (they depend on s only): in flight with the reset scan
  // and the frame loads, stored at the end; lane l holds elements 4l .. 4l + 3
  u32x4u pv[2];
  if (EARLY) {
#pragma unroll
    for (int q = 0; q < 2; q++) {
      if (q >= P.ntab) break;
      const uint32_t* __restrict__ src = (const uint32_t*)P.t[q].src + s * P.t[q].width;
      const int w = (int)P.t[q].width, c = 4 * lane;
      if (c + 3 < w) {
        pv[q] = *reinterpret_cast<const u32x4u*>(src + c);
      } else {
#pragma unroll
        for (int k = 0; k < 4; k++) pv[q][k] = c + k < w ? src[c + k] : 0u;
      }
    }
  }
  const int back = t - 1 - lane;
  // the reset scan's byte loaded first and unconditionally (a clamped slot): waiting for it later
  // (in-order vmcnt) leaves the frame loads issued after it in flight
  const bool scan = lane < F - 1 && back >= 0;
  uint32_t dz = dones[(int64_t)max(back, 0) * dts + (int64_t)e * des];
  // element c of the row: zero below Z (the history a reset cleared), slot 0's stack below Bnd
  // (positions before the rollout: init position j + t, i.e. init row + t W + c), then the
  // env's frames tau = t - (F - 1) + j .. t — one contiguous run in the env-major frame table
  const int row = F * W;
  const int Bnd = (t < F - 1 ? F - 1 - t : 0) * W;
  const S* __restrict__ srcA = init + (int64_t)e * row + (int64_t)t * W;
  const int64_t offB = ((int64_t)e * T + t - (F - 1)) * W;  // frames + offB + c, for c >= Bnd only
  D* __restrict__ out = dst + i * (int64_t)row;
  if constexpr (std::is_same<S, float>::value && std::is_same<D, float>::value) {
    // 4-byte accesses, 64 consecutive elements per wave instruction, every load unconditional (a
    // clamped address past the row's end, the source picked by Bnd with a select): the compiler
    // keeps all of a pass's loads in flight at once.  They depend on the row index only, so they
    // are issued before the reset scan resolves (one dependent round trip instead of two); the
    // history a reset cleared (below Z) is zeroed afterwards.  A 705-wide stack is one pass.
    constexpr int KD = 12;
    for (int base = 0; base < row; base += 64 * KD) {
      float v[KD];
#pragma unroll
      for (int k = 0; k < KD; k++) {
        const int c = min(base + lane + 64 * k, row - 1);
        // one load from a selected address (not two predicated loads and a select)
        const uintptr_t a = c < Bnd ? (uintptr_t)(srcA + c) : (uintptr_t)(frames + offB + c);
        v[k] = *reinterpret_cast<const __attribute__((address_space(1))) float*>(a);  // a global load
      }
      // the scan byte is consumed only now, after the frame loads have been issued
      asm volatile("" : "+v"(dz));
      const uint64_t m = __ballot(scan && dz != 0);
      const int Z = (m ? F - 1 - (__ffsll((unsigned long long)m) - 1) : 0) * W;  // positions j < jz are zero
#pragma unroll
      for (int k = 0; k < KD; k++) {
        const int c = base + lane + 64 * k;
        if (c < row) out[c] = c < Z ? 0.f : v[k];
      }
    }
  } else {
    const uint64_t m = __ballot(scan && dz != 0);
    const int Z = (m ? F - 1 - (__ffsll((unsigned long long)m) - 1) : 0) * W;
    auto elem = [&](int c) -> float {
      return c < Z ? 0.f : (c < Bnd ? (float)srcA[c] : (float)frames[offB + c]);
    };
    constexpr int KB = 16;
    for (int base = 0; base < row; base += 64 * KB) {
      float v[KB];
#pragma unroll
      for (int k = 0; k < KB; k++) {
        const int c = base + lane + 64 * k;
        v[k] = c < row ? elem(c) : 0.f;
      }
#pragma unroll
      for (int k = 0; k < KB; k++) {
        const int c = base + lane + 64 * k;
        if (c < row) out[c] = (D)v[k];
      }
    }
  }
  if (EARLY) {
#pragma unroll
    for (int q = 0; q < 2; q++) {
      if (q >= P.ntab) break;
      uint32_t* __restrict__ d = (uint32_t*)P.t[q].dst + i * P.t[q].width;
      const int w = (int)P.t[q].width, c = 4 * lane;
      if (c + 3 < w) {
        *reinterpret_cast<u32x4u*>(d + c) = pv[q];
      } else {
#pragma unroll
        for (int k = 0; k < 4; k++)
          if (c + k < w) d[c + k] = pv[q][k];
      }
    }
    return;
  }
#pragma unroll
  for (int q = 0; q < 2; q++) {  // constant indices: no dynamic indexing of the kernel argument
    if (q >= P.ntab) break;
    const GatherTab& G = P.t[q];
    if (G.cvt == 1)
      gather_row_bf16<_Float16>((const _Float16*)G.src + s * G.width, (__bf16*)G.dst + i * G.width, G.width, lane);
    else if (G.cvt == 2)
      gather_row_bf16<float>((const float*)G.src + s * G.width, (__bf16*)G.dst + i * G.width, G.width, lane);
    else if (G.es == 4)
      gather_row<uint32_t>((const uint32_t*)G.src + s * G.width, (uint32_t*)G.dst + i * G.width, G.width, lane);
    else
      gather_row<uint16_t>((const uint16_t*)G.src + s * G.width, (uint16_t*)G.dst + i * G.width, G.width, lane);
  }
}

}  // namespace

extern "C" int hg_gather_stacked(const int64_t* idx, int64_t rows, const void* frames, const void* init,
                                 const uint8_t* dones, int64_t dones_ts, int64_t dones_es, int T, int N, int F, int W,
                                 int src_dtype, void* dst, int dst_dtype, const hg_gather_table* tabs, int ntab,
                                 void* stream) {
  if (!idx || rows <= 0 || !frames || !init || !dones || !dst || T <= 0 || N <= 0 || F <= 0 || F > 64 || W <= 0 ||
      (int64_t)F * W > 0x7fffffff || ntab < 0 || ntab > 2 || (ntab > 0 && !tabs))
    return HG_ERR_ARG;
  PlainTabs P;
  P.ntab = 0;
  for (int t = 0; t < ntab; t++) {  // the plain rows of the same storage rows (T*N of them)
    const hg_gather_table& g = tabs[t];
    if (!g.src || !g.dst || g.width <= 0) return HG_ERR_ARG;
    const auto bytes = [](int ty) { return ty == HG_DTYPE_F32 ? 4 : (ty == HG_DTYPE_F16 || ty == HG_DTYPE_BF16) ? 2 : 0; };
    const int sb = bytes(g.src_dtype), db = bytes(g.dst_dtype);
    if (!sb || !db) return HG_ERR_ARG;
    int cvt = 0;
    if (g.src_dtype != g.dst_dtype) {
      if (g.dst_dtype != HG_DTYPE_BF16) return HG_ERR_ARG;
      cvt = g.src_dtype == HG_DTYPE_F16 ? 1 : 2;
    }
    P.t[P.ntab++] = GatherTab{g.src, g.dst, g.width, sb, cvt};
  }
  P.early = 1;
  for (int t = 0; t < P.ntab; t++) P.early &= (P.t[t].es == 4 && P.t[t].cvt == 0 && P.t[t].width <= 64 * PK);
  const int64_t blocks = (rows + TPB / 64 - 1) / (TPB / 64);
  if (blocks > 0x7fffffff) return HG_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const dim3 g((unsigned)blocks), b(TPB);
#define HG_GS(ST, DT)                                                                                          \
  do {                                                                                                        \
    if (P.early)                                                                                              \
      hipLaunchKernelGGL((k_gather_stacked<ST, DT, true>), g, b, 0, s, idx, rows, (const ST*)frames,          \
                         (const ST*)init, dones, dones_ts, dones_es, T, N, F, W, (DT*)dst, P);                \
    else                                                                                                      \
      hipLaunchKernelGGL((k_gather_stacked<ST, DT, false>), g, b, 0, s, idx, rows, (const ST*)frames,         \
                         (const ST*)init, dones, dones_ts, dones_es, T, N, F, W, (DT*)dst, P);                \
  } while (0)
  if (src_dtype == HG_DTYPE_F32 && dst_dtype == HG_DTYPE_F32) HG_GS(float, float);
  else if (src_dtype == HG_DTYPE_F32 && dst_dtype == HG_DTYPE_BF16) HG_GS(float, __bf16);
  else if (src_dtype == HG_DTYPE_F16 && dst_dtype == HG_DTYPE_F16) HG_GS(_Float16, _Float16);
  else if (src_dtype == HG_DTYPE_F16 && dst_dtype == HG_DTYPE_BF16) HG_GS(_Float16, __bf16);
  else if (src_dtype == HG_DTYPE_F16 && dst_dtype == HG_DTYPE_F32) HG_GS(_Float16, float);
  else return HG_ERR_ARG;
#undef HG_GS
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}

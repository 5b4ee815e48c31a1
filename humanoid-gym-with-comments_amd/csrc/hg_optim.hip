// hg_optim.hip — fused global-norm gradient clipping + Adam for the PPO update (gfx950).
//
// Replaces, on the device path, the reference's per-minibatch
//   nn.utils.clip_grad_norm_(parameters, max_grad_norm); optimizer.step()
// (humanoid/algo/ppo/ppo.py:212-214; torch.optim.Adam defaults betas (0.9, 0.999), eps 1e-8).
// Two launches over a list of up to HG_MAX_TENSORS parameter tensors, passed by value:
//   k_sqnorm: per-block partial sums of g^2 (fixed chunk -> block map, deterministic), and each
//             tensor's first block increments that tensor's step counter;
//   k_adam:   every block reduces the partials in a fixed order (deterministic total norm),
//             clip_coef = min(max_norm / (||g|| + 1e-6), 1) as clip_grad_norm_, then Adam:
//               m = b1 m + (1 - b1) g';  v = b2 v + (1 - b2) g'^2
//               p -= (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
//             with g' = g * clip_coef and the learning rate read from device memory (so the
//             adaptive-KL schedule never leaves the GPU and the step is graph-capturable).
// HBM per step: 7 x 4 B per parameter (read p, g, m, v; write p, m, v) + 4 B for the norm pass.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/hgsim.h"

namespace {

constexpr int CHUNK = 4096;   // elements per block
constexpr int TPB = 256;

__global__ void __launch_bounds__(TPB) k_sqnorm(hg_tensor_list T, float* __restrict__ partial) {
  const int b = blockIdx.x;
  int t = 0;
  while (t + 1 < T.count && T.chunk_start[t + 1] <= b) t++;
  const int64_t off = (int64_t)(b - T.chunk_start[t]) * CHUNK;
  const int64_t n = T.numel[t];
  const float* g = T.grad[t];
  float s = 0.f;
  for (int64_t i = off + threadIdx.x; i < off + CHUNK && i < n; i += TPB) {
    const float x = g[i];
    s += x * x;
  }
  // wave reduction (fixed order), then across the block's 4 waves
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  __shared__ float ws[TPB / 64];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float tot = 0.f;
    for (int w = 0; w < TPB / 64; w++) tot += ws[w];
    partial[b] = tot;
    if (b == T.chunk_start[t] && T.step[t]) *T.step[t] += 1.0f;
  }
}

__global__ void __launch_bounds__(TPB) k_adam(hg_tensor_list T, const float* __restrict__ partial, int nblocks,
                                             const float* __restrict__ lr_ptr, float beta1, float beta2, float eps,
                                             float max_norm) {
  __shared__ float s_coef;
  if (threadIdx.x < 64) {
    float s = 0.f;
    for (int i = threadIdx.x; i < nblocks; i += 64) s += partial[i];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (threadIdx.x == 0) {
      float c = 1.0f;
      if (max_norm > 0.f) {
        const float total = sqrtf(s);
        c = fminf(max_norm / (total + 1e-6f), 1.0f);
      }
      s_coef = c;
    }
  }
  __syncthreads();
  const float coef = s_coef;
  const int b = blockIdx.x;
  int t = 0;
  while (t + 1 < T.count && T.chunk_start[t + 1] <= b) t++;
  const int64_t off = (int64_t)(b - T.chunk_start[t]) * CHUNK;
  const int64_t n = T.numel[t];
  const float step = T.step[t] ? *T.step[t] : 1.0f;
  const float lr = *lr_ptr;
  const float bc1 = 1.0f - powf(beta1, step);
  const float bc2 = 1.0f - powf(beta2, step);
  const float step_size = lr / bc1;
  const float bc2_sqrt = sqrtf(bc2);
  float* __restrict__ p = T.param[t];
  const float* __restrict__ g = T.grad[t];
  float* __restrict__ m = T.exp_avg[t];
  float* __restrict__ v = T.exp_avg_sq[t];
  for (int64_t i = off + threadIdx.x; i < off + CHUNK && i < n; i += TPB) {
    const float gi = g[i] * coef;
    const float mi = beta1 * m[i] + (1.0f - beta1) * gi;
    const float vi = beta2 * v[i] + (1.0f - beta2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] -= step_size * mi / denom;
  }
}

}  // namespace

extern "C" int hg_adam_step(const hg_tensor_list* T, const float* lr, float beta1, float beta2, float eps,
                            float max_norm, float* partial, void* stream) {
  if (!T || !lr || !partial || T->count < 1 || T->count > HG_MAX_TENSORS) return HG_ERR_ARG;
  const int nblocks = T->chunk_start[T->count];
  if (nblocks <= 0) return HG_ERR_ARG;
  for (int t = 0; t < T->count; t++) {
    const int64_t need = (T->numel[t] + CHUNK - 1) / CHUNK;
    if (!T->param[t] || !T->grad[t] || !T->exp_avg[t] || !T->exp_avg_sq[t] ||
        T->chunk_start[t + 1] - T->chunk_start[t] != need)
      return HG_ERR_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_sqnorm, dim3(nblocks), dim3(TPB), 0, s, *T, partial);
  hipLaunchKernelGGL(k_adam, dim3(nblocks), dim3(TPB), 0, s, *T, partial, nblocks, lr, beta1, beta2, eps, max_norm);
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}

extern "C" int hg_adam_chunk(void) { return CHUNK; }

// ---------------------------------------------------------------------------------------------
// Adaptive-KL learning rate (ppo.py:162-176): one launch for the KL mean, one for the rule, so
// the schedule stays on the device (and inside the captured update graph).
//   kl_row = sum_a [ log(s/s_old + 1e-5) + (s_old^2 + (m_old - m)^2) / (2 s^2) - 0.5 ]
//   kl     = mean_rows kl_row           (row sums in fp32 in action order; per-block then final
//                                        fp64 sums in a fixed order: deterministic)
//   lr     = kl > 2d ? max(lr/1.5, lr_min) : (0 < kl < d/2 ? min(lr*1.5, lr_max) : lr)   (fp64)
// ---------------------------------------------------------------------------------------------
namespace {
__global__ void __launch_bounds__(256) k_kl_partial(const float* __restrict__ mu, const float* __restrict__ sigma,
                                                   const float* __restrict__ old_mu,
                                                   const float* __restrict__ old_sigma, int64_t rows, int A,
                                                   double* __restrict__ partial) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double acc = 0.0;
  if (r < rows) {
    float s = 0.f;
    for (int a = 0; a < A; a++) {
      const int64_t i = r * A + a;
      const float sg = sigma[i], so = old_sigma[i], d = old_mu[i] - mu[i];
      s += logf(sg / so + 1.0e-5f) + (so * so + d * d) / (2.0f * (sg * sg)) - 0.5f;
    }
    acc = (double)s;
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  __shared__ double ws[4];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = (ws[0] + ws[1]) + (ws[2] + ws[3]);
}

__global__ void __launch_bounds__(64) k_kl_final(const double* __restrict__ partial, int nb, int64_t rows,
                                                 float* __restrict__ kl_out) {
  double acc = 0.0;
  for (int i = threadIdx.x; i < nb; i += 64) acc += partial[i];
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if (threadIdx.x == 0) *kl_out = (float)(acc / (double)rows);
}

__global__ void k_lr_rule(const float* __restrict__ kl, double* __restrict__ lr64, float* __restrict__ lr32,
                          double desired, double lr_min, double lr_max) {
  const double k = (double)*kl;
  double lr = *lr64;
  if (k > desired * 2.0) lr = fmax(lr / 1.5, lr_min);
  else if (k < desired / 2.0 && k > 0.0) lr = fmin(lr * 1.5, lr_max);
  *lr64 = lr;
  *lr32 = (float)lr;
}
}  // namespace

extern "C" int hg_kl_mean(const float* mu, const float* sigma, const float* old_mu, const float* old_sigma,
                          int64_t rows, int num_actions, float* kl_out, double* scratch, void* stream) {
  if (!mu || !sigma || !old_mu || !old_sigma || !kl_out || !scratch || rows <= 0 || num_actions <= 0)
    return HG_ERR_ARG;
  const int nb = (int)((rows + 255) / 256);
  hipLaunchKernelGGL(k_kl_partial, dim3(nb), dim3(256), 0, (hipStream_t)stream, mu, sigma, old_mu, old_sigma, rows,
                     num_actions, scratch);
  hipLaunchKernelGGL(k_kl_final, dim3(1), dim3(64), 0, (hipStream_t)stream, scratch, nb, rows, kl_out);
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}

extern "C" int hg_kl_lr_rule(const float* kl, double* lr64, float* lr32, double desired_kl, double lr_min,
                             double lr_max, void* stream) {
  if (!kl || !lr64 || !lr32) return HG_ERR_ARG;
  hipLaunchKernelGGL(k_lr_rule, dim3(1), dim3(1), 0, (hipStream_t)stream, kl, lr64, lr32, desired_kl, lr_min, lr_max);
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}

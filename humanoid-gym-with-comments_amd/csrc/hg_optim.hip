// hg_optim.hip — fused global-norm gradient clipping + Adam for the PPO update (gfx950).
//
// Replaces, on the device path, the reference's per-minibatch
//   nn.utils.clip_grad_norm_(parameters, max_grad_norm); optimizer.step()
// (humanoid/algo/ppo/ppo.py:212-214; torch.optim.Adam defaults betas (0.9, 0.999), eps 1e-8).
// Two launches over a list of up to HG_MAX_TENSORS parameter tensors, passed by value:
//   k_sqnorm: per-block partial sums of g^2 (fixed chunk -> block map, deterministic), and each
//             tensor's first block increments that tensor's step counter;
//   k_adam:   every block reduces the partials in one fixed order (deterministic total norm; its
//             own chunk's loads issued before that reduction),
//             clip_coef = min(max_norm / (||g|| + 1e-6), 1) as clip_grad_norm_, then Adam:
//               m = b1 m + (1 - b1) g';  v = b2 v + (1 - b2) g'^2
//               p -= (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
//             with g' = g * clip_coef and the learning rate read from device memory (so the
//             adaptive-KL schedule never leaves the GPU and the step is graph-capturable).
// HBM per step: 7 x 4 B per parameter (read p, g, m, v; write p, m, v) + 4 B for the norm pass.
#include <algorithm>
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/hgsim.h"

namespace {

// 1024 elements per block, 4 per thread with all loads issued before the arithmetic: ~1000
// blocks for the 1.03M policy parameters (4 waves per SIMD) instead of 275 latency-bound ones
constexpr int CHUNK = 1024;
constexpr int TPB = 256;
constexpr int PER = CHUNK / TPB;

__global__ void __launch_bounds__(TPB) k_sqnorm(hg_tensor_list T, float* __restrict__ partial) {
  const int b = blockIdx.x;
  int t = 0;
  while (t + 1 < T.count && T.chunk_start[t + 1] <= b) t++;
  const int64_t off = (int64_t)(b - T.chunk_start[t]) * CHUNK;
  const int64_t n = T.numel[t];
  const float* g = T.grad[t];
  float x[PER];
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const int64_t i = off + threadIdx.x + k * TPB;
    x[k] = i < n ? g[i] : 0.f;
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < PER; k++) s += x[k] * x[k];
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
  // the chunk's parameter / gradient / moment loads go out first, so their latency overlaps the
  // norm reduction (a barrier would otherwise hold them back)
  const int b = blockIdx.x;
  int t = 0;
  while (t + 1 < T.count && T.chunk_start[t + 1] <= b) t++;
  const int64_t off = (int64_t)(b - T.chunk_start[t]) * CHUNK;
  const int64_t n = T.numel[t];
  float* __restrict__ p = T.param[t];
  const float* __restrict__ g = T.grad[t];
  float* __restrict__ m = T.exp_avg[t];
  float* __restrict__ v = T.exp_avg_sq[t];
  float gk[PER], mk[PER], vk[PER], pk[PER];
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const int64_t i = off + threadIdx.x + k * TPB;
    if (i < n) { gk[k] = g[i]; mk[k] = m[i]; vk[k] = v[i]; pk[k] = p[i]; }
  }
  // total squared norm from the k_sqnorm partials, the same fixed order in every block: thread t
  // sums partials t, t + 256, ... (independent loads), then the wave and the four waves in order
  __shared__ float ws[TPB / 64];
  float s = 0.f;
#pragma unroll 4
  for (int i = threadIdx.x; i < nblocks; i += TPB) s += partial[i];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  float coef = 1.0f;
  if (max_norm > 0.f) {
    const float total = sqrtf((ws[0] + ws[1]) + (ws[2] + ws[3]));
    coef = fminf(max_norm / (total + 1e-6f), 1.0f);
  }
  const float step = T.step[t] ? *T.step[t] : 1.0f;
  const float lr = *lr_ptr;
  const float bc1 = 1.0f - powf(beta1, step);
  const float bc2 = 1.0f - powf(beta2, step);
  const float step_size = lr / bc1;
  const float bc2_sqrt = sqrtf(bc2);
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const int64_t i = off + threadIdx.x + k * TPB;
    if (i < n) {
      const float gi = gk[k] * coef;
      const float mi = beta1 * mk[k] + (1.0f - beta1) * gi;
      const float vi = beta2 * vk[k] + (1.0f - beta2) * gi * gi;
      m[i] = mi;
      v[i] = vi;
      const float denom = sqrtf(vi) / bc2_sqrt + eps;
      p[i] = pk[k] - step_size * mi / denom;
    }
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

// ---------------------------------------------------------------------------------------------
// Fused PPO minibatch loss (ppo.py:155-210).  One thread per sample row:
//   logp   = sum_a [ -(a - mu)^2 / (2 s^2) - log s - log sqrt(2 pi) ]
//   ratio  = exp(logp - old_logp)
//   surr   = max(-A ratio, -A clamp(ratio, lo, hi))
//   vloss  = max((v - R)^2, (T + clamp(v - T, -c, c) - R)^2)      (or (R - v)^2)
//   lvloss = sum_k (p_k - t_k)^2                                   (MSE numerator)
//   kl     = sum_a [ log(s / s_old + 1e-5) + (s_old^2 + (mu_old - mu)^2) / (2 s^2) - 0.5 ]
// and the row's gradient contributions d loss / d {mu, std, v, p}; the entropy term depends only
// on std and is added once by the final kernel.  torch's backward conventions: maximum splits the
// gradient evenly on ties, clamp passes it on [lo, hi] inclusive.
// ---------------------------------------------------------------------------------------------
namespace {
constexpr int LOSS_TPB = 64;        // one wave per block: 384 blocks at the 24576-row minibatch
constexpr int LOSS_MAX_A = 32;
constexpr float LOG_SQRT_2PI = 0.91893853320467274178f;

__device__ inline float max_w(float x, float y) { return x > y ? 1.f : (x == y ? 0.5f : 0.f); }

__global__ void __launch_bounds__(LOSS_TPB) k_ppo_loss_rows(hg_ppo_batch Bt, int64_t rows, int A, float lo, float hi,
                                                           float vclip, int clipped_value, float c_s, float c_v,
                                                           float c_l, float* __restrict__ g_mu,
                                                           float* __restrict__ g_v, float* __restrict__ g_p,
                                                           double* __restrict__ partial) {
  const int64_t r = (int64_t)blockIdx.x * LOSS_TPB + threadIdx.x;
  const int K = 4 + A;
  // per-row terms: [0] surrogate, [1] value loss, [2] lin-vel squared error, [3] kl, [4+a] d std_a
  float t_surr = 0.f, t_v = 0.f, t_l = 0.f, t_kl = 0.f;
  float gs[LOSS_MAX_A];
#pragma unroll
  for (int a = 0; a < LOSS_MAX_A; a++) gs[a] = 0.f;
  if (r < rows) {
    const float* mu = Bt.mu + r * Bt.mu_ld;
    const float* act = Bt.actions + r * Bt.actions_ld;
    const float* omu = Bt.old_mu + r * Bt.old_mu_ld;
    const float* osg = Bt.old_sigma + r * Bt.old_sigma_ld;
    float logp = 0.f;
#pragma unroll
    for (int a = 0; a < LOSS_MAX_A; a++) {
      if (a >= A) break;
      const float s = Bt.std[a], m = mu[a];
      const float d = act[a] - m;
      logp += -(d * d) / (2.0f * (s * s)) - logf(s) - LOG_SQRT_2PI;
      const float so = osg[a], dm = omu[a] - m;
      t_kl += logf(s / so + 1.0e-5f) + (so * so + dm * dm) / (2.0f * (s * s)) - 0.5f;
    }
    const float ratio = expf(logp - Bt.old_logp[r * Bt.old_logp_ld]);
    const float adv = Bt.advantages[r * Bt.advantages_ld];
    const float rc = fminf(fmaxf(ratio, lo), hi);
    const float s1 = -adv * ratio, s2 = -adv * rc;
    t_surr = fmaxf(s1, s2);
    const float in_r = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;
    const float d_ratio = max_w(s1, s2) * (-adv) + max_w(s2, s1) * (-adv) * in_r;
    const float d_logp = c_s * d_ratio * ratio;
#pragma unroll
    for (int a = 0; a < LOSS_MAX_A; a++) {
      if (a >= A) break;
      const float s = Bt.std[a];
      const float d = act[a] - mu[a];
      const float inv_s2 = 1.0f / (s * s);
      g_mu[r * A + a] = d_logp * d * inv_s2;
      gs[a] = d_logp * (d * d * inv_s2 / s - 1.0f / s);
    }
    // value loss
    const float v = Bt.value[r * Bt.value_ld], R = Bt.returns[r * Bt.returns_ld];
    float dv;
    if (clipped_value) {
      const float T = Bt.target_values[r * Bt.target_values_ld];
      const float dvt = v - T;
      const float vc = T + fminf(fmaxf(dvt, -vclip), vclip);
      const float l1 = (v - R) * (v - R), l2 = (vc - R) * (vc - R);
      t_v = fmaxf(l1, l2);
      const float in_v = (dvt >= -vclip && dvt <= vclip) ? 1.f : 0.f;
      dv = max_w(l1, l2) * 2.0f * (v - R) + max_w(l2, l1) * 2.0f * (vc - R) * in_v;
    } else {
      t_v = (R - v) * (R - v);
      dv = 2.0f * (v - R);
    }
    g_v[r] = c_v * dv;
    // lin-vel MSE
    const float* p = Bt.lin_vel + r * Bt.lin_vel_ld;
    const float* tg = Bt.lin_vel_target + r * Bt.lin_vel_target_ld;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const float e = p[k] - tg[k];
      t_l += e * e;
      g_p[r * 3 + k] = c_l * 2.0f * e;
    }
  }
  // wave reduction in float64, fixed order
  auto wsum = [](double x) {
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    return x;
  };
  double* out = partial + (int64_t)blockIdx.x * K;
  const double s0 = wsum(t_surr), s1 = wsum(t_v), s2 = wsum(t_l), s3 = wsum(t_kl);
  if (threadIdx.x == 0) {
    out[0] = s0;
    out[1] = s1;
    out[2] = s2;
    out[3] = s3;
  }
#pragma unroll
  for (int a = 0; a < LOSS_MAX_A; a++) {
    if (a >= A) break;
    const double s = wsum(gs[a]);
    if (threadIdx.x == 0) out[4 + a] = s;
  }
}

constexpr int FIN_WAVES = 16;
struct LrRule {  // the adaptive-KL rule folded into the loss's final launch (lr64 NULL: none)
  double* lr64;
  float* lr32;
  double desired, lr_min, lr_max;
};
__global__ void __launch_bounds__(64 * FIN_WAVES) k_ppo_loss_final(const double* __restrict__ partial, int nb,
                                                                  int64_t rows, int A, const float* __restrict__ std,
                                                                  float c_v, float c_e, float c_l,
                                                                  float* __restrict__ loss_out,
                                                                  float* __restrict__ stats, int accum,
                                                                  float* __restrict__ g_std, LrRule rule) {
  // one wave per column (columns w, w + 16, ..): lane l sums blocks l, l + 64, .. in order (all
  // its loads in flight at once), then one fixed-order wave reduction — deterministic, and the
  // column chains run side by side instead of one after another in a single block's threads
  __shared__ double col[4 + LOSS_MAX_A];
  __shared__ double ent_a[LOSS_MAX_A];
  const int K = 4 + A;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // the entropy's per-action terms by the last wave's lanes (fp64 log, in parallel; summed in
  // action order below)
  if (wv == FIN_WAVES - 1 && lane < A) ent_a[lane] = 0.5 + (double)LOG_SQRT_2PI + log((double)std[lane]);
  for (int k = wv; k < K; k += FIN_WAVES) {
    double x = 0.0;
#pragma unroll 8
    for (int b = lane; b < nb; b += 64) x += partial[(int64_t)b * K + k];
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    if (lane == 0) col[k] = x;
  }
  __syncthreads();
  if (threadIdx.x < A) {
    const float s = std[threadIdx.x];
    // entropy = mean_rows sum_a (0.5 + log sqrt(2 pi) + log s_a): d/ds_a = 1/s_a
    g_std[threadIdx.x] = (float)col[4 + threadIdx.x] - c_e / s;
  }
  if (threadIdx.x == 0) {
    const double n = (double)rows;
    double ent = 0.0;
    for (int a = 0; a < A; a++) ent += ent_a[a];
    const double surr = col[0] / n, vl = col[1] / n, lv = col[2] / (3.0 * n), kl = col[3] / n;
    loss_out[0] = (float)(surr + (double)c_v * vl - (double)c_e * ent + (double)c_l * lv);
    stats[0] = accum ? stats[0] + (float)vl : (float)vl;
    stats[1] = accum ? stats[1] + (float)surr : (float)surr;
    stats[2] = accum ? stats[2] + (float)lv : (float)lv;
    stats[3] = (float)kl;
    if (rule.lr64) {
      // the adaptive schedule on this minibatch's KL mean, as k_lr_rule reads it (float -> fp64)
      const double k = (double)(float)kl;
      double lr = *rule.lr64;
      if (k > rule.desired * 2.0) lr = fmax(lr / 1.5, rule.lr_min);
      else if (k < rule.desired / 2.0 && k > 0.0) lr = fmin(lr * 1.5, rule.lr_max);
      *rule.lr64 = lr;
      *rule.lr32 = (float)lr;
    }
  }
}

__global__ void __launch_bounds__(256) k_ppo_loss_bwd(const float* __restrict__ g, int64_t rows, int A,
                                                     float* __restrict__ g_mu, float* __restrict__ g_std,
                                                     float* __restrict__ g_v, float* __restrict__ g_p) {
  const float s = *g;
  const int64_t n_mu = rows * A, n_v = rows, n_p = rows * 3;
  const int64_t tot = n_mu + n_v + n_p + A;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < tot; i += (int64_t)gridDim.x * 256) {
    if (i < n_mu) g_mu[i] *= s;
    else if (i < n_mu + n_v) g_v[i - n_mu] *= s;
    else if (i < n_mu + n_v + n_p) g_p[i - n_mu - n_v] *= s;
    else g_std[i - n_mu - n_v - n_p] *= s;
  }
}
}  // namespace

extern "C" int64_t hg_ppo_loss_scratch(int64_t rows, int num_actions) {
  return ((rows + LOSS_TPB - 1) / LOSS_TPB) * (4 + (int64_t)num_actions);
}

namespace {
int launch_ppo_loss(const hg_ppo_batch* B, int64_t rows, int A, float clip_lo, float clip_hi, float value_clip,
                    int clipped_value_loss, float value_loss_coef, float entropy_coef, float lin_vel_coef,
                    float* loss_out, float* stats_out, int accumulate_stats, float* grad_mu, float* grad_std,
                    float* grad_value, float* grad_lin_vel, double* scratch, LrRule rule, void* stream) {
  if (!B || rows <= 0 || A <= 0 || A > LOSS_MAX_A || !loss_out || !stats_out || !grad_mu || !grad_std ||
      !grad_value || !grad_lin_vel || !scratch || !B->mu || !B->std || !B->value || !B->lin_vel ||
      !B->lin_vel_target || !B->actions || !B->old_logp || !B->advantages || !B->returns || !B->old_mu ||
      !B->old_sigma || (clipped_value_loss && !B->target_values))
    return HG_ERR_ARG;
  const int64_t nb64 = (rows + LOSS_TPB - 1) / LOSS_TPB;
  if (nb64 > INT32_MAX) return HG_ERR_ARG;
  const int nb = (int)nb64;
  const double n = (double)rows;
  const float c_s = (float)(1.0 / n), c_v = (float)((double)value_loss_coef / n),
              c_l = (float)((double)lin_vel_coef / (3.0 * n));
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_ppo_loss_rows, dim3(nb), dim3(LOSS_TPB), 0, s, *B, rows, A, clip_lo, clip_hi, value_clip,
                     clipped_value_loss, c_s, c_v, c_l, grad_mu, grad_value, grad_lin_vel, scratch);
  hipLaunchKernelGGL(k_ppo_loss_final, dim3(1), dim3(64 * FIN_WAVES), 0, s, scratch, nb, rows, A, B->std, value_loss_coef,
                     entropy_coef, lin_vel_coef, loss_out, stats_out, accumulate_stats, grad_std, rule);
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}
}  // namespace

extern "C" int hg_ppo_loss(const hg_ppo_batch* B, int64_t rows, int A, float clip_lo, float clip_hi, float value_clip,
                           int clipped_value_loss, float value_loss_coef, float entropy_coef, float lin_vel_coef,
                           float* loss_out, float* stats_out, int accumulate_stats, float* grad_mu, float* grad_std,
                           float* grad_value, float* grad_lin_vel, double* scratch, void* stream) {
  return launch_ppo_loss(B, rows, A, clip_lo, clip_hi, value_clip, clipped_value_loss, value_loss_coef, entropy_coef,
                         lin_vel_coef, loss_out, stats_out, accumulate_stats, grad_mu, grad_std, grad_value,
                         grad_lin_vel, scratch, LrRule{nullptr, nullptr, 0.0, 0.0, 0.0}, stream);
}

extern "C" int hg_ppo_loss_lr(const hg_ppo_batch* B, int64_t rows, int A, float clip_lo, float clip_hi,
                              float value_clip, int clipped_value_loss, float value_loss_coef, float entropy_coef,
                              float lin_vel_coef, float* loss_out, float* stats_out, int accumulate_stats,
                              float* grad_mu, float* grad_std, float* grad_value, float* grad_lin_vel, double* scratch,
                              double* lr64, float* lr32, double desired_kl, double lr_min, double lr_max,
                              void* stream) {
  if (!lr64 || !lr32) return HG_ERR_ARG;
  return launch_ppo_loss(B, rows, A, clip_lo, clip_hi, value_clip, clipped_value_loss, value_loss_coef, entropy_coef,
                         lin_vel_coef, loss_out, stats_out, accumulate_stats, grad_mu, grad_std, grad_value,
                         grad_lin_vel, scratch, LrRule{lr64, lr32, desired_kl, lr_min, lr_max}, stream);
}

extern "C" int hg_ppo_loss_backward(const float* grad_loss, int64_t rows, int A, float* grad_mu, float* grad_std,
                                    float* grad_value, float* grad_lin_vel, void* stream) {
  if (!grad_loss || rows <= 0 || A <= 0 || !grad_mu || !grad_std || !grad_value || !grad_lin_vel) return HG_ERR_ARG;
  const int64_t tot = rows * (A + 4) + A;
  const int nb = (int)std::min<int64_t>((tot + 255) / 256, 1024);
  hipLaunchKernelGGL(k_ppo_loss_bwd, dim3(nb), dim3(256), 0, (hipStream_t)stream, grad_loss, rows, A, grad_mu,
                     grad_std, grad_value, grad_lin_vel);
  return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}

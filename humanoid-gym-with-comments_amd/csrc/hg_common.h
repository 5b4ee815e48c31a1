// hg_common.h — device-side helpers shared by the hg_sim kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hgsim.h"

#define HG_NB 13
#define HG_ND 12
#define HG_NV 18
#define HG_OBS1 47
#define HG_PRIV1 73

// ------------------------------------------------------------------------------------------------
// arena: SoA per-env fields, each row padded to `np` elements (np = N rounded up to 64)
// ------------------------------------------------------------------------------------------------
struct HgState {
  int n, np;
  float* root;        // [13][np]
  float* dof_pos;     // [12][np]
  float* dof_vel;     // [12][np]
  float* contact;     // [13*3][np] SoA
  float* rigid;       // [13*13][np] SoA
  float* torques;     // [12][np]
  float* actions;     // [12][np]
  float* last_actions;
  float* last_last_actions;
  float* last_dof_vel;    // [12][np]
  float* last_root_vel;   // [6][np]
  float* commands;        // [4][np]
  float* obs;             // [n][(frame_stack - 1 + HW) * 47] history windows (hg_api.hip)
  float* priv;            // [n][(c_frame_stack - 1 + HW) * 73]
  float* rew;             // [np]
  uint8_t* reset_buf;     // [np]
  uint8_t* time_out;      // [np]
  int64_t* ep_len;        // [np]
  float* ep_sums;         // [22][np]
  float* feet_air_time;   // [2][np]
  uint8_t* last_contacts; // [2][np]
  float* feet_height;     // [2][np]
  float* last_feet_z;     // [2][np]
  float* friction;        // [np]
  float* body_mass;       // [np]
  float* push_force;      // [3][np]
  float* push_torque;     // [3][np]
  float* base_lin_vel;    // [3][np]
  float* base_ang_vel;    // [3][np]
  float* proj_gravity;    // [3][np]
  float* base_euler;      // [3][np]
  float* ref_dof_pos;     // [12][np]
  float* env_origins;     // [3][np]
  float* ep_stats;        // [24] (+ accumulators [24] after)
  float* lambda;          // [HG_LAMW][np] solver warm-start impulses
  int32_t* nonfinite;     // [np]
  int32_t* terrain_level; // [np]
  int32_t* terrain_type;  // [np]
  int32_t* rows_dropped;  // [np] rows / contact points the row budget dropped (K_step, summed over substeps)
  float* obs_noise;       // [np][48] N(0,1) observation noise of the next post launch (K_step epilogue;
                          // per-env rows, so each wave writes whole cache lines)
  uint64_t* noise_counter;// [1] the post counter obs_noise was drawn for (~0: none)
  int32_t* env_rows;      // [np] constraint rows of each env's last substep (K_step), the cost the next
                          // step's wave balancing sorts by
  int32_t* env_order;     // [np] K_step's env order: within each XCD's env range, heaviest first
  int balance;            // 1: K_step maps block -> env pair through env_order (hg_create: HG_WAVE_BALANCE)
  const hg_cfg* cfg;      // device copy
  const hg_model* model;  // device copy
};

// the rollout-storage slot a step's post launch also fills (hg_set_rollout_sink): rewards [n] f32,
// dones [n] u8 and (optional) time-out flags [n] u8 — what hg_rollout_env writes with the value
// bootstrap deferred; all NULL: no sink
struct HgSink {
  float* rew;
  uint8_t* dones;
  uint8_t* time_outs;
};

// one observation history window table for the post launch: row e = win + e * rowlen, frame slots of
// `width` floats; this launch writes the new frame into slot head + frames - 1, zeroes slots
// head .. head + frames - 2 of reset envs and, when shift_src >= 0, first moves slots
// shift_src .. shift_src + frames - 2 to 0 .. frames - 2
struct HgWindow {
  float* win;
  int64_t rowlen;
  int width, frames, head, shift_src;
};

// contact forces / rigid states are SoA too (field-major, [b*3+i][np] and [b*13+f][np]); the torch
// views keep the reference's [N,13,3] / [N,13,13] shapes with strides (1, 3 np, np) / (1, 13 np, np)
#define HG_CF(S, e, b, i) ((S).contact[(size_t)((b) * 3 + (i)) * (S).np + (e)])
#define HG_RS(S, e, b, f) ((S).rigid[(size_t)((b) * 13 + (f)) * (S).np + (e)])

// ------------------------------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al. SC'11).  Keyed by the run seed; counter = (a, b, c, purpose).
// ------------------------------------------------------------------------------------------------
struct u4 { uint32_t x, y, z, w; };

__host__ __device__ inline u4 philox4x32_10(u4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; r++) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    u4 n = {hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    c = n;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

enum HgRngPurpose : uint32_t {
  RNG_ACT_DELAY = 1, RNG_ACT_NOISE = 2, RNG_OBS_NOISE = 3, RNG_CMD = 4, RNG_PUSH = 5,
  RNG_RESET_DOF = 6, RNG_RESET_ROOT = 7, RNG_TERRAIN = 8,
};

// uniform in [0,1): 24 high bits
__host__ __device__ inline float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }
// uniform in (0,1]
__host__ __device__ inline float u01_open0(uint32_t x) { return (float)((x >> 8) + 1u) * (1.0f / 16777216.0f); }

__device__ inline u4 rng4(const hg_cfg* cfg, uint32_t env, uint64_t step, uint32_t block, uint32_t purpose) {
  u4 c = {env + (uint32_t)cfg->env_offset, (uint32_t)step, (block & 0xFFFFu) | ((uint32_t)(step >> 32) << 16), purpose};
  return philox4x32_10(c, (uint32_t)cfg->seed, (uint32_t)(cfg->seed >> 32));
}

// Box–Muller: 4 uniforms -> 4 standard normals
__device__ inline void normals4(u4 r, float* z) {
  const float two_pi = 6.283185307179586f;
  float r0 = sqrtf(-2.0f * logf(u01_open0(r.x)));
  float r1 = sqrtf(-2.0f * logf(u01_open0(r.z)));
  float s0, c0, s1, c1;
  sincosf(two_pi * u01(r.y), &s0, &c0);
  sincosf(two_pi * u01(r.w), &s1, &c1);
  z[0] = r0 * c0; z[1] = r0 * s0; z[2] = r1 * c1; z[3] = r1 * s1;
}

// ------------------------------------------------------------------------------------------------
// small vector math
// ------------------------------------------------------------------------------------------------
struct f3 { float x, y, z; };
__device__ __forceinline__ f3 mk(float x, float y, float z) { return {x, y, z}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ f3 operator*(float s, f3 a) { return {s * a.x, s * a.y, s * a.z}; }
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

// xyzw quaternion rotate-inverse, as isaacgym.torch_utils.quat_rotate_inverse
__device__ __forceinline__ f3 quat_rotate_inverse(float qx, float qy, float qz, float qw, f3 v) {
  f3 qv = mk(qx, qy, qz);
  f3 a = (2.0f * qw * qw - 1.0f) * v;
  f3 b = (qw * 2.0f) * cross(qv, v);
  f3 c = (2.0f * dot(qv, v)) * qv;
  return a - b + c;
}
__device__ __forceinline__ f3 quat_apply(float qx, float qy, float qz, float qw, f3 v) {
  f3 xyz = mk(qx, qy, qz);
  f3 t = 2.0f * cross(xyz, v);
  return v + qw * t + cross(xyz, t);
}

// K_step's env order for wave balancing (HgState::env_order; k_step maps its blocks through it):
// per XCD env range (k_step's block -> pair map: XCD x owns pairs p0 .. p0 + cnt - 1 of the nb =
// ceil(n / 2) pairs), a stable counting sort of the range's envs by the PGS groups of their last
// substep (HgState::env_rows), heaviest first (12 bins: ceil(rows / 3) capped at 11).  One
// 256-thread block per range, run as extra blocks of the post launch (k_window_stats), so the
// order is ready for the next step's K_step without a launch of its own.
constexpr int HG_ORD_T = 256, HG_ORD_BINS = 12;
__device__ __forceinline__ int hg_order_bin(int rows) {
  return HG_ORD_BINS - 1 - min((max(rows, 0) + 2) / 3, HG_ORD_BINS - 1);
}
__device__ inline void hg_env_order_block(const int32_t* __restrict__ rows, int32_t* __restrict__ order, int n,
                                          int xcd) {
  __shared__ int c[HG_ORD_BINS * HG_ORD_T];
  __shared__ int ws[HG_ORD_T];
  const int nb = (n + 1) / 2, t = threadIdx.x;
  const int cnt = (nb >> 3) + (xcd < (nb & 7) ? 1 : 0);
  const int p0 = xcd * (nb >> 3) + min(xcd, nb & 7);
  const int e0 = 2 * p0, m = max(0, min(n, 2 * (p0 + cnt)) - e0);
  const int per = (m + HG_ORD_T - 1) / HG_ORD_T;
  const int a0 = e0 + min(m, t * per), a1 = e0 + min(m, (t + 1) * per);
  for (int k = 0; k < HG_ORD_BINS; k++) c[k * HG_ORD_T + t] = 0;
  for (int e = a0; e < a1; e++) c[hg_order_bin(rows[e]) * HG_ORD_T + t] += 1;  // own column: no atomics
  __syncthreads();
  // exclusive prefix of c in (bin, thread) order: thread t owns flat entries [12 t, 12 t + 12)
  int s = 0;
  for (int i = 0; i < HG_ORD_BINS; i++) s += c[HG_ORD_BINS * t + i];
  ws[t] = s;
  __syncthreads();
  for (int off = 1; off < HG_ORD_T; off <<= 1) {
    const int v = t >= off ? ws[t - off] : 0;
    __syncthreads();
    ws[t] += v;
    __syncthreads();
  }
  int run = ws[t] - s;
  for (int i = 0; i < HG_ORD_BINS; i++) {
    const int v = c[HG_ORD_BINS * t + i];
    c[HG_ORD_BINS * t + i] = run;
    run += v;
  }
  __syncthreads();
  for (int e = a0; e < a1; e++) order[e0 + c[hg_order_bin(rows[e]) * HG_ORD_T + t]++] = e;
}

// One wave's 16 x 16 tile of x W^T on v_mfma_f32_16x16x4_f32 (A[i = l & 15][k = l >> 4], B[k = l >> 4]
// [j = l & 15], C row 4 (l >> 4) + q, column l & 15): lane group g = l >> 4 owns the 8 consecutive k
// [8g, 8g + 8) of each 32-wide chunk (xr / wr point at its row's element 8g); MFMA step s takes
// k = 8g + s, two accumulators (even / odd steps) cover the dependent-accumulator latency, the next
// chunk's loads are issued before the current chunk's MFMAs.  k past the end loads 0 (the last,
// partial chunk only).  VEC: rows 16-byte aligned.  Used by k_linear_act16 (hg_linear.hip) and the
// rollout's fused policy tail (hg_rollout.hip), which therefore produce the same bits.
typedef float hg_f32x4 __attribute__((ext_vector_type(4)));
typedef float hg_f32x4u __attribute__((ext_vector_type(4), aligned(4)));
template <bool VEC, bool TAIL>
__device__ __forceinline__ void hg_ld8k(const float* __restrict__ p, int k0, int K, float v[8]) {
#pragma unroll
  for (int q = 0; q < 2; q++) {
    if (!TAIL) {
      if (VEC) {
        const float4 t = *reinterpret_cast<const float4*>(p + 4 * q);
        v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
      } else {
        const hg_f32x4u t = *reinterpret_cast<const hg_f32x4u*>(p + 4 * q);
        v[4 * q] = t[0]; v[4 * q + 1] = t[1]; v[4 * q + 2] = t[2]; v[4 * q + 3] = t[3];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; j++) v[4 * q + j] = (k0 + 4 * q + j < K) ? p[4 * q + j] : 0.f;
    }
  }
}
template <bool VEC>
__device__ __forceinline__ void hg_lin16_acc(const float* __restrict__ xr, const float* __restrict__ wr, int K, int g,
                                             hg_f32x4& acc0, hg_f32x4& acc1) {
  acc0 = (hg_f32x4)0.f;
  acc1 = (hg_f32x4)0.f;
  const int kfull = K & ~31;
  float a[2][8], w[2][8];
  if (kfull > 0) {
    hg_ld8k<VEC, false>(xr, 0, K, a[0]);
    hg_ld8k<VEC, false>(wr, 0, K, w[0]);
  }
  for (int kb = 0; kb < kfull; kb += 64) {
#pragma unroll
    for (int j = 0; j < 2; j++) {
      const int kn = kb + 32 * (j + 1);
      if (kn < kfull) {
        hg_ld8k<VEC, false>(xr + kn, kn, K, a[j ^ 1]);
        hg_ld8k<VEC, false>(wr + kn, kn, K, w[j ^ 1]);
      }
      if (kb + 32 * j < kfull) {
#pragma unroll
        for (int s2 = 0; s2 < 8; s2 += 2) {
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j][s2], w[j][s2], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j][s2 + 1], w[j][s2 + 1], acc1, 0, 0, 0);
        }
      }
    }
  }
  if (kfull < K) {
    hg_ld8k<VEC, true>(xr + kfull, kfull, K - 8 * g, a[0]);
    hg_ld8k<VEC, true>(wr + kfull, kfull, K - 8 * g, w[0]);
#pragma unroll
    for (int s2 = 0; s2 < 8; s2 += 2) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0][s2], w[0][s2], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0][s2 + 1], w[0][s2 + 1], acc1, 0, 0, 0);
    }
  }
}

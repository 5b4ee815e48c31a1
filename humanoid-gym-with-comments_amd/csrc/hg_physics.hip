// hg_physics.hip — K_step: lane-parallel articulated dynamics for CDNA4 (gfx950).
//
// Same algorithm and results as oracle/physics_ref.c, mapped onto the hardware:
//   * 32 lanes per env, 2 envs per 64-lane wave, block = 1 wave; 4096 envs -> 2048 waves
//     (8 per CU).  Every per-env working array lives in LDS (~11 KB/env), nothing spills.
//   * Phases run lane-parallel: 12 joint rotations; the two 6-link leg chains (FK, RNEA forward
//     and backward) on 2 lanes; 13 bodies' inertia/force terms; 12 mass-matrix columns;
//     row-parallel Cholesky of M (18 lanes); explicit M^-1 by 18 parallel triangular solves;
//     one constraint row per lane (<= 32 rows: sole/base contact normals+tangents, joint
//     limits) with its Jacobian row held in the lane's registers; the Delassus matrix
//     W = J M^-1 J^T one row per lane.
//   * Projected Gauss-Seidel entirely in registers: lane r keeps the row velocity v_r = J_r nu
//     and its Delassus row W[r][0..31]; every lane of an env keeps a copy of the 32 impulses;
//     a row update reads v_r with v_readlane (no cross-lane reductions) and applies
//     W[:][r] dlambda as one FMA per lane; the row loop is unrolled so all indices are static.  Gauss-Seidel order (normal, then the tangent pair, row by row) is
//     the oracle's, so the PGS iterates are the same sequence as physics_ref.c.
// Replaces humanoid_env.py:620-649 (+ refreshes :776-778), like v1.
#include "hg_common.h"


namespace {

constexpr int RMAX = 32;

struct RowC {  // per-row constants of the PGS, one 16-byte broadcast read
  float tgt, invD, invD2;  // target velocity, 1/W_rr, 1/W_(r+1)(r+1) (tangent pair partner)
  int kind;                // 0 normal, 1 tangent-1 (pair head), 2 tangent-2, 3 joint limit
};

struct __align__(16) EnvSh {
  float root[16];
  float q[12], qd[12], act[12], tau[12];
  float pd_kp[12], pd_kd[12], pd_lim[12], pd_tgt[12];  // PD constants / position target per joint
  float nu[20];
  float h[20];
  float lamst[64];
  float R[13][9];
  float axp[13][3];  // joint axis in the parent-body frame (jrot * axis)
  float o[13][3], a[13][3], w[13][3], v[13][3];
  float cm[13], cs[13][3], cJ[13][6];
  union {
    struct { float al[13][3], ac[13][3], f[13][3], n[13][3]; } kin;  // A2..A5 scratch
    struct { float M[18][20]; float Minv[18][20]; float invd[20]; } fac;                 // A6..A12
    struct { float rigid[13 * 13]; float cf[13 * 3]; } out;                              // epilogue staging
  } u;
  float Y[RMAX][18];
  RowC rc[RMAX];
  float rLam[RMAX];
  float rx[RMAX][3], rd[RMAX][3];   // row geometry: point (base-centred) and direction
  int rPt[RMAX], rBody[RMAX];
  float cf[13][3];
  float base_f[6], base_cm, base_cs[3], base_cJ[6];
  float mass0, fric;
  int nrows, bad;
};

__device__ __forceinline__ f3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }
__device__ __forceinline__ void st3(float* p, f3 v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; }
__device__ __forceinline__ f3 mv3(const float* R, f3 v) {
  return mk(R[0] * v.x + R[1] * v.y + R[2] * v.z, R[3] * v.x + R[4] * v.y + R[5] * v.z,
            R[6] * v.x + R[7] * v.y + R[8] * v.z);
}
__device__ __forceinline__ void mm3(const float* A, const float* B, float* C) {
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) C[i * 3 + j] = A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
}
__device__ __forceinline__ f3 symv(const float* S, f3 v) {
  return mk(S[0] * v.x + S[3] * v.y + S[4] * v.z, S[3] * v.x + S[1] * v.y + S[5] * v.z,
            S[4] * v.x + S[5] * v.y + S[2] * v.z);
}

__device__ void ground(const hg_cfg* cfg, float x, float y, float* h, f3* n) {
  if (cfg->terrain_type == 0 || cfg->heightfield == nullptr) { *h = 0; *n = mk(0, 0, 1); return; }
  const float hs = cfg->hf_horizontal_scale, vs = cfg->hf_vertical_scale;
  float fx = (x + cfg->hf_border) / hs, fy = (y + cfg->hf_border) / hs;
  int i = (int)floorf(fx), j = (int)floorf(fy);
  i = max(0, min(i, cfg->hf_rows - 2));
  j = max(0, min(j, cfg->hf_cols - 2));
  float u = fminf(fmaxf(fx - i, 0.f), 1.f), v = fminf(fmaxf(fy - j, 0.f), 1.f);
  const int16_t* hf = cfg->heightfield;
  const int C = cfg->hf_cols;
  float h00 = vs * hf[i * C + j], h10 = vs * hf[(i + 1) * C + j];
  float h01 = vs * hf[i * C + j + 1], h11 = vs * hf[(i + 1) * C + j + 1];
  float dhdx, dhdy;
  // cells split along the (i,j)-(i+1,j+1) diagonal, as convert_heightfield_to_trimesh tessellates
  if (u >= v) { *h = h00 + u * (h10 - h00) + v * (h11 - h10); dhdx = (h10 - h00) / hs; dhdy = (h11 - h10) / hs; }
  else { *h = h00 + v * (h01 - h00) + u * (h11 - h01); dhdx = (h11 - h01) / hs; dhdy = (h01 - h00) / hs; }
  float inv = rsqrtf(dhdx * dhdx + dhdy * dhdy + 1);
  *n = mk(-dhdx * inv, -dhdy * inv, inv);
}


// ---- kinematics as a parallel scan over each leg (lanes 1..6 left leg, 7..12 right leg; every
// lane of the env runs it, lanes 0 and 13..31 on clamped indices, so the DPP exchanges never
// read a disabled lane).  A body's world transform is the base frame composed with the prefix
// product of its leg's local transforms (Lr_j, jp_j), and every velocity/acceleration recursion
// of kin_chain is a prefix sum of per-body terms:
//   w_b   = w_0 + sum_j qd_j a_j                 v_b   = v_0 + sum_j w_p(j) x r_j
//   alp_b =       sum_j w_p(j) x qd_j a_j        acc_b = acc_0 + sum_j alp_p(j) x r_j + w_p(j) x (w_p(j) x r_j)
// Hillis-Steele steps 1, 2, 4 with DPP row_shr (the leg lies inside one 16-lane DPP row), so the
// 6-link chains take 3 dependent steps per quantity instead of 6, with no LDS round trips.
template <int N>
__device__ __forceinline__ float shr(float x) {  // lane i <- lane i - N within the 16-lane row
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x110 | N, 0xF, 0xF, true));
}
// the DPP reads must run with every lane of the row active (a disabled source lane reads as 0):
// each step computes unconditionally and keeps or drops the result with a select, never a branch
// the compiler could sink the DPP into
__device__ __forceinline__ float keep_dpp(float x) {
  asm volatile("" : "+v"(x));
  return x;
}
template <int N>
__device__ __forceinline__ void scan_step(f3& v, int k) {
  const f3 u = mk(keep_dpp(shr<N>(v.x)), keep_dpp(shr<N>(v.y)), keep_dpp(shr<N>(v.z)));
  const bool take = k >= N;
  v = mk(take ? u.x + v.x : v.x, take ? u.y + v.y : v.y, take ? u.z + v.z : v.z);
}
__device__ __forceinline__ void scan3(f3& v, int k) {
  scan_step<1>(v, k);
  scan_step<2>(v, k);
  scan_step<4>(v, k);
}
template <int N>
__device__ __forceinline__ void tf_step(float* P, f3& t, int k) {
  float Q[9];
#pragma unroll
  for (int i = 0; i < 9; i++) Q[i] = keep_dpp(shr<N>(P[i]));
  const f3 u = mk(keep_dpp(shr<N>(t.x)), keep_dpp(shr<N>(t.y)), keep_dpp(shr<N>(t.z)));
  // (Q, u) o (P, t) = (Q P, u + Q t), kept where the partner is in the same leg
  float QP[9];
  mm3(Q, P, QP);
  const f3 tn = u + mv3(Q, t);
  const bool take = k >= N;
#pragma unroll
  for (int i = 0; i < 9; i++) P[i] = take ? QP[i] : P[i];
  t = mk(take ? tn.x : t.x, take ? tn.y : t.y, take ? tn.z : t.z);
}
__device__ __forceinline__ f3 shr1_or(f3 v, int k, f3 base) {  // parent's value (base for link 0)
  const f3 u = mk(keep_dpp(shr<1>(v.x)), keep_dpp(shr<1>(v.y)), keep_dpp(shr<1>(v.z)));
  return k == 0 ? base : u;
}

struct KinLane {  // one lane's body after kin_scan (lane 0: the base; lanes 13..31: don't-care)
  float R[9];
  f3 o, w, al, ac;
};

__device__ KinLane kin_scan(EnvSh& E, const hg_model* M, int l, float gz, bool bias) {
  const bool body = l >= 1 && l <= 12;
  const int b = body ? l : 1;
  const int k = (b - 1) % 6;  // link index within the leg
  // base frame (every lane, from the root quaternion)
  float R0[9];
  {
    const float x = E.root[3], y = E.root[4], z = E.root[5], w = E.root[6];
    R0[0] = 1 - 2 * (y * y + z * z); R0[1] = 2 * (x * y - z * w);     R0[2] = 2 * (x * z + y * w);
    R0[3] = 2 * (x * y + z * w);     R0[4] = 1 - 2 * (x * x + z * z); R0[5] = 2 * (y * z - x * w);
    R0[6] = 2 * (x * z - y * w);     R0[7] = 2 * (y * z + x * w);     R0[8] = 1 - 2 * (x * x + y * y);
  }
  const f3 v0 = mk(E.nu[0], E.nu[1], E.nu[2]), w0 = mk(E.nu[3], E.nu[4], E.nu[5]);
  // local transform of body b: Lr = jrot * rot(axis, q), origin jp (parent frame)
  const f3 ax = ld3(M->axis[b]);
  float P[9];
  {
    float Rq[9], s, c;
    sincosf(E.q[b - 1], &s, &c);
    const float vv = 1 - c;
    Rq[0] = c + ax.x * ax.x * vv;        Rq[1] = ax.x * ax.y * vv - ax.z * s; Rq[2] = ax.x * ax.z * vv + ax.y * s;
    Rq[3] = ax.y * ax.x * vv + ax.z * s; Rq[4] = c + ax.y * ax.y * vv;        Rq[5] = ax.y * ax.z * vv - ax.x * s;
    Rq[6] = ax.z * ax.x * vv - ax.y * s; Rq[7] = ax.z * ax.y * vv + ax.x * s; Rq[8] = c + ax.z * ax.z * vv;
    mm3(M->joint_rot[b], Rq, P);
  }
  f3 t = ld3(M->joint_pos[b]);
  tf_step<1>(P, t, k);
  tf_step<2>(P, t, k);
  tf_step<4>(P, t, k);
  float Rb[9];
  mm3(R0, P, Rb);
  const f3 ob = mv3(R0, t);
  const f3 ab = mv3(Rb, ax);  // R_b axis = R_parent jrot axis (the joint rotation fixes its axis)
  const float qd = E.nu[5 + b];
  const f3 qa = qd * ab;
  f3 wb = qa;
  scan3(wb, k);
  wb = w0 + wb;
  const f3 op = shr1_or(ob, k, mk(0, 0, 0));
  const f3 wp = shr1_or(wb, k, w0);
  const f3 r = ob - op;
  f3 vb = cross(wp, r);
  scan3(vb, k);
  vb = v0 + vb;
  f3 alb = mk(0, 0, 0), acb = mk(0, 0, 0);
  if (bias) {
    alb = cross(wp, qa);
    scan3(alb, k);
    const f3 alp = shr1_or(alb, k, mk(0, 0, 0));
    acb = cross(alp, r) + cross(wp, cross(wp, r));
    scan3(acb, k);
    acb = mk(0, 0, -gz) + acb;
  }
  KinLane K;
  if (body) {
#pragma unroll
    for (int i = 0; i < 9; i++) E.R[b][i] = Rb[i];
    st3(E.o[b], ob); st3(E.a[b], ab); st3(E.w[b], wb); st3(E.v[b], vb);
    if (bias) { st3(E.u.kin.al[b], alb); st3(E.u.kin.ac[b], acb); }
  } else if (l == 0) {
#pragma unroll
    for (int i = 0; i < 9; i++) E.R[0][i] = R0[i];
    st3(E.o[0], mk(0, 0, 0)); st3(E.v[0], v0); st3(E.w[0], w0);
    if (bias) { st3(E.u.kin.al[0], mk(0, 0, 0)); st3(E.u.kin.ac[0], mk(0, 0, -gz)); }
  }
  const bool base = l == 0;
#pragma unroll
  for (int i = 0; i < 9; i++) K.R[i] = base ? R0[i] : Rb[i];
  K.o = base ? mk(0, 0, 0) : ob;
  K.w = base ? w0 : wb;
  K.al = base ? mk(0, 0, 0) : alb;
  K.ac = base ? mk(0, 0, -gz) : acb;
  return K;
}

// ---- A4 + A5 in registers after kin_scan: per-body inertia / RNEA forces / composite seeds (lane
// b), then the leg's backward recursions as suffix sums with DPP row_shl (partner lane b + N in the
// same 16-lane row, kept where link k + N stays in the leg):
//   F_k = sum_{j>=k} f_j,  N_k = sum_{j>=k} n_j + sum_{j>=k} o_j x f_j - o_k x F_k
//   (= kin_chain's n_k + N_{k+1} + (o_{k+1} - o_k) x F_{k+1} unrolled), composite mass / first /
//   second moments as plain suffix sums; h_k = a_k . N_k.
template <int N>
__device__ __forceinline__ float shl(float x) {  // lane i <- lane i + N within the 16-lane row
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x100 | N, 0xF, 0xF, true));
}
template <int N>
__device__ __forceinline__ void sfx_step(float* v, int n, int k) {
  const bool take = k + N <= 5;
  for (int i = 0; i < n; i++) {
    const float u = keep_dpp(shl<N>(v[i]));
    v[i] = take ? v[i] + u : v[i];
  }
}

__device__ void rnea_scan(EnvSh& E, const hg_model* M, int l, const KinLane& K, float scale0) {
  const int b = l < 13 ? l : 0;
  const bool leg = l >= 1 && l <= 12;
  const int k = leg ? (l - 1) % 6 : 6;  // lanes outside the legs take no partner
  const f3 o = K.o;
  const f3 cb = o + mv3(K.R, ld3(M->com[b]));
  float Iw[6];
  {
    const float* I = M->inertia[b];
    const float* Rm = K.R;
    float Im[9] = {I[0], I[3], I[4], I[3], I[1], I[5], I[4], I[5], I[2]};
    float T9[9];
    mm3(Rm, Im, T9);
    float W9[9];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
      for (int j = 0; j < 3; j++) W9[i * 3 + j] = T9[i * 3] * Rm[j * 3] + T9[i * 3 + 1] * Rm[j * 3 + 1] + T9[i * 3 + 2] * Rm[j * 3 + 2];
    Iw[0] = W9[0]; Iw[1] = W9[4]; Iw[2] = W9[8]; Iw[3] = W9[1]; Iw[4] = W9[2]; Iw[5] = W9[5];
  }
  float mb = M->mass[b];
  if (b == 0) {
    mb = E.mass0;
#pragma unroll
    for (int i = 0; i < 6; i++) Iw[i] *= scale0;
  }
  const f3 wb = K.w, alb = K.al, acb = K.ac;
  const f3 d = cb - o;
  const f3 acc = acb + cross(alb, d) + cross(wb, cross(wb, d));
  const f3 fb = mb * acc;
  const f3 nb = symv(Iw, alb) + cross(wb, symv(Iw, wb)) + cross(d, fb);
  const float cc = dot(cb, cb);
  const f3 of = cross(o, fb);
  // [F(3), S_n(3), S_of(3), m, m c(3), J(6)]
  float v[19] = {fb.x, fb.y, fb.z, nb.x, nb.y, nb.z, of.x, of.y, of.z, mb, mb * cb.x, mb * cb.y, mb * cb.z,
                 Iw[0] + mb * (cc - cb.x * cb.x), Iw[1] + mb * (cc - cb.y * cb.y), Iw[2] + mb * (cc - cb.z * cb.z),
                 Iw[3] - mb * cb.x * cb.y, Iw[4] - mb * cb.x * cb.z, Iw[5] - mb * cb.y * cb.z};
  sfx_step<1>(v, 19, k);
  sfx_step<2>(v, 19, k);
  sfx_step<4>(v, 19, k);
  const f3 F = mk(v[0], v[1], v[2]);
  const f3 Nk = mk(v[3], v[4], v[5]) + mk(v[6], v[7], v[8]) - cross(o, F);
  if (l < 13) {
    st3(E.u.kin.f[b], F); st3(E.u.kin.n[b], Nk);
    E.cm[b] = v[9];
    st3(E.cs[b], mk(v[10], v[11], v[12]));
#pragma unroll
    for (int i = 0; i < 6; i++) E.cJ[b][i] = v[13 + i];
    if (leg) E.h[5 + b] = dot(ld3(E.a[b]), Nk);
  }
}

__device__ __forceinline__ void mat_to_quat(const float* m, float* q) {
  float tr = m[0] + m[4] + m[8];
  if (tr > 0) {
    float s = sqrtf(tr + 1) * 2;
    q[3] = 0.25f * s; q[0] = (m[7] - m[5]) / s; q[1] = (m[2] - m[6]) / s; q[2] = (m[3] - m[1]) / s;
  } else if (m[0] > m[4] && m[0] > m[8]) {
    float s = sqrtf(1 + m[0] - m[4] - m[8]) * 2;
    q[3] = (m[7] - m[5]) / s; q[0] = 0.25f * s; q[1] = (m[1] + m[3]) / s; q[2] = (m[2] + m[6]) / s;
  } else if (m[4] > m[8]) {
    float s = sqrtf(1 + m[4] - m[0] - m[8]) * 2;
    q[3] = (m[2] - m[6]) / s; q[0] = (m[1] + m[3]) / s; q[1] = 0.25f * s; q[2] = (m[5] + m[7]) / s;
  } else {
    float s = sqrtf(1 + m[8] - m[0] - m[4]) * 2;
    q[3] = (m[3] - m[1]) / s; q[0] = (m[2] + m[6]) / s; q[1] = (m[5] + m[7]) / s; q[2] = 0.25f * s;
  }
  if (q[3] < 0) { q[0] = -q[0]; q[1] = -q[1]; q[2] = -q[2]; q[3] = -q[3]; }
}

__device__ __forceinline__ float readlane_f(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
// value of lane r of this lane's env (lanes 0..31 or 32..63): both reads are scalar, the pick
// is one v_cndmask (no divergent branch around the convergent readlane)
#define RL(x, r) hsel(half, readlane_f((x), (r)), readlane_f((x), 32 + (r)))
typedef float f32x16 __attribute__((ext_vector_type(16)));
// v_permlane32_swap: x' = (x.lo | z.lo), z' = (x.hi | z.hi)
__device__ __forceinline__ void swap32(float x, float z, float& xo, float& zo) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(z), false, false);
  xo = __uint_as_float(r[0]);
  zo = __uint_as_float(r[1]);
}
__device__ __forceinline__ float hsel(int half, float lo, float hi) { return half ? hi : lo; }
// the lane index through an empty volatile asm: lane masks built from it are recomputed where
// they are used (one v_cmp) instead of being hoisted out of the substep loop into SGPR pairs
// that spill to VGPR lanes (two v_readlane per restore)
__device__ __forceinline__ int lane_opaque(int l) {
  asm volatile("" : "+v"(l));
  return l;
}

}  // namespace

// FIXED = asset.fix_base_link, a compile-time constant so the factorised size and every
// floating-base branch resolve at compile time (no per-entry scalar branches in the Cholesky)
template <bool FIXED>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2))) k_step(HgState S, const float* __restrict__ actions_in, uint64_t step_counter) {
  __shared__ EnvSh shm[2];
  const int half = threadIdx.x >> 5;
  int l = threadIdx.x & 31;
  // XCD-aware env mapping: workgroups are dispatched round-robin over the 8 XCDs (block b ->
  // XCD b % 8), each with its own L2.  Giving every XCD a contiguous range of env pairs keeps the
  // 16 envs of one 64-byte SoA line on one L2, so their 4-byte state stores merge there instead of
  // being written back as 8 partial lines from 8 caches.
  const int nb = gridDim.x, xcd = blockIdx.x & 7, kx = blockIdx.x >> 3;
  const int pair = xcd * (nb >> 3) + min(xcd, nb & 7) + kx;
  const int e_raw = pair * 2 + half;
  const bool valid = e_raw < S.n;
  const int e = valid ? e_raw : S.n - 1;
  EnvSh& E = shm[half];
  const hg_cfg* cfg = S.cfg;
  const hg_model* M = S.model;
  const int np = S.np;
  const float dt = cfg->sim_dt;
  const float inv_dt = 1.0f / dt;
  constexpr bool fixed = FIXED;
  const float gz = cfg->gravity_z;

  // ---------------- prologue: actions (humanoid_env.py:624-635) + state load
  if (l < 12) {
    const float delay = u01(rng4(cfg, e, step_counter, 0, RNG_ACT_DELAY).x);
    float z4[4];
    normals4(rng4(cfg, e, step_counter, l >> 2, RNG_ACT_NOISE), z4);
    const float z = z4[l & 3];
    float a = actions_in[(size_t)e * HG_ND + l];
    const float prev = S.actions[l * np + e];
    a = (1.0f - delay) * a + delay * prev;
    a += cfg->dynamic_randomization * z * a;
    a = fminf(fmaxf(a, -cfg->clip_actions), cfg->clip_actions);
    E.act[l] = a;
    if (valid) S.actions[l * np + e] = a;
    E.q[l] = S.dof_pos[l * np + e];
    E.qd[l] = S.dof_vel[l * np + e];
  }
  if (l < 13) E.root[l] = S.root[l * np + e];
  for (int i = l; i < HG_LAMW; i += 32) E.lamst[i] = S.lambda[i * np + e];
  if (l == 0) {
    E.mass0 = S.body_mass[e];
    E.fric = S.friction[e];
    E.bad = 0;
  }
  __syncthreads();
  const float scale0 = E.mass0 / M->mass[0];
  // PD constants of this lane's joint staged in LDS for all substeps (one global load each per
  // launch instead of per substep); the position target is constant over the policy step
  if (l < 12) {
    E.pd_kp[l] = cfg->kp[l];
    E.pd_kd[l] = cfg->kd[l];
    E.pd_lim[l] = cfg->torque_limit[l];
    E.pd_tgt[l] = E.act[l] * cfg->action_scale + cfg->default_dof_pos[l];
  }
  const int decimation = cfg->decimation;

  for (int sub = 0; sub < decimation; sub++) {
    // lane masks are rebuilt per substep (v_cmp) instead of living across the loop in SGPR pairs
    asm volatile("" : "+v"(l));
    // ---- A1: torques (_compute_torques, humanoid_env.py:910-925), generalized velocity
    if (l < 12) {
      float t = E.pd_kp[l] * (E.pd_tgt[l] - E.q[l]) - E.pd_kd[l] * E.qd[l];
      E.tau[l] = fminf(fmaxf(t, -E.pd_lim[l]), E.pd_lim[l]);
      E.nu[6 + l] = E.qd[l];
    }
    if (l < 6) E.nu[l] = fixed ? 0.f : E.root[7 + l];
    __syncthreads();
    // ---- A2/A3: kinematics + RNEA forward
    // one register-resident pass over the legs: kinematics (prefix scans), then the per-body
    // forces and the backward recursions (suffix scans) — no barrier until the base totals
    const KinLane K = kin_scan(E, M, l, gz, true);
    rnea_scan(E, M, l, K, scale0);
    __syncthreads();
    // base totals (lane 0) — read the kinematics scratch before M overwrites it
    if (l == 0) {
      f3 f0 = ld3(E.u.kin.f[0]) + ld3(E.u.kin.f[1]) + ld3(E.u.kin.f[7]);
      f3 n0 = ld3(E.u.kin.n[0]) + ld3(E.u.kin.n[1]) + cross(ld3(E.o[1]), ld3(E.u.kin.f[1])) + ld3(E.u.kin.n[7]) +
              cross(ld3(E.o[7]), ld3(E.u.kin.f[7]));
      E.h[0] = f0.x; E.h[1] = f0.y; E.h[2] = f0.z; E.h[3] = n0.x; E.h[4] = n0.y; E.h[5] = n0.z;
      E.base_cm = E.cm[0] + E.cm[1] + E.cm[7];
      f3 s = ld3(E.cs[0]) + ld3(E.cs[1]) + ld3(E.cs[7]);
      st3(E.base_cs, s);
#pragma unroll
      for (int i = 0; i < 6; i++) E.base_cJ[i] = E.cJ[0][i] + E.cJ[1][i] + E.cJ[7][i];
    }
    __syncthreads();
    for (int i = l; i < 18 * 20; i += 32) (&E.u.fac.M[0][0])[i] = 0.f;
    __syncthreads();
    // ---- A6/A7: base block (lane 0); joint columns of M (lanes 1..12)
    if (l == 0) {
      const float m0 = E.base_cm;
      f3 s = ld3(E.base_cs);
      const float* J0 = E.base_cJ;
      float (*A)[20] = E.u.fac.M;
      A[0][0] = A[1][1] = A[2][2] = m0;
      A[3][1] = -s.z; A[3][2] = s.y;
      A[4][0] = s.z;  A[4][2] = -s.x;
      A[5][0] = -s.y; A[5][1] = s.x;
      A[3][3] = J0[0]; A[4][4] = J0[1]; A[5][5] = J0[2];
      A[4][3] = J0[3]; A[5][3] = J0[4]; A[5][4] = J0[5];
    } else if (l <= 12) {
      const int b = l, col = 5 + b;
      f3 a = ld3(E.a[b]), o = ld3(E.o[b]);
      f3 cs = ld3(E.cs[b]);
      f3 F = cross(a, cs - E.cm[b] * o);
      f3 L = symv(E.cJ[b], a) - cross(cs, cross(a, o));
      float (*A)[20] = E.u.fac.M;
      A[col][0] = F.x; A[col][1] = F.y; A[col][2] = F.z;
      A[col][3] = L.x; A[col][4] = L.y; A[col][5] = L.z;
      const int first = b <= 6 ? 1 : 7;
      for (int kb = b; kb >= first; kb--) A[col][5 + kb] = dot(ld3(E.a[kb]), L - cross(ld3(E.o[kb]), F));
      A[col][col] += M->armature[b];
    }
    __syncthreads();
    // ---- A8: Cholesky in registers, in the legs-first order [left leg, right leg, base]
    // (new index i <-> dof o(i) = i < 12 ? 6 + i : i - 12).  M's arrow structure (each leg
    // couples only to itself and the base) then gives L no left-right-leg block, so those
    // columns are skipped.  Lane i holds row i; column j's entries L[k][j] reach the other rows
    // by v_readlane (no LDS round trips, no barriers).  Fixed base: the base block (i >= 12) is
    // dropped.  Entries right of a lane's diagonal are never read.
    constexpr int nf = fixed ? 12 : 18;  // factorised size
    {
      float a[18];
      bool nonpd = false;
      const int ol = l < 12 ? 6 + l : l - 12;  // this lane's dof
#pragma unroll
      for (int k = 0; k < 18; k++) {
        const int ok = k < 12 ? 6 + k : k - 12;
        // M holds the lower triangle in dof order (upper entries are zero)
        a[k] = (l < 18) ? (ol >= ok ? E.u.fac.M[l < 18 ? ol : 0][ok] : E.u.fac.M[ok][l < 18 ? ol : 0]) : 0.f;
      }
      asm volatile("" ::: "memory");
      // column broadcast through LDS: every lane writes its (unscaled) column-j entry, then reads
      // the pivot and the trailing entries back as half-wave broadcasts; the rank-1 update is then
      // ONE FMA per trailing entry for both envs of the wave.  Same-wave LDS accesses complete in
      // order, so no barrier.  Y (written only in A12) holds the scratch column.
      float* colbuf = &E.Y[0][0];
#pragma unroll
      for (int j = 0; j < nf; j++) {
        if (l < 18) colbuf[l] = a[j];
        const float d = colbuf[j];
        nonpd |= !(d > 0.f);
        const float inv = __builtin_amdgcn_rsqf(fmaxf(d, 1e-20f));  // 1 ulp, see the readlane form
        const float t = a[j] * (inv * inv);  // L[l][j] / L[j][j]
        a[j] = (lane_opaque(l) >= j) ? a[j] * inv : a[j];
#pragma unroll
        for (int k = j + 1; k < nf; k++) {
          if (j < 6 && k >= 6 && k < 12) continue;  // structural zero: left-leg pivot, right-leg row
          a[k] -= t * colbuf[k];  // L[l][j] L[k][j] = (a_lj / d) a_kj
        }
      }
      if (l < 18) {
#pragma unroll
        for (int k = 0; k < 18; k++) E.u.fac.M[l][k] = a[k];
        // 1 / L_ll from the lane's own row (same-lane LDS write then read: no barrier needed)
        E.u.fac.invd[l] = __builtin_amdgcn_rcpf(E.u.fac.M[l][l < 18 ? l : 0]);
      }
      if (l == 0 && nonpd) E.bad = 1;
    }
    __syncthreads();
    // ---- A9: explicit M^-1: lane i solves L L^T x = e_i in the legs-first order (skipping the
    // structural zeros) and stores column i back in dof order
    if (l < 18) {
      float y[18];
#pragma unroll
      for (int k = 0; k < 18; k++) y[k] = 0.f;
      if (l < nf) {
        const float (*A)[20] = E.u.fac.M;
#pragma unroll
        for (int k = 0; k < 18; k++) {
          if (k >= nf) continue;
          float s = (k == l) ? 1.f : 0.f;
#pragma unroll
          for (int m = 0; m < k; m++) {
            if (k >= 6 && k < 12 && m < 6) continue;
            s -= A[k][m] * y[m];
          }
          y[k] = s * E.u.fac.invd[k];
          __builtin_amdgcn_sched_barrier(0);  // keep the row's LDS loads next to their use
        }
#pragma unroll
        for (int k = 17; k >= 0; k--) {
          if (k >= nf) continue;
          const float xk = y[k] * E.u.fac.invd[k];
          y[k] = xk;
#pragma unroll
          for (int m = 0; m < k; m++) {
            if (k >= 6 && k < 12 && m < 6) continue;
            y[m] -= A[k][m] * xk;
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      const int ol = l < 12 ? 6 + l : l - 12;
#pragma unroll
      for (int k = 0; k < 18; k++) {
        const int ok = k < 12 ? 6 + k : k - 12;
        E.u.fac.Minv[ok][ol] = (k < nf && l < nf) ? y[k] : 0.f;
      }
    }
    __syncthreads();
    // ---- A10: unconstrained velocity nu* = nu + dt M^-1 (tau - h)
    float nu_star = 0.f;
    if (l < 18) {
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < 18; k++) acc += E.u.fac.Minv[l][k] * ((k >= 6 ? E.tau[k - 6] : 0.f) - E.h[k]);
      nu_star = E.nu[l] + dt * acc;
    }
    __syncthreads();
    if (l < 18) E.nu[l] = nu_star;
    // ---- A11: contact / limit detection and row allocation (whole contact triples first)
    {
      bool act_c = false, act_l = false;
      f3 cx = mk(0, 0, 0), cn = mk(0, 0, 1);
      float phi = 0.f, gapv = 0.f, sgnv = 1.f;
      if (l < 16 && l < M->num_contacts && !fixed) {
        const int b = M->contact_body[l];
        cx = ld3(E.o[b]) + mv3(E.R[b], ld3(M->contact_pos[l]));
        float hg;
        ground(cfg, cx.x + E.root[0], cx.y + E.root[1], &hg, &cn);
        phi = (cx.z + E.root[2] - hg) * cn.z;
        act_c = phi < cfg->contact_offset;
      } else if (l >= 16 && l < 28) {
        const int j = l - 16;
        const float glo = E.q[j] - M->lower[j + 1], ghi = M->upper[j + 1] - E.q[j];
        if (glo < 0.01f) { act_l = true; gapv = glo; sgnv = 1.f; }
        else if (ghi < 0.01f) { act_l = true; gapv = ghi; sgnv = -1.f; }
      }
      const uint64_t bal_c = __ballot(act_c), bal_l = __ballot(act_l);
      const uint32_t mc = (uint32_t)(bal_c >> (32 * half)) & 0xFFFFu;
      const uint32_t ml = ((uint32_t)(bal_l >> (32 * half)) >> 16) & 0xFFFu;
      const int nc = min(__popc(mc), RMAX / 3);
      const int nrows = min(RMAX, 3 * nc + __popc(ml));
      const float beta = cfg->baumgarte, vmax = cfg->max_depenetration_vel;
      if (l == 0) E.nrows = nrows;
      if (l >= nrows) { E.rc[l].kind = 2; E.rc[l].tgt = 0.f; E.rc[l].invD = 0.f; E.rc[l].invD2 = 0.f; }
      if (l < 16) {
        const int rank = __popc(mc & ((1u << l) - 1u));
        if (act_c && rank < nc) {
          const int start = 3 * rank;
          f3 t1 = mk(1, 0, 0) - cn.x * cn;
          t1 = rsqrtf(dot(t1, t1)) * t1;
          f3 t2 = cross(cn, t1);
          const float tgt = phi >= 0.f ? -phi * inv_dt : fminf(-beta * phi * inv_dt, vmax);
          for (int d = 0; d < 3; d++) {
            const int r = start + d;
            f3 dir = d == 0 ? cn : (d == 1 ? t1 : t2);
            st3(E.rx[r], cx); st3(E.rd[r], dir);
            E.rc[r].kind = d; E.rc[r].tgt = d == 0 ? tgt : 0.f;
            E.rPt[r] = l; E.rBody[r] = M->contact_body[l];
            E.rLam[r] = E.lamst[l * 3 + d];
          }
        } else if (l < HG_NC) {
          E.lamst[l * 3 + 0] = E.lamst[l * 3 + 1] = E.lamst[l * 3 + 2] = 0.f;
        }
      } else if (l < 28) {
        const int j = l - 16;
        const int r = 3 * nc + __popc(ml & ((1u << j) - 1u));
        if (act_l && r < RMAX) {
          E.rc[r].kind = 3; E.rc[r].tgt = gapv >= 0.f ? -gapv * inv_dt : fminf(-beta * gapv * inv_dt, vmax);
          E.rPt[r] = j; E.rBody[r] = -1;
          E.rd[r][0] = sgnv;
          E.rLam[r] = E.lamst[HG_NC * 3 + j];
        } else {
          E.lamst[HG_NC * 3 + j] = 0.f;
        }
      }
    }
    __syncthreads();
    const int nrows = E.nrows;
    // ---- A12: Jacobian row (registers), Y = M^-1 J^T, 1/D, J nu*
    float J[18];
#pragma unroll
    for (int i = 0; i < 18; i++) J[i] = 0.f;
    float vrow = 0.f;
    const bool own = l < nrows;
    if (own) {
      const int kind = E.rc[l].kind;
      if (kind == 3) {
        const int j = E.rPt[l];
#pragma unroll
        for (int jj = 0; jj < 12; jj++) J[6 + jj] = (jj == j) ? E.rd[l][0] : 0.f;
      } else {
        const f3 x = ld3(E.rx[l]), d = ld3(E.rd[l]);
        const int b = E.rBody[l];
        J[0] = d.x; J[1] = d.y; J[2] = d.z;
        const f3 xd = cross(x, d);
        J[3] = xd.x; J[4] = xd.y; J[5] = xd.z;
        const int lo = b >= 7 ? 7 : 1;
#pragma unroll
        for (int k = 1; k <= 12; k++) {
          const bool anc = b != 0 && k >= lo && k <= b && (k <= 6) == (b <= 6);
          J[5 + k] = anc ? dot(d, cross(ld3(E.a[k]), x - ld3(E.o[k]))) : 0.f;
        }
      }
    }
    // ---- Y = M^-1 J^T and W = J Y on the matrix cores (v_mfma_f32_32x32x2_f32), one 32x32
    // product per env.  MFMA operand i/kk = lane%32 / lane/32, so the wave's two envs are
    // interleaved with v_permlane32_swap: swap(X, Z) -> (X.lo|Z.lo, X.hi|Z.hi).
    //   Y_h (dof x row): 9 k-pairs (2p, 2p+1); A = M^-1_h (rows >= 18 zero) read from LDS,
    //   B = J_h^T.  D layout: lane (kk, n), vgpr v holds Y_h[8(v/4) + 4kk + v%4][n].
    //   W_h = J_h Y_h: contraction pairs follow that layout, k = 8(q/4) + q%4 (+4 for kk = 1),
    //   so Y's accumulators are the B operands as they stand.
    f32x16 dy0 = {0}, dy1 = {0}, dw0 = {0}, dw1 = {0};
#pragma unroll
    for (int p = 0; p < 9; p++) {
      const float am0 = (l < 18) ? shm[0].u.fac.Minv[l < 18 ? l : 0][2 * p + half] : 0.f;
      const float am1 = (l < 18) ? shm[1].u.fac.Minv[l < 18 ? l : 0][2 * p + half] : 0.f;
      float b0, b1;
      swap32(J[2 * p], J[2 * p + 1], b0, b1);
      dy0 = __builtin_amdgcn_mfma_f32_32x32x2f32(am0, b0, dy0, 0, 0, 0);
      dy1 = __builtin_amdgcn_mfma_f32_32x32x2f32(am1, b1, dy1, 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 10; q++) {
      const int klo = 8 * (q / 4) + q % 4, khi = klo + 4;
      float a0, a1;
      swap32(J[klo], khi < 18 ? J[khi < 18 ? khi : 0] : 0.f, a0, a1);
      dw0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, dy0[q], dw0, 0, 0, 0);
      dw1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, dy1[q], dw1, 0, 0, 0);
    }
    // Y rows to LDS for the velocity update (A15): this lane holds Y_h[i][l] for its 10 dofs
#pragma unroll
    for (int v = 0; v < 10; v++) {
      const int i = 8 * (v / 4) + 4 * half + v % 4;
      if (i < 18) { shm[0].Y[l][i] = dy0[v]; shm[1].Y[l][i] = dy1[v]; }
    }
    // gather each env's W column l into its own lanes: wA[v] = W[8(v/4) + v%4][l],
    // wB[v] = W[8(v/4) + 4 + v%4][l]  (W symmetric: column l == row l)
    float wA[16], wB[16];
#pragma unroll
    for (int v = 0; v < 16; v++) swap32(dw0[v], dw1[v], wA[v], wB[v]);
    float wrow[RMAX];
#pragma unroll
    for (int m = 0; m < RMAX; m++) wrow[m] = (m % 8 < 4) ? wA[4 * (m / 8) + m % 8] : wB[4 * (m / 8) + m % 8 - 4];
    if (own) {
      float D = 0.f;
#pragma unroll
      for (int m = 0; m < RMAX; m++) D = (l == m) ? wrow[m] : D;
      float v0 = 0.f;
#pragma unroll
      for (int i = 0; i < 18; i++) v0 += J[i] * E.nu[i];
#pragma unroll
      for (int m = 0; m < RMAX; m++)
        if (m < nrows) v0 += wrow[m] * E.rLam[m];
      E.rc[l].invD = __builtin_amdgcn_rcpf(D);
      vrow = v0;
    }
    __syncthreads();
    if (own && E.rc[l].kind == 1) E.rc[l].invD2 = E.rc[l + 1].invD;
    // rows that are a no-op in BOTH envs of the wave (tangent partner rows, unused rows) are
    // skipped by a scalar branch: with contacts allocated first as triples they line up
    const uint64_t live_b = __ballot(own && E.rc[l].kind != 2);
    const uint32_t live_rows = __builtin_amdgcn_readfirstlane((uint32_t)live_b | (uint32_t)(live_b >> 32));
    __syncthreads();
    // ---- A14: projected Gauss-Seidel, rows in order (normal, then its tangent pair).  The row
    // velocity v_r lives in lane r and is read with v_readlane; the impulses are replicated: every
    // lane of an env holds all 32 of its env's impulses in registers (uniform per half-wave), so
    // reading and updating lambda_r costs no cross-lane traffic.  The update is uniform over the
    // env's 32 lanes and branch-free (both halves of the wave run it whatever their row kinds):
    //   normal / limit row:  lambda <- max(lambda + (tgt - v) / D, 0)
    //   tangent pair (r, r+1): unconstrained 2-D step, projected onto the disc mu * lambda_n,
    //   lambda_n being the normal impulse updated one row earlier
    //   kind 2 / unused rows: no-op (rc.kind = 2 for rows >= nrows)
    {
      float lam[RMAX];
#pragma unroll
      for (int m = 0; m < RMAX; m++) lam[m] = m < nrows ? E.rLam[m] : 0.f;
      const float mu = 0.5f * (E.fric + cfg->ground_friction);
      const int npgs = cfg->pgs_iterations;
      for (int it = 0; it < npgs; it++) {
        float prev_ln = 0.f;
#pragma unroll
        for (int r = 0; r < RMAX; r++) {
          if (live_rows & (1u << r)) {
          const RowC c = E.rc[r];
          const float vr = RL(vrow, r), lr = lam[r];
          const bool isF = c.kind == 1, isN = c.kind == 0 || c.kind == 3;
          const float ln = fmaxf(lr + (c.tgt - vr) * c.invD, 0.f);
          float dl0 = isN ? ln - lr : 0.f;
          if (r + 1 < RMAX) {
            const float vr2 = RL(vrow, r + 1), lr2 = lam[r + 1];
            float l1 = lr - vr * c.invD, l2 = lr2 - vr2 * c.invD2;
            const float lim = mu * prev_ln, nn2 = l1 * l1 + l2 * l2;
            const float sc = nn2 > lim * lim ? lim * __builtin_amdgcn_rsqf(nn2) : 1.f;
            dl0 = isF ? l1 * sc - lr : dl0;
            const float dl1 = isF ? l2 * sc - lr2 : 0.f;
            vrow += wrow[r] * dl0 + wrow[r + 1] * dl1;
            lam[r + 1] += dl1;
          } else {
            vrow += wrow[r] * dl0;
          }
          lam[r] += dl0;
          prev_ln = isN ? ln : prev_ln;
          }
        }
      }
      // ---- A15: nu = nu* + Y^T lambda; contact forces; warm-start store
      if (l == 0) {
#pragma unroll
        for (int m = 0; m < RMAX; m++)
          if (m < nrows) E.rLam[m] = lam[m];
      }
    }
    for (int i = l; i < 13 * 3; i += 32) (&E.cf[0][0])[i] = 0.f;
    __syncthreads();
    const float mylam = own ? E.rLam[l] : 0.f;
    float nu_new = 0.f;
    if (l < 18) {
      float s = E.nu[l];
      for (int r = 0; r < nrows; r++) s += E.Y[r][l] * E.rLam[r];
      nu_new = s;
    }
    if (own) {
      const int kind = E.rc[l].kind;
      if (kind == 3) {
        E.lamst[HG_NC * 3 + E.rPt[l]] = mylam;
      } else {
        E.lamst[E.rPt[l] * 3 + kind] = mylam;
        const int b = E.rBody[l];
        const float s = mylam * inv_dt;
        atomicAdd(&E.cf[b][0], E.rd[l][0] * s);
        atomicAdd(&E.cf[b][1], E.rd[l][1] * s);
        atomicAdd(&E.cf[b][2], E.rd[l][2] * s);
      }
    }
    const bool fin = (l >= 18) || isfinite(nu_new);
    if ((uint32_t)(__ballot(!fin) >> (32 * half)) != 0u && l == 0) E.bad = 1;
    __syncthreads();
    if (l < 18) E.nu[l] = nu_new;
    __syncthreads();
    // ---- A16: integrate (semi-implicit Euler; exact quaternion exponential)
    if (l < 12) {
      E.qd[l] = E.nu[6 + l];
      E.q[l] += dt * E.qd[l];
    }
    if (l == 0) {
      if (!fixed) {
        for (int i = 0; i < 3; i++) { E.root[7 + i] = E.nu[i]; E.root[10 + i] = E.nu[3 + i]; E.root[i] += dt * E.nu[i]; }
        float* Q = E.root + 3;
        const float wx = E.nu[3], wy = E.nu[4], wz = E.nu[5];
        const float wn = sqrtf(wx * wx + wy * wy + wz * wz);
        const float th = wn * dt;
        if (th > 0.f) {
          float sh, ch;
          sincosf(0.5f * th, &sh, &ch);
          const float s = sh / wn;
          const float dq0 = wx * s, dq1 = wy * s, dq2 = wz * s, dq3 = ch;
          const float x = dq3 * Q[0] + dq0 * Q[3] + dq1 * Q[2] - dq2 * Q[1];
          const float y = dq3 * Q[1] - dq0 * Q[2] + dq1 * Q[3] + dq2 * Q[0];
          const float z = dq3 * Q[2] + dq0 * Q[1] - dq1 * Q[0] + dq2 * Q[3];
          const float w = dq3 * Q[3] - dq0 * Q[0] - dq1 * Q[1] - dq2 * Q[2];
          const float inv = rsqrtf(x * x + y * y + z * z + w * w);
          Q[0] = x * inv; Q[1] = y * inv; Q[2] = z * inv; Q[3] = w * inv;
        }
      } else {
        for (int i = 7; i < 13; i++) E.root[i] = 0.f;
      }
    }
    __syncthreads();
    // a non-finite env keeps stepping (NaNs cannot hang the solver: every loop bound is
    // uniform) and is replaced by the recovery state in the epilogue
  }

  // ---------------- epilogue: rigid-body states (refresh_rigid_body_state_tensor) + store
  // observation noise of the post launch that follows this step (env.step passes it
  // step_counter + 1): 12 lanes per env draw one Philox block each here, where lanes are idle,
  // instead of one K_post thread drawing all twelve in sequence.  K_post checks the counter.
  if (cfg->add_noise && l < 12 && valid) {
    float z4[4];
    normals4(rng4(cfg, e, step_counter + 1, l, RNG_OBS_NOISE), z4);
    // per-env rows [e][48]: lanes 0..11 of the wave's two envs store 384 contiguous bytes (whole
    // cache lines; the former [48][np] columns were 8-byte pieces the L2 fetched lines for)
    *reinterpret_cast<float4*>(S.obs_noise + (size_t)e * 48 + 4 * l) = make_float4(z4[0], z4[1], z4[2], z4[3]);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *S.noise_counter = step_counter + 1;
  const bool bad = E.bad != 0;
  if (l < 6) E.nu[l] = E.root[7 + l];
  if (l < 12) E.nu[6 + l] = E.qd[l];
  __syncthreads();
  kin_scan(E, M, l, gz, false);
  __syncthreads();
  // stage the [13][13] rigid states and [13][3] contact forces in LDS, then store each env's
  // rows as one contiguous run (AoS, the reference's tensor layout)
  if (l < 13) {
    const int b = l;
    float qq[4];
    mat_to_quat(E.R[b], qq);
    float* o = E.u.out.rigid + b * 13;
    o[0] = E.o[b][0] + E.root[0];
    o[1] = E.o[b][1] + E.root[1];
    o[2] = E.o[b][2] + E.root[2];
    o[3] = qq[0]; o[4] = qq[1]; o[5] = qq[2]; o[6] = qq[3];
    o[7] = E.v[b][0]; o[8] = E.v[b][1]; o[9] = E.v[b][2];
    o[10] = E.w[b][0]; o[11] = E.w[b][1]; o[12] = E.w[b][2];
  }
  for (int i = l; i < 13 * 3; i += 32) E.u.out.cf[i] = (&E.cf[0][0])[i];
  __syncthreads();
  if (!valid) return;
  if (bad) {
    // non-finite recovery: keep the pre-step state, push the base below ground so the
    // termination check resets the env; count the event
    if (l == 0) {
      S.nonfinite[e] += 1;
      S.root[2 * np + e] = -10.f;
      HG_CF(S, e, 0, 2) = 1e3f;
    }
    if (l < 12) S.dof_vel[l * np + e] = 0.f;
    return;
  }
  float* rs = &HG_RS(S, e, 0, 0);
  for (int i = l; i < 13 * 13; i += 32) rs[i] = E.u.out.rigid[i];
  float* cfo = &HG_CF(S, e, 0, 0);
  for (int i = l; i < 13 * 3; i += 32) cfo[i] = E.u.out.cf[i];
  if (l < 13) S.root[l * np + e] = E.root[l];
  if (l < 12) {
    S.dof_pos[l * np + e] = E.q[l];
    S.dof_vel[l * np + e] = E.qd[l];
    S.torques[l * np + e] = E.tau[l];
  }
  for (int i = l; i < HG_LAMW; i += 32) S.lambda[i * np + e] = E.lamst[i];
}

extern "C" int hg_launch_step(const HgState* S, const float* actions, uint64_t step_counter, int fixed_base,
                               hipStream_t stream) {
  const int grid = (S->n + 1) / 2;
  if (fixed_base)
    hipLaunchKernelGGL(k_step<true>, dim3(grid), dim3(64), 0, stream, *S, actions, step_counter);
  else
    hipLaunchKernelGGL(k_step<false>, dim3(grid), dim3(64), 0, stream, *S, actions, step_counter);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

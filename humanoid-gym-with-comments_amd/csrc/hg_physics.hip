// hg_physics.hip — K_step: fused action preprocessing + decimation x (PD torques + articulated
// dynamics + contact/limit solve + integration) + rigid-body state refresh, for the XBot-L model.
//
// Replaces (reference humanoid/envs/custom/humanoid_env.py):
//   :620-635  action delay blend / multiplicative noise / clip      (prologue)
//   :639-649  for decimation: _compute_torques (:910-925) + gym.simulate + refresh_dof_state
//   :776-778  refresh actor_root / net_contact_force / rigid_body_state
// The dynamics algorithm is the one of oracle/physics_ref.c, in fp32.
//
// v1 mapping: one env per lane; all state SoA ([field][np]) so a wave's loads/stores of one
// field are contiguous.  The 10 substeps run inside the kernel with state in registers/scratch,
// so HBM sees the state once per policy step.
#include "hg_common.h"

namespace {

struct Mdl {  // model in registers-friendly form, read through a uniform pointer
  const hg_model* m;
};

__device__ __forceinline__ void mat3_mul(const float* A, const float* B, float* C) {
  float T[9];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) T[i * 3 + j] = A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
#pragma unroll
  for (int i = 0; i < 9; i++) C[i] = T[i];
}
__device__ __forceinline__ f3 mat3_vec(const float* R, f3 v) {
  return mk(R[0] * v.x + R[1] * v.y + R[2] * v.z, R[3] * v.x + R[4] * v.y + R[5] * v.z,
            R[6] * v.x + R[7] * v.y + R[8] * v.z);
}
__device__ __forceinline__ f3 sym_vec(const float* S, f3 v) {
  return mk(S[0] * v.x + S[3] * v.y + S[4] * v.z, S[3] * v.x + S[1] * v.y + S[5] * v.z,
            S[4] * v.x + S[5] * v.y + S[2] * v.z);
}
__device__ __forceinline__ void rot_sym(const float* R, const float* I, float* o) {
  float Im[9] = {I[0], I[3], I[4], I[3], I[1], I[5], I[4], I[5], I[2]};
  float T[9];
  mat3_mul(R, Im, T);
  float W[9];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) W[i * 3 + j] = T[i * 3] * R[j * 3] + T[i * 3 + 1] * R[j * 3 + 1] + T[i * 3 + 2] * R[j * 3 + 2];
  o[0] = W[0]; o[1] = W[4]; o[2] = W[8]; o[3] = W[1]; o[4] = W[2]; o[5] = W[5];
}
__device__ __forceinline__ void quat_to_mat(float x, float y, float z, float w, float* R) {
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - z * w);     R[2] = 2 * (x * z + y * w);
  R[3] = 2 * (x * y + z * w);     R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - x * w);
  R[6] = 2 * (x * z - y * w);     R[7] = 2 * (y * z + x * w);     R[8] = 1 - 2 * (x * x + y * y);
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
__device__ __forceinline__ void axis_angle(f3 k, float th, float* R) {
  float s, c;
  sincosf(th, &s, &c);
  float v = 1 - c;
  R[0] = c + k.x * k.x * v;       R[1] = k.x * k.y * v - k.z * s; R[2] = k.x * k.z * v + k.y * s;
  R[3] = k.y * k.x * v + k.z * s; R[4] = c + k.y * k.y * v;       R[5] = k.y * k.z * v - k.x * s;
  R[6] = k.z * k.x * v - k.y * s; R[7] = k.z * k.y * v + k.x * s; R[8] = c + k.z * k.z * v;
}

__device__ __forceinline__ f3 ldm3(const float (*a)[3], int b) { return mk(a[b][0], a[b][1], a[b][2]); }

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

struct Kin {
  f3 o[HG_NB], a[HG_NB], c[HG_NB], w[HG_NB], v[HG_NB];
  float Iw[HG_NB][6], m[HG_NB];
  float R[HG_NB][9];
};

__device__ void kinematics(const hg_model* M, const float* quat, const float* q, const float* nu,
                           float mass0, Kin& k) {
  quat_to_mat(quat[0], quat[1], quat[2], quat[3], k.R[0]);
  k.o[0] = mk(0, 0, 0);
  k.a[0] = mk(0, 0, 0);
  k.v[0] = mk(nu[0], nu[1], nu[2]);
  k.w[0] = mk(nu[3], nu[4], nu[5]);
  for (int b = 1; b < HG_NB; b++) {
    const int p = M->parent[b];
    float Rj[9], Rq[9];
    mat3_mul(k.R[p], M->joint_rot[b], Rj);
    f3 ax = ldm3(M->axis, b);
    axis_angle(ax, q[b - 1], Rq);
    mat3_mul(Rj, Rq, k.R[b]);
    k.o[b] = k.o[p] + mat3_vec(k.R[p], ldm3(M->joint_pos, b));
    k.a[b] = mat3_vec(Rj, ax);
    f3 r = k.o[b] - k.o[p];
    k.v[b] = k.v[p] + cross(k.w[p], r);
    k.w[b] = k.w[p] + nu[5 + b] * k.a[b];
  }
  const float scale0 = mass0 / M->mass[0];
  for (int b = 0; b < HG_NB; b++) {
    k.c[b] = k.o[b] + mat3_vec(k.R[b], ldm3(M->com, b));
    rot_sym(k.R[b], M->inertia[b], k.Iw[b]);
    k.m[b] = M->mass[b];
  }
  k.m[0] = mass0;
#pragma unroll
  for (int i = 0; i < 6; i++) k.Iw[0][i] *= scale0;
}

__device__ void bias_forces(const hg_model* M, const Kin& k, const float* nu, float gz, float* h) {
  f3 alpha[HG_NB], acc[HG_NB], f[HG_NB], n[HG_NB];
  alpha[0] = mk(0, 0, 0);
  acc[0] = mk(0, 0, -gz);
  for (int b = 1; b < HG_NB; b++) {
    const int p = M->parent[b];
    f3 r = k.o[b] - k.o[p];
    alpha[b] = alpha[p] + cross(k.w[p], nu[5 + b] * k.a[b]);
    acc[b] = acc[p] + cross(alpha[p], r) + cross(k.w[p], cross(k.w[p], r));
  }
  for (int b = 0; b < HG_NB; b++) {
    f3 d = k.c[b] - k.o[b];
    f3 ac = acc[b] + cross(alpha[b], d) + cross(k.w[b], cross(k.w[b], d));
    f[b] = k.m[b] * ac;
    n[b] = sym_vec(k.Iw[b], alpha[b]) + cross(k.w[b], sym_vec(k.Iw[b], k.w[b])) + cross(d, f[b]);
  }
  for (int b = HG_NB - 1; b >= 1; b--) {
    const int p = M->parent[b];
    h[5 + b] = dot(k.a[b], n[b]);
    f3 r = k.o[b] - k.o[p];
    f[p] = f[p] + f[b];
    n[p] = n[p] + n[b] + cross(r, f[b]);
  }
  h[0] = f[0].x; h[1] = f[0].y; h[2] = f[0].z;
  h[3] = n[0].x; h[4] = n[0].y; h[5] = n[0].z;
}

// lower triangle of M (row-major 18x18) via composite rigid bodies
__device__ void mass_matrix(const hg_model* M, const Kin& k, float* A) {
  float cm[HG_NB], cJ[HG_NB][6];
  f3 cs[HG_NB];
  for (int b = 0; b < HG_NB; b++) {
    f3 c = k.c[b];
    float mb = k.m[b], cc = dot(c, c);
    cm[b] = mb;
    cs[b] = mb * c;
    cJ[b][0] = k.Iw[b][0] + mb * (cc - c.x * c.x);
    cJ[b][1] = k.Iw[b][1] + mb * (cc - c.y * c.y);
    cJ[b][2] = k.Iw[b][2] + mb * (cc - c.z * c.z);
    cJ[b][3] = k.Iw[b][3] - mb * c.x * c.y;
    cJ[b][4] = k.Iw[b][4] - mb * c.x * c.z;
    cJ[b][5] = k.Iw[b][5] - mb * c.y * c.z;
  }
  for (int b = HG_NB - 1; b >= 1; b--) {
    const int p = M->parent[b];
    cm[p] += cm[b];
    cs[p] = cs[p] + cs[b];
#pragma unroll
    for (int i = 0; i < 6; i++) cJ[p][i] += cJ[b][i];
  }
  for (int i = 0; i < HG_NV * HG_NV; i++) A[i] = 0;
  f3 s = cs[0];
  A[0 * 18 + 0] = A[1 * 18 + 1] = A[2 * 18 + 2] = cm[0];
  // [s]x block at rows 3..5, cols 0..2
  A[3 * 18 + 1] = -s.z; A[3 * 18 + 2] = s.y;
  A[4 * 18 + 0] = s.z;  A[4 * 18 + 2] = -s.x;
  A[5 * 18 + 0] = -s.y; A[5 * 18 + 1] = s.x;
  A[3 * 18 + 3] = cJ[0][0]; A[4 * 18 + 4] = cJ[0][1]; A[5 * 18 + 5] = cJ[0][2];
  A[4 * 18 + 3] = cJ[0][3]; A[5 * 18 + 3] = cJ[0][4]; A[5 * 18 + 4] = cJ[0][5];
  for (int b = 1; b < HG_NB; b++) {
    const int col = 5 + b;
    f3 a = k.a[b], o = k.o[b];
    f3 F = cross(a, cs[b] - cm[b] * o);
    f3 L = sym_vec(cJ[b], a) - cross(cs[b], cross(a, o));
    A[col * 18 + 0] = F.x; A[col * 18 + 1] = F.y; A[col * 18 + 2] = F.z;
    A[col * 18 + 3] = L.x; A[col * 18 + 4] = L.y; A[col * 18 + 5] = L.z;
    for (int kb = b; kb >= 1; kb = M->parent[kb]) {
      float val = dot(k.a[kb], L - cross(k.o[kb], F));
      A[col * 18 + 5 + kb] = val;  // row col, column 5+kb <= col : lower triangle
    }
    A[col * 18 + col] += M->armature[b];
  }
}

// in-place Cholesky of the lower triangle of the n x n block starting at (off, off)
__device__ bool cholesky(float* A, int off) {
  for (int j = off; j < HG_NV; j++) {
    float d = A[j * 18 + j];
    for (int kk = off; kk < j; kk++) d -= A[j * 18 + kk] * A[j * 18 + kk];
    if (!(d > 0.f)) return false;
    d = sqrtf(d);
    A[j * 18 + j] = d;
    const float inv = 1.0f / d;
    for (int i = j + 1; i < HG_NV; i++) {
      float s = A[i * 18 + j];
      for (int kk = off; kk < j; kk++) s -= A[i * 18 + kk] * A[j * 18 + kk];
      A[i * 18 + j] = s * inv;
    }
  }
  return true;
}
__device__ void chol_solve(const float* L, int off, float* x) {
  for (int i = 0; i < off; i++) x[i] = 0;
  for (int i = off; i < HG_NV; i++) {
    float s = x[i];
    for (int kk = off; kk < i; kk++) s -= L[i * 18 + kk] * x[kk];
    x[i] = s / L[i * 18 + i];
  }
  for (int i = HG_NV - 1; i >= off; i--) {
    float s = x[i];
    for (int kk = i + 1; kk < HG_NV; kk++) s -= L[kk * 18 + i] * x[kk];
    x[i] = s / L[i * 18 + i];
  }
}

#define MAX_ROWS (HG_NC * 3 + HG_ND)

struct Rows {
  float J[MAX_ROWS][HG_NV];
  float Y[MAX_ROWS][HG_NV];
  float D[MAX_ROWS], target[MAX_ROWS], lam[MAX_ROWS];
  int8_t kind[MAX_ROWS], pt[MAX_ROWS], body[MAX_ROWS];
};

// one substep; returns false on a non-finite state
__device__ bool substep(const hg_cfg* cfg, const hg_model* M, float* root, float* q, float* qd,
                        float* lamst, const float* tau, float mass0, float fric, float* cf,
                        Kin& k, float* A, Rows& rw) {
  const float dt = cfg->sim_dt;
  const bool fixed = cfg->fix_base_link != 0;
  float nu[HG_NV];
#pragma unroll
  for (int i = 0; i < 3; i++) { nu[i] = fixed ? 0.f : root[7 + i]; nu[3 + i] = fixed ? 0.f : root[10 + i]; }
#pragma unroll
  for (int j = 0; j < HG_ND; j++) nu[6 + j] = qd[j];
  kinematics(M, root + 3, q, nu, mass0, k);
  float h[HG_NV];
  bias_forces(M, k, nu, cfg->gravity_z, h);
  mass_matrix(M, k, A);
  const int off = fixed ? 6 : 0;
  if (!cholesky(A, off)) return false;
  float acc[HG_NV];
#pragma unroll
  for (int i = 0; i < HG_NV; i++) acc[i] = (i >= 6 ? tau[i - 6] : 0.f) - h[i];
  chol_solve(A, off, acc);
#pragma unroll
  for (int i = 0; i < HG_NV; i++) nu[i] += dt * acc[i];

  // ---- constraint rows ----
  int nr = 0;
  const float mu = 0.5f * (fric + cfg->ground_friction);
  const float beta = cfg->baumgarte, vmax = cfg->max_depenetration_vel, offc = cfg->contact_offset;
  if (!fixed) {
    int nct = 0;
    for (int c = 0; c < M->num_contacts; c++) {
      const int b = M->contact_body[c];
      f3 x = k.o[b] + mat3_vec(k.R[b], ldm3(M->contact_pos, c));
      float hg;
      f3 nrm;
      ground(cfg, x.x + root[0], x.y + root[1], &hg, &nrm);
      float phi = (x.z + root[2] - hg) * nrm.z;
      if (!(phi < offc) || nct >= 10) {  // at most 10 contacts (30 rows), candidate order
        lamst[c * 3 + 0] = lamst[c * 3 + 1] = lamst[c * 3 + 2] = 0.f;
        continue;
      }
      nct++;
      f3 ref = mk(1, 0, 0);
      f3 t1 = ref - dot(ref, nrm) * nrm;
      t1 = rsqrtf(dot(t1, t1)) * t1;
      f3 t2 = cross(nrm, t1);
      for (int d = 0; d < 3; d++) {
        f3 e = d == 0 ? nrm : (d == 1 ? t1 : t2);
        float* J = rw.J[nr];
        J[0] = e.x; J[1] = e.y; J[2] = e.z;
        f3 xe = cross(x, e);
        J[3] = xe.x; J[4] = xe.y; J[5] = xe.z;
        for (int j = 0; j < HG_ND; j++) J[6 + j] = 0.f;
        for (int kb = b; kb >= 1; kb = M->parent[kb]) J[5 + kb] = dot(e, cross(k.a[kb], x - k.o[kb]));
        rw.target[nr] = d == 0 ? (phi >= 0 ? -phi / dt : fminf(-beta * phi / dt, vmax)) : 0.f;
        rw.lam[nr] = lamst[c * 3 + d];
        rw.kind[nr] = d;
        rw.pt[nr] = c;
        rw.body[nr] = b;
        nr++;
      }
    }
  }
  const float lim_margin = 0.01f;
  for (int j = 0; j < HG_ND; j++) {
    float glo = q[j] - M->lower[j + 1], ghi = M->upper[j + 1] - q[j];
    float sgn, gap;
    if (glo < lim_margin) { sgn = 1.f; gap = glo; }
    else if (ghi < lim_margin) { sgn = -1.f; gap = ghi; }
    else { lamst[HG_NC * 3 + j] = 0.f; continue; }
    if (nr >= 32) { lamst[HG_NC * 3 + j] = 0.f; continue; }  // at most 32 rows
    float* J = rw.J[nr];
    for (int i = 0; i < HG_NV; i++) J[i] = 0.f;
    J[6 + j] = sgn;
    rw.target[nr] = gap >= 0 ? -gap / dt : fminf(-beta * gap / dt, vmax);
    rw.lam[nr] = lamst[HG_NC * 3 + j];
    rw.kind[nr] = 3;
    rw.pt[nr] = j;
    rw.body[nr] = -1;
    nr++;
  }
  for (int r = 0; r < nr; r++) {
    float* Y = rw.Y[r];
    const float* J = rw.J[r];
    for (int i = 0; i < HG_NV; i++) Y[i] = J[i];
    chol_solve(A, off, Y);
    float D = 0.f;
    for (int i = 0; i < HG_NV; i++) D += J[i] * Y[i];
    rw.D[r] = D;
    const float l = rw.lam[r];
    for (int i = 0; i < HG_NV; i++) nu[i] += Y[i] * l;
  }
  for (int it = 0; it < cfg->pgs_iterations; it++) {
    for (int r = 0; r < nr; r++) {
      const int kd = rw.kind[r];
      float v = 0.f;
      for (int i = 0; i < HG_NV; i++) v += rw.J[r][i] * nu[i];
      float ln = fmaxf(rw.lam[r] + (rw.target[r] - v) / rw.D[r], 0.f);
      float dl = ln - rw.lam[r];
      rw.lam[r] = ln;
      for (int i = 0; i < HG_NV; i++) nu[i] += rw.Y[r][i] * dl;
      if (kd == 0) {
        float v1 = 0.f, v2 = 0.f;
        for (int i = 0; i < HG_NV; i++) { v1 += rw.J[r + 1][i] * nu[i]; v2 += rw.J[r + 2][i] * nu[i]; }
        float l1 = rw.lam[r + 1] - v1 / rw.D[r + 1], l2 = rw.lam[r + 2] - v2 / rw.D[r + 2];
        float lim = mu * ln, nn = sqrtf(l1 * l1 + l2 * l2);
        if (nn > lim) { float s = lim / nn; l1 *= s; l2 *= s; }
        float d1 = l1 - rw.lam[r + 1], d2 = l2 - rw.lam[r + 2];
        rw.lam[r + 1] = l1;
        rw.lam[r + 2] = l2;
        for (int i = 0; i < HG_NV; i++) nu[i] += rw.Y[r + 1][i] * d1 + rw.Y[r + 2][i] * d2;
        r += 2;
      }
    }
  }
  for (int i = 0; i < HG_NB * 3; i++) cf[i] = 0.f;
  for (int r = 0; r < nr; r++) {
    if (rw.kind[r] == 3) { lamst[HG_NC * 3 + rw.pt[r]] = rw.lam[r]; continue; }
    lamst[rw.pt[r] * 3 + rw.kind[r]] = rw.lam[r];
    const int b = rw.body[r];
    const float s = rw.lam[r] / dt;
    cf[b * 3 + 0] += rw.J[r][0] * s;
    cf[b * 3 + 1] += rw.J[r][1] * s;
    cf[b * 3 + 2] += rw.J[r][2] * s;
  }
  bool ok = true;
#pragma unroll
  for (int i = 0; i < HG_NV; i++) ok = ok && isfinite(nu[i]);
  if (!ok) return false;
#pragma unroll
  for (int j = 0; j < HG_ND; j++) { qd[j] = nu[6 + j]; q[j] += dt * qd[j]; }
  if (!fixed) {
#pragma unroll
    for (int i = 0; i < 3; i++) { root[7 + i] = nu[i]; root[10 + i] = nu[3 + i]; root[i] += dt * nu[i]; }
    float* Q = root + 3;
    float wx = nu[3], wy = nu[4], wz = nu[5];
    float wn = sqrtf(wx * wx + wy * wy + wz * wz);
    float th = wn * dt;
    if (th > 0.f) {
      float sh, ch;
      sincosf(0.5f * th, &sh, &ch);
      float s = sh / wn;
      float dq0 = wx * s, dq1 = wy * s, dq2 = wz * s, dq3 = ch;
      float x = dq3 * Q[0] + dq0 * Q[3] + dq1 * Q[2] - dq2 * Q[1];
      float y = dq3 * Q[1] - dq0 * Q[2] + dq1 * Q[3] + dq2 * Q[0];
      float z = dq3 * Q[2] + dq0 * Q[1] - dq1 * Q[0] + dq2 * Q[3];
      float w = dq3 * Q[3] - dq0 * Q[0] - dq1 * Q[1] - dq2 * Q[2];
      float inv = rsqrtf(x * x + y * y + z * z + w * w);
      Q[0] = x * inv; Q[1] = y * inv; Q[2] = z * inv; Q[3] = w * inv;
    }
  } else {
#pragma unroll
    for (int i = 7; i < 13; i++) root[i] = 0.f;
  }
  return true;
}

}  // namespace

// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_step(HgState S, const float* __restrict__ actions_in,
                                             uint64_t step_counter) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= S.n) return;
  const hg_cfg* cfg = S.cfg;
  const hg_model* M = S.model;
  const int np = S.np;
  // ---- prologue: action delay blend, multiplicative noise, clip (humanoid_env.py:624-635)
  float act[HG_ND];
  {
    u4 rd = rng4(cfg, e, step_counter, 0, RNG_ACT_DELAY);
    const float delay = u01(rd.x);
    float z[12];
    for (int b = 0; b < 3; b++) normals4(rng4(cfg, e, step_counter, b, RNG_ACT_NOISE), z + 4 * b);
    const float clipv = cfg->clip_actions, dr = cfg->dynamic_randomization;
#pragma unroll
    for (int j = 0; j < HG_ND; j++) {
      float a = actions_in[(size_t)e * HG_ND + j];
      float prev = S.actions[j * np + e];
      a = (1.0f - delay) * a + delay * prev;
      a += dr * z[j] * a;
      a = fminf(fmaxf(a, -clipv), clipv);
      act[j] = a;
      S.actions[j * np + e] = a;
    }
  }
  // ---- load state
  float root[13], q[HG_ND], qd[HG_ND], lam[HG_LAMW];
#pragma unroll
  for (int i = 0; i < 13; i++) root[i] = S.root[i * np + e];
#pragma unroll
  for (int j = 0; j < HG_ND; j++) { q[j] = S.dof_pos[j * np + e]; qd[j] = S.dof_vel[j * np + e]; }
  for (int i = 0; i < HG_LAMW; i++) lam[i] = S.lambda[i * np + e];
  const float mass0 = S.body_mass[e], fric = S.friction[e];
  float tau[HG_ND], cf[HG_NB * 3];
  Kin k;
  float A[HG_NV * HG_NV];
  Rows rw;
  bool ok = true;
  for (int s = 0; s < cfg->decimation; s++) {
    // _compute_torques (humanoid_env.py:910-925)
#pragma unroll
    for (int j = 0; j < HG_ND; j++) {
      float t = cfg->kp[j] * (act[j] * cfg->action_scale + cfg->default_dof_pos[j] - q[j]) - cfg->kd[j] * qd[j];
      tau[j] = fminf(fmaxf(t, -cfg->torque_limit[j]), cfg->torque_limit[j]);
    }
    if (!substep(cfg, M, root, q, qd, lam, tau, mass0, fric, cf, k, A, rw)) { ok = false; break; }
  }
  if (!ok) {
    // non-finite recovery: freeze the env where it was at the start of the step (the caller's
    // termination check resets it), count the event
    S.nonfinite[e] += 1;
#pragma unroll
    for (int i = 0; i < 13; i++) root[i] = S.root[i * np + e];
    root[2] = -10.f;  // far below ground -> base contact -> reset
#pragma unroll
    for (int j = 0; j < HG_ND; j++) { q[j] = S.dof_pos[j * np + e]; qd[j] = 0.f; }
    for (int i = 0; i < HG_LAMW; i++) lam[i] = 0.f;
    for (int i = 0; i < HG_NB * 3; i++) cf[i] = 0.f;
    cf[2] = 1e3f;
  }
  // ---- store state
#pragma unroll
  for (int i = 0; i < 13; i++) S.root[i * np + e] = root[i];
#pragma unroll
  for (int j = 0; j < HG_ND; j++) {
    S.dof_pos[j * np + e] = q[j];
    S.dof_vel[j * np + e] = qd[j];
    S.torques[j * np + e] = tau[j];
  }
  for (int i = 0; i < HG_LAMW; i++) S.lambda[i * np + e] = lam[i];
  for (int i = 0; i < HG_NB * 3; i++) S.contact[(size_t)e * (HG_NB * 3) + i] = cf[i];
  // ---- rigid body states (refresh_rigid_body_state_tensor)
  {
    float nu[HG_NV];
#pragma unroll
    for (int i = 0; i < 6; i++) nu[i] = root[7 + i];
#pragma unroll
    for (int j = 0; j < HG_ND; j++) nu[6 + j] = qd[j];
    kinematics(M, root + 3, q, nu, mass0, k);
    for (int b = 0; b < HG_NB; b++) {
      float qq[4];
      mat_to_quat(k.R[b], qq);
      float* o = &HG_RS(S, e, b, 0);
      o[0] = k.o[b].x + root[0];
      o[1] = k.o[b].y + root[1];
      o[2] = k.o[b].z + root[2];
      o[3] = qq[0]; o[4] = qq[1]; o[5] = qq[2]; o[6] = qq[3];
      o[7] = k.v[b].x; o[8] = k.v[b].y; o[9] = k.v[b].z;
      o[10] = k.w[b].x; o[11] = k.w[b].y; o[12] = k.w[b].z;
    }
  }
}

extern "C" int hg_launch_step(const HgState* S, const float* actions, uint64_t step_counter, hipStream_t stream) {
  const int block = 64;
  const int grid = (S->n + block - 1) / block;
  hipLaunchKernelGGL(k_step, dim3(grid), dim3(block), 0, stream, *S, actions, step_counter);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

/*
 * physics_ref.c — CPU reference simulator for the XBot-L articulation.
 *
 * TEST INFRASTRUCTURE ONLY (the "oracle").  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library.  The product path (humanoid-gym-with-comments_amd/csrc)
 * never links or calls it.
 *
 * What it restates.  The reference's physics is Isaac Gym Preview 4 / PhysX (gym.simulate,
 * humanoid/envs/custom/humanoid_env.py:639-649), a closed third-party binary that is absent from
 * /root/reference and not installable offline: physics parity against the reference is UNPINNED
 * (SURVEY.md §8c).  This file is the build's documented algorithm, written
 * as plainly as possible — dense matrices, serial loops — so the optimised HIP kernel can be
 * checked against it, and pinned by analytic known-answer tests (free fall, pendulum energy,
 * static standing support, momentum conservation) in tests/test_physics_oracle.py.
 *
 * Pieces that DO follow reference code line by line:
 *   - PD torques: humanoid_env.py:910-925 (_compute_torques), applied every substep (:639-645)
 *   - parameters: humanoid_config.py:273-315 (dt, gravity, contact offset, depenetration)
 *
 * Algorithm per substep (dt = sim.dt), generalized velocity nu = [v_base(3) w_base(3) qd(12)],
 * all vectors in a world-aligned frame centred on the base origin:
 *   1. PD torques tau = clip(kp (target - q) - kd qd, +-limit) (humanoid_env.py:910-925); a joint
 *      whose torque is not clipped has its damping term integrated implicitly: dt*kd is added to
 *      its diagonal of M (exact for the linear damping term; keeps armature 0 — the asset's value,
 *      humanoid_config.py:118 — stable with kd = 10 on the light foot at dt = 1 ms),
 *   2. forward kinematics, 3. bias forces h (RNEA, gravity as base acceleration),
 *   4. joint-space inertia M (composite-rigid-body, + armature + implicit damping), 5. Cholesky,
 *   6. nu* = nu + dt M^-1 (tau - h),
 *   7. constraint rows, at most 32 per env, in this order:
 *        contacts (normal + 2 tangents each, at most 9 points, in priority order: foot-sole points,
 *        shin and thigh capsule end spheres vs the ground, then the self-collision pairs
 *        (humanoid_config.py:103: leg-vs-leg capsules, each hand vs its side's thigh and shin, the
 *        base-box bottom face vs the thighs), then the base-box corners; speculative within
 *        contact_offset, Baumgarte-corrected below zero), then joint limits, then the joint
 *        friction rows (URDF dynamics friction, 0.1 N m on the ankles: |lambda| <= f dt; larger
 *        bounds first, then the joint within its leg, left before right); rows past the budget
 *        (and contact points past 9) are dropped and counted;
 *      solved by projected Gauss-Seidel on impulses with Y = M^-1 J^T (warm-started from the
 *      previous substep); friction cone |lambda_t| <= mu lambda_n with mu = mean(env friction,
 *      ground friction) against the ground (PhysX average combine) and the env friction between
 *      the robot's own shapes,
 *   8. semi-implicit Euler: q += dt qd, p += dt v, quaternion by exact exponential map.
 *
 * Precision: `real` is double by default; -DREF_FLOAT builds an fp32 variant (used to size the
 * fp32 parity tolerance: |gpu - ref64| <= k |ref32 - ref64| + eps).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/hgsim.h"

#ifdef REF_FLOAT
typedef float real;
#define R(x) ((float)(x))
#else
typedef double real;
#define R(x) ((double)(x))
#endif

/* REF_APPROX_QUOT (with REF_FLOAT): the fp32 variant "f32q" whose quotients are formed as the HIP
 * kernel forms them (csrc/hg_physics.hip: v_rcp_f32 / v_rsq_f32 products instead of correctly
 * rounded divisions in the Cholesky pivots and solves, the PGS 1 / D, the friction-disc scale, the
 * segment-segment closest points, the pair normals and the tangent basis), each as a product with
 * a correctly rounded reciprocal — the kernel's 1-ulp quotients in kind, not bit for bit.  Used to
 * classify K_step outliers (scripts/classify_kstep_outlier.py): does an fp32 build with the
 * kernel's quotient structure deviate where the plain fp32 build does not? */
#ifdef REF_APPROX_QUOT
#define QDIV(a, b) ((a) * (R(1) / (b)))
#define RSQRT(x) (R(1) / sqrt(x))
#else
#define QDIV(a, b) ((a) / (b))
#define RSQRT(x) (R(1) / sqrt(x))
#endif
#define NB 13
#define ND 12
#define NV 18
#define NC_MAX HG_MAX_CONTACTS
#define NCAP HG_MAX_CAPSULES
#define NP_MAX HG_MAX_PAIRS
#define LAMW HG_LAMW
#define LAM_PAIR (NC_MAX * 3)              /* warm-start slots: ground candidate c -> 3c + d */
#define LAM_LIM (NC_MAX * 3 + NP_MAX * 3)  /* pair p -> LAM_PAIR + 3p + d; limit j -> LAM_LIM + j */
#define LAM_FRIC (LAM_LIM + ND)            /* joint friction j -> LAM_FRIC + j */
#define MAX_ROWS 32
#define MAX_CONTACT_POINTS 9

typedef struct {
  int nb, nc, nfoot, nleg, ncap, npair;
  int parent[NB];
  int cbody[NC_MAX], capbody[NCAP], capkind[NCAP], pair[NP_MAX][2];
  real jpos[NB][3], jrot[NB][9], axis[NB][3];
  real mass[NB], com[NB][3], inertia[NB][6], armature[NB], lower[NB], upper[NB], jfric[NB];
  real cpos[NC_MAX][3], crad[NC_MAX];
  real cap0[NCAP][3], cap1[NCAP][3], caprad[NCAP];
} Model;

/* ---------------------------------------------------------------- small vector algebra */
static inline void v3_cross(const real* a, const real* b, real* o) {
  real x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
  o[0] = x; o[1] = y; o[2] = z;
}
static inline real v3_dot(const real* a, const real* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static inline void mat3_vec(const real* Rm, const real* v, real* o) {
  real x = Rm[0] * v[0] + Rm[1] * v[1] + Rm[2] * v[2];
  real y = Rm[3] * v[0] + Rm[4] * v[1] + Rm[5] * v[2];
  real z = Rm[6] * v[0] + Rm[7] * v[1] + Rm[8] * v[2];
  o[0] = x; o[1] = y; o[2] = z;
}
static inline void mat3_mul(const real* A, const real* B, real* C) {
  real T[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) T[i * 3 + j] = A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
  memcpy(C, T, sizeof(T));
}
/* symmetric 3x3 stored as xx yy zz xy xz yz */
static inline void sym_vec(const real* S, const real* v, real* o) {
  real x = S[0] * v[0] + S[3] * v[1] + S[4] * v[2];
  real y = S[3] * v[0] + S[1] * v[1] + S[5] * v[2];
  real z = S[4] * v[0] + S[5] * v[1] + S[2] * v[2];
  o[0] = x; o[1] = y; o[2] = z;
}
/* world inertia R I R^T for symmetric I */
static void rot_sym(const real* Rm, const real* I, real* o) {
  real Im[9] = {I[0], I[3], I[4], I[3], I[1], I[5], I[4], I[5], I[2]};
  real T[9], W[9];
  mat3_mul(Rm, Im, T);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) W[i * 3 + j] = T[i * 3] * Rm[j * 3] + T[i * 3 + 1] * Rm[j * 3 + 1] + T[i * 3 + 2] * Rm[j * 3 + 2];
  o[0] = W[0]; o[1] = W[4]; o[2] = W[8]; o[3] = W[1]; o[4] = W[2]; o[5] = W[5];
}
static void quat_to_mat(const real* q, real* Rm) { /* xyzw */
  real x = q[0], y = q[1], z = q[2], w = q[3];
  Rm[0] = 1 - 2 * (y * y + z * z); Rm[1] = 2 * (x * y - z * w);     Rm[2] = 2 * (x * z + y * w);
  Rm[3] = 2 * (x * y + z * w);     Rm[4] = 1 - 2 * (x * x + z * z); Rm[5] = 2 * (y * z - x * w);
  Rm[6] = 2 * (x * z - y * w);     Rm[7] = 2 * (y * z + x * w);     Rm[8] = 1 - 2 * (x * x + y * y);
}
static void mat_to_quat(const real* m, real* q) { /* xyzw, Shepperd */
  real tr = m[0] + m[4] + m[8];
  if (tr > 0) {
    real s = sqrt(tr + 1) * 2;
    q[3] = R(0.25) * s; q[0] = (m[7] - m[5]) / s; q[1] = (m[2] - m[6]) / s; q[2] = (m[3] - m[1]) / s;
  } else if (m[0] > m[4] && m[0] > m[8]) {
    real s = sqrt(1 + m[0] - m[4] - m[8]) * 2;
    q[3] = (m[7] - m[5]) / s; q[0] = R(0.25) * s; q[1] = (m[1] + m[3]) / s; q[2] = (m[2] + m[6]) / s;
  } else if (m[4] > m[8]) {
    real s = sqrt(1 + m[4] - m[0] - m[8]) * 2;
    q[3] = (m[2] - m[6]) / s; q[0] = (m[1] + m[3]) / s; q[1] = R(0.25) * s; q[2] = (m[5] + m[7]) / s;
  } else {
    real s = sqrt(1 + m[8] - m[0] - m[4]) * 2;
    q[3] = (m[3] - m[1]) / s; q[0] = (m[2] + m[6]) / s; q[1] = (m[5] + m[7]) / s; q[2] = R(0.25) * s;
  }
  if (q[3] < 0) { q[0] = -q[0]; q[1] = -q[1]; q[2] = -q[2]; q[3] = -q[3]; }
}
/* rotation by angle about unit axis (Rodrigues) */
static void axis_angle(const real* k, real th, real* Rm) {
  real c = cos(th), s = sin(th), v = 1 - c;
  Rm[0] = c + k[0] * k[0] * v;        Rm[1] = k[0] * k[1] * v - k[2] * s; Rm[2] = k[0] * k[2] * v + k[1] * s;
  Rm[3] = k[1] * k[0] * v + k[2] * s; Rm[4] = c + k[1] * k[1] * v;        Rm[5] = k[1] * k[2] * v - k[0] * s;
  Rm[6] = k[2] * k[0] * v - k[1] * s; Rm[7] = k[2] * k[1] * v + k[0] * s; Rm[8] = c + k[2] * k[2] * v;
}

static void load_model(const hg_model* hm, Model* m) {
  m->nb = hm->num_bodies; m->nc = hm->num_contacts; m->nfoot = hm->num_foot_contacts;
  m->nleg = hm->num_leg_contacts; m->ncap = hm->num_capsules; m->npair = hm->num_pairs;
  for (int b = 0; b < NB; b++) {
    m->parent[b] = hm->parent[b];
    for (int i = 0; i < 3; i++) { m->jpos[b][i] = hm->joint_pos[b][i]; m->axis[b][i] = hm->axis[b][i]; m->com[b][i] = hm->com[b][i]; }
    for (int i = 0; i < 9; i++) m->jrot[b][i] = hm->joint_rot[b][i];
    for (int i = 0; i < 6; i++) m->inertia[b][i] = hm->inertia[b][i];
    m->mass[b] = hm->mass[b]; m->armature[b] = hm->armature[b]; m->jfric[b] = hm->joint_friction[b];
    m->lower[b] = hm->lower[b]; m->upper[b] = hm->upper[b];
  }
  for (int c = 0; c < NC_MAX; c++) {
    m->cbody[c] = hm->contact_body[c];
    m->crad[c] = hm->contact_radius[c];
    for (int i = 0; i < 3; i++) m->cpos[c][i] = hm->contact_pos[c][i];
  }
  for (int k = 0; k < NCAP; k++) {
    m->capbody[k] = hm->capsule_body[k];
    m->capkind[k] = hm->capsule_kind[k];
    m->caprad[k] = hm->capsule_radius[k];
    for (int i = 0; i < 3; i++) { m->cap0[k][i] = hm->capsule_p0[k][i]; m->cap1[k][i] = hm->capsule_p1[k][i]; }
  }
  for (int p = 0; p < NP_MAX; p++) { m->pair[p][0] = hm->pair[p][0]; m->pair[p][1] = hm->pair[p][1]; }
}

/* ---------------------------------------------------------------- terrain */
/* plane z = 0, or the triangulated heightfield (row index = x, column = y, origin at -border) */
static void ground(const hg_cfg* cfg, const int16_t* hf, real x, real y, real* h, real* n) {
  if (cfg->terrain_type == 0 || hf == NULL) { *h = 0; n[0] = 0; n[1] = 0; n[2] = 1; return; }
  real hs = cfg->hf_horizontal_scale, vs = cfg->hf_vertical_scale;
  real fx = (x + cfg->hf_border) / hs, fy = (y + cfg->hf_border) / hs;
  int i = (int)floor(fx), j = (int)floor(fy);
  if (i < 0) i = 0; if (j < 0) j = 0;
  if (i > cfg->hf_rows - 2) i = cfg->hf_rows - 2; if (j > cfg->hf_cols - 2) j = cfg->hf_cols - 2;
  real u = fx - i, v = fy - j;
  if (u < 0) u = 0; if (u > 1) u = 1; if (v < 0) v = 0; if (v > 1) v = 1;
  real h00 = vs * hf[i * cfg->hf_cols + j], h10 = vs * hf[(i + 1) * cfg->hf_cols + j];
  real h01 = vs * hf[i * cfg->hf_cols + j + 1], h11 = vs * hf[(i + 1) * cfg->hf_cols + j + 1];
  real dhdx, dhdy;
  // cells split along the (i,j)-(i+1,j+1) diagonal, as convert_heightfield_to_trimesh tessellates
  if (u >= v) { *h = h00 + u * (h10 - h00) + v * (h11 - h10); dhdx = (h10 - h00) / hs; dhdy = (h11 - h10) / hs; }
  else { *h = h00 + v * (h01 - h00) + u * (h11 - h01); dhdx = (h11 - h01) / hs; dhdy = (h01 - h00) / hs; }
  real inv = 1 / sqrt(dhdx * dhdx + dhdy * dhdy + 1);
  n[0] = -dhdx * inv; n[1] = -dhdy * inv; n[2] = inv;
}

/* ---------------------------------------------------------------- one substep */
typedef struct {
  real Rb[NB][9], o[NB][3], c[NB][3], a[NB][3], Iw[NB][6], m[NB];
  real w[NB][3], v[NB][3];
} Kin;

static void kinematics(const Model* m, const real* quat, const real* q, const real* nu, real mass0,
                       Kin* k) {
  quat_to_mat(quat, k->Rb[0]);
  k->o[0][0] = k->o[0][1] = k->o[0][2] = 0;
  for (int i = 0; i < 3; i++) { k->v[0][i] = nu[i]; k->w[0][i] = nu[3 + i]; }
  for (int b = 1; b < NB; b++) {
    int p = m->parent[b];
    real Rj[9], Rq[9], t[3];
    mat3_mul(k->Rb[p], m->jrot[b], Rj);
    axis_angle(m->axis[b], q[b - 1], Rq);
    mat3_mul(Rj, Rq, k->Rb[b]);
    mat3_vec(k->Rb[p], m->jpos[b], t);
    for (int i = 0; i < 3; i++) k->o[b][i] = k->o[p][i] + t[i];
    mat3_vec(Rj, m->axis[b], k->a[b]);
    /* velocities */
    real r[3], wxr[3];
    for (int i = 0; i < 3; i++) r[i] = k->o[b][i] - k->o[p][i];
    v3_cross(k->w[p], r, wxr);
    real qd = nu[5 + b];
    for (int i = 0; i < 3; i++) { k->v[b][i] = k->v[p][i] + wxr[i]; k->w[b][i] = k->w[p][i] + k->a[b][i] * qd; }
  }
  real scale0 = mass0 / m->mass[0];
  for (int b = 0; b < NB; b++) {
    real t[3];
    mat3_vec(k->Rb[b], m->com[b], t);
    for (int i = 0; i < 3; i++) k->c[b][i] = k->o[b][i] + t[i];
    rot_sym(k->Rb[b], m->inertia[b], k->Iw[b]);
    k->m[b] = m->mass[b];
    if (b == 0) { k->m[0] = mass0; for (int i = 0; i < 6; i++) k->Iw[0][i] *= scale0; }
  }
}

/* bias forces h(q, nu) incl. gravity (RNEA with nu_dot = 0, base acceleration = -g) */
static void bias_forces(const Model* m, const Kin* k, const real* nu, real gz, real* h) {
  real alpha[NB][3], acc[NB][3], f[NB][3], n[NB][3];
  for (int i = 0; i < 3; i++) { alpha[0][i] = 0; acc[0][i] = 0; }
  acc[0][2] = -gz;
  for (int b = 1; b < NB; b++) {
    int p = m->parent[b];
    real r[3], t1[3], t2[3], wqd[3];
    real qd = nu[5 + b];
    for (int i = 0; i < 3; i++) { r[i] = k->o[b][i] - k->o[p][i]; wqd[i] = k->a[b][i] * qd; }
    v3_cross(k->w[p], wqd, t1);
    for (int i = 0; i < 3; i++) alpha[b][i] = alpha[p][i] + t1[i];
    v3_cross(alpha[p], r, t1);
    v3_cross(k->w[p], r, t2);
    v3_cross(k->w[p], t2, t2);
    for (int i = 0; i < 3; i++) acc[b][i] = acc[p][i] + t1[i] + t2[i];
  }
  for (int b = 0; b < NB; b++) {
    real d[3], t1[3], t2[3], ac[3], Iw_w[3], Ia[3];
    for (int i = 0; i < 3; i++) d[i] = k->c[b][i] - k->o[b][i];
    v3_cross(alpha[b], d, t1);
    v3_cross(k->w[b], d, t2);
    v3_cross(k->w[b], t2, t2);
    for (int i = 0; i < 3; i++) ac[i] = acc[b][i] + t1[i] + t2[i];
    sym_vec(k->Iw[b], k->w[b], Iw_w);
    sym_vec(k->Iw[b], alpha[b], Ia);
    v3_cross(k->w[b], Iw_w, t1);
    for (int i = 0; i < 3; i++) { f[b][i] = k->m[b] * ac[i]; n[b][i] = Ia[i] + t1[i]; }
    v3_cross(d, f[b], t2);
    for (int i = 0; i < 3; i++) n[b][i] += t2[i];
  }
  for (int b = NB - 1; b >= 1; b--) {
    int p = m->parent[b];
    h[5 + b] = v3_dot(k->a[b], n[b]);
    real r[3], t[3];
    for (int i = 0; i < 3; i++) r[i] = k->o[b][i] - k->o[p][i];
    v3_cross(r, f[b], t);
    for (int i = 0; i < 3; i++) { f[p][i] += f[b][i]; n[p][i] += n[b][i] + t[i]; }
  }
  for (int i = 0; i < 3; i++) { h[i] = f[0][i]; h[3 + i] = n[0][i]; }
}

/* joint-space inertia by composite rigid bodies */
static void mass_matrix(const Model* m, const Kin* k, real M[NV][NV]) {
  real cm[NB], cs[NB][3], cJ[NB][6];
  for (int b = 0; b < NB; b++) {
    const real* c = k->c[b];
    real mb = k->m[b], cc = v3_dot(c, c);
    cm[b] = mb;
    for (int i = 0; i < 3; i++) cs[b][i] = mb * c[i];
    cJ[b][0] = k->Iw[b][0] + mb * (cc - c[0] * c[0]);
    cJ[b][1] = k->Iw[b][1] + mb * (cc - c[1] * c[1]);
    cJ[b][2] = k->Iw[b][2] + mb * (cc - c[2] * c[2]);
    cJ[b][3] = k->Iw[b][3] - mb * c[0] * c[1];
    cJ[b][4] = k->Iw[b][4] - mb * c[0] * c[2];
    cJ[b][5] = k->Iw[b][5] - mb * c[1] * c[2];
  }
  for (int b = NB - 1; b >= 1; b--) {
    int p = m->parent[b];
    cm[p] += cm[b];
    for (int i = 0; i < 3; i++) cs[p][i] += cs[b][i];
    for (int i = 0; i < 6; i++) cJ[p][i] += cJ[b][i];
  }
  memset(M, 0, sizeof(real) * NV * NV);
  /* base block */
  const real* s = cs[0];
  for (int i = 0; i < 3; i++) M[i][i] = cm[0];
  real S[3][3] = {{0, -s[2], s[1]}, {s[2], 0, -s[0]}, {-s[1], s[0], 0}};
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) { M[3 + i][j] = S[i][j]; M[j][3 + i] = S[i][j]; }
  real Jm[3][3] = {{cJ[0][0], cJ[0][3], cJ[0][4]}, {cJ[0][3], cJ[0][1], cJ[0][5]}, {cJ[0][4], cJ[0][5], cJ[0][2]}};
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) M[3 + i][3 + j] = Jm[i][j];
  /* joint columns */
  for (int b = 1; b < NB; b++) {
    int col = 5 + b;
    const real* a = k->a[b];
    const real* o = k->o[b];
    real sm[3], F[3], L[3], axo[3], t[3];
    for (int i = 0; i < 3; i++) sm[i] = cs[b][i] - cm[b] * o[i];
    v3_cross(a, sm, F);
    sym_vec(cJ[b], a, L);
    v3_cross(a, o, axo);
    v3_cross(cs[b], axo, t);
    for (int i = 0; i < 3; i++) L[i] -= t[i];
    for (int i = 0; i < 3; i++) { M[i][col] = M[col][i] = F[i]; M[3 + i][col] = M[col][3 + i] = L[i]; }
    for (int kb = b; kb >= 1; kb = m->parent[kb]) {
      real ok[3], oxF[3], mom[3];
      for (int i = 0; i < 3; i++) ok[i] = k->o[kb][i];
      v3_cross(ok, F, oxF);
      for (int i = 0; i < 3; i++) mom[i] = L[i] - oxF[i];
      real val = v3_dot(k->a[kb], mom);
      M[5 + kb][col] = val;
      M[col][5 + kb] = val;
    }
    M[col][col] += m->armature[b];
  }
}

static int cholesky(real* A, int n, int ld) { /* in-place lower */
  for (int j = 0; j < n; j++) {
    real d = A[j * ld + j];
    for (int k = 0; k < j; k++) d -= A[j * ld + k] * A[j * ld + k];
    if (!(d > 0)) return -1;
    d = sqrt(d);
    A[j * ld + j] = d;
    for (int i = j + 1; i < n; i++) {
      real s = A[i * ld + j];
      for (int k = 0; k < j; k++) s -= A[i * ld + k] * A[j * ld + k];
      A[i * ld + j] = QDIV(s, d);
    }
  }
  return 0;
}
static void chol_solve(const real* L, int n, int ld, real* x) {
  for (int i = 0; i < n; i++) {
    real s = x[i];
    for (int k = 0; k < i; k++) s -= L[i * ld + k] * x[k];
    x[i] = QDIV(s, L[i * ld + i]);
  }
  for (int i = n - 1; i >= 0; i--) {
    real s = x[i];
    for (int k = i + 1; k < n; k++) s -= L[k * ld + i] * x[k];
    x[i] = QDIV(s, L[i * ld + i]);
  }
}

typedef struct {
  int kind;      /* 0 contact normal, 1 tangent-1, 2 tangent-2, 3 joint limit, 4 joint friction */
  int lam_idx;   /* warm-start slot */
  int bpos, bneg;/* contact force +lambda d / dt on bpos, -lambda d / dt on bneg (-1: none) */
  real d[3];     /* contact direction (world) */
  real mu;       /* friction coefficient of the contact (normal rows) */
  real J[NV], Y[NV], D, target, lo, hi, lam;
} Row;

/* J += sign * (Jacobian of the point x (base-centred) on body b) projected on d */
static void add_point_jac(const Model* m, const Kin* k, int b, const real* x, const real* d, real sign, real* J) {
  real xd[3];
  v3_cross(x, d, xd);
  for (int i = 0; i < 3; i++) { J[i] += sign * d[i]; J[3 + i] += sign * xd[i]; }
  for (int kb = b; kb >= 1; kb = m->parent[kb]) {
    real rr[3], axr[3];
    for (int i = 0; i < 3; i++) rr[i] = x[i] - k->o[kb][i];
    v3_cross(k->a[kb], rr, axr);
    J[5 + kb] += sign * v3_dot(d, axr);
  }
}

static real clamp01(real x) { return x < 0 ? 0 : (x > 1 ? 1 : x); }

/* closest points of segments [p1,q1], [p2,q2] (Ericson, Real-Time Collision Detection 5.1.9) */
static void seg_seg(const real* p1, const real* q1, const real* p2, const real* q2, real* c1, real* c2) {
  real d1[3], d2[3], r[3];
  for (int i = 0; i < 3; i++) { d1[i] = q1[i] - p1[i]; d2[i] = q2[i] - p2[i]; r[i] = p1[i] - p2[i]; }
  const real a = v3_dot(d1, d1), e = v3_dot(d2, d2), f = v3_dot(d2, r);
  const real c = v3_dot(d1, r), b = v3_dot(d1, d2);
  const real denom = a * e - b * b;
  real s = denom > R(1e-6) * a * e ? clamp01(QDIV(b * f - c * e, denom)) : 0;
  real t = QDIV(b * s + f, e);
  if (t < 0) { t = 0; s = clamp01(QDIV(-c, a)); }
  else if (t > 1) { t = 1; s = clamp01(QDIV(b - c, a)); }
  for (int i = 0; i < 3; i++) { c1[i] = p1[i] + d1[i] * s; c2[i] = p2[i] + d2[i] * t; }
}

/* tangent basis of a contact normal n (reference axis x, or y when n is close to x) */
static void tangents(const real* n, real* t1, real* t2) {
  real ref[3] = {0, 0, 0};
  ref[fabs(n[0]) < R(0.9) ? 0 : 1] = 1;
  const real dd = v3_dot(ref, n);
  for (int i = 0; i < 3; i++) t1[i] = ref[i] - dd * n[i];
#ifdef REF_APPROX_QUOT
  const real itn = RSQRT(v3_dot(t1, t1));
  for (int i = 0; i < 3; i++) t1[i] *= itn;
#else
  const real tn = sqrt(v3_dot(t1, t1));
  for (int i = 0; i < 3; i++) t1[i] /= tn;
#endif
  v3_cross(n, t1, t2);
}

/* full generalized solve: M x = b restricted to free dofs (fixed base -> 12 joint dofs) */
static void msolve(const real* L, int off, int n, real* x) {
  real t[NV];
  for (int i = 0; i < n; i++) t[i] = x[off + i];
  chol_solve(L, n, NV, t);
  for (int i = 0; i < NV; i++) x[i] = (i >= off) ? t[i - off] : 0;
}

/* contact candidate: ground point/sphere c, or capsule pair p */
typedef struct {
  int active, lam_base, bpos, bneg;
  real phi, n[3], xpos[3], xneg[3], mu;
} Contact;

static void substep(const hg_cfg* cfg, const Model* m, const int16_t* hf, real* root, real* q,
                    real* qd, real* lamst, const real* act, real* tau, real mass0, real fric, real* cf_out,
                    int* nonfinite, int* dropped) {
  const real dt = cfg->sim_dt;
  /* 1. PD torques; implicit damping on the joints whose torque is not clipped */
  real madd[ND];
  for (int j = 0; j < ND; j++) {
    const real t = R(cfg->kp[j]) * (act[j] * R(cfg->action_scale) + R(cfg->default_dof_pos[j]) - q[j]) -
                   R(cfg->kd[j]) * qd[j];
    const real lim = cfg->torque_limit[j];
    const int sat = t < -lim || t > lim;
    tau[j] = t < -lim ? -lim : (t > lim ? lim : t);
    madd[j] = sat ? 0 : dt * R(cfg->kd[j]);
  }
  real nu[NV];
  for (int i = 0; i < 3; i++) { nu[i] = root[7 + i]; nu[3 + i] = root[10 + i]; }
  for (int j = 0; j < ND; j++) nu[6 + j] = qd[j];
  const int fixed = cfg->fix_base_link;
  if (fixed) for (int i = 0; i < 6; i++) nu[i] = 0;
  Kin k;
  kinematics(m, root + 3, q, nu, mass0, &k);
  real h[NV], M[NV][NV];
  bias_forces(m, &k, nu, cfg->gravity_z, h);
  mass_matrix(m, &k, M);
  for (int j = 0; j < ND; j++) M[6 + j][6 + j] += madd[j];
  const int off = fixed ? 6 : 0, n = NV - off;
  real Lm[NV * NV];
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) Lm[i * NV + j] = M[off + i][off + j];
  if (cholesky(Lm, n, NV) != 0) { *nonfinite = 1; return; }
  real acc[NV];
  for (int i = 0; i < NV; i++) acc[i] = (i >= 6 ? tau[i - 6] : 0) - h[i];
  msolve(Lm, off, n, acc);
  for (int i = 0; i < NV; i++) nu[i] += dt * acc[i];

  /* ---- contact detection, in priority order ---- */
  const real beta = cfg->baumgarte, vmax = cfg->max_depenetration_vel, off_c = cfg->contact_offset;
  Contact cand[NC_MAX + NP_MAX];
  int ncand = 0;
  for (int item = 0; item < m->nc + m->npair; item++) {
    /* items: ground candidates [0, nleg), pairs, ground candidates [nleg, nc) */
    Contact* ct = &cand[ncand++];
    memset(ct, 0, sizeof(*ct));
    const int is_pair = item >= m->nleg && item < m->nleg + m->npair;
    if (!is_pair) {
      const int c = item < m->nleg ? item : item - m->npair;
      const int b = m->cbody[c];
      real x[3];
      mat3_vec(k.Rb[b], m->cpos[c], x);
      for (int i = 0; i < 3; i++) x[i] += k.o[b][i];
      real hg, nrm[3];
      ground(cfg, hf, x[0] + root[0], x[1] + root[1], &hg, nrm);
      const real r = m->crad[c];
      ct->phi = (x[2] + root[2] - hg) * nrm[2] - r;
      for (int i = 0; i < 3; i++) { ct->n[i] = nrm[i]; ct->xpos[i] = x[i] - r * nrm[i]; }
      ct->bpos = b; ct->bneg = -1;
      ct->mu = R(0.5) * (fric + cfg->ground_friction);
      ct->lam_base = 3 * c;
      ct->active = !fixed && ct->phi < off_c;
    } else {
      const int p = item - m->nleg;
      const int ca = m->pair[p][0], cb = m->pair[p][1];
      const int ba = m->capbody[ca], bb = m->capbody[cb];
      real a0[3], a1[3], b0[3], b1[3], pa[3], pb[3], dv[3];
      mat3_vec(k.Rb[ba], m->cap0[ca], a0); mat3_vec(k.Rb[ba], m->cap1[ca], a1);
      mat3_vec(k.Rb[bb], m->cap0[cb], b0); mat3_vec(k.Rb[bb], m->cap1[cb], b1);
      for (int i = 0; i < 3; i++) { a0[i] += k.o[ba][i]; a1[i] += k.o[ba][i]; b0[i] += k.o[bb][i]; b1[i] += k.o[bb][i]; }
      const real rb = m->caprad[cb];
      real ra = m->caprad[ca], dist;
      if (m->capkind[ca] == 1) {
        /* base-box bottom face (base frame: z = cap0.z over [cap0.x, cap1.x] x [cap0.y, cap1.y],
           outward normal -z) vs the end sphere of capsule cb that lies closer to it */
        const real* R0 = k.Rb[0];
        real h[2], xy[2][2];
        const real* ends[2] = {b0, b1};
        for (int s = 0; s < 2; s++) {  /* end sphere in the base frame: R0^T x */
          const real* x = ends[s];
          xy[s][0] = R0[0] * x[0] + R0[3] * x[1] + R0[6] * x[2];
          xy[s][1] = R0[1] * x[0] + R0[4] * x[1] + R0[7] * x[2];
          h[s] = m->cap0[ca][2] - (R0[2] * x[0] + R0[5] * x[1] + R0[8] * x[2]);  /* depth below the face */
        }
        const int s = h[1] < h[0] ? 1 : 0;
        const int inside = xy[s][0] >= m->cap0[ca][0] && xy[s][0] <= m->cap1[ca][0] &&
                           xy[s][1] >= m->cap0[ca][1] && xy[s][1] <= m->cap1[ca][1];
        for (int i = 0; i < 3; i++) {
          ct->n[i] = -R0[i * 3 + 2];
          pb[i] = ends[s][i];
          pa[i] = ends[s][i] - h[s] * ct->n[i];
        }
        ra = 0;
        dist = inside ? h[s] : R(1e3);
      } else {
        seg_seg(a0, a1, b0, b1, pa, pb);
        for (int i = 0; i < 3; i++) dv[i] = pb[i] - pa[i];
        dist = sqrt(v3_dot(dv, dv));
        if (dist > R(1e-9)) for (int i = 0; i < 3; i++) ct->n[i] = QDIV(dv[i], dist);
        else { ct->n[0] = 0; ct->n[1] = -1; ct->n[2] = 0; }  /* left -> right is -y in the base frame */
      }
      ct->phi = dist - ra - rb;
      for (int i = 0; i < 3; i++) { ct->xpos[i] = pb[i] - rb * ct->n[i]; ct->xneg[i] = pa[i] + ra * ct->n[i]; }
      ct->bpos = bb; ct->bneg = ba;
      ct->mu = fric;
      ct->lam_base = LAM_PAIR + 3 * p;
      ct->active = ct->phi < off_c;
    }
  }
  /* ---- rows: contacts (<= MAX_CONTACT_POINTS), joint limits, joint friction; the rest dropped ---- */
  static __thread Row rows[MAX_ROWS];
  int nr = 0, npts = 0;
  for (int ci = 0; ci < ncand; ci++) {
    Contact* ct = &cand[ci];
    if (ct->active && npts >= MAX_CONTACT_POINTS) *dropped += 3;
    if (!ct->active || npts >= MAX_CONTACT_POINTS) { for (int d = 0; d < 3; d++) lamst[ct->lam_base + d] = 0; continue; }
    npts++;
    real t1[3], t2[3];
    tangents(ct->n, t1, t2);
    const real* dirs[3] = {ct->n, t1, t2};
    for (int d = 0; d < 3; d++) {
      Row* r = &rows[nr++];
      memset(r, 0, sizeof(*r));
      r->kind = d; r->lam_idx = ct->lam_base + d;
      r->bpos = ct->bpos; r->bneg = ct->bneg;
      for (int i = 0; i < 3; i++) r->d[i] = dirs[d][i];
      add_point_jac(m, &k, ct->bpos, ct->xpos, dirs[d], 1, r->J);
      if (ct->bneg >= 0) add_point_jac(m, &k, ct->bneg, ct->xneg, dirs[d], -1, r->J);
      if (d == 0) r->target = ct->phi >= 0 ? -ct->phi / dt : fmin(-beta * ct->phi / dt, vmax);
      r->mu = ct->mu;
      r->lam = lamst[r->lam_idx];
    }
  }
  const real lim_margin = R(0.01);
  for (int j = 0; j < ND; j++) {
    real glo = q[j] - m->lower[j + 1], ghi = m->upper[j + 1] - q[j];
    real sgn, gap;
    if (glo < lim_margin) { sgn = 1; gap = glo; }
    else if (ghi < lim_margin) { sgn = -1; gap = ghi; }
    else { lamst[LAM_LIM + j] = 0; continue; }
    if (nr >= MAX_ROWS) { lamst[LAM_LIM + j] = 0; *dropped += 1; continue; }
    Row* r = &rows[nr++];
    memset(r, 0, sizeof(*r));
    r->kind = 3; r->lam_idx = LAM_LIM + j; r->bpos = r->bneg = -1;
    r->J[6 + j] = sgn;
    r->target = gap >= 0 ? -gap / dt : fmin(-beta * gap / dt, vmax);
    r->lam = lamst[r->lam_idx];
  }
  /* friction rows: larger bounds first, then the joint within its leg, left before right */
  int forder[ND];
  for (int j = 0; j < ND; j++) forder[j] = j;
  for (int a = 1; a < ND; a++)
    for (int b = a; b > 0; b--) {
      const int x = forder[b - 1], y = forder[b];
      const real fx = m->jfric[x + 1], fy = m->jfric[y + 1];
      const int swap = fy > fx || (fy == fx && (y % 6 < x % 6 || (y % 6 == x % 6 && y < x)));
      if (!swap) break;
      forder[b - 1] = y; forder[b] = x;
    }
  for (int jj = 0; jj < ND; jj++) {
    const int j = forder[jj];
    const real f = m->jfric[j + 1];
    if (!(f > 0)) { lamst[LAM_FRIC + j] = 0; continue; }
    if (nr >= MAX_ROWS) { lamst[LAM_FRIC + j] = 0; *dropped += 1; continue; }
    Row* r = &rows[nr++];
    memset(r, 0, sizeof(*r));
    r->kind = 4; r->lam_idx = LAM_FRIC + j; r->bpos = r->bneg = -1;
    r->J[6 + j] = 1;
    r->lo = -f * dt; r->hi = f * dt;
    r->lam = lamst[r->lam_idx];
  }
  for (int r = 0; r < nr; r++) {
    for (int i = 0; i < NV; i++) rows[r].Y[i] = rows[r].J[i];
    msolve(Lm, off, n, rows[r].Y);
    rows[r].D = 0;
    for (int i = 0; i < NV; i++) rows[r].D += rows[r].J[i] * rows[r].Y[i];
    /* warm start */
    for (int i = 0; i < NV; i++) nu[i] += rows[r].Y[i] * rows[r].lam;
  }
  /* ---- projected Gauss-Seidel: rows in order; a contact's tangent pair right after its normal ---- */
  for (int it = 0; it < cfg->pgs_iterations; it++) {
    for (int r = 0; r < nr; r++) {
      Row* rn = &rows[r];
      real v = 0;
      for (int i = 0; i < NV; i++) v += rn->J[i] * nu[i];
      real ln = rn->lam + QDIV(rn->target - v, rn->D);
      if (rn->kind == 4) ln = ln < rn->lo ? rn->lo : (ln > rn->hi ? rn->hi : ln);
      else if (ln < 0) ln = 0;
      const real dl = ln - rn->lam;
      rn->lam = ln;
      for (int i = 0; i < NV; i++) nu[i] += rn->Y[i] * dl;
      if (rn->kind == 0) {
        Row* r1 = &rows[r + 1];
        Row* r2 = &rows[r + 2];
        real v1 = 0, v2 = 0;
        for (int i = 0; i < NV; i++) { v1 += r1->J[i] * nu[i]; v2 += r2->J[i] * nu[i]; }
        real l1 = r1->lam - QDIV(v1, r1->D), l2 = r2->lam - QDIV(v2, r2->D);
        const real lim = rn->mu * rn->lam, nn = sqrt(l1 * l1 + l2 * l2);
#ifdef REF_APPROX_QUOT
        if (nn > lim) { const real sc = lim * RSQRT(l1 * l1 + l2 * l2); l1 *= sc; l2 *= sc; }
#else
        if (nn > lim) { const real sc = lim / nn; l1 *= sc; l2 *= sc; }
#endif
        const real d1 = l1 - r1->lam, d2 = l2 - r2->lam;
        r1->lam = l1; r2->lam = l2;
        for (int i = 0; i < NV; i++) nu[i] += r1->Y[i] * d1 + r2->Y[i] * d2;
        r += 2;
      }
    }
  }
  /* contact forces (last substep) and warm-start store */
  for (int b = 0; b < NB * 3; b++) cf_out[b] = 0;
  for (int r = 0; r < nr; r++) {
    Row* rr = &rows[r];
    lamst[rr->lam_idx] = rr->lam;
    if (rr->kind > 2) continue;
    for (int i = 0; i < 3; i++) {
      const real f = rr->d[i] * rr->lam / dt;
      cf_out[rr->bpos * 3 + i] += f;
      if (rr->bneg >= 0) cf_out[rr->bneg * 3 + i] -= f;
    }
  }
  /* integrate */
  int bad = 0;
  for (int i = 0; i < NV; i++) if (!isfinite(nu[i])) bad = 1;
  if (bad) { *nonfinite = 1; return; }
  for (int j = 0; j < ND; j++) { qd[j] = nu[6 + j]; q[j] += dt * qd[j]; }
  if (!fixed) {
    for (int i = 0; i < 3; i++) { root[7 + i] = nu[i]; root[10 + i] = nu[3 + i]; root[i] += dt * nu[i]; }
    real* Q = root + 3;
    real w[3] = {nu[3], nu[4], nu[5]};
    real th = sqrt(v3_dot(w, w)) * dt;
    if (th > 0) {
      real s = sin(th / 2) / (th / dt), c = cos(th / 2);
      real dq[4] = {w[0] * s, w[1] * s, w[2] * s, c};
      real x = dq[3] * Q[0] + dq[0] * Q[3] + dq[1] * Q[2] - dq[2] * Q[1];
      real y = dq[3] * Q[1] - dq[0] * Q[2] + dq[1] * Q[3] + dq[2] * Q[0];
      real z = dq[3] * Q[2] + dq[0] * Q[1] - dq[1] * Q[0] + dq[2] * Q[3];
      real ww = dq[3] * Q[3] - dq[0] * Q[0] - dq[1] * Q[1] - dq[2] * Q[2];
      real nq = sqrt(x * x + y * y + z * z + ww * ww);
      Q[0] = x / nq; Q[1] = y / nq; Q[2] = z / nq; Q[3] = ww / nq;
    }
  } else {
    for (int i = 7; i < 13; i++) root[i] = 0;
  }
}

static void rigid_states(const Model* m, const real* root, const real* q, const real* qd, real mass0,
                         real* out) {
  real nu[NV];
  for (int i = 0; i < 3; i++) { nu[i] = root[7 + i]; nu[3 + i] = root[10 + i]; }
  for (int j = 0; j < ND; j++) nu[6 + j] = qd[j];
  Kin k;
  kinematics(m, root + 3, q, nu, mass0, &k);
  for (int b = 0; b < NB; b++) {
    real* o = out + b * 13;
    for (int i = 0; i < 3; i++) o[i] = k.o[b][i] + root[i];
    mat_to_quat(k.Rb[b], o + 3);
    for (int i = 0; i < 3; i++) { o[7 + i] = k.v[b][i]; o[10 + i] = k.w[b][i]; }
  }
}

/* ---------------------------------------------------------------- public (ctypes) API */
/* One policy step (cfg->decimation substeps) for n envs, AoS arrays:
 *   root[n][13], q[n][12], qd[n][12], lam[n][LAMW] (in/out), actions[n][12] (already
 *   delayed/noised/clipped as in humanoid_env.py:620-635), mass0[n] (base mass after DR),
 *   fric[n];  outputs torques[n][12] (last substep), contact[n][13][3], rigid[n][13][13],
 *   nonfinite[n], dropped[n] (+= rows / contact points over the budget, summed over the
 *   substeps).  Returns 0. */
#if defined(REF_FLOAT) && defined(REF_APPROX_QUOT)
#define API(name) name##_f32q
#elif defined(REF_FLOAT)
#define API(name) name##_f32
#else
#define API(name) name##_f64
#endif
int API(ref_step)(const hg_cfg* cfg, const hg_model* hm, const int16_t* hf, int n, real* root,
                  real* q, real* qd, real* lam, const real* actions, const real* mass0,
                  const real* fric, real* torques, real* contact, real* rigid, int32_t* nonfinite,
                  int32_t* dropped) {
  Model m;
  load_model(hm, &m);
#pragma omp parallel for schedule(static)
  for (int e = 0; e < n; e++) {
    real* re = root + (size_t)e * 13;
    real* qe = q + (size_t)e * ND;
    real* qde = qd + (size_t)e * ND;
    const real* ae = actions + (size_t)e * ND;
    real tau[ND];
    int bad = 0, drop = 0;
    for (int s = 0; s < cfg->decimation && !bad; s++)
      substep(cfg, &m, hf, re, qe, qde, lam + (size_t)e * LAMW, ae, tau, mass0[e], fric[e],
              contact + (size_t)e * NB * 3, &bad, &drop);
    dropped[e] += drop;
    for (int j = 0; j < ND; j++) torques[(size_t)e * ND + j] = tau[j];
    nonfinite[e] = bad;
    rigid_states(&m, re, qe, qde, mass0[e], rigid + (size_t)e * NB * 13);
  }
  return 0;
}

/* Expose the dynamics terms for analytic tests: M (18x18 incl. armature) and h. */
int API(ref_dynamics)(const hg_model* hm, const real* root, const real* q, const real* qd,
                      real mass0, real gz, real* M_out, real* h_out) {
  Model m;
  load_model(hm, &m);
  real nu[NV];
  for (int i = 0; i < 3; i++) { nu[i] = root[7 + i]; nu[3 + i] = root[10 + i]; }
  for (int j = 0; j < ND; j++) nu[6 + j] = qd[j];
  Kin k;
  kinematics(&m, root + 3, q, nu, mass0, &k);
  real M[NV][NV];
  mass_matrix(&m, &k, M);
  bias_forces(&m, &k, nu, gz, h_out);
  memcpy(M_out, M, sizeof(M));
  return 0;
}

int API(ref_lamw)(void) { return LAMW; }

/* host threads of the OpenMP env loop (bench.py cpu_baseline: all cores, then one core) */
#ifndef REF_FLOAT
void ref_set_threads(int n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
#else
  (void)n;
#endif
}
#endif

/* Forward kinematics of n states without stepping: rigid[n][13][13] (position, quaternion xyzw,
 * linear and angular velocity of every body, world frame) — the rigid_states() that ends every
 * ref_step, exposed so tests can pin the joint conventions against an independent FK
 * (tests/test_fk_mjcf.py, oracle/mjcf_fk.py). */
int API(ref_rigid_states)(const hg_model* hm, int n, const real* root, const real* q, const real* qd,
                          const real* mass0, real* rigid) {
  Model m;
  load_model(hm, &m);
  for (int e = 0; e < n; e++)
    rigid_states(&m, root + (size_t)e * 13, q + (size_t)e * ND, qd + (size_t)e * ND, mass0[e],
                 rigid + (size_t)e * NB * 13);
  return 0;
}

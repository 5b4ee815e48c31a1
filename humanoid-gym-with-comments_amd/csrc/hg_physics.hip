// hg_physics.hip — K_step: lane-parallel articulated dynamics for CDNA4 (gfx950).
//
// Replaces the reference's step() preamble + decimation x (_compute_torques, gym.simulate) + the
// state refreshes (humanoid_env.py:620-649, 776-778).  Same algorithm and results as
// oracle/physics_ref.c (the build's documented physics), mapped onto the hardware:
//   * 32 lanes per env, 2 envs per 64-lane wave, block = 1 wave; 4096 envs -> 2048 waves (8 per
//     CU, 2 per SIMD).  Per-env working arrays live in LDS, the hot per-lane state in registers.
//   * Kinematics + RNEA as DPP prefix / suffix scans over the two 6-link legs (one lane per
//     link); composite-rigid-body mass-matrix columns one per lane.
//   * PD torques with the damping term integrated implicitly on unclipped joints (dt*kd on M's
//     diagonal; armature 0 as the asset).
//   * Cholesky of M in registers (lane i = row i, legs-first order, arrow structure skipped), with
//     g = L^-1 (tau - h) carried along as an extra column; no explicit inverse.
//   * Contacts: one candidate per lane — sole points / capsule end spheres vs plane or
//     heightfield, self-collision pairs (leg-vs-leg capsules, hands vs thigh / shin, base-box
//     bottom face vs thighs; segment closest points) — items past lane 31 in a second round;
//     ranked by ballot/popcount; at most 9 points (27 rows), then joint limits, then the
//     joint-friction rows, largest bound first, left / right alike (<= 32; dropped rows counted
//     per env).
//   * Lane r owns constraint row r: Jacobian row in registers, z_r = L^-1 J_r^T by a per-lane
//     forward solve (L broadcast from LDS), the Delassus matrix W = Z^T Z on the matrix cores
//     (v_mfma_f32_32x32x2f32, 9 per env; the wave's two envs interleaved with v_permlane32_swap).
//   * Projected Gauss-Seidel in registers over 3-row groups (a contact's normal + tangent pair,
//     or up to three single rows): one v_readlane round per group, the in-group couplings from
//     W's 3x3 block, the other rows' velocities updated by one FMA each.  The iterate sequence
//     is the oracle's row-by-row Gauss-Seidel.
//   * nu_new = nu + L^-T (dt g + Z^T lambda): one column-oriented back substitution.
#include "hg_common.h"

namespace {

constexpr int RMAX = 32;          // constraint rows per env (one per lane)
constexpr int NGRP = 11;          // PGS groups of 3 row slots (the 33rd slot is virtual, always empty)
constexpr int MAX_PTS = 9;        // contact points per env (27 rows)
constexpr int LAM_PAIR = HG_MAX_CONTACTS * 3;           // warm-start slots (oracle/physics_ref.c)
constexpr int LAM_LIM = LAM_PAIR + HG_MAX_PAIRS * 3;
constexpr int LAM_FRIC = LAM_LIM + HG_ND;
constexpr float BIG = 3.0e38f;

struct __align__(16) GroupC {  // PGS constants of one 3-slot group (a, b, c): four 16-byte reads
  float invD[3];
  float Wba, Wca, Wcb;     // W[b][a], W[c][a], W[c][b]
  float tgt[3], lo[3], hi[3];
  float mu;                // >= 0: (a, b, c) = a contact's normal and tangent pair (friction
                           // coefficient); +inf: single rows (the disc test never scales them)
};
static_assert(sizeof(GroupC) == 64, "GroupC is four 16-byte LDS reads");

struct ContactC {  // one active contact: points on the two bodies (base-centred), normal + tangents
  float xP[3], xN[3];
  float dir[3][3];
  int bP, bN;              // +lambda d on bP, -lambda d on bN (-1: the ground)
  int lam_base;            // warm-start slots lam_base + 0..2
  int pad;
};

struct __align__(16) EnvSh {
  float root[16];
  float q[12], qd[12], act[12], tau[12];
  float pd_kp[12], pd_kd[12], pd_lim[12], pd_tgt[12], pd_arm[12], madd[12];
  alignas(16) float nu[20];
  alignas(16) float h[20];
  alignas(16) float gv[20];  // g = L^-1 (tau - h), legs-first order
  alignas(16) float invd[20];  // 1 / L_kk
  float lamst[HG_LAMW];
  float R[13][9];
  float o[13][3], a[13][3], w[13][3], v[13][3];
  float cm[13], cs[13][3], cJ[13][6];
  union alignas(16) {
    struct { float al[13][3], ac[13][3], f[13][3], n[13][3]; } kin;  // RNEA scratch
    float Z[RMAX][20];                                                 // z_r rows, legs-first order
    struct { float rigid[13 * 13]; float cf[13 * 3]; } out;            // epilogue staging
  } u;
  alignas(16) float L[18][20];  // M (dof order, lower) then its Cholesky factor (legs-first order)
  // Cholesky column / right-hand-side broadcasts: one slot per lane (every lane writes, no
  // exec-mask branch), rows 0..17 read back as 16-byte groups
  alignas(16) float colbuf[32];
  alignas(16) float colbuf2[32];
  alignas(16) float bbuf[32];
  alignas(16) GroupC grp[NGRP];
  ContactC ct[MAX_PTS];
  float rd[RMAX][3];       // joint rows: sign in rd[r][0]
  int rbP[RMAX], rbN[RMAX];// joint rows: rbP = -1 - dof
  int rlam[RMAX];          // warm-start slot
  alignas(16) float rLam[RMAX];
  float cf[13][3];
  float base_cm, base_cs[3], base_cJ[6];
  float mass0, fric;
  int nrows, npts, bad;
  int drop;                // rows / contact points over the budget this launch (HG_T_ROWS_DROPPED)
};
static_assert(offsetof(EnvSh, L) % 16 == 0 && offsetof(EnvSh, invd) % 16 == 0 && offsetof(EnvSh, gv) % 16 == 0 &&
              offsetof(EnvSh, u) % 16 == 0, "16-byte LDS row accesses (ld_vec / st_vec)");

__device__ __forceinline__ f3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }
__device__ __forceinline__ void st3(float* p, f3 v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; }
// N consecutive floats from / to 16-byte-aligned LDS as 16-byte accesses with immediate offsets
// (N rounded up to a multiple of 4 on loads: the rows read this way are padded to 20 floats)
// out must hold N rounded up to a multiple of 4
__device__ __forceinline__ void ld_vec(const float* p, float* out, int N) {  // N: constant after unrolling
#pragma unroll
  for (int q = 0; q < 5; q++) {
    if (4 * q >= N) break;
    const float4 t = reinterpret_cast<const float4*>(p)[q];
    out[4 * q] = t.x; out[4 * q + 1] = t.y; out[4 * q + 2] = t.z; out[4 * q + 3] = t.w;
  }
}
template <int N>
__device__ __forceinline__ void st_vec(float* p, const float* in) {
#pragma unroll
  for (int q = 0; q < N / 4; q++)
    reinterpret_cast<float4*>(p)[q] = make_float4(in[4 * q], in[4 * q + 1], in[4 * q + 2], in[4 * q + 3]);
  if (N % 4 >= 2) reinterpret_cast<float2*>(p)[2 * (N / 4)] = make_float2(in[N & ~3], in[(N & ~3) + 1]);
  if (N % 2) p[N - 1] = in[N - 1];
}
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

// The launch's physics scalars, passed by value as a kernel argument: the substep loop reads them
// with scalar loads from the kernarg segment (invariant) instead of vector loads of hg_cfg, which
// the compiler cannot keep across the kernel's stores and reloads through the vector cache on the
// chain of every substep (detection, PGS bounds).  Filled from the host hg_cfg by hg_launch_step.
struct StepParams {
  float dt, gz, contact_offset, vmax, beta, ground_friction;
  int decimation, pgs_iterations, heightfield_on;  // heightfield_on: terrain_type != 0 and a heightfield
  int hf_rows, hf_cols;
  float hs, vs, border;
  const int16_t* hf;
};

__device__ void ground(const StepParams& P, float x, float y, float* h, f3* n) {
  if (!P.heightfield_on) { *h = 0; *n = mk(0, 0, 1); return; }
  const float hs = P.hs, vs = P.vs;
  float fx = (x + P.border) / hs, fy = (y + P.border) / hs;
  int i = (int)floorf(fx), j = (int)floorf(fy);
  i = max(0, min(i, P.hf_rows - 2));
  j = max(0, min(j, P.hf_cols - 2));
  float u = fminf(fmaxf(fx - i, 0.f), 1.f), v = fminf(fmaxf(fy - j, 0.f), 1.f);
  const int16_t* hf = P.hf;
  const int C = P.hf_cols;
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
// materialise a value here (an LDS read completes before the selects that use it instead of being
// sunk behind an exec-mask branch)
__device__ __forceinline__ void pin(float& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin(int& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin(f3& v) { pin(v.x); pin(v.y); pin(v.z); }
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

// One lane's model constants for kin_scan (body bk: the lane's joint body, lanes outside 1..12 on
// body 1) and rnea_scan (body br: lanes 0..12, others on the base).  Issued at the head of the
// substep, ahead of A1 and its barrier, so their global round trip overlaps that phase instead of
// sitting on the chain inside kin_scan / rnea_scan; the body indices go through an empty asm so the
// loads stay in the loop (not hoisted out and then re-read next to their uses under the loop's
// register pressure).
struct ModelLane {
  f3 ax, jp, com;
  float jr[9], I[6], m;
};
__device__ __forceinline__ ModelLane load_model_lane(const hg_model* M, int l) {
  int bk = l >= 1 && l <= 12 ? l : 1, br = l < 13 ? l : 0;
  asm volatile("" : "+v"(bk), "+v"(br));
  ModelLane ML;
  ML.ax = ld3(M->axis[bk]);
  ML.jp = ld3(M->joint_pos[bk]);
#pragma unroll
  for (int i = 0; i < 9; i++) ML.jr[i] = M->joint_rot[bk][i];
  ML.com = ld3(M->com[br]);
#pragma unroll
  for (int i = 0; i < 6; i++) ML.I[i] = M->inertia[br][i];
  ML.m = M->mass[br];
  return ML;
}

struct KinLane {  // one lane's body after kin_scan (lane 0: the base; lanes 13..31: don't-care)
  float R[9];
  f3 o, w, al, ac;
};

__device__ KinLane kin_scan(EnvSh& E, const ModelLane& ML, int l, float gz, bool bias) {
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
  const f3 ax = ML.ax;
  float P[9];
  {
    float Rq[9], s, c;
    sincosf(E.q[b - 1], &s, &c);
    const float vv = 1 - c;
    Rq[0] = c + ax.x * ax.x * vv;        Rq[1] = ax.x * ax.y * vv - ax.z * s; Rq[2] = ax.x * ax.z * vv + ax.y * s;
    Rq[3] = ax.y * ax.x * vv + ax.z * s; Rq[4] = c + ax.y * ax.y * vv;        Rq[5] = ax.y * ax.z * vv - ax.x * s;
    Rq[6] = ax.z * ax.x * vv - ax.y * s; Rq[7] = ax.z * ax.y * vv + ax.x * s; Rq[8] = c + ax.z * ax.z * vv;
    mm3(ML.jr, Rq, P);
  }
  f3 t = ML.jp;
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

__device__ void rnea_scan(EnvSh& E, const ModelLane& ML, int l, const KinLane& K, float scale0) {
  const int b = l < 13 ? l : 0;
  const bool leg = l >= 1 && l <= 12;
  const int k = leg ? (l - 1) % 6 : 6;  // lanes outside the legs take no partner
  const f3 o = K.o;
  const f3 cb = o + mv3(K.R, ML.com);
  float Iw[6];
  {
    const float* I = ML.I;
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
  float mb = ML.m;
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

// the value of lane R of this lane's 32-lane env half as ONE ds_swizzle (bit mode: and_mask 0,
// or_mask R): no SGPR round trip, no per-env select
template <int R>
__device__ __forceinline__ float bcast32(float x) {
  static_assert(R >= 0 && R < 32, "lane in the half");
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(x), R << 5));
}
__device__ __forceinline__ float clampf(float x, float lo, float hi) { return __builtin_amdgcn_fmed3f(x, lo, hi); }
// bcast32 for a row index that is a compile-time constant after unrolling
__device__ __forceinline__ float swz(float x, int r) {
  switch (r) {
#define HG_SWZ(R) case R: return bcast32<R>(x);
    HG_SWZ(0) HG_SWZ(1) HG_SWZ(2) HG_SWZ(3) HG_SWZ(4) HG_SWZ(5) HG_SWZ(6) HG_SWZ(7) HG_SWZ(8) HG_SWZ(9)
    HG_SWZ(10) HG_SWZ(11) HG_SWZ(12) HG_SWZ(13) HG_SWZ(14) HG_SWZ(15) HG_SWZ(16) HG_SWZ(17) HG_SWZ(18)
    HG_SWZ(19) HG_SWZ(20) HG_SWZ(21) HG_SWZ(22) HG_SWZ(23) HG_SWZ(24) HG_SWZ(25) HG_SWZ(26) HG_SWZ(27)
    HG_SWZ(28) HG_SWZ(29) HG_SWZ(30) HG_SWZ(31)
#undef HG_SWZ
    default: return 0.f;
  }
}
typedef float f32x16 __attribute__((ext_vector_type(16)));
// v_permlane32_swap: x' = (x.lo | z.lo), z' = (x.hi | z.hi)
__device__ __forceinline__ void swap32(float x, float z, float& xo, float& zo) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(z), false, false);
  xo = __uint_as_float(r[0]);
  zo = __uint_as_float(r[1]);
}
// the lane index through an empty volatile asm: lane masks built from it are recomputed where
// they are used (one v_cmp) instead of being hoisted out of the substep loop into SGPR pairs
// that spill to VGPR lanes (two v_readlane per restore)
__device__ __forceinline__ int lane_opaque(int l) {
  asm volatile("" : "+v"(l));
  return l;
}


// closest points of the segments [p1,q1], [p2,q2] (Ericson 5.1.9; as oracle/physics_ref.c seg_seg).
// The quotients are products with v_rcp_f32 reciprocals (1 ulp) instead of correctly rounded
// divisions (about nine instructions each): a and e are squared segment lengths of the model's
// capsules (> 0), and denom is used only above 1e-6 a e
__device__ __forceinline__ void seg_seg(f3 p1, f3 q1, f3 p2, f3 q2, f3& c1, f3& c2) {
  const f3 d1 = q1 - p1, d2 = q2 - p2, r = p1 - p2;
  const float a = dot(d1, d1), e = dot(d2, d2), f = dot(d2, r);
  const float c = dot(d1, r), b = dot(d1, d2);
  const float denom = a * e - b * b;
  const float ra = __builtin_amdgcn_rcpf(a), re = __builtin_amdgcn_rcpf(e);
  float s = denom > 1e-6f * a * e ? fminf(fmaxf((b * f - c * e) * __builtin_amdgcn_rcpf(denom), 0.f), 1.f) : 0.f;
  float t = (b * s + f) * re;
  if (t < 0.f) { t = 0.f; s = fminf(fmaxf(-c * ra, 0.f), 1.f); }
  else if (t > 1.f) { t = 1.f; s = fminf(fmaxf((b - c) * ra, 0.f), 1.f); }
  c1 = p1 + s * d1;
  c2 = p2 + t * d2;
}

// ---- contact candidates (A9).  One candidate per lane: a ground candidate c (sole point /
// capsule end sphere on body b0 vs plane or heightfield) or a self-collision pair p of capsules
// (a on b0, b on b1; normal from a to b; +lambda d on b1, -lambda d on b0).  Per-lane model
// constants k: ground [0..2] point, [3] radius; pair [0..5] a's segment, [6..11] b's segment,
// [12] a's radius (< 0: a is the base-box bottom face, [0..5] its corner extremes in the base
// frame), [13] b's radius.  As oracle/physics_ref.c substep's detection loop.
struct Cand {
  f3 cn, xP, xN;
  float phi, mu;
  int bP, bN, lam_base;
  bool act;
};

// item -> (pair?, ground index c, pair index p, bodies, constants), in the oracle's item order
__device__ __forceinline__ bool load_item(const hg_model* M, int item, int nleg, int npair, int& c, int& p, int& b0,
                                          int& b1, float* k) {
  const bool pr = item >= nleg && item < nleg + npair;
  c = min(item < nleg ? item : item - npair, HG_MAX_CONTACTS - 1);
  p = min(max(item - nleg, 0), HG_MAX_PAIRS - 1);
  if (!pr) {
    b0 = M->contact_body[c];
    b1 = -1;
    k[0] = M->contact_pos[c][0]; k[1] = M->contact_pos[c][1]; k[2] = M->contact_pos[c][2];
    k[3] = M->contact_radius[c];
#pragma unroll
    for (int i = 4; i < 14; i++) k[i] = 0.f;
  } else {
    const int ca = M->pair[p][0], cb = M->pair[p][1];
    b0 = M->capsule_body[ca];
    b1 = M->capsule_body[cb];
#pragma unroll
    for (int i = 0; i < 3; i++) {
      k[i] = M->capsule_p0[ca][i]; k[3 + i] = M->capsule_p1[ca][i];
      k[6 + i] = M->capsule_p0[cb][i]; k[9 + i] = M->capsule_p1[cb][i];
    }
    k[12] = M->capsule_kind[ca] == 1 ? -1.f : M->capsule_radius[ca];
    k[13] = M->capsule_radius[cb];
  }
  return pr;
}

__device__ __forceinline__ Cand detect(const EnvSh& E, const StepParams& P, bool is_pair, int c, int p, int b0, int b1,
                                       const float* k, bool fixed) {
  Cand C;
  C.cn = mk(0, 0, 1); C.xP = mk(0, 0, 0); C.xN = mk(0, 0, 0);
  C.phi = 0.f; C.mu = 0.f; C.bP = -1; C.bN = -1; C.lam_base = 0; C.act = false;
  if (!is_pair) {
    const f3 x = ld3(E.o[b0]) + mv3(E.R[b0], mk(k[0], k[1], k[2]));
    float hg;
    ground(P, x.x + E.root[0], x.y + E.root[1], &hg, &C.cn);
    const float r = k[3];
    C.phi = (x.z + E.root[2] - hg) * C.cn.z - r;
    C.xP = x - r * C.cn;
    C.bP = b0;
    C.mu = 0.5f * (E.fric + P.ground_friction);
    C.lam_base = 3 * c;
    C.act = !fixed && C.phi < P.contact_offset;
    return C;
  }
  const f3 ob = ld3(E.o[b1]);
  const f3 q0 = ob + mv3(E.R[b1], mk(k[6], k[7], k[8])), q1 = ob + mv3(E.R[b1], mk(k[9], k[10], k[11]));
  const float rb = k[13];
  f3 pa, pb;
  float dist, ra;
  if (k[12] < 0.f) {
    // base-box bottom face (base frame z = k[2] over [k0, k3] x [k1, k4], outward normal -z of
    // the base) vs the closer end sphere of capsule b
    const float* R0 = E.R[0];
    const float h0 = k[2] - (R0[2] * q0.x + R0[5] * q0.y + R0[8] * q0.z);
    const float h1 = k[2] - (R0[2] * q1.x + R0[5] * q1.y + R0[8] * q1.z);
    const bool s1 = h1 < h0;
    const f3 e = s1 ? q1 : q0;
    const float h = s1 ? h1 : h0;
    const float ex = R0[0] * e.x + R0[3] * e.y + R0[6] * e.z, ey = R0[1] * e.x + R0[4] * e.y + R0[7] * e.z;
    const bool inside = ex >= k[0] && ex <= k[3] && ey >= k[1] && ey <= k[4];
    C.cn = mk(-R0[2], -R0[5], -R0[8]);
    pb = e;
    pa = e - h * C.cn;
    ra = 0.f;
    dist = inside ? h : 1e3f;
  } else {
    const f3 oa = ld3(E.o[b0]);
    seg_seg(oa + mv3(E.R[b0], mk(k[0], k[1], k[2])), oa + mv3(E.R[b0], mk(k[3], k[4], k[5])), q0, q1, pa, pb);
    const f3 dv = pb - pa;
    // v_sqrt_f32 / v_rcp_f32 (1 ulp) instead of the correctly rounded sequences
    dist = __builtin_amdgcn_sqrtf(dot(dv, dv));
    C.cn = dist > 1e-9f ? __builtin_amdgcn_rcpf(dist) * dv : mk(0.f, -1.f, 0.f);
    ra = k[12];
  }
  C.phi = dist - ra - rb;
  C.xP = pb - rb * C.cn;
  C.xN = pa + ra * C.cn;
  C.bP = b1;
  C.bN = b0;
  C.mu = E.fric;
  C.lam_base = LAM_PAIR + 3 * p;
  C.act = C.phi < P.contact_offset;
  return C;
}

// an active candidate of contact rank `rank` (< npts kept): its contact record (the three rows
// read it in A10) and its PGS group; otherwise its warm-start slots are cleared
__device__ __forceinline__ void place_contact(EnvSh& E, const Cand& C, bool act, int rank, int npts, float inv_dt,
                                              float beta, float vmax) {
  if (act && rank < npts) {
    const float tgt = C.phi >= 0.f ? -C.phi * inv_dt : fminf(-beta * C.phi * inv_dt, vmax);
    // tangent basis (reference axis x, or y when the normal is close to x)
    const f3 ref = fabsf(C.cn.x) < 0.9f ? mk(1, 0, 0) : mk(0, 1, 0);
    f3 t1 = ref - dot(ref, C.cn) * C.cn;
    t1 = rsqrtf(dot(t1, t1)) * t1;
    const f3 t2 = cross(C.cn, t1);
    ContactC& R = E.ct[rank];
    st3(R.xP, C.xP); st3(R.xN, C.xN);
    st3(R.dir[0], C.cn); st3(R.dir[1], t1); st3(R.dir[2], t2);
    R.bP = C.bP; R.bN = C.bN; R.lam_base = C.lam_base;
    GroupC& G = E.grp[rank];
    G.mu = C.mu;
    G.tgt[0] = tgt; G.tgt[1] = 0.f; G.tgt[2] = 0.f;
    G.lo[0] = 0.f; G.lo[1] = -BIG; G.lo[2] = -BIG;
    G.hi[0] = BIG; G.hi[1] = BIG; G.hi[2] = BIG;
  } else {
    E.lamst[C.lam_base + 0] = E.lamst[C.lam_base + 1] = E.lamst[C.lam_base + 2] = 0.f;
  }
}

}  // namespace

// FIXED = asset.fix_base_link, a compile-time constant so the factorised size and every
// floating-base branch resolve at compile time
template <bool FIXED>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2))) k_step(HgState S, const float* __restrict__ actions_in, uint64_t step_counter, const StepParams P) {
  __shared__ EnvSh shm[2];
  const int half = threadIdx.x >> 5;
  int l = threadIdx.x & 31;
  // XCD-aware env mapping: workgroups are dispatched round-robin over the 8 XCDs (block b ->
  // XCD b % 8), each with its own L2.  Giving every XCD a contiguous range of env pairs keeps the
  // 16 envs of one 64-byte SoA line on one L2, so their 4-byte state stores merge there instead of
  // being written back as 8 partial lines from 8 caches.
  const int nb = gridDim.x, xcd = blockIdx.x & 7, kx = blockIdx.x >> 3;
  const int p0 = xcd * (nb >> 3) + min(xcd, nb & 7);
  // wave balancing (S.balance): a launch of 2048 one-wave blocks puts block b and block b + 1024
  // on the same SIMD (scripts/probes/placement_probe.hip: every SIMD of the chip gets one block
  // of each half, in dispatch order), i.e. within an XCD block kx and kx + cnt / 2.  A wave's cost
  // is its heavier env's constraint rows (the PGS runs max of the two envs' groups) and the launch
  // ends with its slowest SIMD, so the XCD's env pairs, sorted heaviest first by env_order_block
  // (hg_common.h; run inside the post launch after each step) from the step's rows, go heaviest to block kx and lightest to its SIMD partner.  Every env
  // stays in its XCD's range (the L2 locality of the SoA stores) and its result does not depend
  // on which env shares its wave.
  int pair = p0 + kx;
  if (S.balance) {
    const int cnt = (nb >> 3) + (xcd < (nb & 7) ? 1 : 0), hc = (cnt + 1) >> 1;
    pair = p0 + (kx < hc ? kx : cnt - 1 - (kx - hc));
  }
  const int pos = pair * 2 + half;
  const bool valid = pos < S.n;
  const int e = S.balance ? S.env_order[valid ? pos : S.n - 1] : (valid ? pos : S.n - 1);
  EnvSh& E = shm[half];
  const hg_cfg* cfg = S.cfg;
  const hg_model* M = S.model;
  const int np = S.np;
  const float dt = P.dt;
  const float inv_dt = 1.0f / dt;
  constexpr bool fixed = FIXED;
  constexpr int nf = fixed ? 12 : 18;  // factorised size (legs-first order: left leg, right leg, base)
  const float gz = P.gz;

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
    a = clampf(a, -cfg->clip_actions, cfg->clip_actions);
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
    E.drop = 0;
  }
  __syncthreads();
  const float scale0 = E.mass0 / M->mass[0];
  // PD constants of this lane's joint staged in LDS for all substeps; the position target is
  // constant over the policy step
  if (l < 12) {
    E.pd_kp[l] = cfg->kp[l];
    E.pd_kd[l] = cfg->kd[l];
    E.pd_lim[l] = cfg->torque_limit[l];
    E.pd_arm[l] = M->armature[l + 1];
    E.pd_tgt[l] = E.act[l] * cfg->action_scale + cfg->default_dof_pos[l];
  }
  for (int i = l; i < 18 * 20; i += 32) (&E.L[0][0])[i] = 0.f;  // the left-right cross block stays zero
  const int decimation = P.decimation;
  // per-lane model constants of the detection phase, in registers for the whole launch (they
  // were global loads at the head of every substep's detection): this lane's ground candidate
  // (body, sole point / sphere centre, radius) or capsule pair (bodies, segment ends, radii),
  // and its joint's limits and friction
  const int nleg = M->num_leg_contacts, npair = M->num_pairs, nitems = M->num_contacts + npair;
  int det_c, det_p, det_b0, det_b1;
  float det_k[14];
  const bool det_pair = load_item(M, min(l, nitems - 1), nleg, npair, det_c, det_p, det_b0, det_b1, det_k);
  // the round-2 items' plane early-out (A9) from two per-lane constants (body, reach = the point's
  // distance from the body origin + its radius), so the skipped round reads no model constants
  int r2_b0 = 0;
  float r2_reach = 0.f;
  if (nitems > 32) {
    int cc2, pp2, b02, b12;
    float k2[14];
    const bool pr2 = load_item(M, min(32 + l, nitems - 1), nleg, npair, cc2, pp2, b02, b12, k2);
    r2_b0 = b02;
    r2_reach = pr2 ? 0.f : sqrtf(k2[0] * k2[0] + k2[1] * k2[1] + k2[2] * k2[2]) + k2[3];
  }
  const int lj = l < 12 ? l + 1 : 1;
  const float lim_lo = M->lower[lj], lim_hi = M->upper[lj], jfric = M->joint_friction[lj];
  // this joint's slot among the friction rows: larger friction bounds first, then the joint
  // within its leg, left before right (the rows the budget drops are the smallest bounds, from
  // both legs alike)
  int frank = 0;
  for (int j = 0; j < 12; j++) {
    const float fj = M->joint_friction[j + 1];
    const bool before = fj > jfric || (fj == jfric && (j % 6 < l % 6 || (j % 6 == l % 6 && j < l)));
    frank += (fj > 0.f && before) ? 1 : 0;
  }

  for (int sub = 0; sub < decimation; sub++) {
    // lane masks are rebuilt per substep (v_cmp) instead of living across the loop in SGPR pairs
    asm volatile("" : "+v"(l));
    const ModelLane ML = load_model_lane(M, l);
    // ---- A1: torques (_compute_torques, humanoid_env.py:910-925); implicit damping on the
    // joints whose torque is not clipped: dt*kd joins M's diagonal (with the model armature)
    if (l < 12) {
      const float t = E.pd_kp[l] * (E.pd_tgt[l] - E.q[l]) - E.pd_kd[l] * E.qd[l];
      const float lim = E.pd_lim[l];
      E.tau[l] = clampf(t, -lim, lim);
      const bool sat = t < -lim || t > lim;
      E.madd[l] = E.pd_arm[l] + (sat ? 0.f : dt * E.pd_kd[l]);
      E.nu[6 + l] = E.qd[l];
    }
    if (l < 6) E.nu[l] = fixed ? 0.f : E.root[7 + l];
    __syncthreads();
    // ---- A2..A5: kinematics (prefix scans), per-body forces, backward recursions (suffix scans)
    const KinLane K = kin_scan(E, ML, l, gz, true);
    rnea_scan(E, ML, l, K, scale0);
    __syncthreads();
    // base totals (lane 0) — read the kinematics scratch before M overwrites it.  One total per
    // lane (16 lanes: h 0..5, base_cm, base_cs 0..2, base_cJ 0..5), each with the operations and
    // order of the serial form (f3 sums and cross products component by component): every LDS
    // read of the phase is issued at once instead of lane 0's chain of 16 round trips
    {
      const int t = l < 16 ? l : 15;
      const int c = t < 3 ? t : (t < 6 ? t - 3 : (t >= 7 && t < 10 ? t - 7 : 0));
      const int c1 = c == 2 ? 0 : c + 1, c2 = c == 0 ? 2 : c - 1;  // cross component c = a[c1] b[c2] - a[c2] b[c1]
      const int j = t >= 10 ? t - 10 : 0;
      // rows of the three base-side links' arrays this lane sums: f (t < 3), n + o x f (3..5),
      // cm (6), cs (7..9), cJ (10..15)
      const float* src = t < 3 ? &E.u.kin.f[0][0] : (t < 6 ? &E.u.kin.n[0][0] : (t == 6 ? E.cm : (t < 10 ? &E.cs[0][0] : &E.cJ[0][0])));
      const int pitch = t == 6 ? 1 : (t < 10 ? 3 : 6), col = t == 6 ? 0 : (t < 10 ? c : j);
      float v0 = src[0 * pitch + col], v1 = src[1 * pitch + col], v7 = src[7 * pitch + col];
      const float o1a = E.o[1][c1], o1b = E.o[1][c2], o7a = E.o[7][c1], o7b = E.o[7][c2];
      const float f1a = E.u.kin.f[1][c1], f1b = E.u.kin.f[1][c2], f7a = E.u.kin.f[7][c1], f7b = E.u.kin.f[7][c2];
      pin(v0); pin(v1); pin(v7);
      float r = v0 + v1;
      if (t >= 3 && t < 6) {
        const float x1 = o1a * f1b - o1b * f1a, x7 = o7a * f7b - o7b * f7a;
        r = ((r + x1) + v7) + x7;
      } else {
        r = r + v7;
      }
      float* dst = t < 6 ? &E.h[t] : (t == 6 ? &E.base_cm : (t < 10 ? &E.base_cs[t - 7] : &E.base_cJ[j]));
      if (l < 16) *dst = r;
    }
    __syncthreads();
    // ---- A6/A7: M written straight into the factor's legs-first lower triangle (index i <-> dof
    // o(i) = i < 12 ? 6 + i : i - 12): joint b's lane writes its row b-1 (ancestors in its leg,
    // diagonal + armature + implicit damping) and its column of the six base rows; lane 0 the base
    // block.  The left-right cross block stays zero from the launch-time fill.
    if (l == 0) {
      const float m0 = E.base_cm;
      f3 s = ld3(E.base_cs);
      const float* J0 = E.base_cJ;
      float (*A)[20] = E.L;
      A[12][12] = A[13][13] = A[14][14] = m0;
      A[13][12] = 0.f; A[14][12] = 0.f; A[14][13] = 0.f;
      A[15][12] = 0.f;  A[15][13] = -s.z; A[15][14] = s.y;
      A[16][12] = s.z;  A[16][13] = 0.f;  A[16][14] = -s.x;
      A[17][12] = -s.y; A[17][13] = s.x;  A[17][14] = 0.f;
      A[15][15] = J0[0]; A[16][16] = J0[1]; A[17][17] = J0[2];
      A[16][15] = J0[3]; A[17][15] = J0[4]; A[17][16] = J0[5];
    } else if (l <= 12) {
      const int b = l, i = b - 1;
      f3 a = ld3(E.a[b]), o = ld3(E.o[b]);
      f3 cs = ld3(E.cs[b]);
      f3 F = cross(a, cs - E.cm[b] * o);
      f3 Lm = symv(E.cJ[b], a) - cross(cs, cross(a, o));
      float (*A)[20] = E.L;
      A[12][i] = F.x; A[13][i] = F.y; A[14][i] = F.z;
      A[15][i] = Lm.x; A[16][i] = Lm.y; A[17][i] = Lm.z;
      const int first = b <= 6 ? 1 : 7;
      // the ancestors kb = b, b - 1, .. first as six predicated slots with every LDS read issued
      // up front (the variable-trip loop waited one round trip per ancestor); a slot past the
      // leg's root stores into the row's unused padding column 19
      const float madd = E.madd[b - 1];
      f3 ak[6], ok[6];
#pragma unroll
      for (int m = 0; m < 6; m++) {
        const int kc = b - m >= first ? b - m : b;
        ak[m] = ld3(E.a[kc]);
        ok[m] = ld3(E.o[kc]);
        pin(ak[m]);
        pin(ok[m]);
      }
#pragma unroll
      for (int m = 0; m < 6; m++) {
        const int kb = b - m;
        const float val = dot(ak[m], Lm - cross(ok[m], F));
        A[i][kb >= first ? kb - 1 : 19] = kb == b ? val + madd : val;
      }
    }
    __syncthreads();
    // ---- A8: Cholesky in registers, legs-first order: M's arrow structure gives L no
    // left-right-leg block.  Lane i holds row i; each pivot column is broadcast through LDS (one
    // write, half-wave broadcast reads; same-wave LDS accesses complete in order, so no barrier)
    // and the rank-1 update is one FMA per trailing entry.  The right-hand side b = tau - h rides
    // along in the same broadcasts: g = L^-1 b comes out of the same steps.
    {
      float a[20];  // 18 used; ld_vec fills whole 16-byte groups
      bool nonpd = false;
      const int ol = l < 12 ? 6 + l : l - 12;  // this lane's dof
      ld_vec(E.L[l < 18 ? l : 0], a, 18);
#pragma unroll
      for (int k = 0; k < 18; k++) a[k] = (l < nf && k <= l) ? a[k] : 0.f;
      float bv = (l < 18) ? (ol >= 6 ? E.tau[(ol >= 6 ? ol : 6) - 6] : 0.f) - E.h[l < 18 ? ol : 0] : 0.f;
      asm volatile("" ::: "memory");
      // steps 0..5: the left-leg pivot j and the right-leg pivot 6 + j together (a left-leg row has
      // L[.][6 + j] = 0, so its right-pivot multiplier is 0, and vice versa; base rows take both
      // updates, which commute); steps 6..: the base pivots
      float my_inv = 0.f, my_g = 0.f;  // this lane's pivot (l == j): 1 / L_ll and g_l, stored after the loop
#pragma unroll
      for (int j = 0; j < 6; j++) {
        const int j2 = 6 + j;
        E.colbuf[l] = a[j]; E.colbuf2[l] = a[j2]; E.bbuf[l] = bv;
        float c1[20], c2[20];  // column j (rows 0..7, 12..19) and column j2 (rows 4..19)
        ld_vec(E.colbuf, c1, 8);
        ld_vec(E.colbuf + 12, c1 + 12, 8);
        ld_vec(E.colbuf2 + 4, c2 + 4, 16);
        const float d1 = c1[j], d2 = c2[j2], b1 = E.bbuf[j], b2 = E.bbuf[j2];
        nonpd |= !(d1 > 0.f) || !(d2 > 0.f);
        const float inv1 = __builtin_amdgcn_rsqf(fmaxf(d1, 1e-20f));  // 1 / L_jj (1 ulp)
        const float inv2 = __builtin_amdgcn_rsqf(fmaxf(d2, 1e-20f));
        const float g1 = b1 * inv1, g2 = b2 * inv2;
        const int lo = lane_opaque(l);
        my_inv = lo == j ? inv1 : (lo == j2 ? inv2 : my_inv);
        my_g = lo == j ? g1 : (lo == j2 ? g2 : my_g);
        const float t1 = lo > j ? a[j] * (inv1 * inv1) : 0.f;     // L[l][j] / L[j][j] (0 on right-leg rows)
        const float t2 = lo > j2 ? a[j2] * (inv2 * inv2) : 0.f;   // L[l][j2] / L[j2][j2] (0 on left-leg rows)
        a[j] = lo >= j ? a[j] * inv1 : a[j];
        a[j2] = lo >= j2 ? a[j2] * inv2 : a[j2];
        bv -= t1 * b1 + t2 * b2;                                   // b_l -= L[l][j] g_j + L[l][j2] g_j2
#pragma unroll
        for (int k = j + 1; k < 6; k++) a[k] -= t1 * c1[k];
#pragma unroll
        for (int k = j2 + 1; k < 12; k++) a[k] -= t2 * c2[k];
#pragma unroll
        for (int k = 12; k < nf; k++) a[k] -= t1 * c1[k] + t2 * c2[k];
      }
#pragma unroll
      for (int j = 12; j < nf; j++) {
        E.colbuf[l] = a[j]; E.bbuf[l] = bv;
        float c1[20];  // column j, rows 12..19
        ld_vec(E.colbuf + 12, c1 + 12, 8);
        const float d = c1[j], bj = E.bbuf[j];
        nonpd |= !(d > 0.f);
        const float inv = __builtin_amdgcn_rsqf(fmaxf(d, 1e-20f));
        const float gj = bj * inv;
        my_inv = lane_opaque(l) == j ? inv : my_inv;
        my_g = lane_opaque(l) == j ? gj : my_g;
        const float t = lane_opaque(l) > j ? a[j] * (inv * inv) : 0.f;
        a[j] = (lane_opaque(l) >= j) ? a[j] * inv : a[j];
        bv -= t * bj;
#pragma unroll
        for (int k = j + 1; k < nf; k++) a[k] -= t * c1[k];
      }
      if (l < nf) { E.invd[l] = my_inv; E.gv[l] = my_g; }
      if (l < nf) st_vec<18>(E.L[l], a);
      if (l == 0 && nonpd) E.bad = 1;
    }
    __syncthreads();
    // ---- A9: contact detection (one candidate per lane, in priority order: ground candidates
    // [0, num_leg_contacts), the self-collision pairs, the remaining ground candidates; items
    // 32.. run as a second round on lanes 0..), joint limits, and row allocation by ballot /
    // popcount: contacts (<= 9 points), then joint limits, then joint friction (<= 32 rows; the
    // rest dropped and counted)
    {
      const uint32_t lt = (1u << l) - 1u;
      const float beta = P.beta, vmax = P.vmax;
      // single rows unless a contact claims the group below (mu = +inf: the PGS disc projection
      // never scales a single-row group, see A13)
      if (l < NGRP) E.grp[l].mu = __builtin_huge_valf();
      // round 1: items 0..31 (model constants in registers for the whole launch); round 2 (when
      // the model has more than 32 items): items 32 + l, constants read here.  A contact's rank
      // among the active candidates decides its slot; round 2 ranks after all of round 1, so each
      // round places its contacts before the next runs.  One loop body (not unrolled): one copy of
      // the detection code.
      int npts_all = 0;
      const int rounds = nitems > 32 ? 2 : 1;
#pragma unroll 1
      for (int rnd = 0; rnd < rounds; rnd++) {
        const int item = 32 * rnd + l;
        bool pr = det_pair;
        int cc = det_c, pp = det_p, b0 = det_b0, b1 = det_b1;
        float k[14];
#pragma unroll
        for (int i = 0; i < 14; i++) k[i] = det_k[i];
        if (rnd) {
          // round 2 holds ground candidates (the base-box corners): on a plane, a candidate whose
          // body origin is higher than contact_offset + the point's distance from it + its radius
          // cannot be active.  When no round-2 item of the wave's two envs can be, the round is
          // skipped (bitwise the same result: its warm-start slots are cleared as an inactive
          // candidate's are, and no contact is placed); the test is from the launch-time constants
          // with a 1e-4 margin (conservative: a borderline round runs in full)
          // (a fixed base never activates ground candidates)
          const bool pr2 = item >= nleg && item < nleg + npair;
          const bool can = item < nitems &&
                           (pr2 || (!fixed && (P.heightfield_on ||
                                               E.o[r2_b0][2] + E.root[2] - r2_reach < P.contact_offset + 1e-4f)));
          if (__ballot(can) == 0) {
            const int cs = min(item < nleg ? item : item - npair, HG_MAX_CONTACTS - 1);  // load_item's c
            if (item < nitems) E.lamst[3 * cs + 0] = E.lamst[3 * cs + 1] = E.lamst[3 * cs + 2] = 0.f;
            continue;
          }
          pr = load_item(M, min(item, nitems - 1), nleg, npair, cc, pp, b0, b1, k);
        }
        Cand c;
        if (item < nitems) c = detect(E, P, pr, cc, pp, b0, b1, k, fixed);
        const bool act = item < nitems && c.act;
        const uint32_t mc = (uint32_t)(__ballot(act) >> (32 * half));
        const int n = __popc(mc);
        if (item < nitems)
          place_contact(E, c, act, npts_all + __popc(mc & lt), min(npts_all + n, MAX_PTS), inv_dt, beta, vmax);
        npts_all += n;
      }
      bool act_l = false, has_f = false;
      float gapv = 0.f, sgnv = 1.f, ffric = 0.f;
      if (l < 12) {
        const float glo = E.q[l] - lim_lo, ghi = lim_hi - E.q[l];
        if (glo < 0.01f) { act_l = true; gapv = glo; sgnv = 1.f; }
        else if (ghi < 0.01f) { act_l = true; gapv = ghi; sgnv = -1.f; }
        ffric = jfric;
        has_f = ffric > 0.f;
      }
      const uint32_t ml = (uint32_t)(__ballot(act_l) >> (32 * half)) & 0xFFFu;
      const uint32_t mf = (uint32_t)(__ballot(has_f) >> (32 * half)) & 0xFFFu;
      const int npts = min(npts_all, MAX_PTS);
      const int nlim = __popc(ml), nfr = __popc(mf);
      const int wanted = 3 * npts + nlim + nfr;
      const int nrows = min(RMAX, wanted);
      if (l == 0) {
        E.nrows = nrows;
        E.npts = npts;
        E.drop += (wanted - nrows) + 3 * (npts_all - npts);
      }
      // empty slots
      for (int r = l; r < 3 * NGRP; r += 32) {
        if (r >= nrows) {
          const int g = r / 3, k = r % 3;
          E.grp[g].tgt[k] = 0.f; E.grp[g].lo[k] = 0.f; E.grp[g].hi[k] = 0.f;
        }
      }
      if (l < 12) {
        const int r = 3 * npts + __popc(ml & lt);
        if (act_l && r < RMAX) {
          E.rd[r][0] = sgnv; E.rbP[r] = -1 - l; E.rbN[r] = -1;
          E.rlam[r] = LAM_LIM + l;
          E.rLam[r] = E.lamst[LAM_LIM + l];
          E.grp[r / 3].tgt[r % 3] = gapv >= 0.f ? -gapv * inv_dt : fminf(-beta * gapv * inv_dt, vmax);
          E.grp[r / 3].lo[r % 3] = 0.f; E.grp[r / 3].hi[r % 3] = BIG;
        } else {
          E.lamst[LAM_LIM + l] = 0.f;
        }
        const int rf = 3 * npts + nlim + frank;
        if (has_f && rf < RMAX) {  // joint friction: |lambda| <= f dt
          E.rd[rf][0] = 1.f; E.rbP[rf] = -1 - l; E.rbN[rf] = -1;
          E.rlam[rf] = LAM_FRIC + l;
          E.rLam[rf] = E.lamst[LAM_FRIC + l];
          E.grp[rf / 3].tgt[rf % 3] = 0.f; E.grp[rf / 3].lo[rf % 3] = -ffric * dt; E.grp[rf / 3].hi[rf % 3] = ffric * dt;
        } else {
          E.lamst[LAM_FRIC + l] = 0.f;
        }
      }
    }
    __syncthreads();
    const int nrows = E.nrows;
    const bool own = l < nrows;
    // ---- A10: Jacobian row (registers, dof order), z = L^-1 J^T (legs-first), row velocity
    // J nu* = J nu + dt z . g
    float z[18];
    float v0 = 0.f;
    {
      float J[18];
#pragma unroll
      for (int i = 0; i < 18; i++) J[i] = 0.f;
      const int npts_e = E.npts;
      const bool crow = own && l < 3 * npts_e;   // contact row (else joint friction / limit row)
      const bool jrow = own && !crow;
      // Branch-free over the row kinds: every lane reads its joint-row slot and a (clamped) contact
      // record and builds both rows; the reads are pinned ahead of the selects so they never sit
      // behind an exec-mask branch.
      int jdof = -1 - E.rbP[l];
      float jsgn = E.rd[l][0];
      pin(jdof);
      pin(jsgn);
      const int cidx = crow ? l / 3 : 0, cdir = crow ? l % 3 : 0;
      const ContactC& C = E.ct[cidx];
      f3 d = ld3(C.dir[cdir]), xp = ld3(C.xP), xn = ld3(C.xN);
      int bP = C.bP, bN = C.bN;
      const int lamb = min(max(C.lam_base, 0), HG_LAMW - 3) + cdir;
      float lamv = E.lamst[lamb];
      pin(d); pin(xp); pin(xn); pin(bP); pin(bN); pin(lamv);
      if (crow) { E.rlam[l] = lamb; E.rLam[l] = lamv; }
      // contact row J = J_bP(xP) d - J_bN(xN) d
      const bool pair2 = bN >= 0;
      float Jc[18];
      Jc[0] = pair2 ? 0.f : d.x; Jc[1] = pair2 ? 0.f : d.y; Jc[2] = pair2 ? 0.f : d.z;
      const f3 xd = cross(xp, d) - (pair2 ? cross(xn, d) : mk(0, 0, 0));
      Jc[3] = xd.x; Jc[4] = xd.y; Jc[5] = xd.z;
      {
        // the contact body's leg: links kb0 .. bP (6 at most)
        const bool right = bP >= 7;
        const int kb0 = right ? 7 : 1;
#pragma unroll
        for (int m = 0; m < 6; m++) {
          const int k = kb0 + m;
          f3 ak = ld3(E.a[k]), ok = ld3(E.o[k]);
          pin(ak); pin(ok);
          const float val = (bP > 0 && k <= bP) ? dot(d, cross(ak, xp - ok)) : 0.f;
          Jc[6 + m] = right ? 0.f : val;
          Jc[12 + m] = right ? val : 0.f;
        }
      }
      // the other capsule's chain (self-collision rows), only when the wave has such a row
      if (__ballot(crow && pair2) != 0) {
        const bool right = bN >= 7;
        const int kb0 = right ? 7 : 1;
#pragma unroll
        for (int m = 0; m < 6; m++) {
          const int k = kb0 + m;
          f3 ak = ld3(E.a[k]), ok = ld3(E.o[k]);
          pin(ak); pin(ok);
          const float val = (pair2 && k <= bN) ? dot(d, cross(ak, xn - ok)) : 0.f;
          Jc[6 + m] -= right ? 0.f : val;
          Jc[12 + m] -= right ? val : 0.f;
        }
      }
#pragma unroll
      for (int i = 0; i < 18; i++) J[i] = crow ? Jc[i] : ((jrow && i >= 6 && i - 6 == jdof) ? jsgn : 0.f);
#pragma unroll
      for (int i = 0; i < 18; i++) v0 += J[i] * E.nu[i];
      // forward substitution with L broadcast from LDS (legs-first order; arrow structure)
      float invd[20], gvr[20];
      ld_vec(E.invd, invd, 20);
      ld_vec(E.gv, gvr, 20);
#pragma unroll
      for (int k = 0; k < 18; k++) {
        if (k >= nf) { z[k] = 0.f; continue; }
        float s = J[k < 12 ? 6 + k : k - 12];
        float Lk[20];
        ld_vec(E.L[k], Lk, k);  // row k below the diagonal
#pragma unroll
        for (int m = 0; m < k; m++) {
          if (k >= 6 && k < 12 && m < 6) continue;
          s -= Lk[m] * z[m];
        }
        z[k] = s * invd[k];
      }
#pragma unroll
      for (int k = 0; k < nf; k++) v0 += dt * (z[k] * gvr[k]);  // gv[k >= nf] is never written (fixed base)
    }
    st_vec<18>(E.u.Z[l], z);
    // the group constants below read the neighbouring lanes' rows: a barrier, not program order
    // (per lane, Z[l-1] and Z[l] are different addresses the compiler may reorder around)
    __syncthreads();
    // ---- A11: W = Z^T Z on the matrix cores (v_mfma_f32_32x32x2f32).  MFMA operand i/kk =
    // lane%32 / lane/32, so the wave's two envs are interleaved with v_permlane32_swap:
    // swap(X, Y) -> (X.lo|Y.lo, X.hi|Y.hi) is env 0's / env 1's [32 rows x 2 k] operand, and the
    // same register is the B operand (B[kk][n] = z_n[k]).  D layout: lane (n, kk), vgpr v holds
    // W[8(v/4) + 4kk + v%4][n].
    f32x16 dw0 = {0}, dw1 = {0};
#pragma unroll
    for (int p = 0; p < 9; p++) {
      float a0, a1;
      swap32(z[2 * p], z[2 * p + 1], a0, a1);
      dw0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, a0, dw0, 0, 0, 0);
      dw1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, a1, dw1, 0, 0, 0);
    }
    // gather each env's W column l into its own lanes: wA[v] = W[8(v/4) + v%4][l],
    // wB[v] = W[8(v/4) + 4 + v%4][l]  (W symmetric: column l == row l)
    float wA[16], wB[16];
#pragma unroll
    for (int v = 0; v < 16; v++) swap32(dw0[v], dw1[v], wA[v], wB[v]);
    float wrow[RMAX];
#pragma unroll
    for (int m = 0; m < RMAX; m++) wrow[m] = (m % 8 < 4) ? wA[4 * (m / 8) + m % 8] : wB[4 * (m / 8) + m % 8 - 4];
    // warm-start impulses, replicated in every lane of the env (uniform per half-wave)
    float lam[RMAX];
#pragma unroll
    for (int m = 0; m < RMAX; m++) lam[m] = m < nrows ? E.rLam[m] : 0.f;
    // ---- A12: group constants (1/W_rr and the in-group couplings z_r . z_{r-1}, z_r . z_{r-2}
    // from the Z rows in LDS), warm-started row velocities
    {
      float Dd = 0.f, W1 = 0.f, W2 = 0.f;  // W[l][l], W[l][l-1], W[l][l-2]
      const int l1 = l >= 1 ? l - 1 : 0, l2 = l >= 2 ? l - 2 : 0;
      float z1[20], z2[20];
      ld_vec(E.u.Z[l1], z1, 18);
      ld_vec(E.u.Z[l2], z2, 18);
#pragma unroll
      for (int k = 0; k < 18; k++) {
        Dd += z[k] * z[k];
        W1 += z[k] * z1[k];
        W2 += z[k] * z2[k];
      }
      const int g = l / 3, k = l % 3;
      E.grp[g].invD[k] = own ? __builtin_amdgcn_rcpf(Dd) : 0.f;
      if (k == 1) E.grp[g].Wba = W1;
      // a contact's tangent pair is updated from the same nu (Wcb unused: 0, see A13)
      if (k == 2) { E.grp[g].Wca = W2; E.grp[g].Wcb = g < E.npts ? 0.f : W1; }
      if (l == 31) { E.grp[10].invD[2] = 0.f; E.grp[10].Wca = 0.f; E.grp[10].Wcb = 0.f; }  // virtual slot 32
      float v = v0;
#pragma unroll
      for (int m = 0; m < RMAX; m++) v += wrow[m] * lam[m];
      v0 = own ? v : 0.f;
    }
    __syncthreads();
    // ---- A13: projected Gauss-Seidel over the 3-slot groups.  The impulses are replicated: every
    // lane of an env holds all 32 of its env's impulses (uniform per half-wave); the row velocity
    // v_r lives in lane r and is read with one ds_swizzle broadcast (swz).  Per group (a, b, c):
    //   a: lambda_a <- clamp(lambda_a + (tgt_a - v_a) / W_aa, lo_a, hi_a)   (normal / single row)
    //   b: lambda_b' <- clamp(lambda_b + (tgt_b - v_b - W_ba dl_a) / W_bb, lo_b, hi_b)
    //   c: lambda_c' <- clamp(lambda_c + (tgt_c - v_c - W_ca dl_a - W_cb dl_b') / W_cc, lo_c, hi_c)
    //   (b, c) <- (b', c') scaled onto the disc |.| <= mu lambda_a
    // One instruction stream for both group kinds, through the group constants: a contact's
    // tangent pair has tgt 0, bounds -+BIG (no clamp) and W_cb = 0 (both steps from the same nu,
    // as the oracle); a single-row group has mu = +inf, so the disc never scales it.  Then every
    // row velocity takes the group's three updates (one FMA each).  Groups empty in both envs of
    // the wave are skipped (scalar branch).  Separate contact / single-row streams behind scalar
    // branches (round 5) cut VALU per wave 45.1 k -> 41.8 k but were slower per launch (their
    // extra SALU and taken branches sit on the chain; profiles/r5_kstep/README.md).
    {
      float vrow = v0;
      const int ng = (max(shm[0].nrows, shm[1].nrows) + 2) / 3;
      const int npgs = P.pgs_iterations;
      for (int it = 0; it < npgs; it++) {
#pragma unroll
        for (int g = 0; g < NGRP; g++) {
          if (g < ng) {
            const int ra = 3 * g, rb = 3 * g + 1, rc = 3 * g + 2;
            const bool has_c = rc < RMAX;  // slot 32 of group 10 is virtual
            const int rcc = has_c ? rc : 0;
            const GroupC& G = E.grp[g];
            const float va = swz(vrow, ra), vb = swz(vrow, rb);
            const float vc = has_c ? swz(vrow, rcc) : 0.f;
            const float la = lam[ra], lb = lam[rb], lc = has_c ? lam[rcc] : 0.f;
            const float na = clampf(la + (G.tgt[0] - va) * G.invD[0], G.lo[0], G.hi[0]);
            const float da = na - la;
            const float vb1 = vb + G.Wba * da, vc1 = vc + G.Wca * da;
            const float tb = clampf(lb + (G.tgt[1] - vb1) * G.invD[1], G.lo[1], G.hi[1]);
            const float vc2 = vc1 + G.Wcb * (tb - lb);
            const float tc = clampf(lc + (G.tgt[2] - vc2) * G.invD[2], G.lo[2], G.hi[2]);
            // the oracle's "if (|l| > lim) l *= lim / |l|" as the scale min(1, |lim| / |l|): |l| = 0
            // gives lim * inf (inf or NaN) and min returns 1; a single-row group's lim = mu lambda_a
            // is +-inf or NaN (mu = +inf), so its scale is 1; |.| is a free source modifier
            const float lim = G.mu * na, nn2 = __builtin_fmaf(tc, tc, tb * tb);  // the order of the oracle's l1^2 + l2^2
            const float sc = fminf(1.f, fabsf(lim) * __builtin_amdgcn_rsqf(nn2));
            const float db = __builtin_fmaf(tb, sc, -lb), dc = __builtin_fmaf(tc, sc, -lc);
            vrow = __builtin_fmaf(wrow[ra], da, vrow);
            vrow = __builtin_fmaf(wrow[rb], db, vrow);
            if (has_c) vrow = __builtin_fmaf(wrow[rcc], dc, vrow);
            lam[ra] += da;
            lam[rb] += db;
            if (has_c) lam[rcc] += dc;
          }
        }
      }
      // ---- A14: nu_new = nu + L^-T (dt g + Z^T lambda): lanes = dofs (legs-first order k)
      // every lane computes (lanes >= nf on a clamped column, discarded): no exec-mask branch
      const int lc = l < 18 ? l : 17;
      float y;
      {
        float u = dt * E.gv[lc];
#pragma unroll
        for (int m = 0; m < RMAX; m++) u += E.u.Z[m][lc] * lam[m];
        y = l < nf ? u : 0.f;
      }
      if (l == 0) st_vec<RMAX>(E.rLam, lam);
      // back substitution L^T x = y, column-oriented: the base pivots 17..12, then the two legs'
      // pivots 6 + k and k together (a leg's column has no rows in the other leg, so the two
      // chains are independent): 12 broadcast round trips instead of 18, the same operations per
      // element in the same order
      // (the L entry is read on every lane, pinned before the select, so the compiler does not
      // put the read behind an exec-mask branch)
#pragma unroll
      for (int j = nf - 1; j >= 12; j--) {
        float Ljl = E.L[j][lc];
        asm volatile("" : "+v"(Ljl));
        const float xj = swz(y, j) * E.invd[j];
        y = (l == j) ? xj : ((l < j) ? y - Ljl * xj : y);
      }
#pragma unroll
      for (int k = 5; k >= 0; k--) {
        const int jr = 6 + k, jl = k;
        const bool right = l >= 6 && l < 12;
        const int j = right ? jr : jl;
        float Ljl = E.L[j][lc];
        asm volatile("" : "+v"(Ljl));
        const float xr = swz(y, jr) * E.invd[jr];
        const float xl = swz(y, jl) * E.invd[jl];
        const float xj = right ? xr : xl;
        const int lo = right ? 6 : 0;
        y = (l == j) ? xj : ((l >= lo && l < j) ? y - Ljl * xj : y);
      }
      __syncthreads();
      float nu_new = 0.f;
      const int od = l < 12 ? 6 + l : l - 12;
      if (l < 18) nu_new = E.nu[l < 18 ? od : 0] + (l < nf ? y : 0.f);
      // contact forces (net per body, world frame; only the last substep's are reported) and
      // warm-start store
      const bool last_sub = sub == decimation - 1;
      if (last_sub)
        for (int i = l; i < 13 * 3; i += 32) (&E.cf[0][0])[i] = 0.f;
      const float mylam = own ? E.rLam[l] : 0.f;
      const bool fin = (l >= 18) || isfinite(nu_new);
      if ((uint32_t)(__ballot(!fin) >> (32 * half)) != 0u && l == 0) E.bad = 1;
      __syncthreads();
      if (own) {
        E.lamst[E.rlam[l]] = mylam;
        if (last_sub && l < 3 * E.npts) {
          const ContactC& C = E.ct[l / 3];
          const int bP = C.bP, bN = C.bN;
          const f3 d = ld3(C.dir[l % 3]);
          const float s = mylam * inv_dt;
          atomicAdd(&E.cf[bP][0], d.x * s);
          atomicAdd(&E.cf[bP][1], d.y * s);
          atomicAdd(&E.cf[bP][2], d.z * s);
          if (bN >= 0) {
            atomicAdd(&E.cf[bN][0], -d.x * s);
            atomicAdd(&E.cf[bN][1], -d.y * s);
            atomicAdd(&E.cf[bN][2], -d.z * s);
          }
        }
      }
      if (l < 18) E.nu[od] = nu_new;
    }
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
          const float zq = dq3 * Q[2] + dq0 * Q[1] - dq1 * Q[0] + dq2 * Q[3];
          const float w = dq3 * Q[3] - dq0 * Q[0] - dq1 * Q[1] - dq2 * Q[2];
          const float inv = rsqrtf(x * x + y * y + zq * zq + w * w);
          Q[0] = x * inv; Q[1] = y * inv; Q[2] = zq * inv; Q[3] = w * inv;
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
    // per-env rows [e][48]: lanes 0..11 of the wave's two envs store 384 contiguous bytes
    *reinterpret_cast<float4*>(S.obs_noise + (size_t)e * 48 + 4 * l) = make_float4(z4[0], z4[1], z4[2], z4[3]);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *S.noise_counter = step_counter + 1;
  const bool bad = E.bad != 0;
  if (l < 6) E.nu[l] = E.root[7 + l];
  if (l < 12) E.nu[6 + l] = E.qd[l];
  __syncthreads();
  kin_scan(E, load_model_lane(M, l), l, gz, false);
  __syncthreads();
  // stage the [13][13] rigid states and [13][3] contact forces in LDS, then store them as SoA rows
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
  if (l == 0) S.env_rows[e] = E.nrows;  // the next step's wave balancing
  if (l == 0 && E.drop != 0) S.rows_dropped[e] += E.drop;
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
  // SoA rows: each store instruction writes 32 fields x the wave's two adjacent envs; the
  // XCD-aware env mapping keeps a line's 32 envs on one L2, where the pieces merge
  for (int i = l; i < 13 * 13; i += 32) S.rigid[(size_t)i * np + e] = E.u.out.rigid[i];
  for (int i = l; i < 13 * 3; i += 32) S.contact[(size_t)i * np + e] = E.u.out.cf[i];
  if (l < 13) S.root[l * np + e] = E.root[l];
  if (l < 12) {
    S.dof_pos[l * np + e] = E.q[l];
    S.dof_vel[l * np + e] = E.qd[l];
    S.torques[l * np + e] = E.tau[l];
  }
  for (int i = l; i < HG_LAMW; i += 32) S.lambda[i * np + e] = E.lamst[i];
}

extern "C" int hg_launch_step(const HgState* S, const hg_cfg* hcfg, const float* actions, uint64_t step_counter,
                              hipStream_t stream) {
  const int grid = (S->n + 1) / 2;  // env pairs (env_order: rebuilt by the post launch, hg_envlogic.hip)
  StepParams P;
  P.dt = hcfg->sim_dt;
  P.gz = hcfg->gravity_z;
  P.contact_offset = hcfg->contact_offset;
  P.vmax = hcfg->max_depenetration_vel;
  P.beta = hcfg->baumgarte;
  P.ground_friction = hcfg->ground_friction;
  P.decimation = hcfg->decimation;
  P.pgs_iterations = hcfg->pgs_iterations;
  P.heightfield_on = hcfg->terrain_type != 0 && hcfg->heightfield != nullptr;
  P.hf_rows = hcfg->hf_rows;
  P.hf_cols = hcfg->hf_cols;
  P.hs = hcfg->hf_horizontal_scale;
  P.vs = hcfg->hf_vertical_scale;
  P.border = hcfg->hf_border;
  P.hf = hcfg->heightfield;
  if (hcfg->fix_base_link)
    hipLaunchKernelGGL(k_step<true>, dim3(grid), dim3(64), 0, stream, *S, actions, step_counter, P);
  else
    hipLaunchKernelGGL(k_step<false>, dim3(grid), dim3(64), 0, stream, *S, actions, step_counter, P);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
